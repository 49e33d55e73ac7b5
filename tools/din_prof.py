"""One DIN config-3 pass (675,653 samples, Dice batches of 4096) for
rocprofv3 counter collection (dev tool): python tools/din_prof.py [reps]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "news-recommendation-tc_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from nrk import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 1
n, T, B = bench.DIN_SAMPLES, 50, 4096
sd, feats, enc, dev = bench.din_workload(101, n, T, "cuda")
p = ops.DinParams(sd, *feats, table_dtype="bf16", device="cuda")
ws = ops.din_workspace(p, n, T, "cuda", batch_size=B)
probs = torch.empty(n, dtype=torch.float32, device="cuda")
full = tuple(dev[k] for k in ("user", "item", "hist", "ctx", "mask"))
for _ in range(reps):
    ops.din_forward(p, *full, workspace=ws, out=probs, validate=False, batch_size=B)
torch.cuda.synchronize()
print("ok", float(probs[:4096].mean()))
