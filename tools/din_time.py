"""Time DIN config-3 passes (dev tool, for comparing libnrk builds via
NRK_LIB_PATH): python tools/din_time.py [passes]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "news-recommendation-tc_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from nrk import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
n, T, B = bench.DIN_SAMPLES, 50, 4096
sd, feats, enc, dev = bench.din_workload(101, n, T, "cuda")
p = ops.DinParams(sd, *feats, table_dtype="bf16", device="cuda")
ws = ops.din_workspace(p, n, T, "cuda", batch_size=B)
probs = torch.empty(n, dtype=torch.float32, device="cuda")
full = tuple(dev[k] for k in ("user", "item", "hist", "ctx", "mask"))
for _ in range(2):
    ops.din_forward(p, *full, workspace=ws, out=probs, validate=False, batch_size=B)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    ops.din_forward(p, *full, workspace=ws, out=probs, validate=False, batch_size=B)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
print(f"{os.environ.get('NRK_LIB_PATH', 'default')}: {ms:.3f} ms/pass {n / ms / 1e3:.2f}M pairs/s "
      f"checksum {float(probs.double().sum()):.9f}")
