"""Dev profiling driver (not product): the config-3 DIN pass (bench.din_workload,
675,653 samples, Dice batches of 4096, bf16 tables) run --iters times, for
rocprofv3 --kernel-trace --stats; prints the mean pass time (HIP events)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "news-recommendation-tc_amd"), REPO]
import bench  # noqa: E402
from nrk import ops  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda")
    n, T, B = bench.DIN_SAMPLES, 50, 4096
    sd, feats, enc, d = bench.din_workload(101, n, T, dev)
    p = ops.DinParams(sd, *feats, table_dtype="bf16", device=dev)
    ws = ops.din_workspace(p, n, T, dev, batch_size=B)
    out = torch.empty(n, dtype=torch.float32, device=dev)
    args = tuple(d[k] for k in ("user", "item", "hist", "ctx", "mask"))
    for _ in range(2):
        ops.din_forward(p, *args, workspace=ws, out=out, validate=False, batch_size=B)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * iters)]
    for i in range(iters):
        ev[2 * i].record()
        ops.din_forward(p, *args, workspace=ws, out=out, validate=False, batch_size=B)
        ev[2 * i + 1].record()
    torch.cuda.synchronize()
    ms = [ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(iters)]
    print(f"DIN pass: {np.mean(ms):.3f} ms (min {np.min(ms):.3f}), {n / np.mean(ms) / 1e3:.1f}M pairs/s")


if __name__ == "__main__":
    main()
