"""Dev-only: phase cycles of din_att_tm_kernel (build_stamp/libnrk.so, made
with make devdin DEVDIR=build_stamp DEVFLAGS=-DNRK_TM_STAMP=1): one config-3
DIN pass, then the per-workgroup shader cycles of each phase, averaged."""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "news-recommendation-tc_amd"), REPO]
import bench  # noqa: E402
from nrk import _lib, ops  # noqa: E402

NAMES = ["plan load", "q rows", "c_b MFMA", "pad rows", "D(t)", "P(t)", "main loop", "partial row",
         " step: claim", " step: loads", " step: tile", " step: epilogue"]


def main():
    dev = torch.device("cuda")
    n, T, B = bench.DIN_SAMPLES, 50, 4096
    sd, feats, enc, d = bench.din_workload(101, n, T, dev)
    p = ops.DinParams(sd, *feats, table_dtype="bf16", device=dev)
    ws = ops.din_workspace(p, n, T, dev, batch_size=B)
    out = torch.empty(n, dtype=torch.float32, device=dev)
    args = tuple(d[k] for k in ("user", "item", "hist", "ctx", "mask"))
    for _ in range(3):
        ops.din_forward(p, *args, workspace=ws, out=out, validate=False, batch_size=B)
    torch.cuda.synchronize()
    buf = np.zeros(1024 * 12, np.uint64)
    lib = _lib.lib()
    rc = lib.nrk_dev_tm_stamps(buf.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    st = buf.reshape(1024, 12)
    st = st[st.sum(1) > 0]
    tot = st[:, :8].sum(1).astype(np.float64)
    print(f"workgroups {len(st)}; cycles per workgroup: mean {tot.mean():.0f} min {tot.min():.0f} max {tot.max():.0f}")
    for k, nm in enumerate(NAMES):
        v = st[:, k].astype(np.float64)
        print(f"  {nm:12s} {v.mean():12.0f}  {100 * v.mean() / tot.mean():5.1f}%")


if __name__ == "__main__":
    main()
