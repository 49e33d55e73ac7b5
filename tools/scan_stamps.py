"""Dev-only: phase cycles of ip_scan_kernel (build_sstamp/libnrk.so, made
with make dev DEVDIR=build_sstamp DEVFLAGS=-DNRK_SCAN_STAMP=1): the config-2
screen once, then wave 0's shader cycles per phase, averaged over workgroups."""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "news-recommendation-tc_amd"), REPO]
import bench  # noqa: E402
from nrk import _lib, ops  # noqa: E402

NAMES = ["vmcnt wait", "barrier", "issue + tile", "appends", "inserts"]


def main():
    U, I, D, K = 250_000, 364_047, 32, 31
    dev = torch.device("cuda")
    wl = bench.recall_workload(23, U, I, D, dev)
    item_vec = ops.tt_item_fwd(wl["item_table"], torch.arange(I, dtype=torch.int32, device=dev))
    cat = ops.Catalog(item_vec)
    u = ops.tt_user_fwd(wl["user_table"], wl["item_table"], wl["uid"], wl["hist"], wl["hist_len"], wl["w0"],
                        wl["b0"], wl["w1"], wl["b1"])
    ws = ops.ip_topk_workspace(U, cat, K, dev)
    for _ in range(2):
        ops.ip_topk_scan(u, cat, K, ws)
    torch.cuda.synchronize()
    buf = np.zeros(1024 * 16, np.uint64)
    assert _lib.lib().nrk_dev_scan_stamps(buf.ctypes.data_as(ctypes.c_void_p)) == 0
    for half, name in ((0, "wave 0 (books after its tile)"), (1, "wave NW/2 (books one tile late)")):
        st = buf.reshape(1024, 2, 8)[:, half, :5]
        st = st[st.sum(1) > 0].astype(np.float64)
        tot = st.sum(1)
        print(f"{name}: workgroups {len(st)}; cycles: mean {tot.mean():.0f} min {tot.min():.0f} max {tot.max():.0f}")
        for k, nm in enumerate(NAMES):
            print(f"  {nm:14s} {st[:, k].mean():12.0f}  {100 * st[:, k].mean() / tot.mean():5.1f}%")


if __name__ == "__main__":
    main()
