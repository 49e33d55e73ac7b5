#!/usr/bin/env python3
"""dev: phase cycles of the warp-specialized config-2 scan from a stamp build
(make -C news-recommendation-tc_amd dev DEVDIR=build_wst DEVFLAGS=-DNRK_SCAN_STAMP=1);
NRK_LIB_PATH=.../build_wst/libnrk.so python3 tools/ws_stamps.py.  Slots
(ip_scan_ws_kernel): wave 0 (MFMA) 0 sync, 1 tile, 7 maxima write + issue,
2 end; wave 4 (book) 0 sync, 1 maxima read, 2 appends, 4 inserts, 5 loop."""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "news-recommendation-tc_amd"), REPO]

import bench  # noqa: E402
from nrk import _lib, ops  # noqa: E402

U, I, D, K = 250_000, 364_047, 32, 31
dev = torch.device("cuda", 0)
wl = bench.recall_workload(23, U, I, D, dev)
item_vec = ops.tt_item_fwd(wl["item_table"], torch.arange(I, dtype=torch.int32, device=dev))
cat = ops.Catalog(item_vec)
u = ops.tt_user_fwd(wl["user_table"], wl["item_table"], wl["uid"], wl["hist"], wl["hist_len"],
                    wl["w0"], wl["b0"], wl["w1"], wl["b1"])
ws = ops.ip_topk_workspace(U, cat, K, dev)
for _ in range(3):
    ops.ip_topk_scan(u, cat, K, ws)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (1024 * 16))()
assert _lib.lib().nrk_dev_scan_stamps(buf) == 0
st = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 16).astype(np.float64)
nwg = int((st.sum(1) > 0).sum())
for off, label, names in ((0, "MFMA wave 0", {0: "sync", 1: "tile", 7: "maxima write + issue", 2: "end"}),
                          (8, "book wave 4", {0: "sync", 1: "maxima read", 2: "appends", 4: "inserts", 5: "loop"})):
    x = st[:nwg, off:off + 8]
    tot = x.sum(1)
    print(f"{label}: workgroups {nwg}; cycles: mean {tot.mean():.0f} min {tot.min():.0f} max {tot.max():.0f}")
    for i, n in names.items():
        print(f"  {n:22s} {x[:, i].mean():12.0f} {100 * x[:, i].mean() / tot.mean():6.1f}%")
