#!/usr/bin/env python3
"""dev: phase cycles of the config-2 scan from a stamp build
(make -C news-recommendation-tc_amd dev DEVDIR=build_st DEVFLAGS=-DNRK_SCAN_STAMP=1),
for the first wave of each stagger half.  NRK_LIB_PATH=.../build_st/libnrk.so
python3 tools/scan_stamps.py.  Slots (ip_topk.hip SC_STAMP): 0 vmcnt wait,
1 barrier, 2 issue + tile (late half: issue + ballots), 3 appends, 4 inserts
(late half: inserts + its tile)."""
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
L = _lib.lib()
assert L.nrk_dev_scan_stamps(buf) == 0
st = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 16).astype(np.float64)
nwg = int((st.sum(1) > 0).sum())
names = ["vmcnt wait", "barrier", "issue + tile", "appends", "inserts"]
for half, label in ((0, "wave 0 (books after its tile)"), (8, "wave NW/2 (books one tile late)")):
    x = st[:nwg, half:half + 8]
    tot = x.sum(1)
    print(f"{label}: workgroups {nwg}; cycles: mean {tot.mean():.0f} min {tot.min():.0f} max {tot.max():.0f}")
    for i, n in enumerate(names):
        print(f"  {n:18s} {x[:, i].mean():12.0f} {100 * x[:, i].mean() / tot.mean():6.1f}%")
