"""Per-wave screen phase cycles from the NRK_SCREEN_STATS build (dev tool):
make -C news-recommendation-tc_amd stats; python tools/screen_stats.py"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["NRK_LIB_PATH"] = os.path.join(REPO, "news-recommendation-tc_amd", "build_stats", "libnrk.so")
sys.path[:0] = [os.path.join(REPO, "news-recommendation-tc_amd"), REPO]
import numpy as np, torch
import bench
from nrk import ops, _lib

dev = torch.device("cuda", 0)
U, I, D, K = int(os.environ.get("U", 250000)), 364047, 32, 31
wl = bench.recall_workload(23, U, I, D, dev)
iv = ops.tt_item_fwd(wl["item_table"], torch.arange(I, dtype=torch.int32, device=dev))
cat = ops.Catalog(iv)
u = ops.tt_user_fwd(wl["user_table"], wl["item_table"], wl["uid"], wl["hist"], wl["hist_len"], wl["w0"], wl["b0"], wl["w1"], wl["b1"])
need = _lib.lib().nrk_ip_topk_workspace_bytes(U, I, D, K)
nw = (U + 31) // 32 + 8
ws = torch.zeros(need + nw * 64 + 4096, dtype=torch.uint8, device=dev)
ops.ip_topk_screen(u, cat, K, ws); torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record(); ops.ip_topk_screen(u, cat, K, ws); ev[1].record(); torch.cuda.synchronize()
print("screen ms", ev[0].elapsed_time(ev[1]))
w = ws.cpu().numpy()
ovl = need - ((U * 4 + 255) // 256) * 256  # ovf_list is the last workspace region
st = w[ovl + U * 4: ovl + U * 4 + ((U + 31) // 32) * 64].view(np.uint64).reshape(-1, 8).astype(np.float64)
names = ["wait+barrier", "issue+tile", "append", "flush", "n_flush", "total", "n_append_tiles"]
cols = [0, 1, 3, 4, 5, 6, 7]
tot = st[:, 6].sum()
for nm, c in zip(names, cols):
    print(f"{nm:16s} mean/wave {st[:, c].mean():12.4g}  frac {st[:, c].sum() / tot:.3f}")
print("tiles per wave", (I + 127) // 128, "cycles/tile", st[:, 6].mean() / ((I + 127) // 128))
