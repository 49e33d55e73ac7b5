"""Per-wave screen statistics from the NRK_SCREEN_STATS build (dev tool)."""
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
ws = torch.zeros(need + U * 4 + (U // 32 + 8) * 64 + 4096, dtype=torch.uint8, device=dev)
ops.ip_topk_screen(u, cat, K, ws); torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record(); ops.ip_topk_screen(u, cat, K, ws); ev[1].record(); torch.cuda.synchronize()
print("screen ms", ev[0].elapsed_time(ev[1]))
w = ws.cpu().numpy()
# ovf_list offset = end of required layout minus align256(U*4)
ovl = need - ((U * 4 + 255) // 256) * 256
st = w[ovl + U * 4: ovl + U * 4 + (U // 32) * 64].view(np.uint64).reshape(-1, 8)
nw = (U + 31) // 32
st = st[:nw].astype(np.float64)
for i, name in enumerate(["cyc_wait", "flush", "cyc_comp", "cyc_flush", "cyc_total"]):
    print(f"{name:10s} mean {st[:, i].mean():.4g}  max {st[:, i].max():.4g}")
print("wait frac", st[:, 0].sum() / st[:, 4].sum(), "compute frac", st[:, 2].sum() / st[:, 4].sum(), "flush frac", st[:, 3].sum() / st[:, 4].sum())
print("tiles per wave", (I + 255) // 256)
