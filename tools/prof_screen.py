"""Run only the recall screen/finish a few times (profiling driver, dev tool)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "news-recommendation-tc_amd"), REPO]
import torch
import bench
from nrk import ops

dev = torch.device("cuda", 0)
U, I, D, K = int(os.environ.get("U", 250000)), 364047, 32, 31
wl = bench.recall_workload(23, U, I, D, dev)
iv = ops.tt_item_fwd(wl["item_table"], torch.arange(I, dtype=torch.int32, device=dev))
cat = ops.Catalog(iv)
u = ops.tt_user_fwd(wl["user_table"], wl["item_table"], wl["uid"], wl["hist"], wl["hist_len"], wl["w0"], wl["b0"], wl["w1"], wl["b1"])
ws = ops.ip_topk_workspace(U, cat, K, dev)
s = torch.empty((U, K), dtype=torch.float32, device=dev); r = torch.empty((U, K), dtype=torch.int32, device=dev)
for _ in range(int(os.environ.get("REPS", 2))):
    ops.ip_topk_screen(u, cat, K, ws)
    ops.ip_topk_finish(u, cat, K, ws, s, r)
torch.cuda.synchronize()
print("done")
