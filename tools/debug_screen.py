"""Diagnostics for the ip_topk screen on the bench workload (dev tool)."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "news-recommendation-tc_amd"), REPO]
import numpy as np, torch
import bench
from nrk import ops

dev = torch.device("cuda", 0)
U, I, D, K = int(os.environ.get("U", 250000)), 364047, 32, 31
wl = bench.recall_workload(23, U, I, D, dev)
iv = ops.tt_item_fwd(wl["item_table"], torch.arange(I, dtype=torch.int32, device=dev))
cat = ops.Catalog(iv)
u = ops.tt_user_fwd(wl["user_table"], wl["item_table"], wl["uid"], wl["hist"], wl["hist_len"], wl["w0"], wl["b0"], wl["w1"], wl["b1"])
un = u.cpu().numpy()
print("zero users", float((np.abs(un).sum(1) == 0).mean()), "mean nnz", float((un != 0).sum(1).mean()))
print("nnz hist", np.bincount((un != 0).sum(1), minlength=33))
ws = ops.ip_topk_workspace(U, cat, K, dev)
torch.cuda.synchronize(); t = time.time()
ops.ip_topk_screen(u, cat, K, ws); torch.cuda.synchronize()
print("screen s", time.time() - t)
w = ws.cpu().numpy()
ovf = w[:4].view(np.int32)[0]
cw = 48
off = 256
cand_bytes = ((U * 2 * cw * 8 + 255) // 256) * 256
ucb = ((U * 8 + 255) // 256) * 256
cnt = w[off + cand_bytes + ucb: off + cand_bytes + ucb + U * 2 * 4].view(np.int32).reshape(U, 2)
print("ovf users", ovf, "cand per user mean", cnt.sum(1).mean(), "max", cnt.sum(1).max())
print("cnt hist", np.bincount(cnt.sum(1))[:100])
s = torch.empty((U, K), dtype=torch.float32, device=dev); r = torch.empty((U, K), dtype=torch.int32, device=dev)
t = time.time(); ops.ip_topk_finish(u, cat, K, ws, s, r); torch.cuda.synchronize(); print("finish s", time.time() - t)
# score gap stats
e = s.cpu().numpy()
print("top1 mean", e[:, 0].mean(), "k-th mean", e[:, -1].mean(), "gap k-1..k mean", (e[:, -2] - e[:, -1]).mean())
