"""numpy model of ip_screen's per-lane candidate logic (dev tool)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "news-recommendation-tc_amd"), REPO]
import numpy as np, torch
import bench
from oracle import oracle

U = 2000
wl = bench.recall_workload(23, 250000, 364047, 32, "cpu")
g = lambda k: wl[k].numpy()
users = oracle.tower_user(g("user_table"), g("item_table"), g("uid")[:U], g("hist")[:U], g("hist_len")[:U], g("w0"), g("b0"), g("w1"), g("b1"))
items = oracle.tower_item(g("item_table"), np.arange(364047))
print("zero users", (np.abs(users).sum(1) == 0).mean(), "nnz", np.bincount((users != 0).sum(1), minlength=33))
ub = oracle.bf16_round(users); ib = oracle.bf16_round(items)
S = (ub.astype(np.float64) @ ib.astype(np.float64).T).astype(np.float32)   # approx scores
ex = users.astype(np.float64) @ items.astype(np.float64).T
err = np.abs(S - ex).max(1)
eps = 0.00392 * np.linalg.norm(users, axis=1) * np.linalg.norm(items, axis=1).max()
print("max err / eps", (err / np.maximum(eps, 1e-30)).max())
K = 31
# per-lane: lane h gets rows with ((row % 32) // 4) % 2 == h
rows = np.arange(364047)
half = ((rows % 32) // 4) % 2
ovf = 0; band = []
for u in range(U):
    for h in (0, 1):
        s = S[u, half == h]
        srt = np.sort(s)[::-1]
        th = srt[K - 1]
        b = (s >= th - 2 * eps[u]).sum()
        band.append(b)
print("final band per lane mean", np.mean(band), "max", np.max(band), ">48:", np.sum(np.array(band) > 48))
# distribution of exact ties in approx scores near top
u = int(np.argmax(band) // 2)
print("worst user", u, "nnz", (users[u] != 0).sum(), users[u][users[u] != 0][:8], "eps", eps[u])
s = np.sort(S[u])[::-1][:80]; print(s[:40])
