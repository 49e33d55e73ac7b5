"""Count slow-path events / appends / flushes of the per-lane screen policy
for one wave (32 users x 2 lanes) on the bench workload (dev tool)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "news-recommendation-tc_amd"), REPO]
import numpy as np
import bench
from oracle import oracle

I, K, CL = 364047, 31, 64
wl = bench.recall_workload(23, 250000, I, 32, "cpu")
g = lambda k: wl[k].numpy()
U0 = int(os.environ.get("U0", 0))
users = oracle.tower_user(g("user_table"), g("item_table"), g("uid")[U0:U0+32], g("hist")[U0:U0+32], g("hist_len")[U0:U0+32], g("w0"), g("b0"), g("w1"), g("b1"))
items = oracle.tower_item(g("item_table"), np.arange(I))
def f16(x): return x.astype(np.float16).astype(np.float32)
S = f16(users) @ f16(items).T  # approx scores [32, I]
eps = (2**-10 + 2**-20) * np.linalg.norm(users, axis=1) * np.linalg.norm(items, axis=1).max()
nb = I // 32
S = S[:, : nb * 32].reshape(32, nb, 32)
r = np.arange(16)
rows_h = [((r & 3) + 8 * (r >> 2) + 4 * h) for h in (0, 1)]
lane_scores = np.concatenate([S[:, :, rows_h[0]], S[:, :, rows_h[1]]], 0)  # [64, nb, 16]
lane_eps = np.concatenate([eps, eps])
warm = int(os.environ.get("WARM", 0))
tau = np.full(64, -np.inf, np.float32)
if warm:
    samp = lane_scores[:, :: max(1, nb // warm), :].reshape(64, -1)
    th = -np.sort(-samp, 1)[:, K - 1]
    tau = (th - 2 * lane_eps).astype(np.float32)
lists = [[] for _ in range(64)]
slow = flushes = appends = 0
for t in range(nb):
    sc = lane_scores[:, t, :]
    hit = (sc > tau[:, None])
    if hit.any():
        slow += 1
        if any(len(l) > CL - 16 for l in lists):
            flushes += 1
            for L in range(64):
                if len(lists[L]) >= K:
                    v = np.sort(np.array(lists[L]))[::-1]
                    th = v[K - 1]; cut = th - 2 * lane_eps[L]
                    tau[L] = max(tau[L], cut)
                    lists[L] = [x for x in lists[L] if x >= cut]
        for L in np.nonzero(hit.any(1))[0]:
            new = sc[L][hit[L]]
            appends += len(new)
            lists[L].extend(new.tolist())
print(f"warm={warm} tiles={nb} slow={slow} ({slow/nb:.3f}) flushes={flushes} appends/lane={appends/64:.1f} final list mean={np.mean([len(l) for l in lists]):.1f} max={max(len(l) for l in lists)}")
