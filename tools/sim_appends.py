"""Dev model (not product): the scan's per-lane lists and appends in numpy,
for 128 config-2 users (fp32 scores; eps taken as 0), to price list policies
before building them: the one-pass list ("cur") against a sampled pre-pass of
W tiles that only feeds the lists (ip_scan_kernel's n_pre).  Prints appended
half-block maxima per user and inserts per lane, for the whole catalog and for
one config-4 shard (1/8 of the tiles)."""
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "news-recommendation-tc_amd"), REPO]
import numpy as np
import bench
from oracle import oracle
U = 128
wl = bench.recall_workload(23, 250000, 364047, 32, "cpu")
g = lambda k: wl[k].numpy()
users = oracle.tower_user(g("user_table"), g("item_table"), g("uid")[:U], g("hist")[:U], g("hist_len")[:U], g("w0"), g("b0"), g("w1"), g("b1"))
items = oracle.tower_item(g("item_table"), np.arange(364047))
I = items.shape[0]; nb = (I + 31) // 32; nb4 = (nb // 4) * 4
S = (users.astype(np.float32) @ items.astype(np.float32).T)
S = np.pad(S, ((0, 0), (0, nb * 32 - I)), constant_values=-np.inf)[:, :nb4 * 32]
r = np.arange(32); half = ((r // 4) % 2)
Sb = S.reshape(U, nb4, 32)
hb = np.stack([Sb[:, :, half == h].max(2) for h in (0, 1)], 1)  # U, 2, nblk
T = nb4 // 4
hbt = hb.reshape(U, 2, T, 4)
MT = 16
def run(t_lo, t_hi, policy, W=32):
    apps = np.zeros(U)
    for u in range(U):
        lst = [np.full(MT, -np.inf), np.full(MT, -np.inf)]
        tau = -np.inf
        def ins(h, v):
            l = lst[h]
            if v > l[-1]:
                l[-1] = v; l.sort(); lst[h] = l[::-1].copy()
        def retau():
            return min(lst[0][-1], lst[1][-1])
        start = t_lo
        if policy in ("blk", "tile"):
            for t in range(t_lo, min(t_lo + W, t_hi)):
                for h in (0, 1):
                    if policy == "blk":
                        for b in range(4): ins(h, hbt[u, h, t, b])
                    else:
                        ins(h, hbt[u, h, t].max())
            tau = retau()
            # append-only over the warm-up range
            for t in range(t_lo, min(t_lo + W, t_hi)):
                apps[u] += (hbt[u, :, t] >= tau).sum()
            start = min(t_lo + W, t_hi)
        for t in range(start, t_hi):
            apps[u] += (hbt[u, :, t] >= tau).sum()
            for h in (0, 1): ins(h, hbt[u, h, t].max())
            tau = retau()
    return apps.mean()


def run1(t_lo, t_hi):
    """the one-pass list: appends vs tau, then the tile max enters"""
    apps = np.zeros(U)
    for u in range(U):
        lst = [np.full(MT, -np.inf), np.full(MT, -np.inf)]
        tau = -np.inf
        for t in range(t_lo, t_hi):
            apps[u] += (hbt[u, :, t] >= tau).sum()
            for h in (0, 1):
                v = hbt[u, h, t].max()
                if v > lst[h][-1]:
                    lst[h][-1] = v
                    lst[h] = np.sort(lst[h])[::-1].copy()
            tau = min(lst[0][-1], lst[1][-1])
    return apps.mean()


def run2(t_lo, t_hi, policy, W):
    apps = np.zeros(U); ins_n = np.zeros(U)
    n = t_hi - t_lo; stride = max(1, n // W)
    samp = set(range(t_lo, t_hi, stride)[:W])
    for u in range(U):
        lst = [np.full(MT, -np.inf), np.full(MT, -np.inf)]
        def ins(h, v):
            l = lst[h]
            if v > l[-1]:
                l[-1] = v; l.sort(); lst[h] = l[::-1].copy(); return 1
            return 0
        for t in sorted(samp):
            for h in (0, 1):
                if policy == "blk":
                    for b in range(4): ins(h, hbt[u, h, t, b])
                else: ins(h, hbt[u, h, t].max())
        tau = min(lst[0][-1], lst[1][-1])
        for t in range(t_lo, t_hi):
            apps[u] += (hbt[u, :, t] >= tau).sum()
            if t in samp: continue
            for h in (0, 1): ins_n[u] += ins(h, hbt[u, h, t].max())
            tau = min(lst[0][-1], lst[1][-1])
    return apps.mean(), ins_n.mean()

for name, lo, hi in (("full", 0, T), ("shard", 0, T // 8)):
    print(name, "one-pass: appends/user", round(run1(lo, hi), 1), flush=True)
    for W in (32, 64):
        a, i = run2(lo, hi, "tile", W)
        print(name, f"pre-pass {W}: appends/user", round(a, 1), "inserts/lane", round(i / 2, 1), flush=True)
