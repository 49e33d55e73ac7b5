"""numpy model: an i8 screen against today's fp16 screen at config 2 (dev tool).

Asked by the round-5 verdict before any i8 kernel is built: the i8 error
bound eps, the band (half-blocks whose screened maximum reaches theta - 2 eps),
the refine's prefilter survivors and the appended maxima, per user, for the
bench's own workload (reference-init towers, 250k x 364,047, D = 32, k + 1 = 31).

fp16: both sides scaled by powers of two into [2^13, 2^14), fp32 accumulation;
eps = ||du|| max||v|| + ||u|| max||dv|| + ||du|| max||dv|| + (2^-15 + D 2^-23)
||u|| max||v||  (ip_topk.hip scan_user_setup).
i8: users scaled per user to max |u| -> 127, the catalog by one global scale
to max |v| -> 127 (the MFMA sums exact int32 products: no accumulation term);
eps = ||du|| max||v|| + ||u|| max||dv|| + ||du|| max||dv||.

Half-block h of block b = items 32 b + (r & 3) + 8 (r >> 2) + 4 h (the MFMA
accumulator layout).  theta = the k-th largest half-block maximum (what the
select finds), cut = theta - 2 eps, band = half-blocks with maximum >= cut,
survivors = band items with a screened score >= cut; appends ~ half-block
maxima >= lb - 2 eps, lb ~ the 32nd largest half-block maximum (the final
list bound of the one-pass scan, without its warm-up).
usage: python tools/sim_i8.py [n_users]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "news-recommendation-tc_amd"), REPO]
import numpy as np  # noqa: E402

import bench  # noqa: E402
from oracle import oracle  # noqa: E402

U = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
K = 31
wl = bench.recall_workload(23, 250000, 364047, 32, "cpu")
g = lambda k: wl[k].numpy()  # noqa: E731
sel = np.arange(0, 250000, 250000 // U)[:U]
users = oracle.tower_user(g("user_table"), g("item_table"), g("uid")[sel], g("hist")[sel], g("hist_len")[sel],
                          g("w0"), g("b0"), g("w1"), g("b1"))
items = oracle.tower_item(g("item_table"), np.arange(364047))
I, D = items.shape
nblk = (I + 31) // 32
pad = np.zeros((nblk * 32 - I, D), np.float32)
itp = np.concatenate([items, pad])
r = np.arange(16)
hb_rows = np.array([32 * b + (r & 3) + 8 * (r >> 2) + 4 * h for b in range(nblk) for h in (0, 1)])  # [2 nblk, 16]
valid = hb_rows < I
live = np.linalg.norm(users, axis=1) > 0
print(f"{U} users sampled ({live.sum()} nonzero), catalog {I} x {D}")


def pow2(m):
    e = np.frexp(m)[1]
    return np.ldexp(1.0, 14 - e)


ex = users.astype(np.float64) @ itp.astype(np.float64).T  # exact
vn = np.linalg.norm(items.astype(np.float64), axis=1).max()
res = {}
for mode in ("fp16", "i8"):
    if mode == "fp16":
        sv = pow2(np.abs(items).max())
        vq = (itp * sv).astype(np.float16).astype(np.float64) / sv
        su = pow2(np.abs(users).max(1, keepdims=True))
        uq = (users * su).astype(np.float16).astype(np.float64) / su
        acc = (2.0 ** -15 + D * 2.0 ** -23)
    else:
        sv = 127.0 / np.abs(items).max()
        vq = np.rint(itp * sv) / sv
        su = 127.0 / np.maximum(np.abs(users).max(1, keepdims=True), 1e-30)
        uq = np.rint(users * su) / su
        acc = 0.0
    S = uq @ vq.T
    dv = np.linalg.norm(vq[:I] - items, axis=1).max()
    du = np.linalg.norm(uq - users, axis=1)
    un = np.linalg.norm(users, axis=1)
    eps = du * vn + un * dv + du * dv + acc * un * vn
    assert (np.abs(S - ex)[:, :I].max(1) <= eps + 1e-12).all(), "eps bound violated"
    Sh = np.where(valid[None], S[:, hb_rows], -np.inf)  # [U, 2 nblk, 16]
    hbm = Sh.max(2)
    srt = -np.sort(-hbm, axis=1)
    theta = srt[:, K - 1]
    cut = theta - 2 * eps
    band = (hbm >= cut[:, None]).sum(1)
    surv = ((Sh >= cut[:, None, None]) & (hbm >= cut[:, None])[:, :, None]).sum((1, 2))
    lb = srt[:, 31]
    app = (hbm >= (lb - 2 * eps)[:, None]).sum(1)
    exs = -np.sort(-ex[:, :I], axis=1)
    exact_surv = (ex[:, :I] >= (cut + eps)[:, None]).sum(1)
    m = live
    res[mode] = dict(eps=eps[m].mean() / un[m].mean(), band=band[m].mean(), band_max=band[m].max(),
                     surv=surv[m].mean(), exact=exact_surv[m].mean(), app=app[m].mean(),
                     over288=(band[m] > 288).mean(), over96=(band[m] > 96).mean())
    print(f"{mode:5s} eps/||u|| {res[mode]['eps']:.2e}  band {res[mode]['band']:.1f} (max {res[mode]['band_max']}, "
          f">96 {res[mode]['over96']:.3f}, >288 {res[mode]['over288']:.3f})  prefilter survivors "
          f"{res[mode]['surv']:.1f}  exact >= cut+eps {res[mode]['exact']:.1f}  appends(final-lb model) "
          f"{res[mode]['app']:.1f}  k-th exact score {exs[m, K - 1].mean():.4f}")
print(f"i8 / fp16: band x{res['i8']['band'] / res['fp16']['band']:.2f}, survivors x"
      f"{res['i8']['surv'] / res['fp16']['surv']:.2f}, appends x{res['i8']['app'] / res['fp16']['app']:.2f}")
