"""One-GPU replay of the catalog-sharded recall (BASELINE config 4) with the
owner refine (nrk.dist.owner_replay) (dev tool).

For 250k users x 364,047 items (D = 32, k = 31): the unsharded screen +
finish, then N emulated ranks on one GPU.  Per rank: the screen of its tile
range for every user (+ the bound), the band pack after the bound exchange,
and the owner refine of its user block -- HIP events around each rank's own
kernels, so "per rank" = what one GPU of an N-GPU node would run (the
collectives are not in these numbers).  Checks the result against the
unsharded rows.  usage: python tools/catalog_replay.py [N | RxC]

RxC: the 2-D layout (nrk.dist.layout_2d): R user groups x C catalog shards,
R C ranks; rank (g, c) screens group g's users over catalog shard c and
refines its 1/C of group g's users.
"""
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "news-recommendation-tc_amd"), REPO):
    sys.path.insert(0, p)

import torch  # noqa: E402

from nrk import ops  # noqa: E402
from nrk.dist import HipRangeShard, owner_replay, shard_blocks  # noqa: E402


def main():
    arg = sys.argv[1] if len(sys.argv) > 1 else "8"
    R, C = (int(x) for x in arg.split("x")) if "x" in arg else (1, int(arg))
    N = R * C
    U, I, D, K = 250_000, 364_047, 32, 31
    g = torch.Generator(device="cuda").manual_seed(23)
    users = torch.nn.functional.normalize(torch.relu(torch.randn(U, D, device="cuda", generator=g)), dim=1).contiguous()
    items = torch.nn.functional.normalize(torch.randn(I, D, device="cuda", generator=g), dim=1).contiguous()
    cat = ops.Catalog(items)
    ws = ops.ip_topk_workspace(U, cat, K, "cuda")
    s1 = torch.empty((U, K), dtype=torch.float32, device="cuda")
    r1 = torch.empty((U, K), dtype=torch.int32, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for rep in range(3):
        ev[0].record()
        ops.ip_topk_screen(users, cat, K, ws)
        ev[1].record()
        ops.ip_topk_finish(users, cat, K, ws, s1, r1)
        ev[2].record()
        torch.cuda.synchronize()
    t_scr, t_fin = ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])
    print(f"unsharded: screen {t_scr:.3f} ms, finish {t_fin:.3f} ms, total {t_scr + t_fin:.3f} ms")
    ws1 = ws
    tb = ops.ip_topk_tile_blocks(D)
    from nrk.dist import shard_range

    groups = [shard_range(U, R, gi) for gi in range(R)]  # user groups
    shards = [[HipRangeShard(cat, *shard_blocks(I, C, c, tb), K, hi - lo) for c in range(C)] for lo, hi in groups]
    times = defaultdict(float)

    def timer(phase, r, fn):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        out = fn()
        b.record()
        torch.cuda.synchronize()
        times[(phase, r)] += a.elapsed_time(b)
        return out

    def acnt_stats(ws, n):
        a = lambda x: (x + 255) & ~255  # noqa: E731
        off = 256 + a(8 * n) + 3 * a(4 * n) + a(16 * n)
        ac = ws[off: off + 8 * n].view(torch.int32).view(n, 2).sum(1).float()
        return f"appended maxima per user: mean {ac.mean().item():.1f}, p99 {ac.quantile(0.99).item():.0f}, " \
               f"max {ac.max().item():.0f}"

    print("unsharded", acnt_stats(ws1, U))

    def replay(tm=None):
        outs = []
        for gi, (lo, hi) in enumerate(groups):
            t_g = None if tm is None else (lambda ph, c, fn, gi=gi: tm(ph, gi * C + c, fn))
            outs.append(owner_replay(users[lo:hi].contiguous(), shards[gi], K, timer=t_g))
        return tuple(torch.cat([o[i] for o in outs]) for i in range(3))

    replay()  # warm-up
    print("shard 0", acnt_stats(shards[0][0].ws, groups[0][1] - groups[0][0]))
    times.clear()
    reps = 3
    for _ in range(reps):
        s, r, e = replay(timer)
    torch.cuda.synchronize()
    worst = 0.0
    print(f"layout {R} user group(s) x {C} catalog shard(s) = {N} ranks")
    for k in range(N):
        t = {ph: times[(ph, k)] / reps for ph in ("screen", "band", "refine")}
        tot = sum(t.values())
        worst = max(worst, tot)
        print(f"rank {k} (group {k // C}, shard {k % C}): screen+bound {t['screen']:.3f} ms, band pack "
              f"{t['band']:.3f} ms, owner refine {t['refine']:.3f} ms, total {tot:.3f} ms")
    print(f"max per-rank compute {worst:.3f} ms against {t_scr + t_fin:.3f} ms unsharded "
          f"(x{(t_scr + t_fin) / worst:.2f}, collectives not included)")
    print("owner rows == unsharded:", bool(torch.equal(r, r1)), " scores:", bool(torch.equal(s, s1)))


if __name__ == "__main__":
    main()
