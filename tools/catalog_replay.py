"""One-GPU replay of the catalog-sharded recall (BASELINE config 4) (dev tool).

Times, for 250k users x 364,047 items (D = 32, k = 31): the unsharded screen
and refine, then each of N shards' screen, refine without the bound exchange
and refine with it (the all_reduce(MAX) replayed as a max over the shards'
bounds), and checks the merged result against the unsharded one.
usage: python tools/catalog_replay.py [N]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "news-recommendation-tc_amd"), REPO):
    sys.path.insert(0, p)

import torch  # noqa: E402

from nrk import ops  # noqa: E402
from nrk.dist import HipShard, bound_width, shard_range  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        out = fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps, out


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    U, I, D, K = 250_000, 364_047, 32, 31
    g = torch.Generator(device="cuda").manual_seed(23)
    users = torch.nn.functional.normalize(torch.relu(torch.randn(U, D, device="cuda", generator=g)), dim=1).contiguous()
    items = torch.nn.functional.normalize(torch.randn(I, D, device="cuda", generator=g), dim=1).contiguous()
    full = HipShard(ops.Catalog(items), 0, K, U)
    t_scr, _ = timed(lambda: full.screen(users, 1))
    t_ref, (e1, r1) = timed(lambda: full.finish(users))
    r1 = r1.clone()
    print(f"unsharded: screen {t_scr:.3f} ms, refine {t_ref:.3f} ms")
    shards = [HipShard(ops.Catalog(items[lo:hi].contiguous()), lo, K, U)
              for lo, hi in (shard_range(I, N, r) for r in range(N))]
    m = bound_width(K, N)
    rows = []
    for i, sh in enumerate(shards):
        ts, b = timed(lambda: sh.screen(users, m))
        tr0, _ = timed(lambda: sh.finish(users))
        rows.append((ts, tr0, b.clone()))
    gb = torch.stack([r[2] for r in rows]).contiguous()
    lists = []
    for i, sh in enumerate(shards):
        def both():
            sh.screen(users, m)
            return sh.finish(users, gb)
        tsb, out = timed(both)
        lists.append((out[0].clone(), out[1].clone()))
        ts, tr0, _ = rows[i]
        kept = int((out[1] >= 0).sum())
        print(f"shard {i}: screen {ts:.3f} ms, refine {tr0:.3f} ms (own bound) / {tsb - ts:.3f} ms (global bound), "
              f"kept entries {kept / U:.2f} per user")
    s, r, e = ops.topk_merge(torch.stack([x[0] for x in lists]).contiguous(),
                             torch.stack([x[1] for x in lists]).contiguous(), K)
    torch.cuda.synchronize()
    print("merged == unsharded:", bool(torch.equal(r, r1)))


if __name__ == "__main__":
    main()
