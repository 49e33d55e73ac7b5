"""Shard-path statistics on one GPU (dev tool): per-shard band counts after
the bound exchange, the global bound G vs the cut, owner overflow counts."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "news-recommendation-tc_amd"), REPO]
import torch  # noqa: E402

from nrk import ops  # noqa: E402
from nrk.dist import HipRangeShard, bound_width, shard_blocks  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
U, I, D, K = 250_000, 364_047, 32, 31
g = torch.Generator(device="cuda").manual_seed(23)
users = torch.nn.functional.normalize(torch.relu(torch.randn(U, D, device="cuda", generator=g)), dim=1).contiguous()
items = torch.nn.functional.normalize(torch.randn(I, D, device="cuda", generator=g), dim=1).contiguous()
cat = ops.Catalog(items)
tb = ops.ip_topk_tile_blocks(D)
shards = [HipRangeShard(cat, *shard_blocks(I, N, r, tb), K, U) for r in range(N)]
m = bound_width(K, N)
bs = [sh.screen(users, m) for sh in shards]
bounds = torch.stack(bs).contiguous()
print("m", m, "bounds finite frac", torch.isfinite(bounds).float().mean().item())
G = bounds.permute(1, 0, 2).reshape(U, -1).sort(1, descending=True).values[:, K - 1]
for r, sh in enumerate(shards[:2]):
    c, e = sh.band(bounds)
    uc = ops.ip_topk_ucut(sh.ws, U)
    cf = c.float()
    print(f"shard {r}: band cnt mean {cf[c >= 0].mean().item():.2f}, max {c.max().item()}, overflow {(c < 0).sum().item()}, "
          f"cut >= G - eps everywhere: {bool((uc[:, 0] >= G - uc[:, 1] - 1e-6).all().item())}, "
          f"G finite {torch.isfinite(G).float().mean().item():.3f}")
    print("   sample: G", G[:4].tolist(), "cut", uc[:4, 0].tolist(), "eps", uc[:4, 1].tolist())
