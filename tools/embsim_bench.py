"""Full-size EmbeddingSimilarity timing (dev tool): 364,047 articles x 250-d
(Tianchi articles_emb shape), embedding_topk=20 -> self-search top-21."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "news-recommendation-tc_amd"))
import torch  # noqa: E402

from nrk import ops  # noqa: E402

n, d, k = int(sys.argv[1]) if len(sys.argv) > 1 else 364_047, 250, 21
g = torch.Generator(device="cuda").manual_seed(23)
x = torch.randn(n, d, device="cuda", generator=g)
ws = ops.ip_topk_workspace(n, type("C", (), {"n": n, "d": d})(), k, "cuda")
s = torch.empty((n, k), dtype=torch.float32, device="cuda")
r = torch.empty((n, k), dtype=torch.int32, device="cuda")
for it in range(3):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    ev[0].record()
    xn = ops.row_normalize(x)
    ev[1].record()
    cat = ops.Catalog(xn)
    ev[2].record()
    ops.ip_topk_screen(xn, cat, k, ws)
    ev[3].record()
    ops.ip_topk_finish(xn, cat, k, ws, s, r)
    ev[4].record()
    torch.cuda.synchronize()
    t = [ev[i].elapsed_time(ev[i + 1]) for i in range(4)]
    flop = 2.0 * n * n * d
    print(f"iter {it}: normalize {t[0]:.3f} ms, catalog {t[1]:.3f} ms, screen {t[2]:.2f} ms "
          f"({flop / t[2] / 1e9:.0f} TFLOP/s), finish {t[3]:.2f} ms, total {sum(t):.2f} ms", flush=True)
rr = r.cpu()
print("self at col0 frac:", float((rr[:, 0] == torch.arange(n, dtype=torch.int32)).float().mean()))
