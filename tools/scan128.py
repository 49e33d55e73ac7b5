"""Dev tool: the config-5 recall screen alone (D = 128, random unit vectors,
5M items, --users users): HIP events around nrk_ip_topk_scan / _select /
_finish, and a checksum of the rows (compare across builds)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "news-recommendation-tc_amd"), REPO]
import torch  # noqa: E402

from nrk import ops  # noqa: E402

U = int(sys.argv[1]) if len(sys.argv) > 1 else 250_000
I, D, K = 5_000_000, 128, 31
g = torch.Generator(device="cuda").manual_seed(5)
users = torch.nn.functional.normalize(torch.randn(U, D, device="cuda", generator=g), dim=1).contiguous()
items = torch.nn.functional.normalize(torch.randn(I, D, device="cuda", generator=g), dim=1).contiguous()
cat = ops.Catalog(items)
ws = ops.ip_topk_workspace(U, cat, K, "cuda")
s = torch.empty((U, K), dtype=torch.float32, device="cuda")
r = torch.empty((U, K), dtype=torch.int32, device="cuda")
ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
t = []
for rep in range(4):
    ev[0].record()
    ops.ip_topk_scan(users, cat, K, ws)
    ev[1].record()
    ops.ip_topk_select(users, cat, K, ws)
    ev[2].record()
    ops.ip_topk_finish(users, cat, K, ws, s, r)
    ev[3].record()
    torch.cuda.synchronize()
    if rep:
        t.append([ev[i].elapsed_time(ev[i + 1]) for i in range(3)])
t = torch.tensor(t).mean(0).tolist()
fl = 2.0 * U * I * D
print(f"D=128 U={U}: scan {t[0]:.2f} ms ({fl / t[0] / 1e9:.0f} TFLOP/s = {fl / t[0] / 1e9 / 2500:.3f} of 2.5 PF), "
      f"select {t[1]:.2f} ms, finish {t[2]:.2f} ms; rows checksum {int(r.long().sum())}")
