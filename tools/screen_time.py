"""Time the config-2 screen (and finish) for the variant selected by
NRK_SCREEN_VARIANT, and print a checksum of the top-31 rows (dev tool)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "news-recommendation-tc_amd"), REPO]
import torch  # noqa: E402

import bench  # noqa: E402
from nrk import ops  # noqa: E402

dev = torch.device("cuda", 0)
U, I, D, K = 250_000, 364_047, 32, 31
wl = bench.recall_workload(23, U, I, D, dev)
iv = ops.tt_item_fwd(wl["item_table"], torch.arange(I, dtype=torch.int32, device=dev))
cat = ops.Catalog(iv)
u = ops.tt_user_fwd(wl["user_table"], wl["item_table"], wl["uid"], wl["hist"], wl["hist_len"], wl["w0"], wl["b0"],
                    wl["w1"], wl["b1"])
ws = ops.ip_topk_workspace(U, cat, K, dev)
s = torch.empty((U, K), dtype=torch.float32, device=dev)
r = torch.empty((U, K), dtype=torch.int32, device=dev)
for _ in range(2):
    ops.ip_topk_screen(u, cat, K, ws)
    ops.ip_topk_finish(u, cat, K, ws, s, r)
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
reps = 10
t_s = t_f = 0.0
for _ in range(reps):
    ev[0].record()
    ops.ip_topk_screen(u, cat, K, ws)
    ev[1].record()
    ops.ip_topk_finish(u, cat, K, ws, s, r)
    ev[2].record()
    torch.cuda.synchronize()
    t_s += ev[0].elapsed_time(ev[1])
    t_f += ev[1].elapsed_time(ev[2])
chk = int((r.long() * torch.arange(1, K + 1, device=dev)).sum().item())
print(f"variant {os.environ.get('NRK_SCAN_VARIANT', '0')}: screen {t_s / reps:.3f} ms, finish {t_f / reps:.3f} ms, "
      f"rows checksum {chk}")
