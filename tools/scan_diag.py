"""Dev diagnostic (not product): config-2 screen phases timed with HIP events,
plus the workspace's per-user append counts / overflow count (layout of
ip_ws_layout in csrc/ip_topk.hip)."""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "news-recommendation-tc_amd"), REPO]
import bench  # noqa: E402
from nrk import ops  # noqa: E402


def al(x):
    return (x + 255) & ~255


def main():
    U, I, D, K = 250_000, 364_047, 32, 31
    dev = torch.device("cuda")
    wl = bench.recall_workload(23, U, I, D, dev)
    item_vec = ops.tt_item_fwd(wl["item_table"], torch.arange(I, dtype=torch.int32, device=dev))
    cat = ops.Catalog(item_vec)
    u = ops.tt_user_fwd(wl["user_table"], wl["item_table"], wl["uid"], wl["hist"], wl["hist_len"], wl["w0"],
                        wl["b0"], wl["w1"], wl["b1"])
    ws = ops.ip_topk_workspace(U, cat, K, dev)
    s = torch.empty((U, K), dtype=torch.float32, device=dev)
    r = torch.empty((U, K), dtype=torch.int32, device=dev)
    for _ in range(3):
        ops.ip_topk_scan(u, cat, K, ws)
        ops.ip_topk_select(u, cat, K, ws)
        ops.ip_topk_finish(u, cat, K, ws, s, r)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    t = []
    for _ in range(5):
        ev[0].record()
        ops.ip_topk_scan(u, cat, K, ws)
        ev[1].record()
        ops.ip_topk_select(u, cat, K, ws)
        ev[2].record()
        ops.ip_topk_finish(u, cat, K, ws, s, r)
        ev[3].record()
        torch.cuda.synchronize()
        t.append([ev[i].elapsed_time(ev[i + 1]) for i in range(3)])
    print("scan / select / finish ms:", np.round(np.median(np.array(t), 0), 3).tolist())
    w = ws.cpu().numpy()
    ovf = int(w[:4].view(np.int32)[0])
    off = 256 + al(U * 8) + al(U * 4) * 3 + al(U * 16)
    uinfo = w[256 + al(U * 8) + al(U * 4) * 3: off].view(np.float32)[:U * 4].reshape(U, 4)
    acnt = w[off: off + U * 8].view(np.int32).reshape(U, 2)
    tot = acnt.sum(1)
    print(f"overflowed users: {ovf}; appends per user: mean {tot.mean():.1f} p50 {np.median(tot):.0f} "
          f"p99 {np.percentile(tot, 99):.0f} max {tot.max()}; per half max {acnt.max()}")
    print("uinfo lb: finite", int(np.isfinite(uinfo[:, 0]).sum()), "mean", float(np.nanmean(
        np.where(np.isfinite(uinfo[:, 0]), uinfo[:, 0], np.nan))), "eps_s mean", float(uinfo[:, 1].mean()))


if __name__ == "__main__":
    main()
