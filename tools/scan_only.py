#!/usr/bin/env python3
"""dev: the config-2 recall screen alone (scan / select / finish launch times
by HIP events on the op stream), the appended maxima per user, and a digest
of the final rows + scores so builds can be compared bit for bit.

    NRK_LIB_PATH=news-recommendation-tc_amd/build_<v>/libnrk.so python3 tools/scan_only.py [--check]

Not product code: nothing under pytest / smoke() / bench.py imports it."""
import argparse
import hashlib
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "news-recommendation-tc_amd"), REPO]

import bench  # noqa: E402
from nrk import ops  # noqa: E402


def a256(x):
    return (x + 255) // 256 * 256


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=250_000)
    ap.add_argument("--items", type=int, default=364_047)
    ap.add_argument("--dim", type=int, default=32)
    ap.add_argument("--k", type=int, default=31)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--check", action="store_true", help="first 256 users against the oracle")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    wl = bench.recall_workload(23, a.users, a.items, a.dim, dev)
    item_vec = ops.tt_item_fwd(wl["item_table"], torch.arange(a.items, dtype=torch.int32, device=dev))
    cat = ops.Catalog(item_vec)
    u = ops.tt_user_fwd(wl["user_table"], wl["item_table"], wl["uid"], wl["hist"], wl["hist_len"],
                        wl["w0"], wl["b0"], wl["w1"], wl["b1"])
    U, K = a.users, a.k
    ws = ops.ip_topk_workspace(U, cat, K, dev)
    out_s = torch.empty((U, K), dtype=torch.float32, device=dev)
    out_r = torch.empty((U, K), dtype=torch.int32, device=dev)

    def run(ev=None):
        if ev:
            ev[0].record()
        ops.ip_topk_scan(u, cat, K, ws)
        if ev:
            ev[1].record()
        ops.ip_topk_select(u, cat, K, ws)
        if ev:
            ev[2].record()
        ops.ip_topk_finish(u, cat, K, ws, out_s, out_r)
        if ev:
            ev[3].record()

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(a.reps)]
    for e in evs:
        run(e)
    torch.cuda.synchronize()
    t = np.array([[e[0].elapsed_time(e[1]), e[1].elapsed_time(e[2]), e[2].elapsed_time(e[3])] for e in evs])
    # workspace: hdr 256, ucut U*8, cnt U*4, ovf_flag U*4, ovf_list U*4, uinfo U*16, acnt U*2*4
    off = 256 + a256(U * 8) + 3 * a256(U * 4) + a256(U * 16)
    acnt = ws[off:off + U * 8].view(torch.int32).view(U, 2).cpu().numpy()
    band = ws[256 + a256(U * 8):256 + a256(U * 8) + U * 4].view(torch.int32).cpu().numpy()
    dg = hashlib.sha256(out_r.cpu().numpy().tobytes() + out_s.cpu().numpy().tobytes()).hexdigest()[:16]
    print(f"scan only {t[:, 0].mean():.4f} ms (min {t[:, 0].min():.4f}) select {t[:, 1].mean():.4f} "
          f"finish {t[:, 2].mean():.4f} appended/user {acnt.sum(1).mean():.1f} (max {acnt.max()}) "
          f"band/user {band.mean():.1f} digest {dg}")
    if a.check:
        from oracle import oracle

        so, ro = oracle.ip_topk(u[:256].cpu().numpy(), item_vec.cpu().numpy(), K, nthreads=16)
        ok = np.array_equal(out_r[:256].cpu().numpy(), ro) and np.array_equal(out_s[:256].cpu().numpy(), so)
        print("oracle check (256 users):", "OK" if ok else "MISMATCH")
        if not ok:
            sys.exit(1)


if __name__ == "__main__":
    main()
