#!/usr/bin/env python3
"""dev: the config-3 DIN pass as groups of G Dice batches (one
nrk_din_forward_segments call per group, groups alternating over S streams)
against the one-call pass; bit-identical outputs expected (every Dice batch
keeps its own statistics).  python3 tools/din_groups.py G[,G...] [S]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "news-recommendation-tc_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from nrk import ops  # noqa: E402

groups = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "165,32,16,8").split(",")]
n_str = int(sys.argv[2]) if len(sys.argv) > 2 else 2
reps = 10
n, T, B = bench.DIN_SAMPLES, 50, 4096
sd, feats, enc, dev = bench.din_workload(101, n, T, "cuda")
p = ops.DinParams(sd, *feats, table_dtype="bf16", device="cuda")
full = [dev[k] for k in ("user", "item", "hist", "ctx", "mask")]
ref = torch.empty(n, dtype=torch.float32, device="cuda")
ws_full = ops.din_workspace(p, n, T, "cuda", batch_size=B)
ops.din_forward(p, *full, workspace=ws_full, out=ref, validate=False, batch_size=B)
torch.cuda.synchronize()
streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(n_str - 1)]
for G in groups:
    rows = G * B
    ws = [ops.din_workspace(p, min(rows, n), T, "cuda", batch_size=B) for _ in streams]
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    chunks = [(a, min(n, a + rows)) for a in range(0, n, rows)]

    def one():
        main = torch.cuda.current_stream()
        for st in streams[1:]:
            st.wait_stream(main)
        for i, (a, b) in enumerate(chunks):
            st = streams[i % len(streams)]
            with torch.cuda.stream(st):
                ops.din_forward(p, *(t[a:b] for t in full), workspace=ws[i % len(streams)], out=out[a:b],
                                validate=False, batch_size=B)
        for st in streams:
            if st is not main:
                main.wait_stream(st)

    for _ in range(2):
        one()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        one()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    same = bool(torch.equal(out, ref))
    print(f"groups of {G:4d} batches ({len(chunks)} calls, {len(streams)} streams): {ms:.3f} ms/pass "
          f"{n / ms / 1e3:.1f}M pairs/s  bit-identical {same}", flush=True)
