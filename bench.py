#!/usr/bin/env python3
"""bench.py -- the hot path on synthetic Tianchi-shaped data (BASELINE.json).

One "step" = one pass of the recall hot path over one batch:
  YouTubeDNN user tower for U = 250,000 users (HIP, nrk_tt_user_fwd)
  + exact top-31 inner-product search over the 364,047-item catalog, D = 32
    (HIP: fp16 MFMA screen + fp64 exact refine, nrk_ip_topk_screen/_finish),
i.e. BASELINE config 2 ("YouTubeDNN recall: 250k users x 364k items,
emb_dim=32, top-30, bf16, 1 MI355X").  The item tower + catalog build is the
index build (faiss add) and happens once, before the timed region.
value = recalled user-item pairs / s = users x 30 / step time (rank 0 of the
31 is dropped by recall(), youtubednn_recaller.py:524).

With --gpus N > 1 (torch.distributed.run, one process per GPU, RCCL) the
layouts are (layout_plan):
  * recall, headline value (default --shard users): the users are
    independent units, so every rank runs its own 250k-user problem against
    the whole (replicated, 70 MB) catalog with no data-path collective --
    weak scaling, value = N x 250k x 30 / the slowest rank's step.
  * recall, "config4" beside it (BASELINE config 4; --shard catalog makes it
    the headline): the same 250k users, the catalog's 32-item blocks split
    N-way in whole screen tiles; each rank runs the user tower for its user
    block (all_gather -> every user), screens its item range for every user,
    the ranks exchange the shard bounds (all_gather) and the band candidates
    (all_to_all to the user's owner), and each rank refines its own user
    block exactly (strong scaling: value = 250k x 30 / the slowest rank's
    step).
  * DIN = config 3: the 165 Dice batches of 4096 (last 3,909) split
    round-robin, batch b on rank b mod N (value = 675,653 / the slowest
    rank's pass).
The timed regions are bracketed by barriers and the max over ranks is used.

Extra fields on the JSON line: "roofline" for the dominant kernel (the
fp16 MFMA screen, ip_scan_ws_kernel), "cpu_baseline" (the oracle's per-user
exact scan -- the reference's nq=1 IndexFlatIP shape -- on a bounded user
sample, rank 0, N=1), "din" (BASELINE config 3, DIN scored pairs/s),
"itemcf" and "plugins" (N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(REPO, "news-recommendation-tc_amd"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "recalled pairs/sec (YouTubeDNN top-30) + DIN scored pairs/sec, 1/2/4/8 MI355X"
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


PROFILE_ROUND = "r06"
TRAFFIC_FILE = os.path.join(REPO, "profiles", PROFILE_ROUND + "_traffic.json")
BUSY_FILE = os.path.join(REPO, "profiles", PROFILE_ROUND + "_busy.json")
CSRC = os.path.join(REPO, "news-recommendation-tc_amd", "csrc")


def source_digest():
    """sha256 (16 hex) of the kernel sources the PMC files were measured on:
    tools/pmc_traffic.py / pmc_busy.py stamp it into the profile files, and
    bench.py only reports their numbers while the sources still match."""
    import hashlib

    h = hashlib.sha256()
    for f in sorted(os.listdir(CSRC)):
        if f.endswith((".hip", ".h")):
            h.update(f.encode())
            h.update(open(os.path.join(CSRC, f), "rb").read())
    return h.hexdigest()[:16]


def _profile(path):
    """A committed PMC summary, or None when absent or measured on other
    kernel sources (stale)."""
    if not os.path.exists(path):
        return None
    d = json.load(open(path))
    return d if d.get("sources") == source_digest() else None


def pmc_busy(kernels, default_config):
    """MFMA-busy / VALU-busy / stall shares of ``kernels`` from the committed
    rocprofv3 SQ-counter passes of this bench's default workloads
    (tools/pmc_busy.sh -> tools/pmc_busy.py, calibrated against the pure-MFMA /
    pure-VALU micro-kernels of tools/calib); None off the default config or
    when the file is stale."""
    b = _profile(BUSY_FILE) if default_config else None
    if b is None:
        return None
    out = {}
    for k in kernels:
        # demangled names start with k; a kernel whose name stays mangled
        # (template + lambda) contains it without the namespace
        m = [v for name, v in b["kernels"].items() if name.startswith(k) or k.replace("nrk::", "") in name]
        if m:
            out[k.replace("nrk::", "")] = {x: m[0].get(x) for x in ("mfma_busy", "valu_busy", "wait_any", "wait_inst",
                                                                     "active")}
    return out or None


def _traffic_file():
    return _profile(TRAFFIC_FILE)


def pmc_traffic(kernels, default_config):
    """HBM-side bytes per launch of ``kernels`` (summed) from the committed
    rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this bench at its default
    config (tools/pmc_traffic.py applies the gfx950 corrections); None when
    the run is not at that config or the file is absent."""
    tf = _traffic_file()
    if not default_config or tf is None:
        return None
    ks = tf["kernels"]
    tot = 0.0
    for k in kernels:
        # a name prefix ("nrk::ip_screen_kernel<32,") matches the one
        # instantiation the default config runs
        m = [v for name, v in ks.items() if name == k or name.startswith(k)]
        if len(m) != 1:
            return None
        tot += m[0]["traffic_bytes_per_launch"]
    return tot


def pmc_din_pass(default_config):
    """HBM-side bytes of one whole DIN config-3 pass (every launch of one
    nrk_din_forward_segments call), from the committed PMC passes."""
    tf = _traffic_file()
    if not default_config or tf is None or "din_pass" not in tf:
        return None
    return tf["din_pass"]["traffic_bytes"]


def max_over_ranks(x, device):
    """The max of a host float over the ranks (the slowest rank's time); gloo
    reduces a host tensor."""
    import torch.distributed as dist

    on_host = dist.get_backend() == "gloo"
    t = torch.tensor([x], dtype=torch.float64, device="cpu" if on_host else device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def log(*a):
    # one write per line: ranks share the parent's stderr and run with -u, so
    # print's separate text / newline writes could interleave between ranks
    sys.stderr.write(" ".join(str(x) for x in a) + "\n")
    sys.stderr.flush()


def recall_workload(seed: int, n_users: int, n_items: int, dim: int, device):
    from nrk.data import synth

    clog = synth.make_click_log(n_users=n_users, n_items=n_items, seed=seed)
    T = 30
    u = clog.user_id
    counts = np.bincount(u, minlength=n_users)
    offs = np.concatenate([[0], np.cumsum(counts)[:-1]])
    pos = np.arange(len(u)) - np.repeat(offs, counts)
    keep = pos < T  # the FIRST 30 rows in click_df order (youtubednn_recaller.py:65-66)
    hist = np.zeros((n_users, T), np.int32)
    hist[u[keep], pos[keep]] = clog.click_article_id[keep]
    hlen = np.minimum(counts, T).astype(np.int32)
    torch.manual_seed(23)
    # reference init (youtubednn_recaller.py:119-127): emb N(0, 0.01), xavier Linear, zero bias
    ue = torch.empty(n_users, dim).normal_(0, 0.01)
    ie = torch.empty(n_items, dim).normal_(0, 0.01)
    w0 = torch.empty(64, 2 * dim)
    torch.nn.init.xavier_uniform_(w0)
    w1 = torch.empty(dim, 64)
    torch.nn.init.xavier_uniform_(w1)
    d = lambda t: torch.as_tensor(t).to(device).contiguous()  # noqa: E731
    return {
        "user_table": d(ue), "item_table": d(ie), "uid": d(np.arange(n_users, dtype=np.int32)),
        "hist": d(hist), "hist_len": d(hlen), "w0": d(w0), "b0": d(torch.zeros(64)),
        "w1": d(w1), "b1": d(torch.zeros(dim)), "n_clicks": len(u),
    }


def cpu_baseline_recall(users_np, items_np, k, sample, threads, seconds):
    """The oracle's exact per-user scan (reference nq=1 IndexFlatIP shape),
    chunks of `sample` users until `seconds` of CPU work have been timed."""
    from oracle import oracle

    oracle.ip_topk(users_np[:8], items_np, k, nthreads=threads)  # warm
    done, dt = 0, 0.0
    while dt < seconds and done < len(users_np):
        q = users_np[done:done + sample]
        t0 = time.perf_counter()
        oracle.ip_topk(q, items_np, k, nthreads=threads)
        dt += time.perf_counter() - t0
        done += len(q)
    return done * (k - 1) / dt, dt, done


def cpu_baseline_recall_gemm(users_np, items_np, k, sample, seconds):
    """batched GEMM + top-k on torch-CPU with every host
    thread, chunks of ``sample`` users until ``seconds`` of CPU work."""
    it = torch.from_numpy(items_np)
    torch.topk(torch.from_numpy(users_np[:8]) @ it.T, k, dim=1)  # warm
    done, dt = 0, 0.0
    while dt < seconds and done < len(users_np):
        q = torch.from_numpy(users_np[done:done + sample])
        t0 = time.perf_counter()
        torch.topk(q @ it.T, k, dim=1)
        dt += time.perf_counter() - t0
        done += q.shape[0]
    return done * (k - 1) / dt, dt, done


def cpu_share():
    """Threads for the cpu_baseline legs: every CPU this process may run on
    (sched_getaffinity), capped by a cgroup CPU quota (cpu.max) and by the
    pool's OMP_NUM_THREADS -- on the MI355X pool a one-GPU box is given 16
    CPUs of a 256-CPU host whose affinity mask it shares with other jobs, so
    the affinity count alone would time contention, not the reference.
    Returns (threads, how the number was chosen)."""
    lim = [("sched_getaffinity", len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity")
            else os.cpu_count() or 1)]
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            lim.append(("cgroup cpu.max", max(1, int(q) // int(per))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        lim.append(("OMP_NUM_THREADS", int(omp)))
    t = min(v for _, v in lim)
    return t, ", ".join(f"{n} {v}" for n, v in lim)


def host_info():
    """nproc, CPU model, torch threads, GPU count."""
    model = None
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "cpu_model": model, "torch_threads": torch.get_num_threads(),
            "affinity_cpus": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None,
            "gpus_visible": torch.cuda.device_count()}


def run_plugins(args, device, u_vec, item_vec, sd, feats):
    """Plugin-level throughput: the drop-in entry points a reference user
    calls, timed end to end on the host clock (host prep, H2D, kernels, D2H,
    building the returned Python containers):
      * YoutubeDNNRecaller.batch_recall(all 250k users, topk=30) -> the
        Dict[user, List[(item, score)]] of recall/base.py:24-40;
      * DINRanker.predict() over a 675,653-row main_df (object rows, ids
        found in the dicts), batches of 4096 -> np.ndarray probabilities
        (DIN.py:1219-1283), encoding included (DinEncoder + nrk_gather_rows).
    Setup (dicts, label encoders, tables) is untimed, as the reference's
    set_data / load_model are."""
    import pandas as pd

    from nrk.config import RankConfig
    from nrk.rank.din import DINRanker
    from nrk.recall.youtubednn_recaller import YoutubeDNNRecaller

    out = {}
    U, I = u_vec.shape[0], item_vec.shape[0]
    rec = YoutubeDNNRecaller.from_embeddings(u_vec, item_vec, np.arange(U) * 3 + 1, np.arange(I) * 7 + 11,
                                             device=device)
    uids = (np.arange(U) * 3 + 1).tolist()
    rec.batch_recall(uids[:1000], topk=30)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = rec.batch_recall(uids, topk=30)
    dt = time.perf_counter() - t0
    out["batch_recall"] = {"value": round(sum(len(v) for v in res.values()) / dt, 1), "unit": "recalled pairs/s",
                           "users": U, "seconds": round(dt, 3)}
    del res

    class _Enc:
        def __init__(self, c):
            self.classes_ = c

    rng = np.random.default_rng(5)
    n, T = args.din_samples, 50
    uf, itf, cf = feats
    NU, NI = 200_000, 300_000
    uv = [rng.integers(0, v - 1, NU) for v in DIN_VOCAB_U]
    iv = [rng.integers(0, v - 1, NI) for v in DIN_VOCAB_I]
    upd = {str(u): {f: float(uv[j][u]) for j, f in enumerate(uf)} for u in range(NU)}
    ifd = {str(i): {f: int(iv[j][i]) for j, f in enumerate(itf)} for i in range(NI)}
    L = np.minimum(rng.geometric(1 / 8, NU), 200)
    uhd = {str(u): [str(x) for x in rng.integers(0, NI, L[u])] for u in range(NU)}
    enc = {f: _Enc(np.unique(uv[j].astype(float))) for j, f in enumerate(uf)}
    enc.update({f: _Enc(np.unique(iv[j])) for j, f in enumerate(itf)})
    enc.update({f: _Enc(np.arange(DIN_VOCAB_C - 1)) for f in cf})
    df = pd.DataFrame({"user_id": rng.integers(0, NU, n).astype(str), "item_id": rng.integers(0, NI, n).astype(str)})
    for f in cf:
        df[f] = rng.integers(0, DIN_VOCAB_C - 1, n)
    cfg = RankConfig()
    cfg.din_seq_max_len, cfg.batch_size = T, 4096
    rk = DINRanker(cfg, device=device, table_dtype="bf16").set_data(df, upd, ifd, uhd, uf, itf, cf, enc)
    rk.load_model(sd)
    rk.predict()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    probs = rk.predict()
    dt = time.perf_counter() - t0
    assert probs.shape == (n,) and np.isfinite(probs).all()
    out["din_predict"] = {"value": round(n / dt, 1), "unit": "DIN scored pairs/s (incl. encoding)", "samples": n,
                          "seconds": round(dt, 3)}
    return out


def run_itemcf(args, device):
    """Informational ItemCF leg: the whole similarity
    (nrk_itemcf_sim, item_cf.py:17-89), per-item top-20 (A9) and the recall of
    every user, top-30 (nrk_itemcf_recall, A10), over the same 250k-user
    synthetic click log as the recall bench; timed end to end (including the
    host reads that size the outputs), inputs resident in HBM."""
    from nrk import ops
    from nrk.data import synth

    clog = synth.make_click_log(n_users=args.users, n_items=args.items, seed=23)
    users, offs, items_raw, ts = synth.user_lists(clog)
    ids, dense = np.unique(items_raw, return_inverse=True)
    created = np.random.default_rng(1).random(len(ids))
    hot = np.argsort(-np.bincount(dense, minlength=len(ids)), kind="stable")[:50].astype(np.int32)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
    t_off, t_items, t_ts, t_cr, t_hot = d(offs), d(dense.astype(np.int32)), d(ts), d(created), d(hot)
    q = torch.arange(len(users), dtype=torch.int64, device=device)
    n_pairs = int(((offs[1:] - offs[:-1]) ** 2).sum())

    def one():
        sim = ops.itemcf_sim(t_off, t_items, t_ts, t_cr, len(ids))
        t1 = time.perf_counter()
        nc, nv, nn = ops.itemcf_topn(sim.row_offsets(), sim.j, sim.v, sim.first, 20)
        oi, osc, _, ocnt = ops.itemcf_recall(q, t_off, t_items, nc, nv, nn, t_cr, t_hot, 30)
        torch.cuda.synchronize()
        return t1, oi, ocnt

    one()
    torch.cuda.synchronize()
    # median of 5 end-to-end runs: once, a single slow run moved the 3-run
    # mean of the similarity from 2.3 to 7.6 ms
    reps = 5
    sim_s, rec_s = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        t1, oi, ocnt = one()
        t2 = time.perf_counter()
        sim_s.append(t1 - t0)
        rec_s.append(t2 - t1)
    t_sim, t_rec = float(np.median(sim_s)), float(np.median(rec_s))
    recalled = int(ocnt.sum())
    out = {"unit": "ordered pairs/s (similarity), recalled pairs/s (recall)",
           "users": len(users), "items": len(ids), "ordered_pairs": n_pairs,
           "sim_ms": round(t_sim * 1e3, 3), "sim_pairs_per_s": round(n_pairs / t_sim, 1),
           "sim_roofline": {"bound": "hbm", "bytes_per_pair": 32,
                            "achieved": round(32 * n_pairs / t_sim / 1e9, 1), "peak": PEAK_HBM_GBS,
                            "unit": "GB/s", "frac": round(32 * n_pairs / t_sim / 1e9 / PEAK_HBM_GBS, 4)},
           "recall_ms": round(t_rec * 1e3, 3), "recall_pairs_per_s": round(recalled / t_rec, 1),
           "workload": "250k-user synthetic Tianchi log: ItemCF similarity + top-20 per item + top-30 "
                       "recall of every user", "timing": "median of 5 end-to-end runs after one warm-up"}
    if not args.no_cpu_baseline:
        from oracle import oracle

        threads, why = cpu_share()
        dn = dense.astype(np.int32)

        def prefix(fn, budget, nu=1000):
            # a bounded prefix of the same users, grown 4x until one timed run
            # takes >= budget seconds (or covers them all)
            while True:
                nu = min(nu, len(users))
                t0 = time.perf_counter()
                fn(nu)
                dt = time.perf_counter() - t0
                if dt >= budget or nu == len(users):
                    return nu, dt, int(((offs[1:nu + 1] - offs[:nu]) ** 2).sum())
                nu *= 4

        nu, dt, sp = prefix(lambda nu: oracle.itemcf_sim_omp(offs[:nu + 1], dn[:offs[nu]], ts[:offs[nu]], created,
                                                             len(ids), threads), 3.0, 4000)
        n1, d1, s1 = prefix(lambda nu: oracle.itemcf_sim(offs[:nu + 1], dn[:offs[nu]], ts[:offs[nu]], created,
                                                         len(ids)), 2.0)

        def pyloop(nu):
            uit = {u: list(zip(dn[offs[u]:offs[u + 1]].tolist(), ts[offs[u]:offs[u + 1]].tolist()))
                   for u in range(nu)}
            oracle.itemcf_sim_pyloop(uit, created)

        n2, d2, s2 = prefix(pyloop, 2.0, 250)
        out["cpu_baseline"] = {
            "value": round(sp / dt, 1), "unit": "ordered pairs/s (similarity)", "cores": threads, "kind": "port",
            "threads_from": why,
            "sample": f"first {nu} users, oracle_itemcf_sim_omp (C, OpenMP, rows split i mod {threads}; "
                      f"bit-identical to the sequential sums) ({dt:.1f}s)",
            "variants": [
                {"value": round(s1 / d1, 1), "unit": "ordered pairs/s (similarity)", "cores": 1, "kind": "port",
                 "sample": f"first {n1} users, oracle_itemcf_sim (C, one thread) ({d1:.1f}s)"},
                {"value": round(s2 / d2, 1), "unit": "ordered pairs/s (similarity)", "cores": 1, "kind": "port",
                 "sample": f"first {n2} users, oracle.itemcf_sim_pyloop: item_cf.py:33-84's Python dict loops "
                           f"with numpy-scalar weights, the reference's own per-pair cost ({d2:.1f}s)"}]}
    return out


def fused_ctx_tables(users, items, user_hist, hist_len, device, gi, g, n_cat=461):
    """Config-5 context tables in HBM (synthetic, Tianchi-shaped): article-id
    Word2Vec vectors [I, 64] f32, 250-d float64 content rows (5% missing, 1%
    all zero), MinMax created times (5% missing), categories, each user's
    last-3 history rows + the categories of the whole history, and the
    recall's own user / item vectors for item_user_sim.  Returns (tables,
    None): the spec is fitted on the first chunk."""
    from nrk.features import CtxTables

    I, U, T = items.shape[0], users.shape[0], user_hist.shape[1]
    w2v = (torch.randn(I, 64, device=device, generator=gi) * 0.3).contiguous()
    content = torch.randn(I, 250, device=device, dtype=torch.float64, generator=gi)
    present = torch.rand(I, device=device, generator=gi) >= 0.05
    zero = torch.rand(I, device=device, generator=gi) < 0.01
    content[~present | zero] = 0.0
    flags = (present.to(torch.uint8) | ((present & ~zero).to(torch.uint8) << 1)).contiguous()
    created = torch.rand(I, device=device, dtype=torch.float64, generator=gi)
    created[torch.rand(I, device=device, generator=gi) < 0.05] = float("nan")
    category = torch.randint(0, n_cat, (I,), device=device, generator=gi, dtype=torch.int32)
    N = 3
    L = hist_len.long()
    t = torch.arange(N, device=device)
    # the last min(L, N) history rows, oldest first (user_history_dict[u][-N:]), -1 after
    start = (L - N).clamp(min=0)
    idx = (start[:, None] + t[None, :]).clamp(max=T - 1)
    keep = t[None, :] < L.clamp(max=N)[:, None]
    hl = torch.where(keep, torch.gather(user_hist.long(), 1, idx), torch.full_like(idx, -1)).to(torch.int32).contiguous()
    hn = torch.where(L > 0, L.clamp(max=N), torch.full_like(L, -1)).to(torch.int32).contiguous()
    valid = torch.arange(T, device=device)[None, :] < L[:, None]
    ucat = category[user_hist.long()][valid].contiguous()
    uoff = torch.zeros(U + 1, dtype=torch.int64, device=device)
    uoff[1:] = torch.cumsum(L, 0)
    ones_u = torch.ones(U, dtype=torch.uint8, device=device)
    ones_i = torch.ones(I, dtype=torch.uint8, device=device)
    tensors = {"w2v": w2v, "w2v_ok": ones_i, "content": content.contiguous(), "flags": flags, "created": created,
               "category": category, "hist_last": hl, "hist_n": hn, "ucat_off": uoff,
               "ucat": ucat if ucat.numel() else torch.zeros(1, dtype=torch.int32, device=device),
               "user_yt": users, "user_yt_ok": ones_u, "item_yt": items, "item_yt_ok": ones_i}
    return CtxTables.from_device(tensors, last_n=N), None


def run_fused(args, device, rank, world, dist):
    """BASELINE config 5 (10M users x 5M items, D=128, fused recall -> DIN),
    weak-scaled: every rank recalls its own 10M / N users (--fused-users
    overrides) against the replicated 5M-item catalog, then DIN scores the 30
    recalled pairs of each user in Dice batches of 4096, all on the device.
    One step = the whole share; value = pairs scored by all ranks / the
    slowest rank's time."""
    from nrk import ops
    from nrk.pipeline import FusedRecallRank

    U = args.fused_users or (10_000_000 // world)
    I, D, T, k = args.fused_items, 128, 50, 30
    chunk = min(args.fused_chunk, -(-U // 2048) * 2048)  # users per assemble -> DIN call (chunk * k % 4096 == 0)
    g = torch.Generator(device=device).manual_seed(1000 + rank)
    gi = torch.Generator(device=device).manual_seed(999)  # the catalog is the same on every rank
    items = torch.nn.functional.normalize(torch.randn(I, D, device=device, generator=gi), dim=1).contiguous()
    users = torch.nn.functional.normalize(torch.randn(U, D, device=device, generator=g), dim=1).contiguous()
    cat = ops.Catalog(items)
    rnd = lambda hi, shape, gen: torch.randint(0, hi, shape, device=device, generator=gen, dtype=torch.int32)  # noqa: E731
    user_feat = torch.stack([rnd(v, (U,), g) for v in DIN_VOCAB_U], 1).contiguous()
    item_feat = torch.stack([rnd(v, (I,), gi) for v in DIN_VOCAB_I], 1).contiguous()
    user_hist = rnd(I, (U, T), g)
    hist_len = rnd(T + 1, (U,), g)
    sd, feats, _, _ = din_workload(101, 64, T, "cpu")
    p = ops.DinParams(sd, *feats, table_dtype="bf16", device=device)
    ctx = None
    if not args.fused_hash_ctx:
        ctx = fused_ctx_tables(users, items, user_hist, hist_len, device, gi, g)
    if ctx is None:
        fused = FusedRecallRank(cat, p, user_feat, item_feat, user_hist, hist_len, k=k, chunk_users=chunk)
    else:
        # fit the binning + label codes on the first chunk's raw features
        # (the reference fits on its whole main_df, offline; untimed here)
        from nrk.features import CtxSpec, ctx_feature_names, ctx_features

        n0 = min(U, 4096)
        s0, r0 = ops.ip_topk(users[:n0].contiguous(), cat, k + 1)
        pi = r0[:, 1:].reshape(-1).contiguous()
        ps = s0[:, 1:].to(torch.float64).reshape(-1).contiguous()
        goff = torch.arange(0, (n0 + 1) * k, k, dtype=torch.int64, device=device)
        gus = torch.arange(0, n0, dtype=torch.int32, device=device)
        raw, _ = ctx_features(ctx[0], None, pi, ps, groups=(goff, gus, None))
        names = ctx_feature_names()
        rawn = raw.cpu().numpy()
        cols = {f: (rawn[:, j] if f == "score" else rawn[:, j].astype(np.float32)) for j, f in enumerate(names)}
        cols["recall_in_user_cat"] = rawn[:, -1].astype(np.int8)
        spec = CtxSpec.fit(cols, names)
        fused = FusedRecallRank(cat, p, user_feat, item_feat, user_hist, hist_len, k=k, ctx=(ctx[0], spec),
                                chunk_users=chunk)
    probs = torch.empty(U * k, dtype=torch.float32, device=device)

    def step(ev=None):
        if ev is not None:
            ev[0].record()
        s, r = fused.recall(users)
        if ev is not None:
            ev[1].record()
        fused.rank(s, r, probs)
        if ev is not None:
            ev[2].record()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(evs[i])
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist is not None:
        el = max_over_ranks(el, device)
    rec_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    din_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))
    pairs = U * k * world
    flops = 2.0 * U * I * D
    return {
        "metric": "fused recall->DIN scored pairs/s (BASELINE config 5)", "value": round(pairs / (el / args.steps), 1),
        "unit": "scored pairs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp16 screen + fp64 exact recall; fp32-class DIN, bf16 tables",
        "data": ("synthetic: random unit user / item vectors, uniform feature indices, random-init DIN, "
                 + ("hash-bin context" if args.fused_hash_ctx else
                    "context features computed on the device from synthetic w2v / content / created / "
                    "category tables (nrk_ctx_features)")),
        "config": {"workload": "BASELINE config 5: fused recall (exact top-31 IP, D=128) -> DIN rank of the "
                               "30 recalled items per user", "users_per_gpu": U, "items": I, "dim": D, "topk": k,
                   "seq_len": T, "dice_batch": 4096, "parallelism": f"users-sharded x{world}"},
        "phase_ms": {"recall": round(rec_ms, 3), "assemble_and_din": round(din_ms, 3)},
        "roofline": {"bound": "mfma", "kernel": "ip_screen_kernel<128> + refine (recall phase)",
                     "achieved": round(flops / (rec_ms * 1e-3) / 1e12, 2), "peak": PEAK_BF16_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(flops / (rec_ms * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4)},
    }


DIN_SAMPLES = 675_653  # README.md:28 (BASELINE config 3)
DIN_VOCAB_U = [200, 5000, 6, 200000, 3000]
DIN_VOCAB_I = [462, 3000, 300000, 1500]
DIN_N_CTX, DIN_VOCAB_C = 16, 11
DIN_BYTES_PER_PAIR = 225 * 4 + 225 * 64 + 4  # idx + bf16 rows + output


def din_batches(n, B, world, rank):
    """Config 3 layout over N ranks: the Dice batches of B (last one short)
    round-robin, batch b on rank b mod N.  Returns (this rank's batch ids,
    its sample rows in batch order).  The short last batch is the highest id,
    so it stays last on its rank and every rank's rows split into its own
    batches of B exactly as on one GPU."""
    nb = -(-n // B)
    mine = list(range(rank, nb, world))
    rows = (np.concatenate([np.arange(b * B, min(n, (b + 1) * B)) for b in mine]) if mine
            else np.zeros(0, np.int64))
    return mine, rows


def din_workload(seed, n, T, device, rows=None):
    """Config 3 synthetic: uniform indices, hist_len ~ U[1, T] with 20% all-pad
    rows, torch-default-initialised DINModel-shaped weights (seed 23).  The
    same n samples on every rank; ``rows`` picks this rank's share."""
    torch.manual_seed(23)
    sd = {}
    uf = [f"u{i}" for i in range(len(DIN_VOCAB_U))]
    itf = [f"i{i}" for i in range(len(DIN_VOCAB_I))]
    cf = [f"c{i}" for i in range(DIN_N_CTX)]
    for grp, names, voc in (("user_profile_embedding_dict", uf, DIN_VOCAB_U),
                            ("item_embedding_dict", itf, DIN_VOCAB_I),
                            ("context_embedding_dict", cf, [DIN_VOCAB_C] * DIN_N_CTX)):
        for f, v in zip(names, voc):
            sd[f"{grp}.{f}.weight"] = torch.nn.Embedding(v, 32).weight.detach()
    in_dim = 32 * (len(uf) + len(cf) + 2 * len(itf))
    for name, (o, i) in (("activation_unit.mlp.0", (36, 128 * len(itf))), ("activation_unit.mlp.2", (1, 36)),
                         ("mlp.0", (200, in_dim)), ("mlp.2", (80, 200)), ("mlp.4", (1, 80))):
        lin = torch.nn.Linear(i, o)
        sd[name + ".weight"], sd[name + ".bias"] = lin.weight.detach(), lin.bias.detach()
    rng = np.random.default_rng(seed)
    L = rng.integers(1, T + 1, n)
    L[rng.random(n) < 0.2] = 0
    mask = (np.arange(T)[None] < L[:, None]).astype(np.float32)
    hist = np.stack([rng.integers(0, v, (n, T), dtype=np.int32) for v in DIN_VOCAB_I], 2)
    hist *= mask[:, :, None].astype(np.int32)
    enc = {
        "user": np.stack([rng.integers(0, v, n, dtype=np.int32) for v in DIN_VOCAB_U], 1),
        "item": np.stack([rng.integers(0, v, n, dtype=np.int32) for v in DIN_VOCAB_I], 1),
        "hist": hist,
        "ctx": rng.integers(0, DIN_VOCAB_C, (n, DIN_N_CTX), dtype=np.int32),
        "mask": mask,
    }
    if rows is not None:
        enc = {k: np.ascontiguousarray(v[rows]) for k, v in enc.items()}
    dev = {k: torch.from_numpy(v).to(device) for k, v in enc.items()}
    return sd, (uf, itf, cf), enc, dev


def run_din(args, device, rank, world):
    """BASELINE config 3: every one of the 675,653 samples scored in Dice
    batches of 4096 (last 3,909), all of a rank's batches in one
    nrk_din_forward_segments call; with N ranks batch b runs on rank b mod N
    (din_batches).  The indices are resident in HBM before the timed region."""
    from nrk import ops

    n, T, B = args.din_samples, 50, 4096
    mine, rows = din_batches(n, B, world, rank)
    sd, feats, enc, dev = din_workload(101, n, T, device, rows=rows if world > 1 else None)
    n_loc = int(dev["mask"].shape[0])
    p = ops.DinParams(sd, *feats, table_dtype="bf16", device=device)
    ws = ops.din_workspace(p, max(n_loc, 2), T, device, batch_size=B)
    probs = torch.empty(n_loc, dtype=torch.float32, device=device)
    if n_loc:
        ops.din_validate(p, dev["user"], dev["item"], dev["hist"], dev["ctx"])  # once, untimed
    full = tuple(dev[k] for k in ("user", "item", "hist", "ctx", "mask"))

    def one_pass(ev=None):
        # every Dice batch of this rank (B each, the global last one short)
        # in one nrk_din_forward_segments call
        if ev is not None:
            ev[0].record()
        if n_loc:
            ops.din_forward(p, *full, workspace=ws, out=probs, validate=False, batch_size=B)
        if ev is not None:
            ev[1].record()

    for _ in range(args.din_warmup):
        one_pass()
    torch.cuda.synchronize()
    steps = args.din_steps
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(steps)]
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        one_pass(evs[i])
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = (time.perf_counter() - t0) / steps
    if dist is not None:  # whole-job rate: every rank's pass / the slowest rank's time
        dt = max_over_ranks(dt, device)
    pass_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    value = n / dt  # every sample of the job once / the slowest rank's pass
    achieved = DIN_BYTES_PER_PAIR * n_loc / (pass_ms * 1e-3) / 1e9
    default_cfg = n == DIN_SAMPLES and world == 1
    t = pmc_din_pass(default_cfg)
    din_traffic = round(t) if t else None
    out = {"value": round(value, 1), "unit": "DIN scored pairs/s", "ms_per_pass": round(dt * 1e3, 3),
           "samples": n, "batch": B, "seq_len": T, "dtype": "fp32 math, bf16 tables",
           "parallelism": (f"Dice batches round-robin x{world} (batch b on rank b mod {world}; rank 0: "
                           f"{len(mine)} batches, {n_loc} samples)" if world > 1 else "single"),
           "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                        "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": din_traffic,
                        "traffic_unit": "bytes per pass, every launch of one nrk_din_forward_segments call "
                                        "(profiles/" + PROFILE_ROUND + "_traffic.json din_pass)",
                        "kernel": f"nrk_din_forward_segments ({n_loc} samples in Dice batches of {B}, one call)",
                        "kernel_ms": round(pass_ms, 4),
                        "algorithmic_bytes_per_launch": DIN_BYTES_PER_PAIR * n_loc,
                        "busy": pmc_busy(["nrk::din_tm_plan", "nrk::din_att", "nrk::din_wh", "nrk::din_mlp1",
                                          "nrk::din_mlp2", "nrk::din_head"], default_cfg)}}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle

        m = args.din_cpu_sample
        threads, why = cpu_share()
        torch_threads = torch.get_num_threads()
        torch.set_num_threads(threads)
        sdn = {k: v.numpy() for k, v in sd.items()}
        model = oracle.DinTorchCPU(sdn, feats, round_bf16=True)
        tt = {k: torch.from_numpy(v) if k == "mask" else torch.from_numpy(v.astype(np.int64)) for k, v in enc.items()}
        cdt, nb = 0.0, 0
        while cdt < args.cpu_seconds and (nb + 1) * m <= n:  # whole B-sample batches, like the reference
            sl = {k: v[nb * m:(nb + 1) * m] for k, v in tt.items()}
            t1 = time.perf_counter()
            model(sl["user"], sl["item"], sl["hist"], sl["ctx"], sl["mask"])
            cdt += time.perf_counter() - t1
            nb += 1
        sl0 = {k: v[:m] for k, v in enc.items()}
        po, _, _ = oracle.din_forward(sdn, sl0["user"], sl0["item"], sl0["hist"], sl0["ctx"], sl0["mask"], feats,
                                      round_bf16=True)
        torch.set_num_threads(torch_threads)
        out["cpu_baseline"] = {"value": round(nb * m / cdt, 1), "unit": "DIN scored pairs/s",
                               "cores": threads, "kind": "port", "threads_from": why,
                               "sample": f"{nb} batches x {m} samples of the same workload, torch-CPU eval forward "
                                         f"of DINModel's formulation (oracle.DinTorchCPU, fp32), {cdt:.1f}s"}
        gp = ops.din_forward(p, *(dev[k][:m] for k in ("user", "item", "hist", "ctx", "mask")), workspace=ws)
        err = float(np.abs(gp.cpu().numpy() - po).max())
        log(f"DIN spot-check vs oracle ({m} samples): max |dp| = {err:.2e}")
    return out


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """``--gpus N`` with no torch.distributed launcher around us: start N
    worker processes of this script (one per GPU, RANK = LOCAL_RANK = r,
    WORLD_SIZE = N, 127.0.0.1 rendezvous) and wait for them.  Runs before
    this process touches the GPU (no HIP call, no exec).  Rank 0 prints the
    JSON line; the parent returns non-zero if any rank fails, and stops the
    remaining ranks (by their own PIDs) so none waits forever in a
    collective."""
    import subprocess

    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + list(argv), env=env))
    log(f"[launcher] started {n} ranks: pids {[p.pid for p in procs]}, master 127.0.0.1:{port}")
    rc = 0
    live = list(procs)
    while live:
        time.sleep(0.2)
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                log(f"[launcher] rank {procs.index(p)} exited with {code}; stopping the others")
                for o in live:
                    o.terminate()
    return rc


def layout_plan(args, world):
    """Per-rank work of the N-rank run (the dry run prints it, the workload
    follows it):
      recall: "catalog" (BASELINE config 4, default at N > 1): the ranks
              form an R x C grid (nrk.dist.layout_2d: R = 2 user groups at
              N = 8, else 1); rank r = g C + c screens the 32-item blocks
              shard_blocks(I, C, c, tile) (whole screen tiles) for group g's
              users, runs the tower for and refines its 1 / C of them
              (nrk.dist.grid_ranges); "users": every rank its own U users
              against the whole catalog; N = 1: "single".
      din:    the Dice batches of 4096 round-robin (din_batches)."""
    from nrk.dist import grid_ranges, layout_2d
    from nrk.ops import ip_topk_tile_blocks

    U, I, D = args.users, args.items, args.dim
    layout = "single" if world == 1 else args.shard
    tb = ip_topk_tile_blocks(D)
    owner = getattr(args, "topk", 30) + 1 <= 128
    # the R x C grid of the owner protocol (the merge protocol: one row)
    R, C = layout_2d(world, getattr(args, "user_groups", None) or (None if owner else 1)) if layout == "catalog" \
        else (1, world)
    per = []
    for r in range(world):
        if layout == "catalog":
            (glo, ghi), (ulo, uhi), (blo, bhi) = grid_ranges(U, I, world, R, r, tb)
            per.append({"rank": r, "blocks": [blo, bhi], "items": [min(I, 32 * blo), min(I, 32 * bhi)],
                        "users": [ulo, uhi], "group_users": [glo, ghi]})
        else:
            per.append({"rank": r, "blocks": [0, -(-I // 32)], "items": [0, I], "users": [0, U]})
    grid = f"{R} user groups x {C} catalog shards" if R > 1 else f"{C} catalog shards"
    rec = {"layout": layout, "tile_blocks": tb, "per_rank": per, "user_groups": R,
           "parallelism": {"single": "single",
                           "catalog": (f"catalog-sharded x{world} as {grid} (BASELINE config 4: shard screen, bound "
                                       f"all_gather, band all_to_all, owner refine)" if owner else
                                       f"catalog-sharded x{world} (BASELINE config 4, k + 1 > 128: per-shard exact "
                                       f"top-k, all_to_all to the owner, merge)"),
                           "users": f"users-sharded x{world} (independent replicas)"}[layout]}
    n, B = args.din_samples, 4096
    dper = []
    for r in range(world):
        mine, rows = din_batches(n, B, world, r)
        dper.append({"rank": r, "batches": len(mine), "samples": int(len(rows)),
                     "short_batch": bool(mine) and mine[-1] == -(-n // B) - 1 and n % B != 0})
    din = {"batches": -(-n // B), "batch": B, "per_rank": dper,
           "parallelism": (f"Dice batches round-robin x{world} (batch b on rank b mod {world})" if world > 1
                           else "single")}
    return {"recall": rec, "din": din}


def dry_run(args, world, rank, local):
    """--dry-run: the launcher, rendezvous and layout without the workload
    (CPU tests use it with --backend gloo): every rank joins the process
    group, checks the world with an all_reduce and that the ranks' own shares
    of layout_plan cover the work once (item blocks, user blocks, DIN
    samples), and rank 0 prints a JSON line with the plan."""
    import torch.distributed as dist

    plan = layout_plan(args, world)
    rec, din = plan["recall"]["per_rank"][rank], plan["din"]["per_rank"][rank]
    mine = torch.tensor([1, rec["blocks"][1] - rec["blocks"][0], rec["users"][1] - rec["users"][0],
                         din["samples"], din["batches"]], dtype=torch.int64)
    if world > 1:
        dist.init_process_group(args.backend or "gloo")
        dist.all_reduce(mine)
    tot = [int(x) for x in mine]
    assert tot[0] == world, (tot, world)
    if plan["recall"]["layout"] == "catalog":  # every block once per user group
        assert tot[1] == plan["recall"]["user_groups"] * -(-args.items // 32) and tot[2] == args.users, tot
    assert tot[3] == args.din_samples and tot[4] == plan["din"]["batches"], tot
    log(f"[rank {rank}/{world}] local_rank {local} pid {os.getpid()} backend {args.backend or 'gloo'} (dry run) "
        f"blocks {rec['blocks']} users {rec['users']} din batches {din['batches']} samples {din['samples']}")
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "n_gpus": world, "dry_run": True, "layout": plan,
                          "covered": {"item_blocks": tot[1], "users": tot[2], "din_samples": tot[3],
                                      "din_batches": tot[4]}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without WORLD_SIZE in the env, bench.py starts them itself")
    ap.add_argument("--backend", default=None, help="process-group backend (default nccl = RCCL)")
    ap.add_argument("--dry-run", action="store_true", help="launcher + rendezvous only, no workload")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--users", type=int, default=250_000)
    ap.add_argument("--items", type=int, default=364_047)
    ap.add_argument("--dim", type=int, default=32)
    ap.add_argument("--topk", type=int, default=30)
    ap.add_argument("--cpu-sample", type=int, default=2048)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="CPU work timed for each cpu_baseline leg (chunks of --cpu-sample users / batches)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-din", action="store_true")
    ap.add_argument("--no-itemcf", action="store_true", help="skip the informational ItemCF leg")
    ap.add_argument("--no-plugins", action="store_true", help="skip the plugin-level (end-to-end API) leg")
    ap.add_argument("--fused", action="store_true",
                    help="BASELINE config 5 instead: fused recall -> DIN, 10M users / N per rank x 5M items, D=128")
    ap.add_argument("--fused-users", type=int, default=0, help="users per rank for --fused (default 10M / N)")
    ap.add_argument("--fused-items", type=int, default=5_000_000)
    ap.add_argument("--fused-chunk", type=int, default=131072,
                    help="config 5: users per assemble / context / DIN call (a multiple of 2048: whole Dice batches; "
                         "rank side 359 / 366 / 372 ms per 1.25M-user step at 131072 / 65536 / 32768)")
    ap.add_argument("--fused-hash-ctx", action="store_true",
                    help="config 5 with the synthetic hash-bin context instead of the real context features")
    ap.add_argument("--shard", choices=["users", "catalog"], default="users",
                    help="N>1 recall layout of the headline value: users-sharded (the default: every "
                         "rank its own 250k-user problem against the whole catalog, no data-path "
                         "collective, weak scaling) or catalog-sharded (BASELINE config 4: shard screens, "
                         "bound all_gather, band all_to_all, owner refine; strong scaling)")
    ap.add_argument("--no-config4", action="store_true",
                    help="N>1, --shard users: skip the BASELINE config-4 measurement (catalog-sharded, "
                         "strong scaling) reported beside the headline as \"config4\"")
    ap.add_argument("--user-groups", type=int, default=None,
                    help="config 4: R user groups x N/R catalog shards (nrk.dist.layout_2d; default 1)")
    ap.add_argument("--din-samples", type=int, default=DIN_SAMPLES)
    ap.add_argument("--din-steps", type=int, default=10)
    ap.add_argument("--din-warmup", type=int, default=2)
    ap.add_argument("--din-cpu-sample", type=int, default=4096)
    args = ap.parse_args(argv)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"[rank {rank}] note: WORLD_SIZE={world} from the launcher, --gpus {args.gpus}; using {world}")
    if args.dry_run:
        return dry_run(args, world, rank, local)
    dist = None
    # one GPU per rank; with fewer visible GPUs than ranks (a one-GPU
    # rehearsal of the N-rank layout, --backend gloo) ranks share devices
    ndev = torch.cuda.device_count()
    dev_idx = local % ndev if ndev else local
    if ndev and local >= ndev:
        log(f"[rank {rank}] {ndev} visible GPU(s): rank shares cuda:{dev_idx} (rehearsal, not a measurement)")
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(dev_idx)
        backend = args.backend or "nccl"
        if backend == "nccl":
            dist.init_process_group(backend, device_id=torch.device("cuda", dev_idx))
        else:
            dist.init_process_group(backend)
    device = torch.device("cuda", dev_idx)
    torch.cuda.set_device(device)
    log(f"[rank {rank}/{world}] device {device} ({torch.cuda.get_device_name(device)}), pid {os.getpid()}")

    from nrk import ops

    if args.fused:
        line = run_fused(args, device, rank, world, dist)
        if rank == 0:
            print(json.dumps(line), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return

    def run_recall(shard_mode):
        """One recall measurement: BASELINE config 2 at N = 1, at N > 1 the
        layout ``shard_mode`` ("users": weak-scaled replicas, "catalog":
        config 4).  Returns the step function, outputs and the line fields."""
        rargs = argparse.Namespace(**vars(args))
        rargs.shard = shard_mode
        U, I, D, K = args.users, args.items, args.dim, args.topk + 1
        plan = layout_plan(rargs, world)
        catalog_mode = plan["recall"]["layout"] == "catalog"
        t0 = time.time()
        # users-sharded: every rank its own users (seed 23 + rank); catalog-sharded:
        # one shared workload, rank r screens item blocks [blk_lo, blk_hi)
        wl = recall_workload(23 if catalog_mode else 23 + rank, U, I, D, device)
        item_vec = ops.tt_item_fwd(wl["item_table"], torch.arange(I, dtype=torch.int32, device=device))
        cat = ops.Catalog(item_vec)
        owner = K <= ops.IP_KFAST  # the owner protocol's shard screen; larger k: the merge protocol
        if catalog_mode:
            from nrk.dist import HipRangeShard, HipShard, catalog_sharded_owner, catalog_sharded_topk, gather_users
            from nrk.dist import grid_groups

            me = plan["recall"]["per_rank"][rank]
            (blo, bhi), (ulo, uhi) = me["blocks"], me["users"]
            glo, ghi = me["group_users"]  # this rank's user group (all users when R = 1)
            grp, _, _ = grid_groups(world, plan["recall"]["user_groups"], rank)
            if owner:
                shard = HipRangeShard(cat, blo, bhi, K, ghi - glo)
            else:
                i0, i1 = me["items"]
                shard = HipShard(ops.Catalog(item_vec[i0:i1].contiguous()), i0, K, U)
        else:
            ws = ops.ip_topk_workspace(U, cat, K, device)
            out_s = torch.empty((U, K), dtype=torch.float32, device=device)
            out_r = torch.empty((U, K), dtype=torch.int32, device=device)
        torch.cuda.synchronize()
        log(f"[rank {rank}] setup {time.time() - t0:.1f}s: U={U} I={I} D={D} K={K} clicks={wl['n_clicks']}")

        def step_catalog(ev=None):
            # tower for this rank's user block, all_gather -> every user of the
            # rank's user group on every rank of it; screen this rank's item
            # blocks for those users, all_gather the shard bounds, band pack +
            # all_to_all to each user's owner, exact refine of the own user block
            # (nrk.dist.catalog_sharded_owner; all inside the group)
            if ev is not None:
                ev[0].record()
            u_loc = ops.tt_user_fwd(wl["user_table"], wl["item_table"], wl["uid"][ulo:uhi], wl["hist"][ulo:uhi],
                                    wl["hist_len"][ulo:uhi], wl["w0"], wl["b0"], wl["w1"], wl["b1"], validate=False)
            u = gather_users(u_loc, ghi - glo, group=grp)
            if ev is not None:
                ev[1].record()
            mark = None if ev is None else (lambda ph: ev[2 if ph == "screen" else 3].record())
            if owner:
                res = catalog_sharded_owner(u, shard, K, group=grp, mark=mark)
            else:
                res = catalog_sharded_topk(u, shard, K)
                if mark is not None:
                    mark("screen")
                    mark("exchange")
            if ev is not None:
                ev[4].record()
            return res

        def step(ev=None):
            if catalog_mode:
                return step_catalog(ev)
            if ev is not None:
                ev[0].record()
            u = ops.tt_user_fwd(wl["user_table"], wl["item_table"], wl["uid"], wl["hist"],
                                wl["hist_len"], wl["w0"], wl["b0"], wl["w1"], wl["b1"], validate=False)
            if ev is not None:
                ev[1].record()
            # the screen as its two launches, so the roofline times the MFMA scan alone
            ops.ip_topk_scan(u, cat, K, ws)
            if ev is not None:
                ev[5].record()
            ops.ip_topk_select(u, cat, K, ws)
            if ev is not None:
                ev[2].record()
            ops.ip_topk_finish(u, cat, K, ws, out_s, out_r)
            if ev is not None:
                ev[3].record()
                ev[4].record()
            return u

        # the tower's inputs are validated once here (hist_len in [0, T]: two
        # device syncs); the timed steps run it with validate=False
        ops.tt_user_fwd(wl["user_table"], wl["item_table"], wl["uid"], wl["hist"], wl["hist_len"], wl["w0"],
                        wl["b0"], wl["w1"], wl["b1"])
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(6)] for _ in range(args.steps)]
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t_start = time.perf_counter()
        for i in range(args.steps):
            step(evs[i])
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        elapsed = time.perf_counter() - t_start
        if dist is not None:
            elapsed = max_over_ranks(elapsed, device)
        ms_step = elapsed / args.steps * 1e3
        tower_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
        screen_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))
        finish_ms = float(np.mean([e[2].elapsed_time(e[3]) for e in evs]))
        refine_ms = float(np.mean([e[3].elapsed_time(e[4]) for e in evs]))
        scan_ms = None if catalog_mode else float(np.mean([e[1].elapsed_time(e[5]) for e in evs]))
        select_ms = None if catalog_mode else float(np.mean([e[5].elapsed_time(e[2]) for e in evs]))
        pairs = U * args.topk * (1 if catalog_mode else world)
        value = pairs / (elapsed / args.steps)

        # catalog mode: this rank's screen covers its own item blocks
        n_scr = (min(I, bhi * 32) - blo * 32) if catalog_mode else cat.n
        flops = 2.0 * ((ghi - glo) if catalog_mode else U) * n_scr * D
        kernel_ms = screen_ms if catalog_mode else scan_ms
        achieved = flops / (kernel_ms * 1e-3) / 1e12
        default_cfg = (U, I, D, args.topk) == (250_000, 364_047, 32, 30) and world == 1
        # the config-2 scan runs the warp-specialized kernel (ip_scan_ws_kernel)
        # unless built with -DNRK_SCAN_WS=0
        traffic = pmc_traffic(["nrk::ip_scan_ws_kernel<"], default_cfg) or pmc_traffic(["nrk::ip_scan_kernel<"], default_cfg)
        roofline = {"bound": "mfma", "achieved": round(achieved, 2), "peak": PEAK_BF16_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(achieved / PEAK_BF16_TFLOPS, 4),
                    "traffic": round(traffic) if traffic else None,
                    "traffic_unit": "bytes/launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, profiles/" + PROFILE_ROUND + "_traffic.json; "
                                    "null when absent or measured on other kernel sources)",
                    "kernel": ("ip_scan_ws_kernel (warp-specialized fp16 MFMA 32x32x16 screen) + bound all_gather, "
                               "this rank's item blocks" if catalog_mode else
                               "ip_scan_ws_kernel (warp-specialized fp16 MFMA 32x32x16 screen), HIP events around its launch"),
                    "kernel_ms": round(kernel_ms, 4),
                    "algorithmic_flop_per_launch": flops,
                    # the same flops over the whole timed step (tower + scan + select + finish on
                    # one GPU; this rank's screen share over the slowest rank's step at N > 1):
                    # the roofline fraction ``value`` itself achieves
                    "step_frac": round(flops / (ms_step * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4),
                    "busy": pmc_busy(["nrk::ip_scan_ws_kernel", "nrk::ip_select_kernel", "nrk::ip_refine_kernel",
                                      "nrk::tt_user_kernel"], default_cfg),
                    "busy_source": "profiles/" + PROFILE_ROUND + "_busy.json (rocprofv3 SQ_VALU_MFMA_BUSY_CYCLES, SQ_ACTIVE_INST_VALU, "
                                   "SQ_WAIT_ANY, GRBM_GUI_ACTIVE passes; tools/pmc_busy.py, calibrated by "
                                   "tools/calib)"}
        return {"step": step, "plan": plan, "catalog": catalog_mode, "value": value, "ms_step": ms_step,
                "tower_ms": tower_ms, "screen_ms": screen_ms, "finish_ms": finish_ms, "refine_ms": refine_ms,
                "scan_ms": scan_ms, "select_ms": select_ms, "roofline": roofline,
                "item_vec": item_vec, "out_r": None if catalog_mode else out_r, "U": U, "I": I, "D": D, "K": K}

    U, I, D, K = args.users, args.items, args.dim, args.topk + 1
    rec = run_recall("single" if world == 1 else args.shard)
    step, plan, catalog_mode, value, ms_step = rec["step"], rec["plan"], rec["catalog"], rec["value"], rec["ms_step"]
    tower_ms, screen_ms, finish_ms, refine_ms = rec["tower_ms"], rec["screen_ms"], rec["finish_ms"], rec["refine_ms"]
    scan_ms, select_ms, roofline, item_vec, out_r = (rec["scan_ms"], rec["select_ms"], rec["roofline"],
                                                      rec["item_vec"], rec["out_r"])
    # N > 1 with the users-sharded headline: BASELINE config 4 (the catalog
    # sharded over the same N ranks, strong scaling of one 250k-user problem,
    # the two RCCL exchanges) measured beside it
    config4 = None
    if world > 1 and args.shard == "users" and not args.no_config4:
        del rec
        c4 = run_recall("catalog")
        config4 = {"value": round(c4["value"], 1), "unit": "recalled pairs/s", "ms_per_step": round(c4["ms_step"], 4),
                   "scaling": "strong", "workload": f"BASELINE config 4: the same {U} users x {I} items, D={D}, "
                                                    f"catalog sharded {world}-way (one problem over all ranks)",
                   "parallelism": c4["plan"]["recall"]["parallelism"],
                   "phase_ms": {"tower_and_gather": round(c4["tower_ms"], 4),
                                "screen_and_bound_exchange": round(c4["screen_ms"], 4),
                                "band_pack_and_all_to_all": round(c4["finish_ms"], 4),
                                "owner_refine": round(c4["refine_ms"], 4)},
                   "roofline": c4["roofline"]}
        del c4

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads, why = cpu_share()
        u = step()
        torch.cuda.synchronize()
        v, dt, nu = cpu_baseline_recall(u.cpu().numpy(), item_vec.cpu().numpy(), K,
                                        args.cpu_sample, threads, args.cpu_seconds)
        cpu = {"value": round(v, 1), "unit": "recalled pairs/s", "cores": threads, "kind": "port",
               "threads_from": why, "per_core": round(v / threads, 1),
               "sample": f"first {nu} of the same {U} users x {I} items, exact fp64 top-{K} scan "
                         f"(oracle/nrk_oracle.c, the reference's per-user nq=1 shape, OpenMP over users, "
                         f"{dt:.1f}s)"}
        torch_threads = torch.get_num_threads()
        torch.set_num_threads(threads)
        vg, dtg, nug = cpu_baseline_recall_gemm(u.cpu().numpy(), item_vec.cpu().numpy(), K, args.cpu_sample,
                                                args.cpu_seconds / 2)
        torch.set_num_threads(torch_threads)
        cpu["variants"] = [{"value": round(vg, 1), "unit": "recalled pairs/s", "cores": threads,
                            "kind": "port", "sample": f"first {nug} users, batched fp32 GEMM + torch.topk on "
                                                      f"torch-CPU ({dtg:.1f}s; fp32 scores, not exact ties)"}]
        # correctness spot check of the timed outputs against the oracle
        from oracle import oracle

        so, ro = oracle.ip_topk(u[:64].cpu().numpy(), item_vec.cpu().numpy(), K, nthreads=threads)
        ok = np.array_equal(out_r[:64].cpu().numpy(), ro)
        log(f"spot-check vs oracle (64 users): {'OK' if ok else 'MISMATCH'}")

    din = None
    if not args.no_din:
        din = run_din(args, device, rank, world)
        log(f"DIN: {din['value']:.0f} pairs/s, {din['ms_per_pass']:.1f} ms/pass, device {din['roofline']['kernel_ms']:.3f} ms")

    plugins = None
    if world == 1 and not args.no_plugins:
        sd_p, feats_p, _, _ = din_workload(101, 64, 50, "cpu")
        plugins = run_plugins(args, device, step(), item_vec, sd_p, feats_p)
        log(f"plugins: batch_recall {plugins['batch_recall']['value']:.0f} pairs/s, "
            f"DINRanker.predict {plugins['din_predict']['value']:.0f} pairs/s")

    itemcf = None
    if world == 1 and not args.no_itemcf:
        itemcf = run_itemcf(args, device)
        log(f"ItemCF: sim {itemcf['sim_ms']:.1f} ms, recall {itemcf['recall_ms']:.1f} ms")

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "recalled pairs/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4), "higher_is_better": True,
            "scaling": "strong" if catalog_mode else "weak",
            "vs_baseline": None, "dtype": "fp16",
            "data": "synthetic Tianchi-shaped click log (seeded), random-init YouTubeDNN weights",
            "config": {"workload": (f"BASELINE config 4: YouTubeDNN recall (user tower + exact top-31 IP "
                                    f"search), {U} users x {I} items, D={D}, catalog sharded {world}-way"
                                    if catalog_mode else
                                    "BASELINE config 2: YouTubeDNN recall (user tower + exact top-31 "
                                    "IP search), 250k users x 364,047 items, D=32"
                                    + (f", one such problem per rank ({world} ranks, users-sharded)"
                                       if world > 1 else "")),
                       "users": U, "items": I, "dim": D, "topk": args.topk,
                       "parallelism": plan["recall"]["parallelism"],
                       "din_parallelism": plan["din"]["parallelism"]},
            "phase_ms": ({"tower_and_gather": round(tower_ms, 4), "screen_and_bound_exchange": round(screen_ms, 4),
                          "band_pack_and_all_to_all": round(finish_ms, 4), "owner_refine": round(refine_ms, 4)}
                         if catalog_mode else
                         {"tower": round(tower_ms, 4), "screen": round(screen_ms, 4), "scan": round(scan_ms, 4),
                          "select": round(select_ms, 4), "finish": round(finish_ms, 4)}),
            "roofline": roofline, "cpu_baseline": cpu, "din": din, "itemcf": itemcf, "plugins": plugins,
            "config4": config4, "host": host_info(),
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
