"""CPU oracle for the nrk hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker (or the
timed CPU baseline).  The product path (``nrk``) never imports it and fails
loudly when its HIP library is missing.

Each function restates the reference (file:line cited) in numpy / C:

* ``ip_topk``            -- faiss.IndexFlatIP contract, youtubednn_recaller.py:493-494, :520
* ``youtubednn_recall``  -- YoutubeDNNRecaller.recall, youtubednn_recaller.py:497-535
* ``embedding_similarity`` / ``embedding_sim_dict``
                         -- EmbeddingSimilarity.calculate, similarity/embedding.py:35-62
* ``tower_user``         -- YoutubeDNN.forward + _extract_embeddings re-norm, :129-178, :467-470
* ``tower_item``         -- get_item_embedding + re-norm, :184-188, :485-489
* ``itemcf_sim``         -- ItemCFSimilarity.calculate, item_cf.py:17-89
* ``itemcf_topn``        -- ItemCFRecaller._precompute_topk_similar_items, itemcf_recaller.py:41-54
* ``itemcf_recall``      -- ItemCFRecaller.recall, itemcf_recaller.py:56-129
* ``din_forward``        -- Dice / ActivationUnit / DINModel.forward, DIN.py:29-286
* ``fuse``               -- RecallFusion.fuse, recall/fusion.py:67-342
* ``ctx_features``       -- FeatureExtractor._extract_context_features,
                            features/feature_extractor.py:440-723

Pinning: tests/test_oracle_golden.py checks every function against the golden
fixtures produced by executing the reference (tests/golden/make_golden.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "libnrk_oracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        P = ctypes.c_void_p
        i64, i32, f64 = ctypes.c_int64, ctypes.c_int32, ctypes.c_double
        L.oracle_ip_topk.argtypes = [P, i64, P, i64, ctypes.c_int, ctypes.c_int, P, P, P, ctypes.c_int]
        L.oracle_ip_topk.restype = None
        L.oracle_itemcf_sim.argtypes = [i64, P, P, P, P, i32, f64, f64, f64, f64, f64, i64, P, P, P, P, P]
        L.oracle_itemcf_sim.restype = i64
        L.oracle_itemcf_sim_omp.argtypes = [i64, P, P, P, P, i32, f64, f64, f64, f64, f64, ctypes.c_int, P, P, P,
                                            P, P]
        L.oracle_itemcf_sim_omp.restype = i64
        L.oracle_topn_rows.argtypes = [i64, P, P, P, ctypes.c_int, P, P, P]
        L.oracle_topn_rows.restype = None
        L.oracle_itemcf_recall.argtypes = [i64, P, P, P, P, P, P, ctypes.c_int, P, P, ctypes.c_int,
                                           ctypes.c_int, f64, f64, i32, P, P, P]
        L.oracle_itemcf_recall.restype = None
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


# --------------------------------------------------------------------------
# Recall: exact top-K and the recall() wrapper
# --------------------------------------------------------------------------
def ip_topk(users, items, k, nthreads=0, exact=False):
    """Top-k rows of ``items`` by exact inner product with each user row.

    Returns (scores f32 [nu,k], rows i64 [nu,k]) (+ fp64 exact scores)."""
    users = np.ascontiguousarray(users, dtype=np.float32)
    items = np.ascontiguousarray(items, dtype=np.float32)
    nu, d = users.shape
    ni = items.shape[0]
    s = np.empty((nu, k), np.float32)
    r = np.empty((nu, k), np.int64)
    e = np.empty((nu, k), np.float64) if exact else None
    lib().oracle_ip_topk(_p(users), nu, _p(items), ni, d, k, _p(s), _p(r),
                         _p(e) if exact else None, int(nthreads))
    return (s, r, e) if exact else (s, r)


def youtubednn_recall(scores, rows, user_rawid_2_index, item_index_2_rawid, user_ids, topk):
    """YoutubeDNNRecaller.recall over a precomputed (k+1) search result.

    Drops rank 0 (:524), maps Faiss row r -> item_index_2_rawid[r] (:528-529,
    the A3 quirk), skips labels not in the mapping, unknown users -> []."""
    out = {}
    for u in user_ids:
        idx = user_rawid_2_index.get(u)
        if idx is None or idx >= scores.shape[0]:
            out[u] = []
            continue
        res = []
        for i in range(1, scores.shape[1]):
            r = int(rows[idx, i])
            if r in item_index_2_rawid:
                res.append((item_index_2_rawid[r], float(scores[idx, i])))
            if len(res) >= topk:
                break
        out[u] = res
    return out


def embedding_similarity(emb, topk, nthreads=0):
    """EmbeddingSimilarity.calculate's arithmetic (similarity/embedding.py:35-50):
    numpy float32 row normalisation (:41) then the IndexFlatIP self-search for
    topk+1 neighbours (:46-50).  Returns (normalised rows, scores, rows)."""
    x = np.ascontiguousarray(emb, dtype=np.float32)
    xn = np.ascontiguousarray(x / np.linalg.norm(x, axis=1, keepdims=True))
    s, r = ip_topk(xn, xn, topk + 1, nthreads=nthreads)
    return xn, s, r


def embedding_sim_dict(ids, scores, rows):
    """The dict build of embedding.py:52-62: row -> raw id, column 0 dropped
    (whatever row it holds), later duplicate keys overwrite."""
    i2r = {n: int(x) for n, x in enumerate(ids)}
    out = {}
    for t in range(scores.shape[0]):
        d = out.setdefault(i2r[t], {})
        for r, v in zip(rows[t, 1:].tolist(), scores[t, 1:].tolist()):
            d[i2r[r]] = float(v)
    return out


# --------------------------------------------------------------------------
# Two-tower forward (fp32, numpy)
# --------------------------------------------------------------------------
def tower_user(user_emb, item_emb, uid, hist, hist_len, w0, b0, w1, b1):
    """YoutubeDNN.forward (youtubednn_recaller.py:129-182) + numpy re-norm (:467-470), two layers."""
    return tower_user_layers(user_emb, item_emb, uid, hist, hist_len, [(w0, b0), (w1, b1)])


def tower_user_layers(user_emb, item_emb, uid, hist, hist_len, layers):
    """Any depth: user_tower = [Linear, ReLU, Dropout] per hidden unit
    (youtubednn_recaller.py:105-112); ``layers`` = [(W_l, b_l), ...]."""
    f32 = np.float32
    ue = user_emb[uid].astype(f32)
    he = item_emb[hist].astype(f32)
    T = hist.shape[1]
    mask = (np.arange(T)[None, :] < hist_len[:, None]).astype(f32)[:, :, None]
    avg = (he * mask).sum(1, dtype=f32) / (hist_len.astype(f32)[:, None] + f32(1e-8))
    x = np.concatenate([ue, avg.astype(f32)], 1)
    for w, b in layers:
        x = np.maximum(x @ w.T.astype(f32) + b.astype(f32), 0).astype(f32)
    n = np.maximum(np.sqrt((x * x).sum(1, keepdims=True, dtype=f32)), f32(1e-12))
    x = (x / n).astype(f32)
    n2 = np.linalg.norm(x, axis=1, keepdims=True)
    n2[n2 == 0] = 1
    return (x / n2).astype(f32)


def tower_item(item_emb, ids):
    f32 = np.float32
    x = item_emb[ids].astype(f32)
    n = np.maximum(np.sqrt((x * x).sum(1, keepdims=True, dtype=f32)), f32(1e-12))
    x = (x / n).astype(f32)
    return (x / np.linalg.norm(x, axis=1, keepdims=True)).astype(f32)


# --------------------------------------------------------------------------
# ItemCF
# --------------------------------------------------------------------------
LOC_ALPHA, LOC_ALPHA_REV, LOC_BETA, TIME_ALPHA, CREATED_ALPHA = 1.0, 0.7, 0.9, 0.7, 0.8


def itemcf_sim(offsets, items, ts, created, n_items):
    """Dense-id ItemCF similarity.  Returns (i, j, v, row_rank, cnt) with the
    (i, j) entries in global first-insertion order."""
    offsets = np.ascontiguousarray(offsets, np.int64)
    items = np.ascontiguousarray(items, np.int32)
    ts = np.ascontiguousarray(ts, np.int64)
    created = np.ascontiguousarray(created, np.float64)
    L = np.diff(offsets)
    cap = int((L * L).sum()) + 1
    oi = np.empty(cap, np.int32)
    oj = np.empty(cap, np.int32)
    ov = np.empty(cap, np.float64)
    rank = np.empty(n_items, np.int64)
    cnt = np.empty(n_items, np.int64)
    n = lib().oracle_itemcf_sim(len(offsets) - 1, _p(offsets), _p(items), _p(ts), _p(created),
                                n_items, LOC_ALPHA, LOC_ALPHA_REV, LOC_BETA, TIME_ALPHA,
                                CREATED_ALPHA, cap, _p(oi), _p(oj), _p(ov), _p(rank), _p(cnt))
    assert n >= 0
    return oi[:n], oj[:n], ov[:n], rank, cnt


def itemcf_sim_omp(offsets, items, ts, created, n_items, nthreads):
    """oracle_itemcf_sim on ``nthreads`` OpenMP threads (rows partitioned by
    i % T; bit-identical values, per-thread first-insertion order).  A CPU
    baseline variant (bench.py ItemCF leg), not a checker.  Returns (i, j, v)."""
    offsets = np.ascontiguousarray(offsets, np.int64)
    items = np.ascontiguousarray(items, np.int32)
    ts = np.ascontiguousarray(ts, np.int64)
    created = np.ascontiguousarray(created, np.float64)
    L = np.diff(offsets)
    cap = int((L * L).sum()) + 1
    oi = np.empty(cap, np.int32)
    oj = np.empty(cap, np.int32)
    ov = np.empty(cap, np.float64)
    base = np.zeros(nthreads, np.int64)
    n = np.zeros(nthreads, np.int64)
    lib().oracle_itemcf_sim_omp(len(offsets) - 1, _p(offsets), _p(items), _p(ts), _p(created), n_items,
                                LOC_ALPHA, LOC_ALPHA_REV, LOC_BETA, TIME_ALPHA, CREATED_ALPHA, int(nthreads),
                                _p(oi), _p(oj), _p(ov), _p(base), _p(n))
    take = np.concatenate([np.arange(b, b + c) for b, c in zip(base, n)]) if nthreads else np.zeros(0, np.int64)
    return oi[take], oj[take], ov[take]


def itemcf_sim_pyloop(user_item_time, created):
    """item_cf.py:33-84 as the reference writes it: Python dict loops over
    ``user_item_time`` ({user: [(item, time), ...]}) with WeightCalculator's
    np.exp / np.abs / math.log (weights.py:7-60) per pair.  A CPU baseline
    variant (the reference's own per-pair cost), not a checker.  Returns
    {i: {j: sim}}."""
    import math

    i2i, cnt = {}, {}
    for _, lst in user_item_time.items():
        for loc1, (i, ti) in enumerate(lst):
            cnt[i] = cnt.get(i, 0) + 1
            i2i.setdefault(i, {})
            for loc2, (j, tj) in enumerate(lst):
                if i == j:
                    continue
                la = LOC_ALPHA if loc2 > loc1 else LOC_ALPHA_REV
                loc_w = la * (LOC_BETA ** (np.abs(loc2 - loc1) - 1))
                click_w = np.exp(TIME_ALPHA ** np.abs(ti - tj))
                created_w = np.exp(CREATED_ALPHA ** np.abs(created[i] - created[j]))
                pen = 1.0 / math.log(len(lst) + 1)
                i2i[i].setdefault(j, 0)
                i2i[i][j] += loc_w * click_w * created_w * pen
    for i, row in i2i.items():
        for j, w in row.items():
            row[j] = w / math.sqrt(cnt[i] * cnt[j])
    return i2i


def sim_to_rows(i, j, v, n_items):
    """Group first-insertion-ordered entries into CSR rows (insertion order kept)."""
    order = np.argsort(i, kind="stable")
    off = np.zeros(n_items + 1, np.int64)
    np.add.at(off, i + 1, 1)
    return np.cumsum(off), j[order].astype(np.int32), v[order]


def itemcf_topn(row_off, cols, vals, topn=20):
    n_rows = len(row_off) - 1
    oc = np.full((n_rows, topn), -1, np.int32)
    ov = np.zeros((n_rows, topn), np.float64)
    cnt = np.zeros(n_rows, np.int32)
    lib().oracle_topn_rows(n_rows, _p(np.ascontiguousarray(row_off, np.int64)),
                           _p(np.ascontiguousarray(cols, np.int32)),
                           _p(np.ascontiguousarray(vals, np.float64)), topn, _p(oc), _p(ov), _p(cnt))
    return oc, ov, cnt


def itemcf_recall(q_slot, offsets, items, nbr_cols, nbr_vals, nbr_cnt, created, hot, topk, n_items):
    q_slot = np.ascontiguousarray(q_slot, np.int64)
    nq = len(q_slot)
    topn = nbr_cols.shape[1]
    oi = np.zeros((nq, topk), np.int32)
    os_ = np.zeros((nq, topk), np.float64)
    oc = np.zeros(nq, np.int32)
    hot = np.ascontiguousarray(hot, np.int32)
    lib().oracle_itemcf_recall(nq, _p(q_slot), _p(np.ascontiguousarray(offsets, np.int64)),
                               _p(np.ascontiguousarray(items, np.int32)),
                               _p(np.ascontiguousarray(nbr_cols, np.int32)),
                               _p(np.ascontiguousarray(nbr_vals, np.float64)),
                               _p(np.ascontiguousarray(nbr_cnt, np.int32)), topn,
                               _p(np.ascontiguousarray(created, np.float64)), _p(hot), len(hot),
                               topk, LOC_BETA, CREATED_ALPHA, n_items, _p(oi), _p(os_), _p(oc))
    return oi, os_, oc


# --------------------------------------------------------------------------
# DIN (fp32 numpy restatement of DIN.py:29-286)
# --------------------------------------------------------------------------
def _dice(x):
    f32 = np.float32
    x = x.astype(f32)
    mean = x.mean(0, keepdims=True, dtype=np.float64).astype(f32)
    std = x.astype(np.float64).std(0, ddof=1, keepdims=True).astype(f32)
    xn = (x - mean) / (std + f32(1e-8))
    p = (1.0 / (1.0 + np.exp(-xn.astype(np.float64)))).astype(f32)
    return (p * x + (f32(1) - p) * f32(0.01) * x).astype(f32)


def din_forward(sd, user, item, hist, ctx, mask, feats, round_bf16=False):
    """sd: DINModel state_dict as numpy; feats: (user_feats, item_feats, ctx_feats).

    Returns (probs [B], logits [B], att [B,T]).  ``round_bf16`` rounds every
    embedding table to bf16 first (storage-only bf16, fp32 math)."""
    f32 = np.float32
    uf, itf, cf = feats

    def tab(group, f):
        w = sd[f"{group}.{f}.weight"].astype(f32)
        return bf16_round(w) if round_bf16 else w

    U = np.concatenate([tab("user_profile_embedding_dict", f)[user[:, n]] for n, f in enumerate(uf)], 1)
    Q = np.concatenate([tab("item_embedding_dict", f)[item[:, n]] for n, f in enumerate(itf)], 1)
    K = np.concatenate([tab("item_embedding_dict", f)[hist[:, :, n]] for n, f in enumerate(itf)], 2)
    C = (np.concatenate([tab("context_embedding_dict", f)[ctx[:, n]] for n, f in enumerate(cf)], 1)
         if len(cf) else np.zeros((len(user), 0), f32))
    B, T, d = K.shape
    q = np.broadcast_to(Q[:, None, :], (B, T, d))
    X = np.concatenate([K, q, q - K, q * K], 2).astype(f32)
    a0w, a0b = sd["activation_unit.mlp.0.weight"].astype(f32), sd["activation_unit.mlp.0.bias"].astype(f32)
    a2w, a2b = sd["activation_unit.mlp.2.weight"].astype(f32), sd["activation_unit.mlp.2.bias"].astype(f32)
    h = (X @ a0w.T + a0b).astype(f32)
    h = _dice(h)
    w = (h @ a2w.T + a2b).astype(f32)[:, :, 0]
    w = (w * mask.astype(f32)).astype(f32)
    wh = (w[:, :, None] * K).sum(1, dtype=f32)
    x = np.concatenate([U, C, Q, wh], 1).astype(f32)
    for li in (0, 2):
        x = (x @ sd[f"mlp.{li}.weight"].astype(f32).T + sd[f"mlp.{li}.bias"].astype(f32)).astype(f32)
        x = _dice(x)
    logit = (x @ sd["mlp.4.weight"].astype(f32).T + sd["mlp.4.bias"].astype(f32)).astype(f32)[:, 0]
    prob = (1.0 / (1.0 + np.exp(-logit.astype(np.float64)))).astype(f32)
    return prob, logit, w


class DinTorchCPU:
    """torch-CPU eval forward in the reference's own formulation
    (DINModel.forward, DIN.py:214-286: nn.Embedding lookups, ActivationUnit
    Linear(512->36) on [k, q, q-k, q*k] + Dice + Linear(36->1) * mask, the
    weighted history sum, Linear/Dice MLP, sigmoid) -- the CPU baseline of
    BASELINE.md §3 for config 3, run on pre-encoded int tensors with every
    host thread torch has.  Bench-only (cpu_baseline leg)."""

    def __init__(self, sd, feats, round_bf16=False):
        import torch

        uf, itf, cf = feats
        t = lambda a: torch.from_numpy(np.ascontiguousarray(bf16_round(a) if round_bf16 else a, np.float32))  # noqa
        self.U = [t(sd[f"user_profile_embedding_dict.{f}.weight"]) for f in uf]
        self.I = [t(sd[f"item_embedding_dict.{f}.weight"]) for f in itf]
        self.C = [t(sd[f"context_embedding_dict.{f}.weight"]) for f in cf]
        g = lambda k: torch.from_numpy(np.ascontiguousarray(sd[k], np.float32))  # noqa: E731
        self.a0w, self.a0b = g("activation_unit.mlp.0.weight"), g("activation_unit.mlp.0.bias")
        self.a2w, self.a2b = g("activation_unit.mlp.2.weight"), g("activation_unit.mlp.2.bias")
        self.m = [(g(f"mlp.{i}.weight"), g(f"mlp.{i}.bias")) for i in (0, 2, 4)]

    @staticmethod
    def _dice(x):
        import torch

        mean, std = x.mean(0), x.std(0)
        p = torch.sigmoid((x - mean) / (std + 1e-8))
        return p * x + (1 - p) * 0.01 * x

    def __call__(self, user, item, hist, ctx, mask):
        import torch
        import torch.nn.functional as F

        with torch.no_grad():
            u = torch.cat([E[user[:, n]] for n, E in enumerate(self.U)], 1)
            q = torch.cat([E[item[:, n]] for n, E in enumerate(self.I)], 1)
            k = torch.cat([E[hist[:, :, n]] for n, E in enumerate(self.I)], 2)
            c = torch.cat([E[ctx[:, n]] for n, E in enumerate(self.C)], 1)
            qq = q.unsqueeze(1).expand_as(k)
            h = self._dice(F.linear(torch.cat([k, qq, qq - k, qq * k], -1), self.a0w, self.a0b))
            w = F.linear(h, self.a2w, self.a2b) * mask.unsqueeze(-1)
            x = torch.cat([u, c, q, (w * k).sum(1)], 1)
            x = self._dice(F.linear(x, *self.m[0]))
            x = self._dice(F.linear(x, *self.m[1]))
            return torch.sigmoid(F.linear(x, *self.m[2]).squeeze(-1))


def bf16_round(x):
    """Round-to-nearest-even fp32 -> bf16 -> fp32 (finite inputs)."""
    b = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    b = (b + 0x7FFF + ((b >> 16) & 1)) >> 16
    return (b.astype(np.uint32) << 16).view(np.float32).reshape(np.shape(x))


def fuse(methods, weights, strategy="weighted_avg", norm="local", topk=30, user_history=None, remove_seen=True):
    """RecallFusion.fuse (recall/fusion.py:267-342): ``methods`` = ordered
    {name: {user: [(item, score), ...]}}, ``weights`` = {name: w}.  Plain
    Python floats in the reference's operation order."""
    # normalisation (:289-304)
    normed = {}
    if norm == "global":  # _global_normalize :100-134
        allv = [s for d in methods.values() for lst in d.values() for _, s in lst]
        gmin, gmax = (min(allv), max(allv)) if allv else (0.0, 0.0)
        for m, d in methods.items():
            normed[m] = {u: [(i, (s - gmin) / (gmax - gmin) if gmax > gmin else 1.0) for i, s in lst]
                         for u, lst in d.items()}
    elif norm == "z-score":  # _zscore_normalize :136-187 (numpy mean / std, sigmoid via np.exp)
        for m, d in methods.items():
            allv = [s for lst in d.values() for _, s in lst]
            if not allv:
                normed[m] = {}
                continue
            mu, sd = np.mean(allv), np.std(allv)
            normed[m] = {u: [(i, 1.0 / (1.0 + np.exp(-((s - mu) / sd))) if sd > 0 else 0.5) for i, s in lst]
                         for u, lst in d.items()}
    else:  # _normalize_scores :71-98 per list
        for m, d in methods.items():
            out = {}
            for u, lst in d.items():
                if len(lst) <= 1:
                    out[u] = [(lst[0][0], 1.0)] if lst else []
                    continue
                mn, mx = min(s for _, s in lst), max(s for _, s in lst)
                out[u] = [(i, (s - mn) / (mx - mn) if mx > mn else 1.0) for i, s in lst]
            normed[m] = out
    users = set()
    for d in normed.values():
        users.update(d.keys())
    res = {}
    for u in users:
        src = {}
        for m, d in normed.items():  # _weighted_merge :189-265
            if u not in d:
                continue
            w = weights.get(m, 1.0)
            for r, (i, s) in enumerate(d[u]):
                src.setdefault(i, []).append((w, s, r))
        merged = {}
        for i, ss in src.items():
            if strategy == "weighted_sum":
                merged[i] = sum(w * s for w, s, _ in ss)
            elif strategy == "max_score":
                merged[i] = max(w * s for w, s, _ in ss)
            elif strategy == "harmonic_mean":
                merged[i] = len(ss) / sum(1.0 / (w * s + 1e-8) for w, s, _ in ss)
            elif strategy == "diversity_weighted":
                merged[i] = sum(w * s for w, s, _ in ss) * (1 + len(ss) * 0.1)
            elif strategy == "rrf":
                merged[i] = sum(w / (60 + r) for w, _, r in ss)
            else:
                tw = sum(w for w, _, _ in ss)
                merged[i] = sum(w * s for w, s, _ in ss) / tw if tw > 0 else 0
        if remove_seen and user_history and u in user_history:
            merged = {i: s for i, s in merged.items() if i not in user_history[u]}
        res[u] = sorted(merged.items(), key=lambda x: x[1], reverse=True)[:topk]
    return res


def ctx_features(main_users, main_items, main_scores, user_history, w2v, content, created, ctype, user_yt=None,
                 art_yt=None, last_n=3, emb_dim=64):
    """FeatureExtractor._extract_context_features
    (features/feature_extractor.py:440-723) restated in the reference's own
    numpy operations, per user group.  main_* are the main_df columns (str
    user / item ids, float64 scores); returns {feature: column}."""
    import pandas as pd

    n = len(main_items)
    N = last_n
    sim = np.full((n, N), np.nan, dtype=np.float32)
    tdf = np.zeros((n, N), dtype=np.float32)
    wdf = np.zeros((n, N), dtype=np.float32)
    stats = np.full((n, 4), np.nan, dtype=np.float32)
    ius = np.zeros(n, dtype=np.float32)
    ric = np.zeros(n, dtype=np.int8)
    ucats = {}
    for u, h in user_history.items():  # :497-506
        ucats[u] = {ctype[i] for i in h if i in ctype}
    zid = np.zeros(emb_dim, dtype=np.float32)
    zc = np.zeros(250, dtype=np.float32)
    groups = pd.Series(np.arange(n)).groupby(pd.Series(main_users)).apply(lambda s: s.to_numpy())
    items = np.asarray(main_items, dtype=object)
    for u, rows in groups.items():  # :527-690
        u = str(u)
        if u not in user_history:
            continue
        hist = user_history[u][-N:]
        rec = items[rows]
        if user_yt is not None and art_yt is not None:
            ue = user_yt.get(u)
            if ue is not None:
                ie = np.array([art_yt.get(i, zid) for i in rec], dtype=np.float32)
                ius[rows] = ie @ ue
        rid = np.array([w2v.get(i, zid) for i in rec], dtype=np.float32)
        rc = np.array([content.get(i, zc) for i in rec], dtype=np.float32)
        rt = np.array([created.get(i, np.nan) for i in rec], dtype=np.float32)
        for k, h in enumerate(hist):
            hid, hc, ht = w2v.get(h), content.get(h), created.get(h, np.nan)
            s = rid @ hid if hid is not None else np.zeros(len(rows), dtype=np.float32)
            if not np.isnan(ht):
                t = np.abs(rt - ht)
                t = np.where(np.isnan(t), 0, t)
            else:
                t = np.zeros(len(rows), dtype=np.float32)
            if hc is not None:
                w = np.linalg.norm(rc - hc[np.newaxis, :], axis=1)
                w = np.where(np.any(rc != 0, axis=1), w, 0)
            else:
                w = np.zeros(len(rows), dtype=np.float32)
            sim[rows, k] = s
            tdf[rows, k] = t
            wdf[rows, k] = w
        us = sim[rows, :]
        with np.errstate(all="ignore"):
            import warnings

            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                stats[rows, 0] = np.nanmax(us, axis=1)
                stats[rows, 1] = np.nanmean(us, axis=1)
                stats[rows, 2] = np.nanmin(us, axis=1)
                stats[rows, 3] = np.nanstd(us, axis=1)
        cats = ucats.get(u, set())
        if cats:
            ric[rows] = np.array([1 if ctype.get(i) in cats else 0 for i in rec], dtype=np.int8)
    out = {"score": np.asarray(main_scores, np.float64)}
    for k in range(N):
        out[f"sim_{k + 1}"], out[f"time_diff_{k + 1}"], out[f"word_diff_{k + 1}"] = sim[:, k], tdf[:, k], wdf[:, k]
    for k, f in enumerate(("sim_max", "sim_mean", "sim_min", "sim_std")):
        out[f] = stats[:, k]
    out["item_user_sim"], out["recall_in_user_cat"] = ius, ric
    return out
