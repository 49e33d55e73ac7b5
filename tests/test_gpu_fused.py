"""GPU parity: the fused recall -> rank hand-off (BASELINE config 5).

nrk_din_assemble is checked element-for-element against a numpy
restatement of the same layout (DIN.py:330-520 encoding: left-aligned last-T
history, index 0 and mask 0 on padding; rank 0 of the recall dropped as
youtubednn_recaller.py:524).  FusedRecallRank is checked against the oracle
for both stages: recall rows / scores bit-exact, DIN probabilities per Dice
batch within 1e-5 (the north_star bar), chunking invisible.
"""
import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu
TOL = 1e-5
M32 = np.uint64(0xFFFFFFFF)


def _mix32(x):
    x = x.astype(np.uint64) & M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & M32
    x ^= x >> np.uint64(16)
    return x


def ref_assemble(rows, scores, user_feat, item_feat, user_hist, hist_len, u0, nu, k, skip, n_ctx, bins, lo, hi, seed):
    P = nu * k
    u = u0 + np.arange(P) // k
    c = np.arange(P) % k + skip
    row = rows[u, c]
    item = np.where(row >= 0, row, 0)
    T = user_hist.shape[1]
    mask = (np.arange(T)[None] < hist_len[u][:, None]).astype(np.float32)
    hist = np.where(mask[:, :, None] > 0, item_feat[user_hist[u]], 0)
    s = scores[u, c].astype(np.float32)
    inv = np.float32(bins) / (np.float32(hi) - np.float32(lo))
    b = np.floor((s - np.float32(lo)) * inv).astype(np.int64)
    ctx = np.zeros((P, n_ctx), np.int64)
    if n_ctx:
        ctx[:, 0] = np.clip(b, 0, bins - 1) + 1
    uu = (u.astype(np.uint64) * np.uint64(0x9E3779B9)) & M32
    for f in range(1, n_ctx):
        h = _mix32(uu ^ _mix32((item.astype(np.uint64) + np.uint64(0x85EBCA6B) * np.uint64(f)) & M32) ^ np.uint64(seed))
        ctx[:, f] = (h % np.uint64(bins)).astype(np.int64) + 1
    return {"user": user_feat[u], "item": item_feat[item], "hist": hist, "ctx": ctx, "mask": mask, "cand": row}


def _world(rng, U, I, D, T, vu, vi):
    users = rng.standard_normal((U, D)).astype(np.float32)
    users /= np.linalg.norm(users, axis=1, keepdims=True)
    items = rng.standard_normal((I, D)).astype(np.float32)
    items /= np.linalg.norm(items, axis=1, keepdims=True)
    user_feat = np.stack([rng.integers(0, v, U) for v in vu], 1).astype(np.int32)
    item_feat = np.stack([rng.integers(0, v, I) for v in vi], 1).astype(np.int32)
    user_hist = rng.integers(0, I, (U, T)).astype(np.int32)
    hist_len = rng.integers(0, T + 1, U).astype(np.int32)
    return users, items, user_feat, item_feat, user_hist, hist_len


def test_din_assemble_vs_numpy():
    from nrk import ops

    rng = np.random.default_rng(5)
    U, I, k_in, T = 300, 1000, 31, 50
    rows = rng.integers(-1, I, (U, k_in)).astype(np.int32)
    scores = (rng.random((U, k_in)) * 2.2 - 1.1).astype(np.float32)  # also outside [lo, hi]
    _, _, user_feat, item_feat, user_hist, hist_len = _world(rng, U, I, 8, T, [7, 50, 3], [9, 40, 200, 5])
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    for u0, nu, k, skip, n_ctx in ((0, U, 30, 1, 16), (17, 100, 5, 3, 1), (299, 1, 31, 0, 0)):
        got = ops.din_assemble(d(rows), d(scores), d(user_feat), d(item_feat), d(user_hist), d(hist_len),
                               u0, nu, k_use=k, skip=skip, n_ctx=n_ctx, ctx_bins=10, seed=77)
        ref = ref_assemble(rows, scores, user_feat, item_feat, user_hist, hist_len, u0, nu, k, skip, n_ctx,
                           10, -1.0, 1.0, 77)
        for key in ("user", "item", "hist", "ctx", "mask", "cand"):
            assert np.array_equal(got[key].cpu().numpy(), ref[key]), key


@pytest.mark.parametrize("chunk", [2048, 4096])
def test_fused_recall_rank_vs_oracle(chunk):
    from nrk import ops
    from nrk.pipeline import FusedRecallRank
    from test_gpu_din import synth_model

    rng = np.random.default_rng(chunk)
    U, I, D, T, k = 2500, 3000, 128, 50, 30
    vu, vi, vc = [50, 300, 7, 2000, 90], [60, 900, 5000, 70], [11] * 16
    users, items, user_feat, item_feat, user_hist, hist_len = _world(rng, U, I, D, T, vu, vi)
    sd, feats = synth_model(rng, vu, vi, vc)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    p = ops.DinParams(sd, *feats, table_dtype="bf16")
    fused = FusedRecallRank(ops.Catalog(d(items)), p, d(user_feat), d(item_feat), d(user_hist), d(hist_len),
                            k=k, chunk_users=chunk)
    s, r = fused.recall(d(users))
    so, ro = oracle.ip_topk(users, items, k + 1)
    assert np.array_equal(r.cpu().numpy().astype(np.int64), ro)
    assert np.array_equal(s.cpu().numpy(), so)
    probs, cand = fused.rank(s, r)
    probs, cand = probs.cpu().numpy(), cand.cpu().numpy()
    a = ref_assemble(ro.astype(np.int32), so, user_feat, item_feat, user_hist, hist_len, 0, U, k, 1, 16,
                     10, -1.0, 1.0, 23)
    assert np.array_equal(cand, a["cand"])
    B = 4096
    for b0 in range(0, U * k, B):
        sl = slice(b0, min(b0 + B, U * k))
        po, _, _ = oracle.din_forward(sd, a["user"][sl], a["item"][sl], a["hist"][sl], a["ctx"][sl], a["mask"][sl],
                                      feats, round_bf16=True)
        np.testing.assert_allclose(probs[sl], po, atol=TOL, rtol=0)


def _ctx_world(rng, users, items, user_hist, hist_len, n_cat=12):
    """Context tables over catalog rows / user rows (str keys for the oracle),
    with gaps: items without a w2v vector / content row / created time, all-zero
    content rows, users without history."""
    I, U = len(items), len(users)
    w2v = {str(i): (rng.standard_normal(64) * 0.3).astype(np.float32) for i in range(I) if rng.random() < 0.9}
    content = {str(i): rng.standard_normal(250) for i in range(I) if rng.random() < 0.9}
    for key in list(content)[:20]:
        content[key] = np.zeros(250)
    created = {str(i): np.float64(rng.random()) for i in range(I) if rng.random() < 0.9}
    ctype = {str(i): int(rng.integers(0, n_cat)) for i in range(I)}
    hist = {str(u): [str(x) for x in user_hist[u, :hist_len[u]]] for u in range(U) if hist_len[u] > 0}
    user_yt = {str(u): users[u] for u in range(U)}
    art_yt = {str(i): items[i] for i in range(I)}
    return w2v, content, created, ctype, hist, user_yt, art_yt


def test_fused_with_context_features():
    """Config-5 path with the reference's context features: the fused
    pipeline's codes are the fitted spec applied to nrk_ctx_features' raw
    values, those raw values match the oracle restatement of
    feature_extractor.py:440-723 (1e-5; exact for the float64 paths), and the
    DIN probabilities match the oracle on the same codes (1e-5)."""
    import warnings

    from nrk import ops
    from nrk.features import CtxSpec, CtxTables, ctx_feature_names, ctx_features
    from nrk.pipeline import FusedRecallRank
    from test_ctxfeat_oracle import apply_spec_host
    from test_gpu_din import synth_model

    warnings.simplefilter("ignore")
    rng = np.random.default_rng(41)
    U, I, D, T, k = 700, 1500, 64, 50, 30
    vu, vi, vc = [50, 300, 7, 2000, 90], [60, 900, 5000, 70], [24] * 16
    users, items, user_feat, item_feat, user_hist, hist_len = _world(rng, U, I, D, T, vu, vi)
    w2v, content, created, ctype, hist, user_yt, art_yt = _ctx_world(rng, users, items, user_hist, hist_len)
    tables = CtxTables([str(i) for i in range(I)], [str(u) for u in range(U)], w2v, content, created, ctype, hist,
                       user_yt=user_yt, item_yt=art_yt)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    so, ro = oracle.ip_topk(users, items, k + 1)
    names = ctx_feature_names()
    pu = np.repeat(np.arange(U), k).astype(np.int32)
    pi = ro[:, 1:].reshape(-1).astype(np.int32)
    ps = so[:, 1:].reshape(-1).astype(np.float64)
    raw, _ = ctx_features(tables, d(pu), d(pi), d(ps))
    raw = raw.cpu().numpy()
    exp = oracle.ctx_features([str(u) for u in pu], [str(i) for i in pi], ps, hist, w2v, content, created, ctype,
                              user_yt, art_yt)
    for j, f in enumerate(names):
        if f.startswith("sim") or f == "item_user_sim":
            np.testing.assert_allclose(raw[:, j], exp[f], rtol=1e-5, atol=1e-5, equal_nan=True, err_msg=f)
        else:
            assert np.array_equal(raw[:, j], exp[f].astype(np.float64), equal_nan=True), f
    spec = CtxSpec.fit({f: (raw[:, j].astype(np.float32) if f != "score" else raw[:, j]) for j, f in enumerate(names)},
                       names)
    codes = np.stack([apply_spec_host(spec.specs[j], raw[:, j]) for j in range(len(names))], 1)
    sd, feats = synth_model(rng, vu, vi, vc)
    p = ops.DinParams(sd, *feats, table_dtype="bf16")
    fused = FusedRecallRank(ops.Catalog(d(items)), p, d(user_feat), d(item_feat), d(user_hist), d(hist_len),
                            k=k, chunk_users=2048, ctx=(tables, spec))
    s, r = fused.recall(d(users))
    assert np.array_equal(r.cpu().numpy().astype(np.int64), ro)
    probs, cand = fused.rank(s, r)
    probs = probs.cpu().numpy()
    a = ref_assemble(ro.astype(np.int32), so, user_feat, item_feat, user_hist, hist_len, 0, U, k, 1, 16,
                     10, -1.0, 1.0, 23)
    B = 4096
    for b0 in range(0, U * k, B):
        sl = slice(b0, min(b0 + B, U * k))
        po, _, _ = oracle.din_forward(sd, a["user"][sl], a["item"][sl], a["hist"][sl], codes[sl], a["mask"][sl],
                                      feats, round_bf16=True)
        np.testing.assert_allclose(probs[sl], po, atol=TOL, rtol=0)


def test_fused_rejects_bad_tables():
    from nrk import ops
    from nrk.pipeline import FusedRecallRank
    from test_gpu_din import synth_model

    rng = np.random.default_rng(3)
    U, I, D, T = 100, 300, 32, 50
    vu, vi, vc = [50, 300, 7, 2000, 90], [60, 900, 5000, 70], [11] * 16
    users, items, user_feat, item_feat, user_hist, hist_len = _world(rng, U, I, D, T, vu, vi)
    sd, feats = synth_model(rng, vu, vi, vc)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    p = ops.DinParams(sd, *feats, table_dtype="bf16")
    bad_hist = user_hist.copy()
    bad_hist[5, 3] = I  # out of the item table
    with pytest.raises(ValueError):
        FusedRecallRank(ops.Catalog(d(items)), p, d(user_feat), d(item_feat), d(bad_hist), d(hist_len))
    bad_feat = item_feat.copy()
    bad_feat[7, 2] = 5000  # == vocab
    with pytest.raises(ValueError):
        FusedRecallRank(ops.Catalog(d(items)), p, d(user_feat), d(bad_feat), d(user_hist), d(hist_len))
    bad_len = hist_len.copy()
    bad_len[0] = T + 1
    with pytest.raises(ValueError):
        FusedRecallRank(ops.Catalog(d(items)), p, d(user_feat), d(item_feat), d(user_hist), d(bad_len))
