"""GPU parity: DIN forward (src/rank/DIN.py:29-212 DINModel.forward in eval
mode) through the C ABI (nrk_din_forward).

Checker: the reference's own outputs (tests/golden/din_small.npz, fp32
tables) and the CPU oracle (oracle.din_forward) for other shapes and for
bf16-stored tables.  Tolerance: 1e-5 on probabilities and logits (the
north_star floating-point bar; absolute, plus 1e-5 relative for logits).
"""
import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _sd(g):
    return {k[4:]: g[k] for k in g.files if k.startswith("sd::")}


def _feats(g):
    return [list(map(str, g[k])) for k in ("user_feats", "item_feats", "ctx_feats")]


def _run(sd, feats, batch, table_dtype="fp32"):
    from nrk import ops

    p = ops.DinParams(sd, *feats, table_dtype=table_dtype, device="cuda")
    d = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to("cuda", dt)  # noqa: E731
    probs, lg = ops.din_forward(p, d(batch["user"], torch.int32), d(batch["item"], torch.int32),
                                d(batch["hist"], torch.int32), d(batch["ctx"], torch.int32),
                                d(batch["mask"], torch.float32), logits=True)
    torch.cuda.synchronize()
    return probs.cpu().numpy(), lg.cpu().numpy()


def _batch(g, tag):
    return {k: g[f"{tag}_{k}"].astype(np.int64 if k != "mask" else np.float32)
            for k in ("user", "item", "hist", "ctx", "mask")}


@pytest.mark.parametrize("tag", ["b512", "b4096", "b37"])
def test_din_golden(golden, tag):
    g = golden("din_small")
    probs, lg = _run(_sd(g), _feats(g), _batch(g, tag))
    np.testing.assert_allclose(probs, g[f"{tag}_probs"], atol=TOL, rtol=0)
    np.testing.assert_allclose(lg, g[f"{tag}_logits"], atol=TOL, rtol=TOL)


@pytest.mark.parametrize("tag", ["b512", "b37"])
def test_din_bf16_tables_vs_oracle(golden, tag):
    g = golden("din_small")
    sd, feats, b = _sd(g), _feats(g), _batch(g, tag)
    probs, lg = _run(sd, feats, b, table_dtype="bf16")
    po, lo, _ = oracle.din_forward(sd, b["user"], b["item"], b["hist"], b["ctx"], b["mask"], feats,
                                   round_bf16=True)
    np.testing.assert_allclose(probs, po, atol=TOL, rtol=0)
    np.testing.assert_allclose(lg, lo, atol=TOL, rtol=TOL)


def synth_model(rng, vocab_u, vocab_i, vocab_c, h1=200, h2=80, scale=0.05, dim=32):
    """Random DINModel-shaped state_dict (DIN.py:133-212 parameter names)
    at embedding width ``dim``."""
    f32 = np.float32
    uf = [f"u{n}" for n in range(len(vocab_u))]
    itf = [f"i{n}" for n in range(len(vocab_i))]
    cf = [f"c{n}" for n in range(len(vocab_c))]
    sd = {}
    for grp, names, voc in (("user_profile_embedding_dict", uf, vocab_u),
                            ("item_embedding_dict", itf, vocab_i),
                            ("context_embedding_dict", cf, vocab_c)):
        for f, v in zip(names, voc):
            sd[f"{grp}.{f}.weight"] = (rng.standard_normal((v, dim)) * 0.1).astype(f32)
    ni = len(itf)
    in_dim = dim * (len(uf) + len(cf) + 2 * ni)
    lin = lambda o, i: (rng.standard_normal((o, i)) * (scale * 8 / np.sqrt(i))).astype(f32)  # noqa: E731
    sd["activation_unit.mlp.0.weight"] = lin(36, 4 * dim * ni)
    sd["activation_unit.mlp.0.bias"] = (rng.standard_normal(36) * 0.1).astype(f32)
    sd["activation_unit.mlp.2.weight"] = lin(1, 36)
    sd["activation_unit.mlp.2.bias"] = np.array([0.1], f32)
    sd["mlp.0.weight"], sd["mlp.0.bias"] = lin(h1, in_dim), (rng.standard_normal(h1) * 0.1).astype(f32)
    sd["mlp.2.weight"], sd["mlp.2.bias"] = lin(h2, h1), (rng.standard_normal(h2) * 0.1).astype(f32)
    sd["mlp.4.weight"], sd["mlp.4.bias"] = lin(1, h2), np.array([-0.2], f32)
    return sd, (uf, itf, cf)


def synth_batch(rng, B, T, vocab_u, vocab_i, vocab_c, p_empty=0.05):
    L = rng.integers(0, T + 1, B)
    L[rng.random(B) < p_empty] = 0
    mask = (np.arange(T)[None] < L[:, None]).astype(np.float32)
    hist = np.stack([rng.integers(0, v, (B, T)) for v in vocab_i], 2) * mask[:, :, None].astype(np.int64)
    return {
        "user": np.stack([rng.integers(0, v, B) for v in vocab_u], 1),
        "item": np.stack([rng.integers(0, v, B) for v in vocab_i], 1),
        "hist": hist,
        "ctx": np.stack([rng.integers(0, v, B) for v in vocab_c], 1) if vocab_c else np.zeros((B, 0), np.int64),
        "mask": mask,
    }


@pytest.mark.parametrize(
    "B,T,n_item,n_ctx,h1,h2",
    [
        (2, 1, 4, 16, 200, 80),
        (3, 50, 4, 16, 200, 80),
        (100, 7, 1, 0, 64, 32),
        (257, 128, 2, 3, 128, 64),
        (1000, 50, 4, 11, 200, 80),
        (5000, 33, 4, 16, 256, 100),
    ],
)
@pytest.mark.parametrize("table_dtype", ["fp32", "bf16"])
def test_din_vs_oracle(B, T, n_item, n_ctx, h1, h2, table_dtype):
    rng = np.random.default_rng(B * 131 + T)
    vu, vi, vc = [50, 300, 7, 2000, 90], [60, 900, 5000, 70][:n_item], [12] * n_ctx
    sd, feats = synth_model(rng, vu, vi, vc, h1, h2)
    b = synth_batch(rng, B, T, vu, vi, vc)
    probs, lg = _run(sd, feats, b, table_dtype)
    po, lo, _ = oracle.din_forward(sd, b["user"], b["item"], b["hist"], b["ctx"], b["mask"], feats,
                                   round_bf16=table_dtype == "bf16")
    np.testing.assert_allclose(probs, po, atol=TOL, rtol=0)
    np.testing.assert_allclose(lg, lo, atol=TOL, rtol=TOL)


@pytest.mark.parametrize(
    "dim,n_item,T,B,table_dtype",
    [
        (16, 4, 50, 700, "bf16"),   # din_embedding_dim 16: tables zero-padded to 32
        (16, 3, 30, 300, "fp32"),   # 3 item features -> padded to 4 with the zero row
        (64, 4, 50, 700, "bf16"),   # 64 = two 32-wide virtual features each -> 8 item features
        (64, 2, 50, 700, "bf16"),   # 2 x 2 = 4 virtual item features: the position-major path with padding rows
        (64, 2, 70, 257, "fp32"),   # T > 64 (general path) at 4 virtual item features
        (8, 1, 20, 129, "bf16"),    # tiny width, one item feature
        (48, 3, 50, 200, "bf16"),   # 48 -> 64 padded, 2 x 3 = 6 -> 8 item features
        (32, 3, 50, 500, "bf16"),   # 3 item features at the native width
        (32, 6, 40, 300, "fp32"),   # 6 -> 8
    ],
)
def test_din_embedding_dims_vs_oracle(dim, n_item, T, B, table_dtype):
    """Any din_embedding_dim (config.py:115) and item-feature count: the
    32-wide virtual-feature layout of ops.DinParams (zero padding, split
    rows, padding features) against the oracle run at the model's own width."""
    rng = np.random.default_rng(dim * 1000 + n_item * 10 + T)
    vu, vi, vc = [50, 300, 7], [60, 900, 5000, 70, 40, 33][:n_item], [12] * 5
    sd, feats = synth_model(rng, vu, vi, vc, dim=dim)
    b = synth_batch(rng, B, T, vu, vi, vc)
    probs, lg = _run(sd, feats, b, table_dtype)
    po, lo, _ = oracle.din_forward(sd, b["user"], b["item"], b["hist"], b["ctx"], b["mask"], feats,
                                   round_bf16=table_dtype == "bf16")
    np.testing.assert_allclose(probs, po, atol=TOL, rtol=0)
    np.testing.assert_allclose(lg, lo, atol=TOL, rtol=TOL)


@pytest.mark.parametrize("dim,n_item", [(64, 2), (64, 1), (128, 1), (16, 3)])
def test_din_virtual_indices_keep_padding_zero(dim, n_item):
    """ops.DinParams' virtual-feature layout keeps the collate's padding (caller
    index 0) at virtual index 0 in every 32-wide half, so the position-major
    plan recognises padding rows (mask 0, every index 0) at any embedding width
    (ADVICE r4), and every other caller index i of feature f addresses the rows
    fb[f] + hh + m i of its halves."""
    from nrk import ops

    rng = np.random.default_rng(dim + n_item)
    vu, vi, vc = [50, 300], [60, 900, 5000][:n_item], [12] * 2
    sd, feats = synth_model(rng, vu, vi, vc, dim=dim)
    p = ops.DinParams(sd, *feats, table_dtype="bf16", device="cuda")
    b = synth_batch(rng, 64, 20, vu, vi, vc, p_empty=0.3)
    t = {k: torch.from_numpy(np.ascontiguousarray(v, np.int32)).cuda() for k, v in b.items() if k != "mask"}
    _, _, hist, _ = p.kernel_indices(t["user"], t["item"], t["hist"], t["ctx"])
    hist = hist.cpu().numpy()
    pad = b["mask"] == 0
    assert pad.any() and (hist[pad] == 0).all()
    m = max(1, -(-dim // 32))
    table = p.table.float().cpu().numpy()
    rb = p.row_base.cpu().numpy()
    emb = sd[f"item_embedding_dict.{feats[1][0]}.weight"]
    r, tt = np.argwhere(~pad)[0]
    i0 = int(b["hist"][r, tt, 0])
    row = np.concatenate([table[rb[p.kn_user + hh] + hist[r, tt, hh]] for hh in range(m)])[:dim]
    np.testing.assert_allclose(row, emb[i0], atol=1e-2)  # bf16 table


def test_din_all_history_masked():
    rng = np.random.default_rng(5)
    vu, vi, vc = [50, 300], [60, 900, 5000, 70], [12, 12]
    sd, feats = synth_model(rng, vu, vi, vc)
    b = synth_batch(rng, 64, 50, vu, vi, vc, p_empty=1.0)
    probs, lg = _run(sd, feats, b)
    po, lo, _ = oracle.din_forward(sd, b["user"], b["item"], b["hist"], b["ctx"], b["mask"], feats)
    np.testing.assert_allclose(probs, po, atol=TOL, rtol=0)


@pytest.mark.parametrize("case", ["holes", "unit_masks", "full", "mixed_len", "t64", "t1"])
def test_din_position_major_edges(case):
    """The position-major attention kernel (bf16 tables, T <= 64) computes
    only rows before each sample's last non-padding row and enters the
    padding rows' h through a per-sample pad row: masks that are not
    prefixes (mask 0 with non-zero indices, mask != 0 with all-zero
    indices, fractional masks), every row real, ragged lengths around the
    16-row tiles, T = 64 and T = 1 -- all against the oracle at 1e-5."""
    rng = np.random.default_rng(["holes", "unit_masks", "full", "mixed_len", "t64", "t1"].index(case) + 71)
    vu, vi, vc = [50, 300, 7], [60, 900, 5000, 70], [12] * 4
    sd, feats = synth_model(rng, vu, vi, vc)
    T = {"t64": 64, "t1": 1}.get(case, 50)
    B = 700
    b = synth_batch(rng, B, T, vu, vi, vc)
    if case == "holes":
        # interior padding-like rows (mask 0, indices 0), masked rows with real
        # indices, and unmasked rows whose indices are all 0
        b["mask"][:, 3:6] = 0.0
        b["hist"][:, 3:5] = 0
        b["hist"][:50, 40] = 7
        b["mask"][60:90, 45] = 1.0
        b["hist"][60:90, 45] = 0
    elif case == "unit_masks":
        b["mask"] = b["mask"] * rng.choice([0.5, 1.0, 2.0], size=b["mask"].shape).astype(np.float32)
    elif case == "full":
        b["mask"][:] = 1.0
        b["hist"] = np.stack([rng.integers(1, v, (B, T)) for v in vi], 2)
    elif case == "mixed_len":
        L = rng.choice([0, 1, 15, 16, 17, 31, 32, 33, T], size=B)
        b["mask"] = (np.arange(T)[None] < L[:, None]).astype(np.float32)
        b["hist"] = b["hist"] * b["mask"][:, :, None].astype(np.int64)
    probs, lg = _run(sd, feats, b, "bf16")
    po, lo, _ = oracle.din_forward(sd, b["user"], b["item"], b["hist"], b["ctx"], b["mask"], feats,
                                   round_bf16=True)
    np.testing.assert_allclose(probs, po, atol=TOL, rtol=0)
    np.testing.assert_allclose(lg, lo, atol=TOL, rtol=TOL)


def test_din_errors():
    from nrk import ops

    rng = np.random.default_rng(1)
    vu, vi, vc = [50], [60, 900, 5000, 70], [12]
    sd, feats = synth_model(rng, vu, vi, vc)
    b = synth_batch(rng, 8, 10, vu, vi, vc)
    b["item"][3, 2] = 5000  # out of the table
    with pytest.raises(ValueError):
        _run(sd, feats, b)
    p = ops.DinParams(sd, *feats, device="cuda")
    one = {k: torch.from_numpy(np.ascontiguousarray(v[:1])).cuda() for k, v in b.items()}
    with pytest.raises(ValueError):  # batch of one: Dice std undefined, rejected at the boundary
        ops.din_forward(p, one["user"].int(), one["item"].int(), one["hist"].int(),
                        one["ctx"].int(), one["mask"].float())


def test_din_config3_batch():
    """Config 3 shapes: B=4096, T=50, Tianchi-sized vocabularies, bf16 tables."""
    rng = np.random.default_rng(3)
    vu, vi, vc = [200, 5000, 6, 200000, 3000], [462, 3000, 300000, 1500], [11] * 16
    sd, feats = synth_model(rng, vu, vi, vc)
    b = synth_batch(rng, 4096, 50, vu, vi, vc)
    probs, lg = _run(sd, feats, b, "bf16")
    po, lo, _ = oracle.din_forward(sd, b["user"], b["item"], b["hist"], b["ctx"], b["mask"], feats,
                                   round_bf16=True)
    np.testing.assert_allclose(probs, po, atol=TOL, rtol=0)
    np.testing.assert_allclose(lg, lo, atol=TOL, rtol=TOL)


@pytest.mark.parametrize("N,S,table_dtype", [(1000, 128, "bf16"), (257, 64, "fp32"), (2 * 4096 + 77, 4096, "bf16"),
                                               (1000, 192, "bf16"), (700, 64, "bf16"), (4096 + 2, 4096, "bf16")])
def test_din_segments_vs_per_batch_oracle(N, S, table_dtype):
    """nrk_din_forward_segments: N samples as consecutive Dice batches of S in
    one call == the oracle run batch by batch (DINRanker.predict's loop);
    a trailing one-row batch is NaN."""
    from nrk import ops

    rng = np.random.default_rng(N + S)
    vu, vi, vc = [50, 300, 7, 2000, 90], [60, 900, 5000, 70], [12] * 16
    sd, feats = synth_model(rng, vu, vi, vc)
    b = synth_batch(rng, N, 50, vu, vi, vc)
    p = ops.DinParams(sd, *feats, table_dtype=table_dtype, device="cuda")
    d = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to("cuda", dt)  # noqa: E731
    probs, lg = ops.din_forward(p, d(b["user"], torch.int32), d(b["item"], torch.int32),
                                d(b["hist"], torch.int32), d(b["ctx"], torch.int32),
                                d(b["mask"], torch.float32), logits=True, batch_size=S)
    probs, lg = probs.cpu().numpy(), lg.cpu().numpy()
    for s in range(0, N, S):
        e = min(N, s + S)
        if e - s == 1:
            assert np.isnan(probs[s]) and np.isnan(lg[s])
            continue
        po, lo, _ = oracle.din_forward(sd, *(b[k][s:e] for k in ("user", "item", "hist", "ctx", "mask")),
                                       feats, round_bf16=table_dtype == "bf16")
        np.testing.assert_allclose(probs[s:e], po, atol=TOL, rtol=0)
        np.testing.assert_allclose(lg[s:e], lo, atol=TOL, rtol=TOL)


def test_din_segments_errors():
    from nrk import ops

    rng = np.random.default_rng(2)
    vu, vi, vc = [50], [60, 900, 5000, 70], [12]
    sd, feats = synth_model(rng, vu, vi, vc)
    b = synth_batch(rng, 300, 10, vu, vi, vc)
    p = ops.DinParams(sd, *feats, device="cuda")
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in b.items()}
    with pytest.raises(ValueError):  # several batches need a multiple-of-64 batch size
        ops.din_forward(p, t["user"].int(), t["item"].int(), t["hist"].int(), t["ctx"].int(),
                        t["mask"].float(), batch_size=100)


def test_din_ranker_predict_batches(golden):
    """DINRanker.predict batching: short last batch scored with its own
    statistics; a trailing batch of one row is NaN as in the reference."""
    from nrk.rank.din import DINScorer

    g = golden("din_small")
    sd, feats, b = _sd(g), _feats(g), _batch(g, "b512")
    sc = DINScorer(sd, *feats)
    out = sc.predict(b, 100)
    for s in range(0, 512, 100):
        e = min(512, s + 100)
        po, _, _ = oracle.din_forward(sd, *(b[k][s:e] for k in ("user", "item", "hist", "ctx", "mask")),
                                      feats)
        np.testing.assert_allclose(out[s:e], po, atol=TOL, rtol=0)
    out2 = sc.predict({k: v[:201] for k, v in b.items()}, 100)
    assert np.isnan(out2[200]) and not np.isnan(out2[:200]).any()
    # multiple-of-64 batch size: the one-call segmented path
    out3 = sc.predict(b, 128)
    for s in range(0, 512, 128):
        po, _, _ = oracle.din_forward(sd, *(b[k][s:s + 128] for k in ("user", "item", "hist", "ctx", "mask")),
                                      feats)
        np.testing.assert_allclose(out3[s:s + 128], po, atol=TOL, rtol=0)
    out4 = sc.predict({k: v[:129] for k, v in b.items()}, 128)
    assert np.isnan(out4[128]) and not np.isnan(out4[:128]).any()


def _reference_rank_and_recommend(main_df, probs, top_k):
    """rank_pipeline.py:162-172, executed with pandas exactly as written there."""
    df = main_df.copy()
    df["rank_score"] = probs
    rec = {}
    for user_id, group in df.groupby("user_id"):
        top_items = group.nlargest(top_k, "rank_score")[["item_id", "rank_score"]]
        rec[str(user_id)] = [(str(row["item_id"]), float(row["rank_score"])) for _, row in top_items.iterrows()]
    return rec


@pytest.mark.parametrize("n_rows,n_users,top_k", [(1, 1, 10), (5000, 700, 10), (20000, 300, 64), (3000, 2999, 3),
                                                  (30000, 200, 150)])
def test_rank_and_recommend_matches_reference(n_rows, n_users, top_k, tmp_path):
    """RankPipeline.rank_and_recommend (rank_pipeline.py:143-191): per-user
    nlargest with first-occurrence ties, NaN after numbers, float-formatted item ids."""
    import pickle

    import pandas as pd

    from nrk.rank.recommend import rank_and_recommend

    rng = np.random.default_rng(n_rows + top_k)
    main_df = pd.DataFrame({"user_id": rng.integers(0, n_users, n_rows) * 3 + 1,
                            "item_id": rng.integers(0, 10**6, n_rows)})
    probs = (np.round(rng.random(n_rows) * 40) / 40).astype(np.float32)  # many exact ties
    probs[rng.random(n_rows) < 0.01] = np.nan
    probs[main_df["user_id"].to_numpy() == main_df["user_id"].iloc[0]] = np.nan  # a user with only NaN scores
    ref = _reference_rank_and_recommend(main_df, probs, top_k)
    path = str(tmp_path / "rec.pkl")
    got = rank_and_recommend(main_df, torch.from_numpy(probs).cuda(), top_k, save_path=path)
    assert list(got) == list(ref)
    sizes = main_df.groupby("user_id").size()

    def same(a, b, n_rows):
        if not np.array_equal([y for _, y in a], [y for _, y in b], equal_nan=True):
            return False
        if n_rows > top_k:  # nlargest's selection path: mergesort, ties in row order
            return a == b or [x for x, _ in a] == [x for x, _ in b]
        # n >= len(group): nlargest falls back to sort_values(kind="quicksort"), whose
        # numpy SIMD argsort orders exact ties hardware-dependently -> equal sets per score
        key = lambda lst: sorted((str(y), x) for x, y in lst)  # noqa: E731
        return key(a) == key(b)

    for u in ref:
        assert same(got[u], ref[u], int(sizes[int(u)])), u
    with open(path, "rb") as f:
        saved = pickle.load(f)
    assert all(same(saved[u], ref[u], int(sizes[int(u)])) for u in ref)
