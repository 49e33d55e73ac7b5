"""GPU parity: ip_topk (faiss.IndexFlatIP replacement) and the two-tower forward.

Checker = the CPU oracle (oracle/) and the golden fixtures from the reference.
Bar: bit-exact row indices (ties -> lower row), scores equal to the fp32
rounding of the exact fp64 score (so exact equality is expected; the
reference's own tolerance 1e-5 is the documented bar).
"""
import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops():
    from nrk import ops as _ops

    return _ops


def _dev(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.cuda()


def _run_topk(ops, users, items, k, row_offset=0):
    cat = ops.Catalog(_dev(items, torch.float32))
    s, r, e = ops.ip_topk(_dev(users, torch.float32), cat, k, row_offset=row_offset, exact=True)
    torch.cuda.synchronize()
    return s.cpu().numpy(), r.cpu().numpy().astype(np.int64), e.cpu().numpy()


@pytest.mark.parametrize("tag", ["a", "b"])
def test_ip_topk_golden(ops, golden, tag):
    g = golden("topk_small")
    k = int(g["k"]) + 1
    s, r, e = _run_topk(ops, g[f"{tag}_users"], g[f"{tag}_items"], k)
    assert np.array_equal(r, g[f"{tag}_I"])
    assert np.array_equal(s, g[f"{tag}_D"])


def test_ip_topk_padding_golden(ops, golden):
    g = golden("topk_small")
    k = g["small_I"].shape[1]
    s, r, _ = _run_topk(ops, g["a_users"][:4], g["a_items"][:10], k)
    assert np.array_equal(r, g["small_I"])
    assert np.array_equal(s, g["small_D"])


def _unit(x):
    n = np.linalg.norm(x, axis=1, keepdims=True)
    n[n == 0] = 1
    return (x / n).astype(np.float32)


@pytest.mark.parametrize(
    "n_users,n_items,d,k",
    [
        (1, 1, 32, 1),
        (3, 31, 32, 31),
        (129, 33, 32, 31),
        (300, 1000, 32, 31),
        (257, 5003, 32, 32),
        (130, 4097, 16, 10),
        (70, 3000, 50, 21),
        (200, 2500, 64, 31),
        (64, 2000, 128, 31),
        (40, 1500, 250, 21),
    ],
)
def test_ip_topk_vs_oracle(ops, n_users, n_items, d, k):
    rng = np.random.default_rng(n_users * 7 + n_items + d)
    users = _unit(rng.standard_normal((n_users, d)))
    items = _unit(rng.standard_normal((n_items, d)))
    s, r, e = _run_topk(ops, users, items, k)
    so, ro, eo = oracle.ip_topk(users, items, k, exact=True)
    assert np.array_equal(r, ro)
    assert np.array_equal(s, so)
    assert np.array_equal(e[ro >= 0], eo[ro >= 0])


@pytest.mark.parametrize(
    "n_users,n_items,d,k",
    [
        (130, 40000, 32, 10),  # UG = 4 scan, 4-slot ring: 312 tiles, list pre-pass of 52
        (300, 12000, 64, 61),  # MT = 32, two waves / SIMD (staggered): 187 tiles
        (257, 20000, 128, 31),  # one block per tile: 625 tiles, pre-pass of 64
        (100, 9000, 250, 21),  # 16-KB tiles: 281 tiles
        (64, 32700, 16, 31),  # 8 blocks per tile: 128 tiles, the smallest range with a pre-pass (21)
    ],
)
def test_ip_topk_list_prepass_vs_oracle(ops, n_users, n_items, d, k):
    """Ranges of >= 128 tiles run the scan's sampled list pre-pass (tile
    maxima of up to 64 tiles spread over the range seed tau, the main pass
    does not insert them again): bit-exact rows and scores against the
    oracle on every scan instantiation it applies to."""
    rng = np.random.default_rng(n_users * 11 + n_items + d)
    users = _unit(rng.standard_normal((n_users, d)))
    items = _unit(rng.standard_normal((n_items, d)))
    s, r, e = _run_topk(ops, users, items, k)
    so, ro, eo = oracle.ip_topk(users, items, k, exact=True)
    assert np.array_equal(r, ro)
    assert np.array_equal(s, so)
    assert np.array_equal(e[ro >= 0], eo[ro >= 0])


@pytest.mark.parametrize(
    "n_users,n_items",
    [
        (1500, 100),  # one tile: a single, short step
        (1500, 7 * 128),  # 7 tiles: no insert-period boundary, the pending maxima flushed at the end
        (1500, 129 * 128),  # 129 tiles + an odd 21-tile pre-pass: 150 tiles in the sequence
        (1500, 130 * 128 - 5),  # 151 tiles (a short last step) and a masked last block
        (1100, 131 * 128 + 77),  # 132 tiles, a partial last tile; 76 users past the first 1,024-user block
    ],
)
def test_ip_topk_ws_steps_vs_oracle(ops, n_users, n_items):
    """The warp-specialized config-2 scan (D = 32, k = 31): two tiles per
    barrier step, main-pass inserts every 8 tiles, the pre-pass and main pass
    as one sequence -- odd sequence lengths, odd pre-passes, ranges shorter
    than the insert period, masked tails and a partial user block, bit-exact
    against the oracle."""
    rng = np.random.default_rng(n_users * 7 + n_items)
    users = _unit(rng.standard_normal((n_users, 32)))
    items = _unit(rng.standard_normal((n_items, 32)))
    s, r, e = _run_topk(ops, users, items, 31)
    so, ro, eo = oracle.ip_topk(users, items, 31, exact=True)
    assert np.array_equal(r, ro)
    assert np.array_equal(s, so)
    assert np.array_equal(e[ro >= 0], eo[ro >= 0])


def test_ip_topk_unnormalised_and_offset(ops):
    rng = np.random.default_rng(3)
    users = (rng.standard_normal((150, 32)) * 5).astype(np.float32)
    items = (rng.standard_normal((2000, 32)) * rng.random((2000, 1)) * 3).astype(np.float32)
    s, r, _ = _run_topk(ops, users, items, 31, row_offset=1000)
    so, ro = oracle.ip_topk(users, items, 31)
    assert np.array_equal(r, ro + 1000)
    assert np.array_equal(s, so)


def test_ip_topk_ties_overflow_fallback(ops):
    # heavy exact duplicates -> candidate band overflows -> exact fallback path
    rng = np.random.default_rng(9)
    base = _unit(rng.standard_normal((4, 32)))
    items = base[rng.integers(0, 4, size=6000)]
    users = _unit(rng.standard_normal((64, 32)))
    users[:8] = 0.0
    users[8:16] = base[rng.integers(0, 4, size=8)]
    s, r, _ = _run_topk(ops, users, items, 31)
    so, ro = oracle.ip_topk(users, items, 31)
    assert np.array_equal(r, ro)
    assert np.array_equal(s, so)


@pytest.mark.parametrize(
    "n_users,n_items,d,k",
    [
        (300, 5000, 32, 61),    # RecallEnsemble's recall(uid, 2 * 30) -> k + 1 = 61 (fusion.py:478)
        (257, 20000, 32, 101),
        (130, 7000, 32, 128),   # largest k on the screen path
        (66, 3001, 16, 64),
        (70, 4000, 64, 77),
        (40, 1500, 250, 65),    # EmbeddingSimilarity width
        (33, 2500, 32, 129),    # exact path (k > 128)
        (20, 1200, 32, 700),
        (9, 500, 32, 600),      # k > n_items: -1 / -FLT_MAX padding
    ],
)
def test_ip_topk_large_k_vs_oracle(ops, n_users, n_items, d, k):
    """k beyond round 2's cap of 32: the screen path up to k = 128, the exact
    path above it; bit-exact rows and scores."""
    rng = np.random.default_rng(n_users + n_items + d + k)
    users = _unit(rng.standard_normal((n_users, d)))
    users[0] = 0.0  # zero user: all-tie row
    items = _unit(rng.standard_normal((n_items, d)))
    s, r, e = _run_topk(ops, users, items, k)
    so, ro, eo = oracle.ip_topk(users, items, k, exact=True)
    assert np.array_equal(r, ro)
    assert np.array_equal(s, so)
    assert np.array_equal(e[ro >= 0], eo[ro >= 0])


@pytest.mark.parametrize("k", [61, 101, 200])
def test_ip_topk_large_k_ties(ops, k):
    """Tie stress at large k: duplicated catalog rows, quantised vectors,
    users equal to catalog rows (exact ties across the k-th place)."""
    rng = np.random.default_rng(k)
    base = _unit(rng.standard_normal((40, 32)))
    items = np.concatenate([base[rng.integers(0, 40, size=3000)],
                            _unit(np.round(rng.standard_normal((3000, 32)) * 2) / 2)]).astype(np.float32)
    users = _unit(rng.standard_normal((96, 32)))
    users[:4] = 0.0
    users[4:24] = base[rng.integers(0, 40, size=20)]
    s, r, _ = _run_topk(ops, users, items, k)
    so, ro = oracle.ip_topk(users, items, k)
    assert np.array_equal(r, ro)
    assert np.array_equal(s, so)


def test_recall_ensemble_style_call(golden):
    """RecallEnsemble.recall calls recall(user_id, topk=topk * 2)
    (fusion.py:478): at BASELINE's top-30 that is a (60 + 1)-deep search
    through YoutubeDNNRecaller.recall, one user at a time."""
    from nrk.recall.youtubednn_recaller import YoutubeDNNRecaller

    g = golden("youtubednn_small")
    ue, ie = g["user_embeddings"], g["item_embeddings"]
    rec = YoutubeDNNRecaller.from_embeddings(ue, ie, user_index_2_rawid=g["user_index_2_rawid"],
                                             item_index_2_rawid=g["item_index_2_rawid"])
    users = [int(u) for u in g["recall_users"][:12]]
    so, ro = oracle.ip_topk(ue.astype(np.float32), ie.astype(np.float32), 61)
    u2i = {int(r): i for i, r in enumerate(g["user_index_2_rawid"])}
    i2r = {i: int(r) for i, r in enumerate(g["item_index_2_rawid"])}
    want = oracle.youtubednn_recall(so, ro, u2i, i2r, users, 60)
    for u in users:
        got = rec.recall(u, topk=60)
        assert [a for a, _ in got] == [a for a, _ in want[u]]
        assert [b for _, b in got] == [b for _, b in want[u]]


def test_recall_lists_match_reference(golden):
    """YoutubeDNNRecaller.recall semantics end to end (drop rank 0, row->raw quirk)."""
    from nrk.recall.youtubednn_recaller import YoutubeDNNRecaller

    g = golden("youtubednn_small")
    rec = YoutubeDNNRecaller.from_embeddings(
        g["user_embeddings"], g["item_embeddings"],
        user_index_2_rawid=g["user_index_2_rawid"], item_index_2_rawid=g["item_index_2_rawid"],
    )
    k = int(g["topk"])
    res = rec.batch_recall([int(u) for u in g["recall_users"]], topk=k)
    ro = g["recall_offsets"]
    for n, u in enumerate(g["recall_users"]):
        got = res[int(u)]
        assert [a for a, _ in got] == g["recall_items"][ro[n]:ro[n + 1]].tolist()
        np.testing.assert_allclose([b for _, b in got], g["recall_scores"][ro[n]:ro[n + 1]], atol=1e-6)
    assert rec.recall(10**9, topk=5) == []


def test_tower_matches_golden(ops, golden):
    from nrk.data import synth

    g = golden("youtubednn_small")
    log = synth.ClickLog(g["click_user"], g["click_item"], g["click_ts"])
    uid, hist, hlen, _, profile = synth.youtubednn_histories(log, int(g["seq_max_len"]))
    out = ops.tt_user_fwd(_dev(g["user_emb"]), _dev(g["item_emb"]), _dev(uid, torch.int32),
                          _dev(hist, torch.int32), _dev(hlen, torch.int32), _dev(g["w0"]),
                          _dev(g["b0"]), _dev(g["w1"]), _dev(g["b1"]))
    it = ops.tt_item_fwd(_dev(g["item_emb"]), _dev(profile, torch.int32))
    np.testing.assert_allclose(out.cpu().numpy(), g["user_embeddings"], atol=1e-6, rtol=0)
    np.testing.assert_allclose(it.cpu().numpy(), g["item_embeddings"], atol=1e-6, rtol=0)


@pytest.mark.parametrize("D,h0", [(16, 64), (32, 64), (64, 128), (32, 100)])
def test_tower_vs_oracle(ops, D, h0):
    rng = np.random.default_rng(D + h0)
    U, I, T, n = 500, 3000, 30, 777
    ue = (rng.standard_normal((U, D)) * 0.01).astype(np.float32)
    ie = (rng.standard_normal((I, D)) * 0.01).astype(np.float32)
    w0 = (rng.standard_normal((h0, 2 * D)) * 0.2).astype(np.float32)
    b0 = (rng.standard_normal(h0) * 0.01).astype(np.float32)
    w1 = (rng.standard_normal((D, h0)) * 0.2).astype(np.float32)
    b1 = (rng.standard_normal(D) * 0.01).astype(np.float32)
    uid = rng.integers(0, U, n)
    hlen = rng.integers(0, T + 1, n)
    hist = rng.integers(0, I, (n, T)) * (np.arange(T)[None] < hlen[:, None])
    out = ops.tt_user_fwd(_dev(ue), _dev(ie), _dev(uid, torch.int32), _dev(hist, torch.int32),
                          _dev(hlen, torch.int32), _dev(w0), _dev(b0), _dev(w1), _dev(b1))
    ref = oracle.tower_user(ue, ie, uid, hist, hlen, w0, b0, w1, b1)
    np.testing.assert_allclose(out.cpu().numpy(), ref, atol=1e-5, rtol=0)


@pytest.mark.parametrize("widths", [[32], [64, 48, 32], [128, 96, 64, 32], [256, 32]])
def test_tower_any_depth_vs_oracle(ops, widths):
    """youtubednn_hidden_units of any length (youtubednn_recaller.py:105-112)."""
    rng = np.random.default_rng(len(widths) * 11 + widths[0])
    U, I, T, n, D = 300, 2000, 30, 555, widths[-1]
    ue = (rng.standard_normal((U, D)) * 0.01).astype(np.float32)
    ie = (rng.standard_normal((I, D)) * 0.01).astype(np.float32)
    layers, fan = [], 2 * D
    for w in widths:
        layers.append(((rng.standard_normal((w, fan)) * 0.2).astype(np.float32),
                       (rng.standard_normal(w) * 0.01).astype(np.float32)))
        fan = w
    uid = rng.integers(0, U, n)
    hlen = rng.integers(0, T + 1, n)
    hist = rng.integers(0, I, (n, T)) * (np.arange(T)[None] < hlen[:, None])
    out = ops.tt_user_fwd_layers(_dev(ue), _dev(ie), _dev(uid, torch.int32), _dev(hist, torch.int32),
                                 _dev(hlen, torch.int32), [(_dev(w), _dev(b)) for w, b in layers])
    ref = oracle.tower_user_layers(ue, ie, uid, hist, hlen, layers)
    np.testing.assert_allclose(out.cpu().numpy(), ref, atol=1e-5, rtol=0)
    if len(widths) == 2 and widths[0] <= 128:  # same bits as the two-layer kernel
        two = ops.tt_user_fwd(_dev(ue), _dev(ie), _dev(uid, torch.int32), _dev(hist, torch.int32),
                              _dev(hlen, torch.int32), *[_dev(a) for wb in layers for a in wb])
        assert torch.equal(two, out)


def test_full_size_topk_properties(ops):
    """Config 2 shapes (250k x 364,047 x 32, k=31): sortedness, exact scores,
    and oracle agreement on a user sample."""
    rng = np.random.default_rng(23)
    U, I, D, K = 250_000, 364_047, 32, 31
    g = torch.Generator(device="cuda").manual_seed(23)
    users = torch.nn.functional.normalize(torch.randn(U, D, device="cuda", generator=g), dim=1)
    items = torch.nn.functional.normalize(torch.randn(I, D, device="cuda", generator=g), dim=1)
    cat = ops.Catalog(items.contiguous())
    s, r, e = ops.ip_topk(users.contiguous(), cat, K, exact=True)
    torch.cuda.synchronize()
    assert bool((r >= 0).all()) and bool((r < I).all())
    assert bool((e[:, :-1] >= e[:, 1:]).all())
    # the bench's launch sequence: the screen as scan + select, then finish
    ws = ops.ip_topk_workspace(U, cat, K, users.device)
    s2 = torch.empty_like(s)
    r2 = torch.empty_like(r)
    ops.ip_topk_scan(users, cat, K, ws)
    ops.ip_topk_select(users, cat, K, ws)
    ops.ip_topk_finish(users, cat, K, ws, s2, r2)
    assert torch.equal(r2, r) and torch.equal(s2, s)
    sample = np.sort(rng.choice(U, 256, replace=False))
    so, ro = oracle.ip_topk(users[sample].cpu().numpy(), items.cpu().numpy(), K, nthreads=8)
    assert np.array_equal(r[sample].cpu().numpy().astype(np.int64), ro)
    assert np.array_equal(s[sample].cpu().numpy(), so)


def test_ip_topk_catalog_body_near_2gib(ops):
    """A packed catalog body just under ip_check's 2 GiB limit (33,554,000
    items x 32 dims = 2,147,457,024 B): the scan's ring prefetches run past
    the last tile (main loop: 3 tiles; list pre-pass: 3 strides of 4,096
    tiles), and their 32-bit DMA offsets must not wrap (a wrapped
    offset read ~2 GB before the buffer).  Rows and scores bit-exact against
    the oracle for 64 users."""
    from nrk import _lib

    I, D, U, K = 33_554_000, 32, 64, 31
    body = -(-I // 32) * 64 * 32
    assert body < 2**31 and _lib.lib().nrk_ip_catalog_bytes(I, D) > 2 * body
    g = torch.Generator(device="cuda").manual_seed(5)
    items = torch.nn.functional.normalize(torch.randn(I, D, device="cuda", generator=g), dim=1).contiguous()
    users = torch.nn.functional.normalize(torch.randn(U, D, device="cuda", generator=g), dim=1).contiguous()
    cat = ops.Catalog(items)
    s, r = ops.ip_topk(users, cat, K)
    torch.cuda.synchronize()
    so, ro = oracle.ip_topk(users.cpu().numpy(), items.cpu().numpy(), K, nthreads=16)
    del cat, items
    assert np.array_equal(r.cpu().numpy(), ro)
    assert np.array_equal(s.cpu().numpy(), so)


@pytest.mark.parametrize("n_shards", [2, 3, 8])
def test_catalog_shards_merge_equals_single(ops, n_shards):
    """Config-4 data path on one GPU: per-shard exact top-k with global rows
    (row_offset) + nrk_topk_merge == the unsharded result, incl. a cross-shard
    exact tie (lower global row wins)."""
    from nrk.dist import HipShard, bound_width, catalog_sharded_topk, shard_range

    rng = np.random.default_rng(n_shards)
    users = _unit(rng.standard_normal((300, 32)))
    users[7] = 0.0  # zero user: all-tie row, lowest global rows win
    items = _unit(rng.standard_normal((5000, 32)))
    items[4990] = items[10]
    K = 31
    so, ro = oracle.ip_topk(users, items, K)
    u = _dev(users)
    for exchange in (False, True):
        shards = []
        for r in range(n_shards):
            lo, hi = shard_range(len(items), n_shards, r)
            shards.append(HipShard(ops.Catalog(_dev(items[lo:hi])), lo, K, len(users)))
        m = bound_width(K, n_shards)
        bounds = torch.stack([sh.screen(u, max(m, 1)) for sh in shards]).contiguous()  # = the all_gather
        lists = [sh.finish(u, bounds if exchange and m else None) for sh in shards]
        es = torch.stack([x[0] for x in lists]).contiguous()
        rs = torch.stack([x[1] for x in lists]).contiguous()
        s, r, e = ops.topk_merge(es, rs, K)
        assert np.array_equal(r.cpu().numpy(), ro), exchange
        assert np.array_equal(s.cpu().numpy(), so), exchange
        if exchange:  # the global bound left each shard about its share of the top-k
            assert int((rs >= 0).sum()) < 2 * len(users) * K
    # the single-rank code path of nrk.dist (no process group)
    s1, r1, _ = catalog_sharded_topk(u, HipShard(ops.Catalog(_dev(items)), 0, K, len(users)), K)
    assert np.array_equal(r1.cpu().numpy(), ro)


@pytest.mark.parametrize("d,k", [(32, 31), (32, 10), (16, 31), (64, 21), (32, 32)])
def test_one_pass_screen_150k_stress_vs_oracle(ops, d, k):
    """The one-pass screen (list pre-pass over sampled tiles, then every
    tile) on a 150k-item catalog: rows and scores bit-exact vs the oracle for
    every user, incl. exact duplicate items in a pre-pass tile and elsewhere,
    a run of duplicates inside one tile, a zero user, a user equal to an item
    and near-tie scores."""
    rng = np.random.default_rng(d * 100 + k)
    n_items = 150_000
    users = _unit(rng.standard_normal((512, d)))
    items = _unit(rng.standard_normal((n_items, d)))
    users[5] = 0.0
    items[140_001] = items[3]       # duplicate in another tile
    items[70_000:70_040] = items[9]  # a run of duplicates inside one tile
    users[6] = items[9]
    users[7] = np.round(users[7] * 8) / 8  # coarse values: many near-ties
    so, ro = oracle.ip_topk(users, items, k, nthreads=8)
    s, r = ops.ip_topk(_dev(users), ops.Catalog(_dev(items)), k)
    assert np.array_equal(r.cpu().numpy(), ro)
    assert np.array_equal(s.cpu().numpy(), so)


@pytest.mark.parametrize("n_shards,k", [(2, 129), (8, 129), (3, 300)])
def test_catalog_shards_large_k_merge(ops, n_shards, k):
    """k > IP_KFAST (no MFMA screen): the catalog-sharded merge protocol takes
    each shard's exact path (no bound exchange) and merges pairwise in a tree
    when n_shards * k exceeds one nrk_topk_merge call (8 x 129, 3 x 300);
    the owner protocol refuses such k with an accurate message."""
    from nrk.dist import HipRangeShard, HipShard, _default_merge, catalog_sharded_topk, shard_range

    rng = np.random.default_rng(k + n_shards)
    users = _unit(rng.standard_normal((150, 32)))
    users[3] = 0.0
    items = _unit(rng.standard_normal((6000, 32)))
    items[5990] = items[10]
    so, ro = oracle.ip_topk(users, items, k)
    u = _dev(users)
    shards = [HipShard(ops.Catalog(_dev(items[lo:hi])), lo, k, len(users))
              for lo, hi in (shard_range(len(items), n_shards, r) for r in range(n_shards))]
    assert not shards[0].bounded
    lists = [sh.finish(u, None) for sh in shards]
    s, r, e = _default_merge(torch.stack([x[0] for x in lists]).contiguous(),
                             torch.stack([x[1] for x in lists]).contiguous(), k)
    assert np.array_equal(r.cpu().numpy(), ro)
    assert np.array_equal(s.cpu().numpy(), so)
    s1, r1, _ = catalog_sharded_topk(u, HipShard(ops.Catalog(_dev(items)), 0, k, len(users)), k)
    assert np.array_equal(r1.cpu().numpy(), ro)
    with pytest.raises(NotImplementedError, match="owner protocol"):
        HipRangeShard(ops.Catalog(_dev(items)), 0, 4, k, len(users))


def test_catalog_shards_bound_full_size(ops):
    """8-shard replay of config 4 at the full catalog (364,047 x 32) with the
    bound exchange: merged rows / scores bit-exact vs the oracle on a sample."""
    from nrk.dist import HipShard, bound_width, shard_range

    U, I, D, K, N = 4096, 364_047, 32, 31, 8
    g = torch.Generator(device="cuda").manual_seed(5)
    users = torch.nn.functional.normalize(torch.randn(U, D, device="cuda", generator=g), dim=1).contiguous()
    items = torch.nn.functional.normalize(torch.randn(I, D, device="cuda", generator=g), dim=1).contiguous()
    shards = [HipShard(ops.Catalog(items[lo:hi].contiguous()), lo, K, U)
              for lo, hi in (shard_range(I, N, r) for r in range(N))]
    m = bound_width(K, N)
    gb = torch.stack([sh.screen(users, m) for sh in shards]).contiguous()
    lists = [sh.finish(users, gb) for sh in shards]
    s, r, e = ops.topk_merge(torch.stack([x[0] for x in lists]).contiguous(),
                             torch.stack([x[1] for x in lists]).contiguous(), K)
    torch.cuda.synchronize()
    sample = np.arange(0, U, 16)
    so, ro = oracle.ip_topk(users[sample].cpu().numpy(), items.cpu().numpy(), K, nthreads=8)
    assert np.array_equal(r[sample].cpu().numpy().astype(np.int64), ro)
    assert np.array_equal(s[sample].cpu().numpy(), so)


@pytest.mark.parametrize("n_shards,k,d", [(2, 31, 32), (3, 31, 32), (8, 31, 32), (8, 61, 32), (4, 10, 32),
                                          (3, 31, 16), (4, 21, 64), (3, 100, 32), (2, 31, 128)])
def test_catalog_owner_refine_equals_single(ops, n_shards, k, d):
    """Config 4, owner refine (nrk.dist.owner_replay: the two exchanges
    in-process): every rank screens its tile range of the shared catalog,
    bands above the global bound go to each user block's owner, which
    refines its users -- rows and scores identical to one GPU, incl. a
    cross-shard exact tie, a zero user and the tie-stress overflow path.
    d = 32 with k <= 31 is the warp-specialized shard scan; the other dims
    run ip_scan_kernel's variants, k = 100 the shard bound pass
    (ip_shard_bound_kernel) instead of the scan's list epilogue."""
    from nrk.dist import HipRangeShard, owner_replay, shard_blocks

    rng = np.random.default_rng(n_shards * 100 + k + d)
    users = _unit(rng.standard_normal((300, d)))
    users[7] = 0.0
    items = _unit(rng.standard_normal((20000, d)))
    items[19990] = items[10]
    items[5000:5600] = items[100]  # dense exact duplicates -> overflowed users take the exact path
    users[9] = items[100]
    so, ro = oracle.ip_topk(users, items, k)
    cat = ops.Catalog(_dev(items))
    tb = ops.ip_topk_tile_blocks(d)
    shards = [HipRangeShard(cat, *shard_blocks(len(items), n_shards, r, tb), k, len(users)) for r in range(n_shards)]
    s, r, e = owner_replay(_dev(users), shards, k)
    assert np.array_equal(r.cpu().numpy(), ro)
    assert np.array_equal(s.cpu().numpy(), so)


def test_catalog_owner_refine_full_size(ops):
    """The 8-shard owner replay at config 2's catalog (364,047 x 32): rows and
    scores bit-exact vs the oracle on a user sample."""
    from nrk.dist import HipRangeShard, owner_replay, shard_blocks

    U, I, D, K, N = 4096, 364_047, 32, 31, 8
    g = torch.Generator(device="cuda").manual_seed(5)
    users = torch.nn.functional.normalize(torch.randn(U, D, device="cuda", generator=g), dim=1).contiguous()
    items = torch.nn.functional.normalize(torch.randn(I, D, device="cuda", generator=g), dim=1).contiguous()
    cat = ops.Catalog(items)
    tb = ops.ip_topk_tile_blocks(D)
    shards = [HipRangeShard(cat, *shard_blocks(I, N, r, tb), K, U) for r in range(N)]
    s, r, e = owner_replay(users, shards, K)
    torch.cuda.synchronize()
    sample = np.arange(0, U, 16)
    so, ro = oracle.ip_topk(users[sample].cpu().numpy(), items.cpu().numpy(), K, nthreads=8)
    assert np.array_equal(r[sample].cpu().numpy().astype(np.int64), ro)
    assert np.array_equal(s[sample].cpu().numpy(), so)


@pytest.mark.parametrize("d", [16, 32, 64])
def test_screen_eps_bounds_the_fp16_rounding(ops, d):
    """The screen's per-user error bound (ucut.y, ip_topk.hip ip_screen_kernel:
    ||du|| max||v|| + ||u|| max||dv|| + ||du|| max||dv|| + accumulation) must
    cover |fp16 score - exact| for every (user, item): the fp16 scores are
    re-derived here exactly (float16 rounding of the power-of-two scaled
    rows, products summed in float64, so no accumulation error -- the
    rounding part of the bound is what is tested).  Rows of very different
    norms and a few tiny components stress both sides."""
    rng = np.random.default_rng(7 + d)
    U, I, K = 384, 20000, 31
    users = (rng.standard_normal((U, d)) * np.exp(rng.standard_normal((U, 1)))).astype(np.float32)
    items = (rng.standard_normal((I, d)) * np.exp(rng.standard_normal((I, 1)))).astype(np.float32)
    items[::97, : d // 4] *= np.float32(1e-6)  # components deep below the fp16 normal range
    cat = ops.Catalog(_dev(items))
    ws = ops.ip_topk_workspace(U, cat, K, "cuda")
    ops.ip_topk_screen(_dev(users), cat, K, ws)
    torch.cuda.synchronize()
    # workspace layout (ip_ws_layout): 256 B header, then ucut float2 [U]
    off = 256
    eps = ws[off: off + U * 8].view(torch.float32).view(U, 2)[:, 1].double().cpu().numpy()

    def p2(maxabs):  # pow2_scale: maps max|x| into [2^13, 2^14)
        _, e = np.frexp(maxabs)
        return np.ldexp(1.0, 14 - e)

    su = p2(np.abs(users).max(1)).astype(np.float32)[:, None]
    sv = np.float32(p2(np.abs(items).max()))
    u16 = (users * su).astype(np.float16).astype(np.float64) / su
    v16 = (items * sv).astype(np.float16).astype(np.float64) / np.float64(sv)
    exact = users.astype(np.float64) @ items.astype(np.float64).T
    err = np.abs(u16 @ v16.T - exact).max(1)
    assert np.all(err <= eps), float((err / eps).max())
    # and it is the tighter form: well under round 1's 2^-10 ||u|| max||v|| worst case
    old = 9.765625e-4 * np.linalg.norm(users.astype(np.float64), axis=1) * np.linalg.norm(items, axis=1).max()
    assert np.all(eps < 0.9 * old), float((eps / old).max())


@pytest.mark.gpu
def test_nonfinite_inputs_rejected():
    """NaN / inf items or users never reach the -fno-honor-nans screen."""
    from nrk import ops

    items = torch.nn.functional.normalize(torch.randn(500, 32, device="cuda"), dim=1).contiguous()
    bad = items.clone()
    bad[7, 3] = float("nan")
    with pytest.raises(ValueError, match="finite"):
        ops.Catalog(bad)
    cat = ops.Catalog(items)
    u = torch.randn(10, 32, device="cuda")
    u[4, 0] = float("inf")
    with pytest.raises(ValueError, match="finite"):
        ops.ip_topk(u, cat, 31)
