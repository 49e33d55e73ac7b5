"""GPU parity: ItemCF similarity (item_cf.py:17-89), per-item top-n
(itemcf_recaller.py:41-54) and the recaller built on them, through the C ABI
(nrk_itemcf_sim / nrk_itemcf_topn).

Checker: the oracle (oracle/nrk_oracle.c, glibc exp/pow) and the reference's
own outputs (tests/golden/itemcf_small.npz).  Keys, dict order, counts and
top-n membership/order are exact; fp64 similarity values agree to rtol 1e-12
(the device exp/pow and libm / numpy's SIMD exp differ in the last ulp).
"""
import numpy as np
import pandas as pd
import pytest
import torch

from nrk.data import synth
from oracle import oracle

pytestmark = pytest.mark.gpu
RTOL = 1e-12


def _inputs(g):
    log = synth.ClickLog(g["click_user"], g["click_item"], g["click_ts"])
    users, offs, items_raw, ts = synth.user_lists(log)
    ids = g["created_ids"]
    dense = np.searchsorted(ids, items_raw).astype(np.int32)
    return users, offs, dense, ts, ids


def _gpu_sim(offs, dense, ts, created, n_items):
    from nrk import ops

    d = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dt)).cuda()  # noqa: E731
    return ops.itemcf_sim(d(offs, np.int64), d(dense, np.int32), d(ts, np.int64), d(created, np.float64), n_items)


def _check_vs_oracle(offs, dense, ts, created, n_items):
    sim = _gpu_sim(offs, dense, ts, created, n_items)
    gi, gj, gv, gf = (t.cpu().numpy() for t in (sim.i, sim.j, sim.v, sim.first))
    oi, oj, ov, rank, cnt = oracle.itemcf_sim(offs, dense, ts, created, n_items)
    assert len(gi) == len(oi)
    # GPU order is (i, j); the oracle's is first insertion -> compare both ways
    order = np.argsort(gf, kind="stable")
    assert np.array_equal(gi[order], oi) and np.array_equal(gj[order], oj)
    np.testing.assert_allclose(gv[order], ov, rtol=RTOL, atol=0)
    assert np.all(np.diff(gi.astype(np.int64) * n_items + gj) > 0)
    assert np.array_equal(sim.cnt.cpu().numpy(), cnt)
    return sim, (oi, oj, ov)


def test_itemcf_sim_vs_oracle_golden_inputs(golden):
    g = golden("itemcf_small")
    users, offs, dense, ts, ids = _inputs(g)
    _check_vs_oracle(offs, dense, ts, g["created_vals"], len(ids))


def test_itemcf_similarity_plugin_matches_reference(golden):
    from nrk.similarity.item_cf import ItemCFSimilarity

    g = golden("itemcf_small")
    df = pd.DataFrame({"user_id": g["click_user"], "click_article_id": g["click_item"],
                       "click_timestamp": g["click_ts"]})
    created = dict(zip(g["created_ids"].tolist(), g["created_vals"].tolist()))
    sim = ItemCFSimilarity().calculate(df, created)
    assert list(sim.keys()) == g["sim_rows"].tolist()
    fi = [i for i, row in sim.items() for _ in row]
    fj = [j for row in sim.values() for j in row]
    fv = [v for row in sim.values() for v in row.values()]
    assert fi == g["sim_i"].tolist() and fj == g["sim_j"].tolist()
    np.testing.assert_allclose(fv, g["sim_v"], rtol=RTOL, atol=0)


def test_itemcf_recall_matches_reference(golden):
    from nrk.config import RecallConfig
    from nrk.data.extractors import csr_to_dict
    from nrk.recall.itemcf_recaller import ItemCFRecaller
    from nrk.similarity.item_cf import ItemCFSimilarity

    g = golden("itemcf_small")
    cfg = RecallConfig(itemcf_sim_item_topk=int(g["sim_item_topk"]))
    log = synth.ClickLog(g["click_user"], g["click_item"], g["click_ts"])
    users, offs, items, ts = synth.user_lists(log)
    created = dict(zip(g["created_ids"].tolist(), g["created_vals"].tolist()))
    res = ItemCFSimilarity(cfg).compute(users, offs, items, ts, created)
    uit = csr_to_dict(users, offs, items, ts)
    hot = g["hot"].tolist()
    for rec in (ItemCFRecaller.from_result(cfg, res, created, uit, hot),
                ItemCFRecaller(cfg, res.to_dict(), created, uit, hot)):
        out = rec.batch_recall([int(u) for u in g["recall_users"]], topk=int(g["topk"]))
        ro = g["recall_offsets"]
        for n, u in enumerate(g["recall_users"]):
            got = out[int(u)]
            assert [a for a, _ in got] == g["recall_items"][ro[n]:ro[n + 1]].tolist(), n
            np.testing.assert_allclose([b for _, b in got], g["recall_scores"][ro[n]:ro[n + 1]], rtol=RTOL)


def _random_lists(rng, n_users, n_items, max_len, repeat_p=0.1):
    L = rng.integers(0, max_len + 1, n_users)
    offs = np.zeros(n_users + 1, np.int64)
    offs[1:] = np.cumsum(L)
    items = rng.integers(0, n_items, offs[-1]).astype(np.int32)
    rep = rng.random(offs[-1]) < repeat_p  # repeated clicks on the previous item
    rep[offs[:-1][L > 0]] = False
    idx = np.nonzero(rep)[0]
    items[idx] = items[idx - 1]
    ts = np.zeros(offs[-1], np.int64)
    for u in range(n_users):
        a, b = offs[u], offs[u + 1]
        ts[a:b] = 1_500_000_000_000 + np.cumsum(rng.integers(0, 4, b - a))  # ties and 1-ms gaps
    created = rng.random(n_items)
    created[rng.integers(0, n_items, n_items // 10)] = 0.5  # equal created times
    return offs, items, ts, created


@pytest.mark.parametrize("n_users,n_items,max_len", [(1, 3, 1), (5, 4, 6), (300, 50, 40),
                                                     (2000, 20000, 25), (50, 1_100_000, 300)])
def test_itemcf_sim_vs_oracle_random(n_users, n_items, max_len):
    rng = np.random.default_rng(n_users + n_items)
    offs, items, ts, created = _random_lists(rng, n_users, n_items, max_len)
    _check_vs_oracle(offs, items, ts, created, n_items)


def test_itemcf_no_pairs():
    offs = np.array([0, 1, 1, 2], np.int64)
    sim = _gpu_sim(offs, np.array([3, 3], np.int32), np.array([5, 6], np.int64), np.zeros(4), 4)
    assert sim.i.numel() == 0
    assert sim.cnt.cpu().tolist() == [0, 0, 0, 2]


@pytest.mark.parametrize("topn", [1, 20, 64, 65, 100, 300])
def test_itemcf_topn_vs_oracle(topn):
    from nrk import ops

    rng = np.random.default_rng(topn)
    n_rows = 700
    lens = rng.integers(0, 300, n_rows)
    lens[:9] = [0, 1, 63, 64, 65, 4096, 4097, 20000, 70000]  # + rows for the workgroup-per-row path
    off = np.zeros(n_rows + 1, np.int64)
    off[1:] = np.cumsum(lens)
    n = int(off[-1])
    vals = np.round(rng.random(n) * 50) / 50  # many exact ties -> insertion order decides
    cols = rng.integers(0, 10**6, n).astype(np.int32)
    first = np.arange(n, dtype=np.int64)
    d = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    gc, gv, gn = ops.itemcf_topn(d(off), d(cols), d(vals), d(first), topn)
    oc, ov, on = oracle.itemcf_topn(off, cols, vals, topn)
    assert np.array_equal(gn.cpu().numpy(), on)
    assert np.array_equal(gc.cpu().numpy(), oc)
    assert np.array_equal(gv.cpu().numpy(), ov)


NEAR_TIE_MAX_FRAC = 1e-5  # at most 1 excused position per 100,000 compared entries


def _near_ties_only(g_idx, o_idx, o_val_ext, valid, rtol=1e-12):
    """Every position where the device's index differs from the oracle's
    holds an oracle value within ``rtol`` of a neighbouring oracle value
    (o_val_ext has one extra column: the first entry past the cut) -- i.e.
    only near-ties that the last ulp of exp / pow can reorder."""
    mism = (g_idx != o_idx) & valid
    r, p = np.nonzero(mism)
    # the count the near-tie rule excuses is part of the
    # result -- bounded here (round 3 measured 0 at full size), not only printed
    print(f"near-tie check: {len(r)} differing positions in {int(np.unique(r).size)} rows "
          f"of {int(valid.sum())} compared entries")
    assert len(r) <= NEAR_TIE_MAX_FRAC * int(valid.sum()), (len(r), int(valid.sum()))
    if len(r) == 0:
        return True
    v = o_val_ext
    tol = rtol * np.abs(v[r, p])
    left = (p > 0) & (np.abs(v[r, p] - v[r, np.maximum(p - 1, 0)]) <= tol)
    right = np.abs(v[r, p] - v[r, p + 1]) <= tol
    return bool((left | right).all())


def test_itemcf_full_size():
    """250k-user / 364,047-item synthetic Tianchi log (BASELINE sizes): the
    whole similarity against the oracle, plus top-20 per item."""
    from nrk import ops

    log = synth.make_click_log(n_users=250_000, n_items=364_047, seed=23)
    users, offs, items_raw, ts = synth.user_lists(log)
    ids, dense = np.unique(items_raw, return_inverse=True)
    created = np.random.default_rng(1).random(len(ids))
    sim, (oi, oj, ov) = _check_vs_oracle(offs, dense.astype(np.int32), ts, created, len(ids))
    gc, gv, gn = ops.itemcf_topn(sim.row_offsets(), sim.j, sim.v, sim.first, 20)
    roff, cols, vals = oracle.sim_to_rows(oi, oj, ov, len(ids))
    oc, ovv, on = oracle.itemcf_topn(roff, cols, vals, 20)
    assert np.array_equal(gn.cpu().numpy(), on)
    # identical except where device / libm last-ulp differences reorder an
    # exact-arithmetic near-tie: every differing position must sit next to an
    # oracle value within 1e-12 of its own (the 21st entry included), and the
    # sorted values agree to 1e-12
    _, ov21, _ = oracle.itemcf_topn(roff, cols, vals, 21)
    valid = np.arange(20)[None, :] < on[:, None]
    assert _near_ties_only(gc.cpu().numpy(), oc, ov21, valid)
    np.testing.assert_allclose(gv.cpu().numpy()[valid], ovv[valid], rtol=1e-12, atol=0)


# ------------------------------------------------------------ A10 recall --
def _emb_dict(g):
    out = {}
    for i, j, v in zip(g["emb_i"].tolist(), g["emb_j"].tolist(), g["emb_v"].tolist()):
        out.setdefault(i, {})[j] = v
    return out


def test_itemcf_recall_with_embedding_content_weight_matches_reference(golden):
    """ItemCFRecaller with the EmbeddingSimilarity content weight (itemcf_recaller.py:98-103)
    against the reference's own output on the same inputs."""
    from nrk.config import RecallConfig
    from nrk.data.extractors import csr_to_dict
    from nrk.recall.itemcf_recaller import ItemCFRecaller
    from nrk.similarity.item_cf import ItemCFSimilarity

    g = golden("itemcf_small")
    cfg = RecallConfig(itemcf_sim_item_topk=int(g["sim_item_topk"]))
    log = synth.ClickLog(g["click_user"], g["click_item"], g["click_ts"])
    users, offs, items, ts = synth.user_lists(log)
    created = dict(zip(g["created_ids"].tolist(), g["created_vals"].tolist()))
    res = ItemCFSimilarity(cfg).compute(users, offs, items, ts, created)
    uit = csr_to_dict(users, offs, items, ts)
    rec = ItemCFRecaller.from_result(cfg, res, created, uit, g["hot"].tolist(), emb_similarity_matrix=_emb_dict(g))
    out = rec.batch_recall([int(u) for u in g["recall_users"]], topk=int(g["topk"]))
    ro = g["emb_recall_offsets"]
    for n, u in enumerate(g["recall_users"]):
        got = out[int(u)]
        assert [a for a, _ in got] == g["emb_recall_items"][ro[n]:ro[n + 1]].tolist(), n
        np.testing.assert_allclose([b for _, b in got], g["emb_recall_scores"][ro[n]:ro[n + 1]], rtol=RTOL)
    # single-user recall() is the same kernel (a batch of one); unknown user -> hot items, int scores
    u0 = int(g["recall_users"][0])
    assert rec.recall(u0, topk=30) == out[u0]
    cold = rec.recall(-5, topk=7)
    assert cold == [(int(h), -x) for x, h in enumerate(g["hot"][:7].tolist())]
    assert all(isinstance(s, int) for _, s in cold)


def _recall_case(rng, n_users, n_items, max_len, topn, n_hot):
    from nrk import ops

    offs, items, ts, created = _random_lists(rng, n_users, n_items, max_len)
    sim = _gpu_sim(offs, items, ts, created, n_items)
    nc, nv, nn = ops.itemcf_topn(sim.row_offsets(), sim.j, sim.v, sim.first, topn)
    hot = rng.permutation(n_items)[:n_hot].astype(np.int32)
    return offs, items, created, nc, nv, nn, hot


@pytest.mark.parametrize("n_users,n_items,max_len,topn,topk,n_hot",
                         [(1, 3, 1, 20, 5, 2), (40, 30, 12, 5, 64, 100), (500, 400, 40, 20, 30, 50),
                          (3000, 20000, 25, 20, 30, 50), (60, 5000, 250, 64, 64, 64),
                          (500, 4000, 40, 20, 100, 300), (300, 2000, 30, 100, 200, 150), (50, 60, 8, 20, 100, 30)])
def test_itemcf_recall_vs_oracle(n_users, n_items, max_len, topn, topk, n_hot):
    """nrk_itemcf_recall vs the C restatement of ItemCFRecaller.recall
    (oracle_itemcf_recall): candidate sums in (loc, x) order, hot fill,
    stable (score desc, insertion order) top-k, unknown users."""
    from nrk import ops

    rng = np.random.default_rng(n_users * 7 + topk)
    offs, items, created, nc, nv, nn, hot = _recall_case(rng, n_users, n_items, max_len, topn, n_hot)
    q = np.concatenate([rng.permutation(n_users), [-1, -1]]).astype(np.int64)  # + two cold-start queries
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    gi, gs, gsrc, gn = ops.itemcf_recall(d(q), d(offs), d(items), nc, nv, nn, d(created), d(hot), topk)
    oi, os_, on = oracle.itemcf_recall(q, offs, items, nc.cpu().numpy(), nv.cpu().numpy(), nn.cpu().numpy(),
                                       created, hot, topk, n_items)
    gi, gs, gsrc, gn = (t.cpu().numpy() for t in (gi, gs, gsrc, gn))
    assert np.array_equal(gn, on)
    for r in range(len(q)):
        m = on[r]
        assert np.array_equal(gi[r, :m], oi[r, :m]), r
        np.testing.assert_allclose(gs[r, :m], os_[r, :m], rtol=RTOL, atol=0)
        assert (gsrc[r, :m] == 2).all() if q[r] < 0 else (gsrc[r, :m] < 2).all()


def test_itemcf_recall_full_size():
    """All 250k users of the synthetic Tianchi log (BASELINE sizes) recalled in
    one call; every list against the C oracle (identical except where the
    device and libm exp/pow differ in the last ulp of near-tied scores)."""
    from nrk import ops

    log = synth.make_click_log(n_users=250_000, n_items=364_047, seed=23)
    users, offs, items_raw, ts = synth.user_lists(log)
    ids, dense = np.unique(items_raw, return_inverse=True)
    dense = dense.astype(np.int32)
    created = np.random.default_rng(1).random(len(ids))
    sim = _gpu_sim(offs, dense, ts, created, len(ids))
    nc, nv, nn = ops.itemcf_topn(sim.row_offsets(), sim.j, sim.v, sim.first, 20)
    hot = np.argsort(-np.bincount(dense, minlength=len(ids)), kind="stable")[:50].astype(np.int32)
    q = np.arange(len(users), dtype=np.int64)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    gi, gs, _, gn = ops.itemcf_recall(d(q), d(offs), d(dense), nc, nv, nn, d(created), d(hot), 30)
    oi, os_, on = oracle.itemcf_recall(q, offs, dense, nc.cpu().numpy(), nv.cpu().numpy(), nn.cpu().numpy(),
                                       created, hot, 30, len(ids))
    assert np.array_equal(gn.cpu().numpy(), on)
    gi = gi.cpu().numpy()
    valid = np.arange(30)[None, :] < on[:, None]
    # exact except certified near-ties (see _near_ties_only), scores to 1e-11
    _, os31, _ = oracle.itemcf_recall(q, offs, dense, nc.cpu().numpy(), nv.cpu().numpy(), nn.cpu().numpy(),
                                      created, hot, 31, len(ids))
    assert _near_ties_only(gi, oi, os31, valid, rtol=1e-11)
    np.testing.assert_allclose(gs.cpu().numpy()[valid], os_[valid], rtol=1e-11, atol=0)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_itemcf_users_sharded_equals_single(world):
    """The data path of nrk.dist.itemcf_sim_sharded on one GPU: per-rank
    nrk_itemcf_pairs (global slots), tuples bucketed by item owner in rank
    order, summed counts, nrk_itemcf_reduce per owner == nrk_itemcf_sim."""
    from nrk import ops
    from nrk.dist import shard_range

    rng = np.random.default_rng(world)
    offs, items, ts, created = _random_lists(rng, 3000, 20000, 25)
    n_items = 20000
    full = _gpu_sim(offs, items, ts, created, n_items)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    parts, base, cnt = [], 0, torch.zeros(n_items, dtype=torch.int64, device="cuda")
    for r in range(world):
        lo, hi = shard_range(len(offs) - 1, world, r)
        a, e = offs[lo], offs[hi]
        k, s, w, c = ops.itemcf_pairs(d(offs[lo:hi + 1] - a), d(items[a:e]), d(ts[a:e]), d(created), n_items,
                                      slot_base=base)
        base += int(((offs[lo + 1:hi + 1] - offs[lo:hi]) ** 2).sum())
        parts.append((k, s, w))
        cnt += c
    b = 1
    while (1 << b) <= n_items:
        b += 1
    per = -(-n_items // world)
    got = []
    for o in range(world):  # owner o receives every rank's tuples for its items, in rank order
        ks, ss, ws_ = [], [], []
        for k, s, w in parts:
            m = ((k >> b) // per == o) & (k != (1 << (2 * b)) - 1)
            ks.append(k[m]), ss.append(s[m]), ws_.append(w[m])
        res = ops.itemcf_reduce(torch.cat(ks), torch.cat(ss), torch.cat(ws_), n_items, cnt)
        got.append(res)
    gi = torch.cat([g.i for g in got]).cpu().numpy()
    gj = torch.cat([g.j for g in got]).cpu().numpy()
    gv = torch.cat([g.v for g in got]).cpu().numpy()
    gf = torch.cat([g.first for g in got]).cpu().numpy()
    assert np.array_equal(gi, full.i.cpu().numpy()) and np.array_equal(gj, full.j.cpu().numpy())
    assert np.array_equal(gf, full.first.cpu().numpy())
    np.testing.assert_allclose(gv, full.v.cpu().numpy(), rtol=1e-12, atol=0)
    assert np.array_equal(cnt.cpu().numpy(), full.cnt.cpu().numpy())
