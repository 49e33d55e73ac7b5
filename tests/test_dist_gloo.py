"""CPU, world_size 2 (gloo): the multi-GPU layouts of the recall path.
The exchange + ownership logic of nrk.dist runs for real over gloo; the
per-shard scan and the merge are the oracle / a numpy stand-in here (the HIP
versions are covered by the -m gpu tests)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _np_merge(exact_lists, row_lists, k):
    e = exact_lists.numpy()
    r = row_lists.numpy()
    G, n, kin = e.shape
    e = e.transpose(1, 0, 2).reshape(n, G * kin)
    r = r.transpose(1, 0, 2).reshape(n, G * kin)
    key_r = np.where(r < 0, np.iinfo(np.int64).max, r)
    key_e = np.where(r < 0, np.inf, -e)
    order = np.lexsort((key_r, key_e), axis=1)[:, :k]
    oe = np.take_along_axis(e, order, 1)
    orow = np.take_along_axis(r, order, 1)
    ok = orow >= 0
    return (torch.from_numpy(np.where(ok, oe, -np.finfo(np.float32).max).astype(np.float32)),
            torch.from_numpy(np.where(ok, orow, -1).astype(np.int32)),
            torch.from_numpy(np.where(ok, oe, -np.inf)))


class _OracleShard:
    """CPU stand-in for nrk.dist.HipShard: the screen's bounds are the
    shard's m largest exact scores minus a margin (valid lower bounds of
    distinct items, like the HIP screen's half-block maxima - eps); finish
    takes the k-th largest of every shard's bounds and returns the shard's
    top-k restricted to exact >= that bound (-1 padded), the contract of
    nrk_ip_topk_apply_bound."""

    def __init__(self, items, lo, k):
        self.items, self.lo, self.k, self.dropped = items, lo, k, 0

    def screen(self, users, m):
        sc = users.double().numpy() @ self.items.astype(np.float64).T
        top = -np.sort(-sc, axis=1)[:, :m] - 1e-9
        if top.shape[1] < m:
            top = np.concatenate([top, np.full((len(top), m - top.shape[1]), -np.inf)], 1)
        return torch.from_numpy(top.astype(np.float32) - np.float32(1e-6))

    def finish(self, users, bounds):
        from oracle import oracle

        s, r, e = oracle.ip_topk(users.numpy(), self.items, self.k, exact=True)
        r = np.where(r >= 0, r + self.lo, -1)
        if bounds is not None:
            L, U, m = bounds.shape
            vals = bounds.permute(1, 0, 2).reshape(U, L * m).double().numpy()
            g = -np.sort(-vals, axis=1)[:, self.k - 1]
            drop = (r >= 0) & (e < g[:, None])
            self.dropped += int(drop.sum())
            r = np.where(drop, -1, r)
            e = np.where(drop, -np.inf, e)
        return torch.from_numpy(e), torch.from_numpy(r.astype(np.int32))


def _worker(rank, world, port, U, I, D, k, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nrk.dist import catalog_sharded_topk, gather_users, shard_range

        rng = np.random.default_rng(7)
        users = rng.standard_normal((U, D)).astype(np.float32)
        items = rng.standard_normal((I, D)).astype(np.float32)
        items[I // 2 + 1] = items[3]  # cross-shard exact tie -> lower row must win
        lo, hi = shard_range(I, world, rank)
        ulo, uhi = shard_range(U, world, rank)
        # the user tower runs per user block; all_gather gives every rank all users
        full = gather_users(torch.from_numpy(users[ulo:uhi]), U)
        assert torch.equal(full, torch.from_numpy(users))
        shard = _OracleShard(items[lo:hi], lo, k)
        s, r, e = catalog_sharded_topk(full, shard, k, merge=_np_merge)
        q.put((rank, ulo, uhi, s.numpy(), r.numpy(), shard.dropped))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("U,I,k", [(37, 101, 31), (64, 40, 31), (5, 7, 10), (50, 400, 8)])
def test_catalog_sharded_matches_single(U, I, k):
    from oracle import oracle

    world, D = 2, 16
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, U, I, D, k, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(7)
    users = rng.standard_normal((U, D)).astype(np.float32)
    items = rng.standard_normal((I, D)).astype(np.float32)
    items[I // 2 + 1] = items[3]
    so, ro = oracle.ip_topk(users, items, k)
    for rank, ulo, uhi, s, r, _ in got:
        assert np.array_equal(r, ro[ulo:uhi]), rank
        assert np.array_equal(s, so[ulo:uhi]), rank
    if I >= 2 * k:  # the global bound cut the shard lists (the refine-shrinking exchange ran)
        assert sum(g[5] for g in got) > 0


class _OwnerShard:
    """CPU stand-in for nrk.dist.HipRangeShard (config 4, owner refine):
    bounds = the range's m largest exact scores minus a margin; band = the
    range's rows with exact >= (k-th largest of every shard's bounds) -
    margin, as int64 entries (the stand-in's own row encoding); the owner's
    refine = exact top-k over the received rows ((score desc, row asc)),
    the whole catalog for users flagged overflowed (one user is forced)."""

    def __init__(self, items, lo, hi, k, force_ovf=None, x_cap=64):
        self.items, self.lo, self.hi, self.k, self.force, self.x_cap = items, lo, hi, k, force_ovf, x_cap

    def screen(self, users, m):
        self.users = users.double().numpy()
        sc = self.users @ self.items[self.lo:self.hi].astype(np.float64).T
        top = -np.sort(-sc, axis=1)[:, :m] - 1e-9
        if top.shape[1] < m:
            top = np.concatenate([top, np.full((len(top), m - top.shape[1]), -np.inf)], 1)
        return torch.from_numpy(top.astype(np.float32) - np.float32(1e-6))

    def band(self, bounds):
        U = self.users.shape[0]
        g = np.full(U, -np.inf)
        if bounds is not None:
            L, _, m = bounds.shape
            vals = bounds.permute(1, 0, 2).reshape(U, L * m).double().numpy()
            if L * m >= self.k:
                g = -np.sort(-vals, axis=1)[:, self.k - 1]
        sc = self.users @ self.items[self.lo:self.hi].astype(np.float64).T
        keep = sc >= (g[:, None] - 1e-6)
        cnt = keep.sum(1)
        cap = self.x_cap  # fixed exchange slots; more -> -1 (exact path on the owner)
        ent = np.zeros((U, cap), np.int64)
        for u in range(U):
            rows = np.nonzero(keep[u])[0] + self.lo
            ent[u, :min(cap, len(rows))] = rows[:cap]
        cnt = np.where(cnt > cap, -1, cnt).astype(np.int32)
        if self.force is not None:
            cnt[self.force] = -1
        self.g = g
        return torch.from_numpy(cnt), torch.from_numpy(ent)

    def ucut(self, lo, hi):
        return torch.from_numpy(np.stack([self.g[lo:hi], np.zeros(hi - lo)], 1).astype(np.float32))

    def refine(self, users, src_cnt, src_ent, ucut, ovf):
        u = users.double().numpy()
        rc, re, ovf = src_cnt.numpy(), src_ent.numpy(), ovf.numpy()
        n, k = len(u), self.k
        s = np.full((n, k), -np.finfo(np.float32).max, np.float32)
        r = np.full((n, k), -1, np.int32)
        e = np.full((n, k), -np.inf)
        for i in range(n):
            got = [re[w, i, :max(0, rc[w, i])] for w in range(rc.shape[0])]
            rows = np.arange(len(self.items)) if ovf[i] else np.unique(np.concatenate(got))
            sc = (u[i] @ self.items[rows].astype(np.float64).T) if len(rows) else np.zeros(0)
            order = np.lexsort((rows, -sc))[:k]
            m = len(order)
            r[i, :m], e[i, :m], s[i, :m] = rows[order], sc[order], sc[order].astype(np.float32)
        return torch.from_numpy(s), torch.from_numpy(r), torch.from_numpy(e)


def _owner_worker(rank, world, port, U, I, D, k, q, x_cap=64):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nrk.dist import catalog_sharded_owner, shard_range

        rng = np.random.default_rng(11)
        users = rng.standard_normal((U, D)).astype(np.float32)
        items = rng.standard_normal((I, D)).astype(np.float32)
        items[I // 2 + 1] = items[3]  # cross-shard exact tie -> lower row must win
        lo, hi = shard_range(I, world, rank)
        shard = _OwnerShard(items, lo, hi, k, force_ovf=2 if rank == world - 1 else None, x_cap=x_cap)
        s, r, e = catalog_sharded_owner(torch.from_numpy(users), shard, k)
        ulo, uhi = shard_range(U, world, rank)
        q.put((rank, ulo, uhi, s.numpy(), r.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,U,I,k,x_cap", [(2, 37, 101, 31, 64), (3, 50, 400, 8, 64), (2, 64, 40, 31, 64),
                                                (3, 5, 7, 10, 64), (3, 50, 400, 8, 3)])
def test_catalog_sharded_owner_refine_matches_single(world, U, I, k, x_cap):
    """Config 4 with owner refine: bound all_gather, the fixed-slot band
    all_to_all (counts + x_cap entries per user and shard; users padded to
    whole blocks), overflowed users (forced, or more than x_cap entries from
    one shard) on the exact path -- the merged result equals one GPU's."""
    from oracle import oracle

    D = 16
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_owner_worker, args=(r, world, port, U, I, D, k, q, x_cap)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(11)
    users = rng.standard_normal((U, D)).astype(np.float32)
    items = rng.standard_normal((I, D)).astype(np.float32)
    items[I // 2 + 1] = items[3]
    so, ro = oracle.ip_topk(users, items, k)
    for rank, ulo, uhi, s, r in got:
        assert np.array_equal(r, ro[ulo:uhi]), rank
        assert np.array_equal(s, so[ulo:uhi]), rank


def _grid_worker(rank, world, port, R, U, I, D, k, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nrk.dist import catalog_sharded_owner, grid_groups, grid_ranges, shard_range

        rng = np.random.default_rng(11)
        users = rng.standard_normal((U, D)).astype(np.float32)
        items = rng.standard_normal((I, D)).astype(np.float32)
        items[I // 2 + 1] = items[3]
        grp, g, c = grid_groups(world, R, rank)
        C = world // R
        (glo, ghi), (ulo, uhi), _ = grid_ranges(U, I, world, R, rank, 1)
        lo, hi = shard_range(I, C, c)  # the stand-in shards by rows
        shard = _OwnerShard(items, lo, hi, k, force_ovf=1 if c == C - 1 else None)
        s, r, e = catalog_sharded_owner(torch.from_numpy(users[glo:ghi]), shard, k, group=grp)
        q.put((rank, ulo, uhi, s.numpy(), r.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,R,U,I,k", [(4, 2, 41, 300, 31), (6, 2, 50, 400, 8), (6, 3, 23, 90, 10)])
def test_grid_owner_refine_matches_single(world, R, U, I, k):
    """Config 4 as an R x C rank grid (nrk.dist.layout_2d / grid_groups):
    each user group runs the owner protocol over its C catalog shards inside
    its own process group (bound all_gather and band all_to_all among C
    ranks); every rank's user block equals one GPU's rows and scores."""
    from oracle import oracle

    D = 16
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grid_worker, args=(r, world, port, R, U, I, D, k, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(11)
    users = rng.standard_normal((U, D)).astype(np.float32)
    items = rng.standard_normal((I, D)).astype(np.float32)
    items[I // 2 + 1] = items[3]
    so, ro = oracle.ip_topk(users, items, k)
    covered = np.zeros(U, np.int32)
    for rank, ulo, uhi, s, r in got:
        covered[ulo:uhi] += 1
        assert np.array_equal(r, ro[ulo:uhi]), rank
        assert np.array_equal(s, so[ulo:uhi]), rank
    assert (covered == 1).all()


def test_layout_2d():
    from nrk.dist import grid_ranges, layout_2d

    assert layout_2d(8) == (1, 8) and layout_2d(4) == (1, 4) and layout_2d(1) == (1, 1) and layout_2d(8, 2) == (2, 4)
    with pytest.raises(ValueError):
        layout_2d(6, 4)
    U, I, tb = 250_000, 364_047, 4
    seen_u, seen_b = np.zeros(U, np.int32), np.zeros(-(-I // 32), np.int32)
    for r in range(8):
        (glo, ghi), (lo, hi), (blo, bhi) = grid_ranges(U, I, 8, 2, r, tb)
        assert glo <= lo <= hi <= ghi and blo % tb == 0
        seen_u[lo:hi] += 1
        seen_b[blo:bhi] += 1
    assert (seen_u == 1).all() and (seen_b == 2).all()  # every item block screened once per user group


def test_shard_blocks_tile_aligned():
    from nrk.dist import shard_blocks

    for n in (1, 5000, 364_047):
        for w in (1, 2, 3, 8):
            spans = [shard_blocks(n, w, r, 4) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == -(-n // 32)
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert all(a[0] % 4 == 0 for a in spans if a[1] > a[0])  # empty tail ranges sit at the end


def test_shard_range_covers():
    from nrk.dist import shard_range

    for n in (0, 1, 7, 364_047):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


# ------------------------------------------------ users-sharded ItemCF --
def _np_pairs(offsets, items, ts, created, n_items, slot_base):
    """Pair tuples of item_cf.py:36-79 (weights.py), global slots; numpy/math."""
    import math

    offs, it, t, cr = offsets.numpy(), items.numpy(), ts.numpy(), created.numpy()
    b = 1
    while (1 << b) <= n_items:
        b += 1
    sent = (1 << (2 * b)) - 1
    keys, slots, w = [], [], []
    cnt = np.zeros(n_items, np.int64)
    base = slot_base
    for u in range(len(offs) - 1):
        a, e = offs[u], offs[u + 1]
        L = e - a
        pen = 1.0 / math.log(L + 1) if L else 0.0
        for x in it[a:e]:
            cnt[x] += 1
        for l1 in range(L):
            for l2 in range(L):
                i, j = int(it[a + l1]), int(it[a + l2])
                if i == j:
                    keys.append(sent)
                    w.append(0.0)
                else:
                    la = 1.0 if l2 > l1 else 0.7
                    lw = la * 0.9 ** (abs(l2 - l1) - 1)
                    cw = math.exp(0.7 ** abs(int(t[a + l1]) - int(t[a + l2])))
                    tw = math.exp(0.8 ** abs(cr[i] - cr[j]))
                    keys.append((i << b) | j)
                    w.append(lw * cw * tw * pen)
                slots.append(base + l1 * L + l2)
        base += L * L
    return (torch.tensor(keys, dtype=torch.int64), torch.tensor(slots, dtype=torch.int32),
            torch.tensor(w, dtype=torch.float64), torch.from_numpy(cnt))


class _Entries:
    def __init__(self, i, j, v, first):
        self.i, self.j, self.v, self.first = i, j, v, first


def _np_reduce(keys, slots, w, n_items, cnt):
    """The owner's reduce: sums in (global) slot order, first slot, / sqrt(cnt_i cnt_j)."""
    import math

    b = 1
    while (1 << b) <= n_items:
        b += 1
    acc = {}
    for k, s, x in zip(keys.tolist(), slots.tolist(), w.tolist()):
        if k == (1 << (2 * b)) - 1:
            continue
        if k not in acc:
            acc[k] = [0.0, s]
        acc[k][0] += x
    ks = sorted(acc)
    c = cnt.numpy()
    i = np.array([k >> b for k in ks], np.int64)
    j = np.array([k & ((1 << b) - 1) for k in ks], np.int64)
    v = np.array([acc[k][0] / math.sqrt(c[a] * c[bb]) for k, a, bb in zip(ks, i, j)])
    return _Entries(i, j, v, np.array([acc[k][1] for k in ks], np.int64))


def _cf_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nrk.dist import itemcf_sim_sharded, shard_range

        rng = np.random.default_rng(11)
        n_users, n_items = 60, 25
        L = rng.integers(0, 9, n_users)
        offs = np.concatenate([[0], np.cumsum(L)]).astype(np.int64)
        items = rng.integers(0, n_items, offs[-1]).astype(np.int32)
        ts = (1_500_000_000_000 + np.cumsum(rng.integers(0, 3, offs[-1]))).astype(np.int64)
        created = rng.random(n_items)
        lo, hi = shard_range(n_users, world, rank)
        a, e = offs[lo], offs[hi]
        res = itemcf_sim_sharded(torch.from_numpy(offs[lo:hi + 1] - a), torch.from_numpy(items[a:e]),
                                 torch.from_numpy(ts[a:e]), torch.from_numpy(created), n_items,
                                 pairs=_np_pairs, reduce=_np_reduce)
        ilo, ihi = shard_range(n_items, world, rank)
        assert ((res.i >= ilo) & (res.i < ihi)).all()
        q.put((rank, res.i, res.j, res.v, res.first))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_itemcf_users_sharded_gloo(world):
    """SURVEY 8e ItemCF: users sharded, one all_to_all by item owner + an
    all_reduce of the click counts -> the same entries, first-encounter slots
    and values as the single-process oracle."""
    from oracle import oracle

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_cf_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = [q.get(timeout=300) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    gi = np.concatenate([g[1] for g in got])
    gj = np.concatenate([g[2] for g in got])
    gv = np.concatenate([g[3] for g in got])
    gf = np.concatenate([g[4] for g in got])
    rng = np.random.default_rng(11)
    n_users, n_items = 60, 25
    L = rng.integers(0, 9, n_users)
    offs = np.concatenate([[0], np.cumsum(L)]).astype(np.int64)
    items = rng.integers(0, n_items, offs[-1]).astype(np.int32)
    ts = (1_500_000_000_000 + np.cumsum(rng.integers(0, 3, offs[-1]))).astype(np.int64)
    created = rng.random(n_items)
    oi, oj, ov, _, _ = oracle.itemcf_sim(offs, items, ts, created, n_items)
    order = np.argsort(gf, kind="stable")  # first-encounter order = the oracle's
    assert np.array_equal(gi[order], oi) and np.array_equal(gj[order], oj)
    np.testing.assert_allclose(gv[order], ov, rtol=1e-12, atol=0)


def test_itemcf_slot_range_guard():
    """the sharded ItemCF's int32 global slots must not wrap."""
    from nrk.dist import SLOT_LIMIT, check_slot_range

    check_slot_range(SLOT_LIMIT - 1)
    with pytest.raises(ValueError):
        check_slot_range(SLOT_LIMIT)
    with pytest.raises(ValueError):
        check_slot_range(3 * (1 << 30))
