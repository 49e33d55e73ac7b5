"""Multi-GPU layouts of the recall path.  One process per GPU,
torch.distributed over RCCL ("nccl" on ROCm), 127.0.0.1 rendezvous.

* users-sharded  -- every rank scores its own contiguous user block against
  the full (replicated) catalog.  No data-path collective (weak scaling).
* catalog-sharded (BASELINE config 4), owner refine (catalog_sharded_owner,
  the default, k <= 128) -- every rank holds the whole packed catalog and
  fp32 rows (69 MB at config 2) and screens only its tile-aligned block
  range for ALL users (gather_users: each rank runs the user tower for its
  own user block, all_gather).  Two exchanges, both fixed-size (no host-side
  sizes, no sync): an all_gather of every shard's m largest screen lower
  bounds per user (nrk_ip_topk_shard_screen), whose k-th largest bounds the
  user's GLOBAL k-th score; each shard packs the half-block ids at or above
  its cut (nrk_ip_topk_shard_band: IP_X_CAP = 32 slots of 4-byte int32
  half-block ids per user, count -1 = more than 32 -> the owner takes that
  user's exact path), and one all_to_all of counts and slots goes to the
  owner of each user block, which runs the exact refine of its users only
  from every shard's slots (nrk_ip_topk_refine_x): the refine shrinks 1/N
  with the screen and no merge is needed.  Same rows and scores as one GPU.
  The ranks may form an R x C grid (layout_2d, bench --user-groups R): R user
  groups, each running this protocol over C catalog shards inside its own
  process group, so the per-user passes cover U / R users (default R = 1).
* catalog-sharded, merge (catalog_sharded_topk) -- each shard holds its own
  rows and refines every user against them (k <= 128: after the bound
  exchange; larger k: the exact path, no exchange) and an all_to_all of the
  shard-local top-k (fp64 exact + int32 global row) goes to the owner,
  where nrk_topk_merge orders by (score desc, row asc), pairwise in a tree
  when the lists exceed one merge (k <= 512).
* users-sharded ItemCF similarity (itemcf_sim_sharded) -- rank r holds the
  click lists of users [lo_r, hi_r) and owns items [ilo_r, ihi_r).  Every
  rank emits the pair tuples (key, GLOBAL slot, weight) of its users; one
  exchange (all_to_all by owner of item i, sources concatenated in rank
  order = global slot order) and an all_reduce of the click counts; the
  owner reduces its tuples (sort by key, sums in slot order, / sqrt(cnt_i
  cnt_j)).  Same entries, values and first-encounter slots as one GPU.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def _staged(t, group=None):
    """gloo with device tensors: collectives staged through host memory (the
    one-GPU rehearsals of the N-rank layouts; RCCL takes device tensors)."""
    return t.is_cuda and dist.is_initialized() and dist.get_backend(group) == "gloo"


def all_gather_into(out, inp, group=None):
    if _staged(out, group):
        o = out.cpu()
        dist.all_gather_into_tensor(o, inp.cpu(), group=group)
        out.copy_(o)
    else:
        dist.all_gather_into_tensor(out, inp, group=group)


def all_to_all(out, inp, out_splits=None, in_splits=None, group=None):
    if _staged(out, group):
        o = out.cpu()
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)


def shard_range(n: int, world: int, rank: int):
    """Contiguous split, ceil(n / world) per rank (the last ranks may be short)."""
    per = -(-n // world)
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


class HipShard:
    """This rank's catalog shard on the HIP path (nrk_ip_topk_screen ->
    nrk_ip_topk_bound / _apply_bound -> nrk_ip_topk_finish), with its
    workspace and outputs allocated once for ``n_users`` queries.  For
    k > ops.IP_KFAST (no MFMA screen; nrk_ip_topk's exact path) there are no
    screen bounds: ``bounded`` is False, screen() returns -inf and finish()
    runs the exact top-k of the shard."""

    def __init__(self, catalog, row_lo: int, k: int, n_users: int):
        from . import ops

        self.ops, self.cat, self.row_lo, self.k = ops, catalog, int(row_lo), int(k)
        self.bounded = self.k <= ops.IP_KFAST
        dev = catalog.items.device
        self.ws = ops.ip_topk_workspace(n_users, catalog, k, dev)
        self.s = torch.empty((n_users, k), dtype=torch.float32, device=dev)
        self.r = torch.empty((n_users, k), dtype=torch.int32, device=dev)
        self.e = torch.empty((n_users, k), dtype=torch.float64, device=dev)

    def screen(self, users, m: int):
        """fp16 MFMA screen; returns this shard's m largest exact lower
        bounds per user (fp32 [U, m]; -inf without a screen)."""
        if not self.bounded:
            return torch.full((users.shape[0], m), float("-inf"), dtype=torch.float32, device=users.device)
        self.ops.ip_topk_screen(users, self.cat, self.k, self.ws)
        return self.ops.ip_topk_bound(users, self.cat, self.k, m, self.ws)

    def finish(self, users, bounds=None):
        """Exact refine -> (exact f64 [U, k], global rows i32 [U, k]) of this
        shard; with ``bounds`` ([n_lists, U, m], every shard's screen bounds)
        the cut is first raised to the k-th largest of each user's values."""
        n = users.shape[0]
        if not self.bounded:
            s, r, e = self.ops.ip_topk(users, self.cat, self.k, row_offset=self.row_lo, exact=True,
                                       workspace=self.ws, check_finite=False)
            return e, r
        if bounds is not None:
            self.ops.ip_topk_apply_bound(bounds, self.k, self.ws)
        self.ops.ip_topk_finish(users, self.cat, self.k, self.ws, self.s[:n], self.r[:n],
                                out_exact=self.e[:n], row_offset=self.row_lo)
        return self.e[:n], self.r[:n]


def bound_width(k: int, world: int) -> int:
    """Bounds per user and shard for the exchange: world * m >= k values
    (so the k-th largest exists) with a little slack, world * m <= 512; 0 =
    no exchange (one rank, or too many ranks for nrk_ip_topk_apply_bound)."""
    if world <= 1:
        return 0
    m = min(256, -(-k // world) + 1)
    return m if world * m <= 512 and world * m >= k else 0


MERGE_MAX = 1024  # entries one nrk_topk_merge call orders per user


def _default_merge(exact_lists, row_lists, k):
    """(score desc, row asc) merge of [G, n, k_in] lists; lists longer than
    one merge call are merged pairwise in a tree (the order is total, so
    the result is the same)."""
    from . import ops

    G, n, k_in = exact_lists.shape
    while G * k_in > MERGE_MAX:
        if 2 * k_in > MERGE_MAX:
            raise NotImplementedError(f"catalog-sharded merge supports k <= {MERGE_MAX // 2}, got {k_in}")
        e_next, r_next = [], []
        for g in range(0, G, 2):
            if g + 1 == G:
                e_next.append(exact_lists[g])
                r_next.append(row_lists[g])
                continue
            _, r2, e2 = ops.topk_merge(exact_lists[g:g + 2].contiguous(), row_lists[g:g + 2].contiguous(), k_in)
            e_next.append(e2)
            r_next.append(r2)
        exact_lists, row_lists = torch.stack(e_next).contiguous(), torch.stack(r_next).contiguous()
        G = exact_lists.shape[0]
    return ops.topk_merge(exact_lists, row_lists, k)


def gather_users(u_local, n_users: int, group=None):
    """Every rank computed the user tower for its own block
    shard_range(n_users, world, rank); all_gather -> the full [n_users, D]
    on every rank (the catalog-sharded screen needs every user)."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1:
        return u_local
    per = -(-n_users // world)
    buf = torch.empty((per * world,) + tuple(u_local.shape[1:]), dtype=u_local.dtype, device=u_local.device)  # rank-major blocks
    send = u_local
    if u_local.shape[0] < per:
        send = torch.zeros((per,) + tuple(u_local.shape[1:]), dtype=u_local.dtype, device=u_local.device)
        send[: u_local.shape[0]] = u_local
    all_gather_into(buf, send.contiguous(), group=group)
    if per * world == n_users:
        return buf
    parts = [buf[r * per: r * per + (shard_range(n_users, world, r)[1] - shard_range(n_users, world, r)[0])]
             for r in range(world)]
    return torch.cat(parts).contiguous()


def catalog_sharded_topk(users, shard, k: int, group=None, merge=None, exchange_bound: bool = True):
    """Exact top-k of ``users`` (replicated on every rank, [U, D]) over the
    catalog split across the ranks of ``group``.  ``shard`` (HipShard, or a
    stand-in with the same screen / finish methods in the gloo tests) holds
    this rank's rows [row_lo, row_lo + n) and reports global rows.

    Two exchanges:
      1. all_gather of every shard's m largest screen bounds per user
         (fp32 [U, m], bound_width(k, world)) between screen and refine: the
         k-th largest of a user's world * m values bounds the user's GLOBAL
         k-th exact score from below, so each shard rescores only the
         candidates that can still reach the merged top-k;
      2. all_to_all of the shard-local top-k (fp64 exact + int32 global row)
         to the owner of each user block, then the (score desc, row asc)
         merge -- the same tie-break as one GPU.
    Returns the merged (scores f32, rows i32, exact f64) of THIS rank's user
    block shard_range(U, world, rank)."""
    merge = merge or _default_merge
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    U = users.shape[0]
    m = bound_width(k, world) if exchange_bound and getattr(shard, "bounded", True) else 0
    b = shard.screen(users, max(m, 1))
    bounds = None
    if m:
        bounds = torch.empty((world * b.shape[0], b.shape[1]), dtype=b.dtype, device=b.device)
        all_gather_into(bounds, b.contiguous(), group=group)
        bounds = bounds.view(world, b.shape[0], b.shape[1])
    e, r = shard.finish(users, bounds)  # [U, k] each
    if world == 1:
        return merge(e.unsqueeze(0).contiguous(), r.unsqueeze(0).contiguous(), k)
    per = -(-U // world)
    pad = per * world - U
    if pad:  # equal blocks for all_to_all_single; padded users are dropped after the merge
        e = torch.cat([e, torch.full((pad, k), float("-inf"), dtype=e.dtype, device=e.device)])
        r = torch.cat([r, torch.full((pad, k), -1, dtype=r.dtype, device=r.device)])
    re = torch.empty_like(e)
    rr = torch.empty_like(r)
    # block s of the send buffer = users of rank s; block s of the receive
    # buffer = shard s's lists for this rank's users
    all_to_all(re, e.contiguous(), group=group)
    all_to_all(rr, r.contiguous(), group=group)
    s_, r_, x_ = merge(re.view(world, per, k), rr.view(world, per, k), k)
    lo, hi = shard_range(U, world, rank)
    return s_[: hi - lo], r_[: hi - lo], x_[: hi - lo]


class HipRangeShard:
    """Config 4 with owner refine: the shared catalog (every rank builds the
    same ops.Catalog over ALL items) and this rank's block range, tile
    aligned (shard_blocks).  screen / band on this rank's range for every
    user; refine for the owner's user block."""

    def __init__(self, catalog, blk_lo: int, blk_hi: int, k: int, n_users: int):
        from . import ops

        self.ops, self.cat, self.k = ops, catalog, int(k)
        self.k_max = ops.IP_KFAST  # the shard screen's list (nrk_ip_topk_shard_screen)
        if self.k > self.k_max:
            raise NotImplementedError(f"HipRangeShard (owner protocol) handles k <= {self.k_max}, got {self.k}; "
                                      "use HipShard + catalog_sharded_topk")
        self.blk_lo, self.blk_hi, self.n_users = int(blk_lo), int(blk_hi), int(n_users)
        self.ws = ops.ip_topk_workspace(n_users, catalog, k, catalog.items.device)
        self.rws = None
        self.x_cap = ops.IP_X_CAP

    def screen(self, users, m: int):
        # scan + the m largest appended maxima as bounds (no per-shard select)
        return self.ops.ip_topk_shard_screen(users, self.cat, self.k, self.blk_lo, self.blk_hi, m, self.ws)

    def band(self, bounds=None):
        # cut = max(own list bound - 2 eps, global bound - eps); entries >= cut,
        # x_cap slots per user for the fixed-size exchange
        return self.ops.ip_topk_shard_band(self.n_users, self.cat, self.k, bounds, self.ws, self.x_cap)

    def ucut(self, lo: int, hi: int):
        return self.ops.ip_topk_ucut(self.ws, self.n_users)[lo:hi].contiguous()

    def refine(self, users, src_cnt, src_ent, ucut, ovf):
        if self.rws is None:
            self.rws = self.ops.ip_topk_workspace(users.shape[0], self.cat, self.k, users.device)
        return self.ops.ip_topk_refine_x(users, self.cat, self.k, src_cnt, src_ent, ucut, ovf, workspace=self.rws)


def shard_blocks(n_items: int, world: int, rank: int, tile_blocks: int):
    """Block range of rank r: whole screen tiles (tile_blocks 32-item blocks)
    split contiguously; the last rank ends at the catalog's last block."""
    nblk = -(-n_items // 32)
    ntile = -(-nblk // tile_blocks)
    lo, hi = shard_range(ntile, world, rank)
    return min(nblk, lo * tile_blocks), min(nblk, hi * tile_blocks)


def exchange_bands(cnt, ent, n_users: int, group=None):
    """The owner exchange, fixed size (no host-side sizes, so no sync): rank
    r holds, per user, cnt [U] int32 (-1 = overflowed) and ent [U, X] (X
    slots of int32 half-block ids on the HIP path); user block o (rows [o * per, (o + 1) * per), per = ceil(U /
    world), = shard_range) goes to owner o with one all_to_all of counts and
    one of entries.  Returns this rank's (src_cnt int32 [world, per],
    src_ent [world, per, X]): source s's band of the owner's users."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    U, X = ent.shape
    if world == 1:
        return cnt.view(1, U), ent.view(1, U, X)
    per = -(-n_users // world)
    if per * world != U:  # pad to whole blocks
        cp = torch.full((per * world,), 0, dtype=cnt.dtype, device=cnt.device)
        cp[:U] = cnt
        ep = torch.zeros((per * world, X), dtype=ent.dtype, device=ent.device)
        ep[:U] = ent
        cnt, ent = cp, ep
    rc = torch.empty_like(cnt)
    all_to_all(rc, cnt.contiguous(), group=group)
    re = torch.empty_like(ent)
    all_to_all(re, ent.contiguous(), group=group)
    return rc.view(world, per), re.view(world, per, X)


def catalog_sharded_owner(users, shard, k: int, group=None, exchange_bound: bool = True, mark=None):
    """Config 4, owner refine (see the module docstring): ``users`` [U, D]
    on every rank, ``shard`` a HipRangeShard (or a stand-in with screen /
    band / ucut / refine in the gloo tests).  Returns (scores f32, rows i32,
    exact f64) of THIS rank's user block shard_range(U, world, rank).
    ``mark(phase)``, if given, is called after the screen + bound exchange
    ("screen") and after the band pack + all_to_all ("exchange") -- bench.py
    records HIP events there."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    U = users.shape[0]
    if k > getattr(shard, "k_max", k):
        raise NotImplementedError(f"the owner protocol's shard screen handles k <= {shard.k_max}; "
                                  f"use catalog_sharded_topk (merge protocol) for k = {k}")
    m = bound_width(k, world) if exchange_bound else 0
    b = shard.screen(users, max(m, 1))
    bounds = None
    if m:
        bounds = torch.empty((world * b.shape[0], b.shape[1]), dtype=b.dtype, device=b.device)
        all_gather_into(bounds, b.contiguous(), group=group)
        bounds = bounds.view(world, b.shape[0], b.shape[1])
    if mark is not None:
        mark("screen")
    cnt, ent = shard.band(bounds)
    rc, re = exchange_bands(cnt, ent, U, group)
    if mark is not None:
        mark("exchange")
    lo, hi = shard_range(U, world, rank)
    ovf = (rc[:, :hi - lo] < 0).any(0).to(torch.int32)
    return shard.refine(users[lo:hi].contiguous(), rc, re, shard.ucut(lo, hi), ovf)


def layout_2d(world: int, R: int | None = None):
    """The config-4 rank grid: R user groups x C catalog shards, R C = world.
    Rank r = g C + c screens group g's users (shard_range(U, R, g)) over
    catalog shard c (shard_blocks(I, C, c, tile)) and refines its 1 / C of
    group g's users; the two exchanges stay inside the group's C ranks.
    Every per-user pass of a rank (the shard screen's list pre-pass share,
    the bound and band passes) covers U / R users instead of U, and each shard's
    tile range is R times longer, which shrinks the sampled pre-pass relative
    to it.  Default R = 1: measured on the one-GPU replay (tools/catalog_replay.py,
    DESIGN 4.6), 2 x 4 runs 1.67 ms per rank against 1.52 for 1 x 8 -- a
    group's 125k users fill only 123 of the 256 CUs at the warp-specialized
    scan's 1,024 users per workgroup -- and 4 x 2 overflows the band
    exchange's 32 slots per user and shard (exact path)."""
    if R is None:
        R = 1
    if R < 1 or world % R:
        raise ValueError(f"{R} user groups do not divide {world} ranks")
    return R, world // R


def grid_groups(world: int, R: int, rank: int):
    """The R process groups of layout_2d (every rank creates all of them, in
    the same order, as torch.distributed requires); returns (this rank's
    group, its group index g, its shard index c).  R = 1: the default group."""
    C = world // R
    if R == 1:
        return None, 0, rank
    groups = [dist.new_group(list(range(g * C, (g + 1) * C))) for g in range(R)]
    return groups[rank // C], rank // C, rank % C


def grid_ranges(n_users: int, n_items: int, world: int, R: int, rank: int, tile_blocks: int):
    """Rank r's share in layout_2d: (group users [glo, ghi), own users
    [lo, hi) (global rows: the users it runs the tower for and refines),
    block range [blo, bhi) of its catalog shard)."""
    C = world // R
    g, c = rank // C, rank % C
    glo, ghi = shard_range(n_users, R, g)
    lo, hi = shard_range(ghi - glo, C, c)
    blo, bhi = shard_blocks(n_items, C, c, tile_blocks)
    return (glo, ghi), (glo + lo, glo + hi), (blo, bhi)


def owner_replay(users, shards, k: int, timer=None):
    """One-process replay of catalog_sharded_owner over ``shards`` (one
    HipRangeShard per emulated rank, all on this device): the two exchanges
    become stacks.  ``timer(phase, rank, fn)`` may wrap each rank's steps
    (tools/catalog_replay.py times them).  Returns the full (scores f32
    [U, k], rows i32 [U, k], exact f64 [U, k])."""
    run = timer or (lambda phase, r, fn: fn())
    world = len(shards)
    U = users.shape[0]
    m = bound_width(k, world)
    bs = [run("screen", r, lambda sh=sh: sh.screen(users, max(m, 1))) for r, sh in enumerate(shards)]
    bounds = torch.stack(bs).contiguous() if m else None
    packs = [run("band", r, lambda sh=sh: sh.band(bounds)) for r, sh in enumerate(shards)]
    per = -(-U // world)
    outs = []
    for o in range(world):
        lo, hi = shard_range(U, world, o)
        rc = torch.zeros((world, per), dtype=torch.int32, device=users.device)
        re = torch.zeros((world, per, packs[0][1].shape[1]), dtype=packs[0][1].dtype, device=users.device)
        for src, (c, ent) in enumerate(packs):
            rc[src, :hi - lo] = c[lo:hi]
            re[src, :hi - lo] = ent[lo:hi]
        ovf = (rc[:, :hi - lo] < 0).any(0).to(torch.int32)
        sh = shards[o]
        outs.append(run("refine", o, lambda sh=sh, lo=lo, hi=hi, rc=rc, re=re, ovf=ovf: sh.refine(
            users[lo:hi].contiguous(), rc, re, sh.ucut(lo, hi), ovf)))
    return tuple(torch.cat([x[i] for x in outs]) for i in range(3))


def _default_pairs(offsets, items, ts, created, n_items, slot_base):
    from . import ops

    return ops.itemcf_pairs(offsets, items, ts, created, n_items, slot_base)


def _default_reduce(keys, slots, w, n_items, cnt):
    from . import ops

    return ops.itemcf_reduce(keys, slots, w, n_items, cnt)


SLOT_LIMIT = (1 << 31) - (1 << 16)  # int32 global slots, minus the radix sort's tile slack


def check_slot_range(total_pairs: int):
    """The pair tuples carry int32 GLOBAL slots (the first-encounter order):
    the whole log's ordered pair count must stay below 2^31 (minus the sort
    tile), or slots would wrap and break the reference's dict order."""
    if total_pairs >= SLOT_LIMIT:
        raise ValueError(f"{total_pairs} ordered pairs: int32 global slots need < {SLOT_LIMIT}")


def itemcf_sim_sharded(offsets, items, ts, created, n_items: int, group=None, pairs=None, reduce=None):
    """ItemCF similarity (item_cf.py:17-89) with users sharded over the ranks
    of ``group``.  ``offsets`` / ``items`` / ``ts`` are THIS rank's users (a
    contiguous block of the global user order, ranks in order); ``created``
    covers all n_items.  Returns this rank's owned entries (rows i in
    shard_range(n_items, world, rank)) as the reducer's result.  ``pairs`` /
    ``reduce`` default to the HIP kernels; tests inject CPU stand-ins."""
    pairs = pairs or _default_pairs
    reduce = reduce or _default_reduce
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    L = offsets[1:] - offsets[:-1]
    n_local = int((L * L).sum())
    dev = offsets.device
    # global slot base: pairs of the ranks before this one
    tot = torch.tensor([n_local], dtype=torch.int64, device=dev)
    if world > 1:
        all_tot = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
        dist.all_gather(all_tot, tot, group=group)
        base = int(sum(int(t) for t in all_tot[:rank]))
        check_slot_range(sum(int(t) for t in all_tot))
    else:
        base = 0
        check_slot_range(n_local)
    keys, slots, w, cnt = pairs(offsets, items, ts, created, n_items, base)
    if world == 1:
        return reduce(keys, slots, w, n_items, cnt)
    dist.all_reduce(cnt, group=group)
    # bucket by owner of item i (key >> b); stable, so each bucket stays in slot order
    b = 1
    while (1 << b) <= n_items:
        b += 1
    per = -(-n_items // world)
    live = torch.nonzero(keys != (1 << (2 * b)) - 1).flatten()  # drop the i == j sentinels
    keys, slots, w = keys[live], slots[live], w[live]
    owner = (keys >> b) // per
    order = torch.sort(owner, stable=True).indices
    send_counts = torch.bincount(owner, minlength=world).to(torch.int64)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    sc, rc = send_counts.tolist(), recv_counts.tolist()
    nr = int(sum(rc))
    rk = torch.empty(nr, dtype=keys.dtype, device=keys.device)
    rs = torch.empty(nr, dtype=slots.dtype, device=slots.device)
    rw = torch.empty(nr, dtype=w.dtype, device=w.device)
    dist.all_to_all_single(rk, keys[order].contiguous(), rc, sc, group=group)
    dist.all_to_all_single(rs, slots[order].contiguous(), rc, sc, group=group)
    dist.all_to_all_single(rw, w[order].contiguous(), rc, sc, group=group)
    return reduce(rk, rs, rw, n_items, cnt)
