"""Multi-GPU layouts of the recall path.  One process per GPU,
torch.distributed over RCCL ("nccl" on ROCm), 127.0.0.1 rendezvous.

* users-sharded  -- every rank scores its own contiguous user block against
  the full (replicated) catalog.  No data-path collective (weak scaling).
* catalog-sharded (BASELINE config 4) -- rank r holds items [lo_r, hi_r) and
  scores ALL users of the batch against its shard (global row ids via
  row_offset).  One exchange step: all_to_all of the shard-local top-k
  (fp64 exact score + int32 global row, 12 B per entry) so that the owner of
  each user block receives every shard's list for its users, then
  nrk_topk_merge orders by (score desc, row asc) -- the same tie-break as a
  single GPU, so the merged lists are identical to the 1-GPU result.
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


def shard_range(n: int, world: int, rank: int):
    """Contiguous split, ceil(n / world) per rank (the last ranks may be short)."""
    per = -(-n // world)
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


def _default_local(users, shard, k, row_lo):
    from . import ops

    s, r, e = ops.ip_topk(users, shard, k, row_offset=row_lo, exact=True)
    return e, r


def _default_merge(exact_lists, row_lists, k):
    from . import ops

    return ops.topk_merge(exact_lists, row_lists, k)


def catalog_sharded_topk(users, shard, row_lo: int, k: int, group=None, local=None, merge=None):
    """Exact top-k of ``users`` (replicated on every rank, [U, D]) over the
    catalog split across the ranks of ``group``.  ``shard`` is this rank's
    ops.Catalog (rows [row_lo, row_lo + shard.ntotal)).  Returns the merged
    (scores f32, rows i32, exact f64) for THIS rank's user block
    shard_range(U, world, rank).  ``local`` / ``merge`` default to the HIP
    kernels; tests inject CPU stand-ins to run the exchange under gloo."""
    local = local or _default_local
    merge = merge or _default_merge
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    U = users.shape[0]
    e, r = local(users, shard, k, row_lo)  # [U, k] each
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
    dist.all_to_all_single(re, e.contiguous(), group=group)
    dist.all_to_all_single(rr, r.contiguous(), group=group)
    s_, r_, x_ = merge(re.view(world, per, k), rr.view(world, per, k), k)
    lo, hi = shard_range(U, world, rank)
    return s_[: hi - lo], r_[: hi - lo], x_[: hi - lo]


def _default_pairs(offsets, items, ts, created, n_items, slot_base):
    from . import ops

    return ops.itemcf_pairs(offsets, items, ts, created, n_items, slot_base)


def _default_reduce(keys, slots, w, n_items, cnt):
    from . import ops

    return ops.itemcf_reduce(keys, slots, w, n_items, cnt)


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
    else:
        base = 0
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
