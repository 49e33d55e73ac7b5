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
