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


def _oracle_local(users, shard, k, row_lo):
    from oracle import oracle

    s, r, e = oracle.ip_topk(users.numpy(), shard, k, exact=True)
    r = np.where(r >= 0, r + row_lo, -1)
    return torch.from_numpy(e), torch.from_numpy(r.astype(np.int32))


def _worker(rank, world, port, U, I, D, k, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nrk.dist import catalog_sharded_topk, shard_range

        rng = np.random.default_rng(7)
        users = rng.standard_normal((U, D)).astype(np.float32)
        items = rng.standard_normal((I, D)).astype(np.float32)
        items[I // 2 + 1] = items[3]  # cross-shard exact tie -> lower row must win
        lo, hi = shard_range(I, world, rank)
        s, r, e = catalog_sharded_topk(torch.from_numpy(users), items[lo:hi], lo, k,
                                       local=_oracle_local, merge=_np_merge)
        ulo, uhi = shard_range(U, world, rank)
        q.put((rank, ulo, uhi, s.numpy(), r.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("U,I,k", [(37, 101, 31), (64, 40, 31), (5, 7, 10)])
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
    for rank, ulo, uhi, s, r in got:
        assert np.array_equal(r, ro[ulo:uhi]), rank
        assert np.array_equal(s, so[ulo:uhi]), rank


def test_shard_range_covers():
    from nrk.dist import shard_range

    for n in (0, 1, 7, 364_047):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
