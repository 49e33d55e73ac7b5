"""GPU: the C-ABI RCCL exchanges (nrk_rccl_*) on a one-rank
communicator -- the box has one GPU, so this checks the binding, the
communicator life cycle and the data movement / merge of each exchange;
the N-rank protocols are covered by the gloo tests (tests/test_dist_gloo.py)
and the one-GPU replays of tests/test_gpu_recall.py."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _comm():
    from nrk import _lib

    L = _lib.lib()
    nb = L.nrk_rccl_unique_id_bytes()
    assert nb == 128
    uid = ctypes.create_string_buffer(nb)
    _lib.check(L.nrk_rccl_get_unique_id(uid), "nrk_rccl_get_unique_id")
    comm = ctypes.c_void_p()
    _lib.check(L.nrk_rccl_comm_init(ctypes.byref(comm), 1, uid, 0), "nrk_rccl_comm_init")
    assert comm.value
    return L, comm


def test_rccl_topk_allgather_merges():
    from nrk import _lib, ops

    L, comm = _comm()
    try:
        rng = np.random.default_rng(3)
        U, k_in, k_out = 300, 31, 20
        ex = np.sort(rng.standard_normal((U, k_in)), axis=1)[:, ::-1].copy()
        ex[:, 5] = ex[:, 4]  # a tie: the lower row must win
        rows = rng.permutation(10_000)[: U * k_in].reshape(U, k_in).astype(np.int32)
        t_ex, t_rows = torch.from_numpy(ex).cuda(), torch.from_numpy(rows).cuda()
        g_ex = torch.empty_like(t_ex)
        g_rows = torch.empty_like(t_rows)
        s = torch.empty((U, k_out), dtype=torch.float32, device="cuda")
        r = torch.empty((U, k_out), dtype=torch.int32, device="cuda")
        e = torch.empty((U, k_out), dtype=torch.float64, device="cuda")
        p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        _lib.check(L.nrk_rccl_topk_allgather(comm, p(t_ex), p(t_rows), U, k_in, k_out, p(g_ex), p(g_rows), p(s),
                                             p(r), p(e), ops._stream()), "nrk_rccl_topk_allgather")
        torch.cuda.synchronize()
        assert torch.equal(g_ex, t_ex) and torch.equal(g_rows, t_rows)
        ms, mr = ops.topk_merge(t_ex[None].contiguous(), t_rows[None].contiguous(), k_out)[:2]
        assert torch.equal(r, mr) and torch.equal(s, ms)
    finally:
        L.nrk_rccl_comm_destroy(comm)


def test_rccl_owner_exchanges_move_blocks():
    from nrk import _lib, ops

    L, comm = _comm()
    try:
        U, m, x = 257, 5, 32
        b = torch.randn(U, m, device="cuda")
        out = torch.empty(1, U, m, device="cuda")
        p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        _lib.check(L.nrk_rccl_bound_allgather(comm, p(b), U, m, p(out), ops._stream()), "bound_allgather")
        cnt = torch.randint(-1, x, (U,), dtype=torch.int32, device="cuda")
        ids = torch.randint(0, 1 << 20, (U, x), dtype=torch.int32, device="cuda")
        oc = torch.empty_like(cnt)
        oi = torch.empty_like(ids)
        _lib.check(L.nrk_rccl_band_alltoall(comm, p(cnt), p(ids), U, x, p(oc), p(oi), ops._stream()),
                   "band_alltoall")
        torch.cuda.synchronize()
        assert torch.equal(out[0], b) and torch.equal(oc, cnt) and torch.equal(oi, ids)
    finally:
        L.nrk_rccl_comm_destroy(comm)


def test_rccl_argument_errors():
    from nrk import _lib

    L = _lib.lib()
    assert L.nrk_rccl_topk_allgather(None, None, None, 10, 31, 31, None, None, None, None, None, None) == \
        _lib.NRK_EINVAL
    assert b"null communicator" in L.nrk_last_error()
    comm = ctypes.c_void_p()
    assert L.nrk_rccl_comm_init(ctypes.byref(comm), 2, ctypes.create_string_buffer(128), 5) == _lib.NRK_EINVAL
