"""CPU: the C-ABI RCCL entry points end their group on every error path
(csrc/rccl_ops.hip, NRK_RCCL_G).  rccl_ops.hip is built here against a test
double of RCCL (tests/rccl_mock) that fails a chosen call between
ncclGroupStart and ncclGroupEnd; after the failure the group depth must be
back to 0 and the next call on the same communicator must run every one of
its sends and receives.  No GPU: the double moves no data."""
import ctypes
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(HERE), "news-recommendation-tc_amd")


@pytest.fixture(scope="module")
def mocklib(tmp_path_factory):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    out = str(tmp_path_factory.mktemp("rcclmock") / "librccl_ops_mock.so")
    # host code only: rccl_ops.hip has no kernels; the mock header shadows <rccl/rccl.h>
    subprocess.run([hipcc, "-O1", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                    "-I", os.path.join(HERE, "rccl_mock"), os.path.join(PKG, "csrc", "rccl_ops.hip"),
                    os.path.join(PKG, "csrc", "nrk_error.cpp"), os.path.join(HERE, "rccl_mock", "mock_rccl.cpp"),
                    "-o", out], check=True, capture_output=True)
    L = ctypes.CDLL(out)
    L.nrk_last_error.restype = ctypes.c_char_p
    return L


P = ctypes.c_void_p
BUF = (ctypes.c_int32 * 64)()
ptr = ctypes.cast(BUF, P)


def band(L, comm, per=4, x_cap=2):
    L.nrk_rccl_band_alltoall.argtypes = [P, P, P, ctypes.c_int64, ctypes.c_int, P, P, P]
    return L.nrk_rccl_band_alltoall(comm, ptr, ptr, per, x_cap, ptr, ptr, None)


def gather(L, comm):
    L.nrk_rccl_topk_allgather.argtypes = [P, P, P, ctypes.c_int64, ctypes.c_int, ctypes.c_int, P, P, P, P, P, P]
    return L.nrk_rccl_topk_allgather(comm, ptr, ptr, 0, 31, 31, ptr, ptr, ptr, ptr, None, None)


@pytest.mark.parametrize("fail_at", [0, 2, 5, 7])
def test_band_alltoall_ends_its_group_on_error(mocklib, fail_at):
    L = mocklib
    comm = P(1)
    L.mock_reset(2, fail_at)  # 2 peers x 4 calls: fail call fail_at
    assert band(L, comm) == 2  # NRK_EHIP
    assert b"invalid argument" in L.nrk_last_error()
    assert L.mock_group_depth() == 0
    L.mock_reset(2, -1)
    assert band(L, comm) == 0
    assert L.mock_group_depth() == 0 and L.mock_ops() == 8


@pytest.mark.parametrize("fail_at", [0, 1])
def test_topk_allgather_ends_its_group_on_error(mocklib, fail_at):
    L = mocklib
    comm = P(1)
    L.mock_reset(1, fail_at)
    L.nrk_rccl_topk_allgather.argtypes = [P, P, P, ctypes.c_int64, ctypes.c_int, ctypes.c_int, P, P, P, P, P, P]
    rc = L.nrk_rccl_topk_allgather(comm, ptr, ptr, 1, 31, 31, ptr, ptr, ptr, ptr, None, None)
    assert rc == 2 and L.mock_group_depth() == 0
