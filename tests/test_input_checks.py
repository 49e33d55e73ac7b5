"""CPU: the host-side input checks that guard the -fno-honor-nans screen
(Makefile) and the DIN tables: NaN / inf inputs are rejected before any
kernel runs."""
import numpy as np
import pytest
import torch


def test_din_params_reject_nonfinite_tables():
    import bench
    from nrk import ops

    sd, feats, _, _ = bench.din_workload(101, 8, 50, "cpu")
    sd = dict(sd)
    w = sd["item_embedding_dict.i0.weight"].clone()
    w[3, 5] = float("nan")
    sd["item_embedding_dict.i0.weight"] = w
    with pytest.raises(ValueError, match="finite"):
        ops.DinParams(sd, *feats, device="cpu")


def test_finite_helper():
    from nrk import ops

    ops._finite(torch.zeros(4), "x")
    ops._finite(torch.zeros(0), "x")
    for bad in (float("nan"), float("inf"), -float("inf")):
        t = torch.zeros(4)
        t[2] = bad
        with pytest.raises(ValueError, match="x must be finite"):
            ops._finite(t, "x")
