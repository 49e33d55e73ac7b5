"""CPU: the CPU-baseline implementations bench.py times are the reference's
computation: the torch-CPU DIN forward (oracle.DinTorchCPU) reproduces the
reference's own probabilities on tests/golden/din_small.npz."""
import numpy as np
import pytest
import torch


@pytest.mark.parametrize("tag", ["b512", "b37"])
def test_din_torch_cpu_matches_reference(golden, tag):
    from oracle import oracle

    g = golden("din_small")
    sd = {k[4:]: g[k] for k in g.files if k.startswith("sd::")}
    feats = (g["user_feats"].tolist(), g["item_feats"].tolist(), g["ctx_feats"].tolist())
    m = oracle.DinTorchCPU(sd, feats)
    t = lambda k: torch.from_numpy(g[f"{tag}_{k}"].astype(np.int64))  # noqa: E731
    p = m(t("user"), t("item"), t("hist"), t("ctx"), torch.from_numpy(g[f"{tag}_mask"].astype(np.float32)))
    np.testing.assert_allclose(p.numpy(), g[f"{tag}_probs"], atol=1e-5, rtol=0)
