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


def _itemcf_golden(g):
    from nrk.data import synth

    log = synth.ClickLog(g["click_user"], g["click_item"], g["click_ts"])
    users, offs, items_raw, ts = synth.user_lists(log)
    ids = g["created_ids"]
    dense = np.searchsorted(ids, items_raw).astype(np.int32)
    return offs, dense, ts, ids


def _as_dict(ids, i, j, v):
    return {(int(ids[a]), int(ids[b])): float(c) for a, b, c in zip(i, j, v)}


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_itemcf_omp_variant_matches_sequential(golden, threads):
    """bench.py's OpenMP ItemCF baseline (oracle_itemcf_sim_omp): the same
    (i, j) entries with bit-identical values as the sequential restatement,
    and the reference's similarities (item_cf.py:33-84) to 1e-12."""
    from oracle import oracle

    g = golden("itemcf_small")
    offs, dense, ts, ids = _itemcf_golden(g)
    i, j, v, _, _ = oracle.itemcf_sim(offs, dense, ts, g["created_vals"], len(ids))
    a, b, c = oracle.itemcf_sim_omp(offs, dense, ts, g["created_vals"], len(ids), threads)
    assert _as_dict(ids, a, b, c) == _as_dict(ids, i, j, v)
    ref = {(int(x), int(y)): float(z) for x, y, z in zip(g["sim_i"], g["sim_j"], g["sim_v"])}
    got = _as_dict(ids, a, b, c)
    assert got.keys() == ref.keys()
    np.testing.assert_allclose([got[k] for k in ref], list(ref.values()), rtol=1e-12, atol=0)


def test_itemcf_pyloop_variant_matches_reference(golden):
    """bench.py's Python-loop ItemCF baseline (the reference's dict loops,
    oracle.itemcf_sim_pyloop) against the reference's own similarity dict,
    in the reference's row and entry order."""
    from oracle import oracle

    g = golden("itemcf_small")
    offs, dense, ts, ids = _itemcf_golden(g)
    cr = g["created_vals"]
    uit = {u: [(int(dense[t]), int(ts[t])) for t in range(offs[u], offs[u + 1])] for u in range(len(offs) - 1)}
    sim = oracle.itemcf_sim_pyloop(uit, cr)
    flat = [(int(ids[i]), int(ids[j]), w) for i, row in sim.items() for j, w in row.items()]
    assert [x[0] for x in flat] == g["sim_i"].tolist()
    assert [x[1] for x in flat] == g["sim_j"].tolist()
    np.testing.assert_allclose([x[2] for x in flat], g["sim_v"], rtol=1e-12, atol=0)
