"""CPU: the fusion oracle (oracle.fuse) reproduces the reference's
RecallFusion.fuse (src/recall/fusion.py:267-342) on the fixture the
reference itself produced (tests/golden/fusion_small.npz), for every
strategy x normalisation and the seen-item filter: same users, same lists in
the same order, bit-identical scores (the z-score sigmoid included: both sides
use numpy's exp on this host)."""
import numpy as np
import pytest

from oracle import oracle

STRATS = ("weighted_sum", "weighted_avg", "max_score", "harmonic_mean", "diversity_weighted", "rrf")


def fusion_inputs(g):
    methods = {}
    for m in g["methods"].tolist():
        u, o, i, s = (g[f"in::{m}::{k}"] for k in ("users", "offsets", "items", "scores"))
        methods[m] = {int(uu): list(zip(i[o[n]:o[n + 1]].tolist(), s[o[n]:o[n + 1]].tolist()))
                      for n, uu in enumerate(u)}
    weights = dict(zip(g["methods"].tolist(), g["weights"].tolist()))
    ho = g["hist_offsets"]
    hist = {int(u): set(g["hist_items"][ho[n]:ho[n + 1]].tolist()) for n, u in enumerate(g["hist_users"])}
    return methods, weights, hist


def expected(g, strat, norm, seen):
    tag = f"out::{strat}::{norm}::{int(seen)}"
    u, o, i, s = (g[f"{tag}::{k}"] for k in ("users", "offsets", "items", "scores"))
    return {int(uu): list(zip(i[o[n]:o[n + 1]].tolist(), s[o[n]:o[n + 1]].tolist())) for n, uu in enumerate(u)}


CASES = [(s, n, False) for s in STRATS for n in ("local", "global", "z-score")] + [("weighted_avg", "global", True)]


@pytest.mark.parametrize("strat,norm,seen", CASES)
def test_fusion_oracle_matches_reference(golden, strat, norm, seen):
    g = golden("fusion_small")
    methods, weights, hist = fusion_inputs(g)
    got = oracle.fuse(methods, weights, strat, norm, 30, hist if seen else None, seen)
    exp = expected(g, strat, norm, seen)
    assert list(got) == list(exp)  # the reference's set iteration order
    for u in exp:
        assert got[u] == exp[u], u
