"""GPU parity: EmbeddingSimilarity (similarity/embedding.py:15-67).

Checkers: numpy itself for the row normalisation (the reference's own line,
embedding.py:41 -- bit-exact expected), the CPU oracle for the self-search,
and the golden dict made by executing the reference (tests/golden/
make_golden.py, gen_embsim) with the IndexFlatIP contract stand-in.
"""
import numpy as np
import pandas as pd
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("d", [1, 5, 8, 16, 31, 32, 100, 128, 129, 200, 250, 256])
def test_row_normalize_bit_exact_vs_numpy(d):
    from nrk import ops

    rng = np.random.default_rng(d)
    n = 777
    x = (rng.standard_normal((n, d)) * rng.uniform(1e-3, 1e3, (n, 1))).astype(np.float32)
    out, nr = ops.row_normalize(torch.from_numpy(x).cuda(), norms=True)
    torch.cuda.synchronize()
    ref_n = np.linalg.norm(x, axis=1)
    ref = x / np.linalg.norm(x, axis=1, keepdims=True)
    assert np.array_equal(nr.cpu().numpy(), ref_n)
    assert np.array_equal(out.cpu().numpy(), ref)


def test_row_normalize_empty():
    from nrk import ops

    out = ops.row_normalize(torch.empty((0, 250), device="cuda"))
    assert out.shape == (0, 250)


def _df(ids, emb, index=None):
    df = pd.DataFrame(emb, columns=[f"emb_{n}" for n in range(emb.shape[1])])
    df.insert(0, "article_id", ids)
    if index is not None:
        df.index = index
    return df


def test_embedding_similarity_matches_reference_golden(golden):
    from nrk.config import RecallConfig
    from nrk.similarity.embedding import EmbeddingSimilarity

    g = golden("embsim_small")
    es = EmbeddingSimilarity(RecallConfig(embedding_topk=int(g["topk"])))
    got = es.calculate(_df(g["ids"], g["emb"], index=np.arange(len(g["ids"]))[::-1] + 3))
    ref = {}
    for i, j, v in zip(g["sim_i"].tolist(), g["sim_j"].tolist(), g["sim_v"].tolist()):
        ref.setdefault(i, {})[j] = v
    assert list(got) == list(ref)
    for i in ref:
        assert list(got[i].items()) == list(ref[i].items())  # keys, order and exact values
    top = es.get_similar_items(int(g["ids"][0]), topk=5)
    assert top == sorted(ref[int(g["ids"][0])].items(), key=lambda x: x[1], reverse=True)[:5]
    assert es.get_similar_items(-12345) == []


@pytest.mark.parametrize("n,d,k", [(3000, 250, 20), (4097, 64, 31), (500, 32, 10), (3000, 250, 50), (2000, 250, 150)])
def test_embedding_similarity_vs_oracle(n, d, k):
    from nrk.similarity.embedding import EmbeddingSimilarity

    rng = np.random.default_rng(n + d)
    emb = rng.standard_normal((n, d)).astype(np.float32)
    emb[n // 2: n // 2 + 30] = emb[:30] * np.float32(4.0)  # exact ties after normalisation
    s, r = EmbeddingSimilarity().compute(torch.from_numpy(emb).cuda(), topk=k)
    torch.cuda.synchronize()
    _, so, ro = oracle.embedding_similarity(emb, k, nthreads=8)
    assert np.array_equal(r.cpu().numpy().astype(np.int64), ro)
    assert np.array_equal(s.cpu().numpy(), so)


def test_embedding_similarity_errors():
    from nrk.config import RecallConfig
    from nrk.similarity.embedding import EmbeddingSimilarity

    emb = np.ones((5, 8), np.float32)
    with pytest.raises(KeyError):  # topk + 1 > n -> -1 label, as the reference's dict lookup
        EmbeddingSimilarity(RecallConfig(embedding_topk=10)).calculate(_df(np.arange(5), emb))
    emb[2] = 0.0
    with pytest.raises(ValueError):
        EmbeddingSimilarity(RecallConfig(embedding_topk=2)).calculate(_df(np.arange(5), emb))
    with pytest.raises(ValueError):
        EmbeddingSimilarity().get_similar_items(1)
