"""GPU: the plugin entry points a reference maintainer calls.

* ``YoutubeDNNRecaller.load_model`` (youtubednn_recaller.py:425-495 driven
  from trained weights + click_df) -> the reference's extracted embeddings
  and its recall() lists (tests/golden/youtubednn_small.npz);
* ``DINRanker.set_data / load_model / predict`` (DIN.py:1219-1283) on the
  reference-encoded fixture (tests/golden/din_encode_small.npz): the device
  encoder (nrk_gather_rows) builds the same index tensors as the reference's
  DINDataset + collate_fn, and the probabilities match the oracle run on the
  reference's own tensors, batch by batch (1e-5)."""
import numpy as np
import pandas as pd
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu


def test_youtubednn_load_model_matches_golden(golden):
    from nrk.config import RecallConfig
    from nrk.recall.youtubednn_recaller import YoutubeDNNRecaller

    g = golden("youtubednn_small")
    cfg = RecallConfig()
    cfg.youtubednn_seq_max_len = int(g["seq_max_len"])
    sd = {"user_embedding.weight": g["user_emb"], "item_embedding.weight": g["item_emb"],
          "user_tower.0.weight": g["w0"], "user_tower.0.bias": g["b0"],
          "user_tower.3.weight": g["w1"], "user_tower.3.bias": g["b1"]}
    click_df = pd.DataFrame({"user_id": g["click_user"], "click_article_id": g["click_item"],
                             "click_timestamp": g["click_ts"]})
    rec = YoutubeDNNRecaller(cfg).load_model(sd, click_df)
    np.testing.assert_allclose(rec.user_embeddings.cpu().numpy(), g["user_embeddings"], atol=1e-6, rtol=0)
    np.testing.assert_allclose(rec.item_embeddings.cpu().numpy(), g["item_embeddings"], atol=1e-6, rtol=0)
    assert [rec.user_index_2_rawid[i] for i in range(len(g["user_index_2_rawid"]))] == \
        g["user_index_2_rawid"].tolist()
    assert [rec.item_index_2_rawid[i] for i in range(len(g["item_index_2_rawid"]))] == \
        g["item_index_2_rawid"].tolist()
    k = int(g["topk"])
    res = rec.batch_recall([int(u) for u in g["recall_users"]], topk=k)
    ro = g["recall_offsets"]
    for n, u in enumerate(g["recall_users"]):
        got = res[int(u)]
        assert [a for a, _ in got] == g["recall_items"][ro[n]:ro[n + 1]].tolist()
        np.testing.assert_allclose([b for _, b in got], g["recall_scores"][ro[n]:ro[n + 1]], atol=1e-6)


class _Enc:
    def __init__(self, classes):
        self.classes_ = classes


def _din_fixture(golden, case):
    g = golden("din_encode_small")
    uf = [k.split("::")[1] for k in g.files if k.startswith("classes::")]
    nu, ni = g["prof_vals"].shape[1], g["ifeat_vals"].shape[1]
    user_f, item_f, ctx_f = uf[:nu], uf[nu:nu + ni], uf[nu + ni:]
    enc = {f: _Enc(g[f"classes::{f}"]) for f in uf}
    upd = {str(u): {f: float(v) for f, v in zip(user_f, row)} for u, row in zip(g["prof_users"], g["prof_vals"])}
    ifd = {str(i): {f: int(v) for f, v in zip(item_f, row)} for i, row in zip(g["ifeat_items"], g["ifeat_vals"])}
    off = g["hist_offsets"]
    uhd = {str(u): [str(x) for x in g["hist_items"][off[n]:off[n + 1]]] for n, u in enumerate(g["hist_users"])}
    df = pd.DataFrame({"user_id": g["main_user"], "item_id": g["main_item"], "label": g["main_label"]})
    for n, f in enumerate(ctx_f):
        df[f] = g["main_ctx"][:, n]
        if case == "obj":
            df[f] = df[f].astype(str)
    # a DINModel-shaped state_dict sized to these encoders (vocab = classes + 1)
    rng = np.random.default_rng(5)
    sd = {}
    for grp, names in (("user_profile_embedding_dict", user_f), ("item_embedding_dict", item_f),
                       ("context_embedding_dict", ctx_f)):
        for f in names:
            sd[f"{grp}.{f}.weight"] = (rng.standard_normal((len(g[f"classes::{f}"]) + 1, 32)) * 0.1).astype(np.float32)
    lin = lambda o, i: (rng.standard_normal((o, i)) / np.sqrt(i)).astype(np.float32)  # noqa: E731
    sd["activation_unit.mlp.0.weight"], sd["activation_unit.mlp.0.bias"] = lin(36, 128 * len(item_f)), \
        (rng.standard_normal(36) * 0.01).astype(np.float32)
    sd["activation_unit.mlp.2.weight"], sd["activation_unit.mlp.2.bias"] = lin(1, 36), np.zeros(1, np.float32)
    in_dim = 32 * (len(user_f) + len(ctx_f) + 2 * len(item_f))
    sd["mlp.0.weight"], sd["mlp.0.bias"] = lin(200, in_dim), np.zeros(200, np.float32)
    sd["mlp.2.weight"], sd["mlp.2.bias"] = lin(80, 200), np.zeros(80, np.float32)
    sd["mlp.4.weight"], sd["mlp.4.bias"] = lin(1, 80), np.zeros(1, np.float32)
    return g, (user_f, item_f, ctx_f), enc, upd, ifd, uhd, df, sd


@pytest.mark.parametrize("case", ["out", "obj"])
@pytest.mark.parametrize("batch_size", [128, 400, 333])
def test_din_ranker_predict(golden, case, batch_size):
    from nrk.config import RankConfig
    from nrk.rank.din import DINRanker

    g, (user_f, item_f, ctx_f), enc, upd, ifd, uhd, df, sd = _din_fixture(golden, case)
    cfg = RankConfig()
    cfg.din_seq_max_len = int(g["T"])
    cfg.batch_size = batch_size
    rk = DINRanker(cfg).set_data(df, upd, ifd, uhd, user_f, item_f, ctx_f, enc).load_model(sd)
    # the device encoder == the reference's collated tensors
    from nrk.rank.encode import iloc_columns

    cols = iloc_columns(df, ["user_id", "item_id"] + ctx_f)
    dev = rk.encoder.encode_device(rk.encoder.device_tables("cuda"), cols["user_id"], cols["item_id"], cols)
    for k in ("user", "item", "hist", "ctx", "mask"):
        assert np.array_equal(dev[k].cpu().numpy(), g[f"{case}_{k}"]), k
    probs = rk.predict()
    assert probs.shape == (len(df),)
    n = len(df)
    for s in range(0, n, batch_size):
        e = min(n, s + batch_size)
        sl = {k: g[f"{case}_{k}"][s:e] for k in ("user", "item", "hist", "ctx", "mask")}
        po, _, _ = oracle.din_forward(sd, sl["user"], sl["item"], sl["hist"], sl["ctx"], sl["mask"],
                                      (user_f, item_f, ctx_f))
        np.testing.assert_allclose(probs[s:e], po, atol=1e-5, rtol=0)


def test_din_ranker_requires_model(golden):
    from nrk.rank.din import DINRanker

    with pytest.raises(ValueError):
        DINRanker().predict()


def test_gather_rows_edges():
    from nrk import ops

    src = torch.arange(12, dtype=torch.int32, device="cuda").reshape(4, 3)
    idx = torch.tensor([3, -1, 0, 4, 1], dtype=torch.int32, device="cuda")
    out = ops.gather_rows(src, idx).cpu().numpy()
    assert out.tolist() == [[9, 10, 11], [0, 0, 0], [0, 1, 2], [0, 0, 0], [3, 4, 5]]
    assert ops.gather_rows(src, idx[:0]).shape == (0, 3)
