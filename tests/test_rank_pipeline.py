"""The Ranker plugin as RankPipeline drives it (src/pipeline/rank_pipeline.py:
80-191): ``DINRanker(config)`` -> ``load()`` -> ``load_model(load_dir)`` ->
``predict()`` -> ``rank_and_recommend``, on an artifact directory laid out the
way the reference's feature step and ``save_model`` write it
(src/utils/config.py:141-161, src/rank/DIN.py:1285-1326).

Checker: tests/golden/rank_pipeline_small.npz, made by EXECUTING the
reference's own DINRanker.load / load_model / predict on the same artifacts
(tests/golden/make_golden.py gen_rank_pipeline) at embedding dims 32, 16 and
64 and batch sizes 128 (a multiple of 64: one segmented call) and 100 (one
call per batch).  Bars: probabilities 1e-5 (north_star); recommendations:
same users, the reference's (item, score) lists with scores at 1e-5 and the
item order equal wherever the reference's scores are more than 2e-5 apart.
"""
import os
import pickle

import numpy as np
import pytest
import torch

DIMS = (32, 16, 64)
TOL = 1e-5


def _feats(g):
    return [list(map(str, g[k])) for k in ("user_feats", "item_feats", "ctx_feats")]


def write_artifacts(g, dim, root):
    """The artifact directory of one fixture set: main_features.csv, the four
    feature pickles, din_model_metadata.pkl, label_encoders.pkl, din_model.pth."""
    import pandas as pd
    from sklearn.preprocessing import LabelEncoder

    uf, itf, cf = _feats(g)
    p = f"d{dim}_"
    save = os.path.join(root, "temp")
    os.makedirs(save, exist_ok=True)
    main = pd.DataFrame(g[p + "main"], columns=["user_id", "item_id"] + cf + ["label"])
    main.to_csv(os.path.join(save, "main_features.csv"), index=False)
    upd = {str(u): dict(zip(uf, map(float, row))) for u, row in zip(g[p + "prof_users"], g[p + "prof_vals"])}
    ifd = {str(i): dict(zip(itf, map(int, row))) for i, row in zip(g[p + "ifeat_items"], g[p + "ifeat_vals"])}
    off, items = g[p + "hist_offsets"], [str(x) for x in g[p + "hist_items"]]
    uhd = {str(u): items[off[n]:off[n + 1]] for n, u in enumerate(g[p + "hist_users"])}
    lists = {"user_profile_features": uf, "item_features": itf, "context_features": cf}
    meta = {"user_profile_features": uf, "item_features": itf, "context_features": cf, "din_embedding_dim": dim,
            "din_attention_hidden_units": [36], "din_mlp_hidden_units": [200, 80], "din_activation": "dice",
            "din_seq_max_len": 30}
    encs = {}
    for f in uf + itf + cf:
        le = LabelEncoder()
        le.classes_ = g[f"{p}classes::{f}"]
        encs[f] = le
    for name, obj in (("user_profile_dict", upd), ("item_features_dict", ifd), ("user_history_dict", uhd),
                      ("feature_lists", lists), ("din_model_metadata", meta), ("label_encoders", encs)):
        with open(os.path.join(save, name + ".pkl"), "wb") as fh:
            pickle.dump(obj, fh)
    sd = {k[len(p) + 4:]: torch.from_numpy(np.array(g[k])) for k in g.files if k.startswith(p + "sd::")}
    torch.save(sd, os.path.join(save, "din_model.pth"))
    return save


class RankPipeline:
    """rank_pipeline.py:12-191 restated over the nrk plugin (the steps the
    serving path runs; extract_features / train stay with the reference)."""

    def __init__(self, config):
        self.config = config
        self.ranker = None

    def load_model(self, model_dir=None):  # :80-105
        from nrk.rank.din import DINRanker

        self.ranker = DINRanker(self.config)
        self.ranker.load()
        self.ranker.load_model(load_dir=model_dir)

    def predict(self, use_pretrained=False, model_dir=None):  # :107-141
        if use_pretrained:
            self.load_model(model_dir=model_dir)
        if self.ranker is None:
            raise ValueError("Model is not trained/loaded. Train or load the model before prediction.")
        return self.ranker.predict()

    def rank_and_recommend(self, top_k=10, save_path=None):  # :143-191
        import pandas as pd
        from nrk.rank.recommend import rank_and_recommend

        probs = self.predict() if self.ranker is None else self.ranker.predict()
        main_df = pd.read_csv(self.config.main_features_path)
        return rank_and_recommend(main_df, probs, top_k=top_k, save_path=save_path)


# ----------------------------------------------------------------- CPU --
@pytest.mark.parametrize("dim", DIMS)
def test_load_and_vocab_match_reference(golden, dim, tmp_path):
    """load() reads the artifacts; _prepare_vocab_dicts re-fits the same
    encoders the reference fitted (classes identical), and the fixture's
    state_dict is exactly the shape set the strict load expects."""
    from nrk.config import RankConfig
    from nrk.rank.din import DINRanker, _expected_state

    g = golden("rank_pipeline_small")
    write_artifacts(g, dim, str(tmp_path))
    r = DINRanker(RankConfig(_project_root=str(tmp_path)))
    r.load()
    assert len(r.main_df) == len(g[f"d{dim}_main"])
    uv, iv, cv = r._prepare_vocab_dicts()
    for f, le in r.label_encoders.items():
        np.testing.assert_array_equal(np.asarray(le.classes_).astype(str), g[f"d{dim}_classes::{f}"].astype(str))
    exp = _expected_state(uv, iv, cv, dim, [200, 80])
    p = f"d{dim}_sd::"
    got = {k[len(p):]: tuple(g[k].shape) for k in g.files if k.startswith(p)}
    assert got == exp


def test_config_paths_without_side_effects(tmp_path):
    from nrk.config import RankConfig

    c = RankConfig(_project_root=str(tmp_path / "proj"))
    assert c.main_features_path == str(tmp_path / "proj" / "temp" / "main_features.csv")
    assert c.feature_lists_path.endswith(os.path.join("temp", "feature_lists.pkl"))
    assert not (tmp_path / "proj").exists()  # the reference makes directories; this config does not
    c2 = RankConfig.from_dict({"batch_size": 64, "din_embedding_dim": 16, "unknown": 1})
    assert c2.batch_size == 64 and c2.din_embedding_dim == 16


def test_load_model_errors(tmp_path):
    from nrk.config import RankConfig
    from nrk.rank.din import DINRanker

    r = DINRanker(RankConfig(_project_root=str(tmp_path)))
    with pytest.raises(FileNotFoundError, match="metadata"):
        r.load_model(str(tmp_path))
    with pytest.raises(ValueError, match="not trained"):
        r.predict()


# ----------------------------------------------------------------- GPU --
@pytest.mark.gpu
@pytest.mark.parametrize("dim", DIMS)
@pytest.mark.parametrize("bs", [128, 100])
def test_rank_pipeline_matches_reference(golden, dim, bs, tmp_path):
    from nrk.config import RankConfig

    g = golden("rank_pipeline_small")
    write_artifacts(g, dim, str(tmp_path))
    cfg = RankConfig(_project_root=str(tmp_path), din_embedding_dim=dim, batch_size=bs)
    pipe = RankPipeline(cfg)
    probs = pipe.predict(use_pretrained=True)
    torch.cuda.synchronize()
    np.testing.assert_allclose(probs, g[f"d{dim}_probs_bs{bs}"], atol=TOL, rtol=0)
    if bs != 128:
        return
    out = str(tmp_path / "final_recommendations.pkl")
    rec = pipe.rank_and_recommend(top_k=5, save_path=out)
    with open(out, "rb") as fh:
        assert pickle.load(fh) == rec
    ru, ri, rs = g[f"d{dim}_rec_user"], g[f"d{dim}_rec_item"], g[f"d{dim}_rec_score"]
    ref = {}
    for u, i, s in zip(ru, ri, rs):
        ref.setdefault(str(u), []).append((str(i), float(s)))
    assert list(rec) == list(ref)
    for u, lst in ref.items():
        got = rec[u]
        assert len(got) == len(lst)
        np.testing.assert_allclose([s for _, s in got], [s for _, s in lst], atol=TOL, rtol=0)
        for n, ((gi, _), (ei, es)) in enumerate(zip(got, lst)):
            if gi != ei:  # only a near-tie of the reference's own scores may swap
                near = [abs(es - s2) <= 2e-5 for _, s2 in lst]
                assert near.count(True) >= 2, (u, n, gi, ei)


@pytest.mark.gpu
def test_load_model_state_dict_mismatch(golden, tmp_path):
    """A din_model.pth whose shapes disagree with the data's vocabularies is
    refused like load_state_dict(strict=True) refuses it."""
    from nrk.config import RankConfig
    from nrk.rank.din import DINRanker

    g = golden("rank_pipeline_small")
    save = write_artifacts(g, 32, str(tmp_path))
    sd = torch.load(os.path.join(save, "din_model.pth"), weights_only=True)
    k = next(k for k in sd if k.startswith("item_embedding_dict."))
    sd[k] = sd[k][:-1]
    torch.save(sd, os.path.join(save, "din_model.pth"))
    r = DINRanker(RankConfig(_project_root=str(tmp_path)))
    r.load()
    with pytest.raises(RuntimeError, match="size mismatch"):
        r.load_model()
