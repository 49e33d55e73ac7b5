"""GPU DIN ranker: drop-in for src/rank/DIN.py's scoring path.

* ``encode_samples`` / ``DinEncoder`` (nrk/rank/encode.py) restate
  DINDataset.__getitem__ + collate_fn (DIN.py:289-520) without a per-row
  loop: the same int index tensors (0 = pad / unknown, class index + 1
  otherwise; LAST T history items, left aligned, prefix mask), the lookups
  gathered on the device for ``DINRanker.predict``.
* ``DINScorer`` holds a trained DINModel's state_dict in kernel layout and
  scores batches with the HIP kernels (nrk_din_forward).
* ``DINRanker`` (a ``BaseRanker``, rank/base.py:10-117) is the plugin
  RankPipeline drives (rank_pipeline.py:96-141): ``load()`` (DIN.py:529-558),
  ``load_model(load_dir)`` (:1328-1399), ``predict()`` (:1219-1283): every
  main_df row in order, batches of ``batch_size``, probabilities positional
  to main_df.  Like the reference, Dice uses the statistics of each batch, so
  a batch is the unit of work; a trailing batch of one row is NaN there (std
  of one sample) and is NaN here too.
"""
from __future__ import annotations

import os
from collections.abc import Mapping
from typing import Optional

import numpy as np
import torch

from .. import ops
from ..config import RankConfig
from .base import BaseRanker, load_pickle


from .encode import DinEncoder, iloc_columns  # noqa: F401  (re-exported)


def encode_samples(user_ids, item_ids, ctx_cols, user_profile_dict, item_features_dict,
                   user_history_dict, user_features, item_features, ctx_features,
                   label_encoders, seq_max_len):
    """DINDataset + collate_fn for a list of samples (host arrays).
    ``user_ids``/``item_ids`` and ``ctx_cols`` (feature -> raw values) as the
    reference reads them from main_df rows (see ``iloc_columns``)."""
    enc = DinEncoder(user_profile_dict, item_features_dict, user_history_dict, user_features,
                     item_features, ctx_features, label_encoders, seq_max_len)
    return enc.encode_host(user_ids, item_ids, ctx_cols)


class DINScorer:
    """Trained DINModel weights (state_dict) on the device, scored by the HIP
    kernels.  ``table_dtype='bf16'`` stores the embedding tables in bf16
    (fp32 arithmetic)."""

    def __init__(self, state_dict, user_features, item_features, ctx_features,
                 table_dtype: str = "fp32", device="cuda"):
        self.device = torch.device(device)
        self.params = ops.DinParams(state_dict, user_features, item_features, ctx_features,
                                    table_dtype=table_dtype, device=self.device)

    def forward(self, user, item, hist, ctx, mask, logits=False):
        """One batch (B >= 2) of int index arrays -> probs (B,) [, logits]."""
        d = self.device
        t = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a)).to(d, dt).contiguous()  # noqa: E731
        return ops.din_forward(self.params, t(user, torch.int32), t(item, torch.int32),
                               t(hist, torch.int32), t(ctx, torch.int32), t(mask, torch.float32),
                               logits=logits)

    def predict(self, enc, batch_size):
        """All rows in order, reference batching (DIN.py:1245-1283).  With a
        batch size that is a multiple of 64 every batch is scored in one
        nrk_din_forward_segments call (each batch keeps its own Dice
        statistics); otherwise one call per batch.  ``enc`` holds numpy
        arrays or device tensors (DinEncoder.encode_device)."""
        n = enc["mask"].shape[0]
        if n >= 2 and (batch_size % 64 == 0 or n <= batch_size):
            d = self.device
            t = lambda a, dt: torch.as_tensor(a).to(d, dt).contiguous()  # noqa: E731
            p = ops.din_forward(self.params, t(enc["user"], torch.int32), t(enc["item"], torch.int32),
                                t(enc["hist"], torch.int32), t(enc["ctx"], torch.int32),
                                t(enc["mask"], torch.float32), batch_size=batch_size)
            return p.cpu().numpy()
        out = np.empty(n, np.float32)
        for s in range(0, n, batch_size):
            e = min(n, s + batch_size)
            if e - s == 1:
                out[s] = np.nan  # std over one sample is NaN in the reference too
                continue
            host = {k: (v.cpu().numpy() if hasattr(v, "cpu") else v) for k, v in enc.items()}
            p = self.forward(host["user"][s:e], host["item"][s:e], host["hist"][s:e],
                             host["ctx"][s:e], host["mask"][s:e])
            out[s:e] = p.cpu().numpy()
        return out


def _expected_state(uv, iv, cv, dim, mlp_hidden):
    """key -> shape of DINModel(uv, iv, cv, dim, [36], mlp_hidden, "dice")'s
    state_dict (DIN.py:133-212; ActivationUnit is built with its defaults,
    :188; each Dice holds an unused ``alpha``)."""
    exp = {}
    for grp, vocab in (("user_profile_embedding_dict", uv), ("item_embedding_dict", iv),
                       ("context_embedding_dict", cv)):
        for f, v in vocab.items():
            exp[f"{grp}.{f}.weight"] = (v, dim)
    item_dim = len(iv) * dim
    exp.update({"activation_unit.mlp.0.weight": (36, 4 * item_dim), "activation_unit.mlp.0.bias": (36,),
                "activation_unit.mlp.1.alpha": (), "activation_unit.mlp.2.weight": (1, 36),
                "activation_unit.mlp.2.bias": (1,)})
    cur = (len(uv) + len(cv)) * dim + 2 * item_dim
    for n, unit in enumerate(mlp_hidden):
        exp[f"mlp.{2 * n}.weight"], exp[f"mlp.{2 * n}.bias"] = (unit, cur), (unit,)
        exp[f"mlp.{2 * n + 1}.alpha"] = ()
        cur = unit
    exp[f"mlp.{2 * len(mlp_hidden)}.weight"], exp[f"mlp.{2 * len(mlp_hidden)}.bias"] = (1, cur), (1,)
    return exp


class DINRanker(BaseRanker):
    """Ranker plugin: drop-in for src/rank/DIN.py's DINRanker on the serving
    path RankPipeline drives (rank_pipeline.py:96-141):
    ``DINRanker(config)`` -> ``load()`` -> ``load_model(load_dir)`` ->
    ``predict()`` (probabilities positional to ``main_df`` rows).

    * ``load`` (DIN.py:529-558) reads ``main_features.csv`` and the
      user-profile / item-feature / user-history / feature-list pickles from
      the ``RankConfig`` paths;
    * ``load_model(load_dir=None)`` (DIN.py:1328-1399) reads
      ``din_model_metadata.pkl`` and ``label_encoders.pkl``, re-fits the
      encoders and vocabularies from the loaded data exactly as the
      reference's ``_prepare_vocab_dicts`` does (:560-619, which overwrites
      the pickled encoders), then ``din_model.pth`` through
      ``torch.load(weights_only=True)`` -- checked like a strict
      ``load_state_dict`` -- into device weights for the HIP kernels;
    * ``predict`` (:1219-1283): every main_df row in order, Dice batches of
      ``config.batch_size``.
    Alternate entry points for in-memory data: ``set_data(...)`` and
    ``load_model(state_dict)``.  Training stays with the reference (out of
    scope); ``train()`` is BaseRanker's no-op."""

    def __init__(self, config: Optional[RankConfig] = None, device="cuda", table_dtype="fp32"):
        super().__init__(config or RankConfig())
        self.device = device
        self.table_dtype = table_dtype
        self.model = None  # DINScorer: the model's weights on the device
        self.label_encoders = {}
        self.encoder = None
        self._tables = None

    @property
    def scorer(self):
        return self.model

    # ------------------------------------------------------------ data --
    def load(self):
        """DIN.py:529-558."""
        import pandas as pd

        self.main_df = pd.read_csv(self.config.main_features_path)
        self.user_profile_dict = load_pickle(self.config.user_profile_dict_path)
        self.item_features_dict = load_pickle(self.config.item_features_dict_path)
        self.user_history_dict = load_pickle(self.config.user_history_dict_path)
        feature_lists = load_pickle(self.config.feature_lists_path)
        self.user_profile_features = feature_lists["user_profile_features"]
        self.item_features = feature_lists["item_features"]
        self.context_features = feature_lists["context_features"]
        self.encoder, self._tables = None, None

    def set_data(self, main_df, user_profile_dict, item_features_dict, user_history_dict,
                 user_profile_features, item_features, context_features, label_encoders):
        """The structures ``load()`` reads, handed over in memory (with the
        encoders the model was trained with)."""
        self.main_df = main_df
        self.user_profile_dict = user_profile_dict
        self.item_features_dict = item_features_dict
        self.user_history_dict = user_history_dict
        self.user_profile_features = list(user_profile_features)
        self.item_features = list(item_features)
        self.context_features = list(context_features)
        self.label_encoders = label_encoders
        self.encoder = DinEncoder(user_profile_dict, item_features_dict, user_history_dict,
                                  self.user_profile_features, self.item_features, self.context_features,
                                  label_encoders, self.config.din_seq_max_len)
        self._tables = None
        return self

    def _prepare_vocab_dicts(self):
        """DIN.py:560-619: one LabelEncoder per feature fitted on the loaded
        data (user / item features on their raw values, context features on
        ``main_df[feat].fillna(0).astype(str)``), stored in
        ``self.label_encoders``; vocabulary = classes + 1."""
        from sklearn.preprocessing import LabelEncoder

        uv, iv, cv = {}, {}, {}
        for feats, dicts, vocab in ((self.user_profile_features, list(self.user_profile_dict.values()), uv),
                                    (self.item_features, list(self.item_features_dict.values()), iv)):
            for feat in feats:
                values = {d[feat] for d in dicts if feat in d}
                if values:
                    le = LabelEncoder()
                    le.fit(list(values))
                    self.label_encoders[feat] = le
                    vocab[feat] = len(le.classes_) + 1
        ctx = self.main_df[self.context_features].copy()
        for feat in self.context_features:
            if feat in ctx.columns:
                le = LabelEncoder()
                ctx[feat] = ctx[feat].fillna(0)
                le.fit(ctx[feat].astype(str))
                self.label_encoders[feat] = le
                cv[feat] = len(le.classes_) + 1
        return uv, iv, cv

    # ----------------------------------------------------------- model --
    def load_model(self, load_dir=None):
        """DIN.py:1328-1399 (``load_dir``: a directory, default
        ``config.save_path``), or a DINModel state_dict (alternate entry)."""
        if isinstance(load_dir, Mapping):
            self.model = DINScorer(load_dir, self.user_profile_features, self.item_features, self.context_features,
                                   table_dtype=self.table_dtype, device=self.device)
            return self
        load_dir = load_dir or self.config.save_path
        metadata_path = os.path.join(load_dir, "din_model_metadata.pkl")
        if not os.path.exists(metadata_path):
            raise FileNotFoundError(f"Model metadata not found at: {metadata_path}")
        metadata = load_pickle(metadata_path)
        self.user_profile_features = metadata["user_profile_features"]
        self.item_features = metadata["item_features"]
        self.context_features = metadata["context_features"]
        encoders_path = os.path.join(load_dir, "label_encoders.pkl")
        self.label_encoders = load_pickle(encoders_path) if os.path.exists(encoders_path) else {}
        uv, iv, cv = self._prepare_vocab_dicts()
        if metadata.get("din_activation", "dice") != "dice":
            raise NotImplementedError("the DIN kernels implement the Dice activation only")
        hidden = list(metadata.get("din_mlp_hidden_units", [200, 80]))
        if len(hidden) != 2:
            raise NotImplementedError("the DIN kernels implement two MLP hidden layers")
        model_path = os.path.join(load_dir, "din_model.pth")
        if not os.path.exists(model_path):
            raise FileNotFoundError(f"Model weights not found at: {model_path}")
        sd = torch.load(model_path, map_location="cpu", weights_only=True)
        exp = _expected_state(uv, iv, cv, int(metadata["din_embedding_dim"]), hidden)
        missing, unexpected = sorted(set(exp) - set(sd)), sorted(set(sd) - set(exp))
        bad = [k for k in exp if k in sd and tuple(sd[k].shape) != exp[k]]
        if missing or unexpected or bad:  # load_state_dict(strict=True) refuses these
            raise RuntimeError(f"Error(s) in loading state_dict for DINModel: missing {missing}, "
                               f"unexpected {unexpected}, size mismatch {bad}")
        self.model = DINScorer(sd, list(uv), list(iv), list(cv), table_dtype=self.table_dtype, device=self.device)
        self.encoder, self._tables = None, None
        return self

    # --------------------------------------------------------- predict --
    def predict(self):
        """DIN.py:1219-1283: probabilities [len(main_df)] float32."""
        if self.model is None:
            raise ValueError("Model is not trained yet. Please train the model before prediction.")
        if not getattr(self, "label_encoders", None):
            encoders_path = os.path.join(self.config.save_path, "label_encoders.pkl")
            if os.path.exists(encoders_path):
                self.label_encoders = load_pickle(encoders_path)
        if getattr(self, "main_df", None) is None:
            raise ValueError("load() or set_data() must be called before predict()")
        if self.encoder is None:
            # the encoded lookup tables, built once per data set (the
            # reference's _build_encoding_cache, DIN.py:330-342, plus the
            # per-user / per-item dict lookups of __getitem__ as table rows)
            self.encoder = DinEncoder(self.user_profile_dict, self.item_features_dict, self.user_history_dict,
                                      self.user_profile_features, self.item_features, self.context_features,
                                      self.label_encoders, self.config.din_seq_max_len)
            self._tables = None
        cols = iloc_columns(self.main_df, ["user_id", "item_id"] + list(self.context_features))
        if self._tables is None:
            self._tables = self.encoder.device_tables(self.model.device)
        enc = self.encoder.encode_device(self._tables, cols["user_id"], cols["item_id"], cols)
        return self.model.predict(enc, self.config.batch_size)
