"""GPU DIN ranker: drop-in for src/rank/DIN.py's scoring path.

* ``encode_samples`` restates DINDataset.__getitem__ + collate_fn
  (DIN.py:289-520) as a vectorised host encoder that produces the same int
  index tensors (0 = pad / unknown, class index + 1 otherwise; LAST T history
  items, left aligned, prefix mask).
* ``DINScorer`` holds a trained DINModel's state_dict in kernel layout and
  scores batches with the HIP kernels (nrk_din_forward).
* ``DINRanker.predict`` mirrors DINRanker.predict (DIN.py:1219-1283): every
  main_df row in order, batches of ``batch_size``, probabilities positional to
  main_df.  Like the reference, Dice uses the statistics of each batch, so a
  batch is the unit of work; a trailing batch of one row is NaN there (std of
  one sample) and is NaN here too.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch

from .. import ops
from ..config import RankConfig


def _cache(label_encoders, feat):
    enc = label_encoders.get(feat) if label_encoders else None
    if enc is None:
        return None
    return {str(c): i + 1 for i, c in enumerate(enc.classes_)}


def _code(cache, raw):
    if cache is None:
        return raw  # DINDataset._encode_feature_fast without an encoder (DIN.py:348-349)
    return cache.get(str(raw), 0)


def iloc_columns(df, cols):
    """Column values exactly as ``main_df.iloc[idx][col]`` presents them
    (DIN.py:369-371, 407).  pandas upcasts a row to the frame's common dtype:
    with float context columns an int user_id reads back as 1013.0, so
    ``str(row["user_id"])`` is "1013.0", misses the str(int) keys of the
    profile / feature / history dicts and every user, item and history
    feature encodes to 0.  That quirk is part of the reference's output and
    is reproduced here, not repaired."""
    if len(df) == 0:
        return {c: [] for c in cols}
    dt = df.iloc[0].dtype
    if dt == object:
        return {c: df[c].tolist() for c in cols}
    return {c: df[c].astype(dt).tolist() for c in cols}


def encode_samples(user_ids, item_ids, ctx_cols, user_profile_dict, item_features_dict,
                   user_history_dict, user_features, item_features, ctx_features,
                   label_encoders, seq_max_len):
    """Vectorised DINDataset + collate_fn.  ``user_ids``/``item_ids`` and
    ``ctx_cols`` (feature -> list of raw values) as the reference reads them
    from main_df rows (see ``iloc_columns``)."""
    n = len(user_ids)
    uc = [_cache(label_encoders, f) for f in user_features]
    ic = [_cache(label_encoders, f) for f in item_features]
    cc = [_cache(label_encoders, f) for f in ctx_features]
    user_vec: Dict[str, List[int]] = {}
    item_vec: Dict[str, List[int]] = {}

    def uvec(u):
        v = user_vec.get(u)
        if v is None:
            prof = user_profile_dict.get(u)
            v = ([_code(c, prof.get(f, 0)) for c, f in zip(uc, user_features)]
                 if prof is not None else [0] * len(user_features))
            user_vec[u] = v
        return v

    def ivec(i):
        v = item_vec.get(i)
        if v is None:
            feat = item_features_dict.get(i)
            v = ([_code(c, feat.get(f, 0)) for c, f in zip(ic, item_features)]
                 if feat is not None else [0] * len(item_features))
            item_vec[i] = v
        return v

    T = seq_max_len
    user = np.zeros((n, len(user_features)), np.int64)
    item = np.zeros((n, len(item_features)), np.int64)
    hist = np.zeros((n, T, len(item_features)), np.int64)
    mask = np.zeros((n, T), np.float32)
    ctx = np.zeros((n, len(ctx_features)), np.int64)
    hist_cache: Dict[str, np.ndarray] = {}
    for r in range(n):
        u = str(user_ids[r])
        it = str(item_ids[r])
        user[r] = uvec(u)
        item[r] = ivec(it)
        h = hist_cache.get(u)
        if h is None:
            lst = user_history_dict.get(u, [])
            if len(lst) > T:
                lst = lst[-T:]  # LAST T (DIN.py:481-482)
            h = np.array([ivec(x) for x in lst], np.int64).reshape(-1, len(item_features))
            hist_cache[u] = h
        L = h.shape[0]
        hist[r, :L] = h
        mask[r, :L] = 1.0
    if len(ctx_features):
        for k, f in enumerate(ctx_features):
            cache = cc[k]
            ctx[:, k] = [_code(cache, v) for v in ctx_cols[f]]
    return {"user": user, "item": item, "hist": hist, "ctx": ctx, "mask": mask}


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
        statistics); otherwise one call per batch."""
        n = enc["mask"].shape[0]
        if n >= 2 and (batch_size % 64 == 0 or n <= batch_size):
            d = self.device
            t = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a)).to(d, dt).contiguous()  # noqa: E731
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
            p = self.forward(enc["user"][s:e], enc["item"][s:e], enc["hist"][s:e],
                             enc["ctx"][s:e], enc["mask"][s:e])
            out[s:e] = p.cpu().numpy()
        return out


class DINRanker:
    """Ranker plugin (rank/base.py:10-117 contract): ``predict()`` returns
    probabilities aligned to ``main_df`` rows.  Data loading (feature CSVs,
    pickles) and training stay with the reference; hand this class the
    loaded structures and the trained state_dict."""

    def __init__(self, config: Optional[RankConfig] = None, device="cuda", table_dtype="fp32"):
        self.config = config or RankConfig()
        self.device = device
        self.table_dtype = table_dtype
        self.scorer = None

    def set_data(self, main_df, user_profile_dict, item_features_dict, user_history_dict,
                 user_profile_features, item_features, context_features, label_encoders):
        self.main_df = main_df
        self.user_profile_dict = user_profile_dict
        self.item_features_dict = item_features_dict
        self.user_history_dict = user_history_dict
        self.user_profile_features = list(user_profile_features)
        self.item_features = list(item_features)
        self.context_features = list(context_features)
        self.label_encoders = label_encoders
        return self

    def load_model(self, state_dict):
        self.scorer = DINScorer(state_dict, self.user_profile_features, self.item_features,
                                self.context_features, table_dtype=self.table_dtype,
                                device=self.device)
        return self

    def predict(self):
        if self.scorer is None:
            raise ValueError("Model is not trained yet. Please train the model before prediction.")
        cols = iloc_columns(self.main_df, ["user_id", "item_id"] + self.context_features)
        enc = encode_samples(cols["user_id"], cols["item_id"], cols,
                             self.user_profile_dict, self.item_features_dict,
                             self.user_history_dict, self.user_profile_features,
                             self.item_features, self.context_features, self.label_encoders,
                             self.config.din_seq_max_len)
        return self.scorer.predict(enc, self.config.batch_size)
