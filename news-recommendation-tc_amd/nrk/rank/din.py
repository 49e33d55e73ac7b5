"""GPU DIN ranker: drop-in for src/rank/DIN.py's scoring path.

* ``encode_samples`` / ``DinEncoder`` (nrk/rank/encode.py) restate
  DINDataset.__getitem__ + collate_fn (DIN.py:289-520) without a per-row
  loop: the same int index tensors (0 = pad / unknown, class index + 1
  otherwise; LAST T history items, left aligned, prefix mask), the lookups
  gathered on the device for ``DINRanker.predict``.
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
        # the encoded lookup tables, built once per data set (the reference's
        # _build_encoding_cache, DIN.py:330-342, plus the per-user / per-item
        # dict lookups of __getitem__ turned into table rows)
        self.encoder = DinEncoder(user_profile_dict, item_features_dict, user_history_dict,
                                  self.user_profile_features, self.item_features, self.context_features,
                                  label_encoders, self.config.din_seq_max_len)
        self._tables = None
        return self

    def load_model(self, state_dict):
        self.scorer = DINScorer(state_dict, self.user_profile_features, self.item_features,
                                self.context_features, table_dtype=self.table_dtype,
                                device=self.device)
        return self

    def predict(self):
        if self.scorer is None:
            raise ValueError("Model is not trained yet. Please train the model before prediction.")
        if getattr(self, "encoder", None) is None:
            raise ValueError("set_data() must be called before predict()")
        cols = iloc_columns(self.main_df, ["user_id", "item_id"] + self.context_features)
        if self._tables is None:
            self._tables = self.encoder.device_tables(self.scorer.device)
        enc = self.encoder.encode_device(self._tables, cols["user_id"], cols["item_id"], cols)
        return self.scorer.predict(enc, self.config.batch_size)
