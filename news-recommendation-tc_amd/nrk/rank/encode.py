"""Vectorised DIN input encoding: DINDataset.__getitem__ + collate_fn
(src/rank/DIN.py:330-520) without a per-row Python loop.

The reference, per main_df row (DIN.py:358-457):
  * ``str(row["user_id"])`` / ``str(row["item_id"])`` keys into
    user_profile_dict / item_features_dict / user_history_dict;
  * every raw feature value -> ``str(raw)`` -> LabelEncoder class index + 1,
    0 when unknown; a feature without an encoder passes its raw value
    through (``_encode_feature_fast``, :330-353);
  * the user's history items encoded the same way, the LAST T kept,
    left-aligned, mask 1 on valid slots (collate_fn :471-520);
  * context features read from the row itself.

Here that becomes (``DinEncoder``):
  * once per data set (``__init__``): one ``Codebook`` per LabelEncoder
    (str(class) -> index + 1, hash lookups through pandas), and three encoded
    tables: user profile codes [n_users, Fu], item feature codes [n_items,
    Fi], and per history user the encoded last-T block [n_hist_users, T, Fi]
    + its mask [n_hist_users, T];
  * per call (``rows``): the main_df columns read with the reference's
    ``iloc`` dtype semantics (``iloc_columns``), factorised, the distinct
    keys ``str()``-ed once, and mapped to table rows (-1 = unknown -> zeros)
    plus the context codes;
  * the gathers table[row] run on the device (``nrk_gather_rows``) for the
    GPU ranker, or in numpy (``encode_host``) for the CPU tests.
"""
from __future__ import annotations

from itertools import chain

import numpy as np
import pandas as pd


def iloc_columns(df, cols):
    """Columns exactly as ``main_df.iloc[idx][col]`` presents them
    (DIN.py:369-371, 407): pandas upcasts a row to the frame's common dtype,
    so with float context columns an int user_id reads back as 1013.0 and
    ``str()`` gives "1013.0" -- which misses the str(int) keys of the
    profile / feature / history dicts, so every user, item and history
    feature encodes to 0.  That quirk is part of the reference's output and
    is reproduced, not repaired.  Returns numpy arrays (numeric dtype: the
    row dtype; object rows: object arrays)."""
    if len(df) == 0:
        return {c: np.array([], dtype=object) for c in cols}
    dt = df.iloc[0].dtype
    if dt == object:
        # an object row holds each column's own value; int64 / float64 / bool
        # columns print the same from their numpy array (fast factorisation)
        out = {}
        for c in cols:
            col = df[c]
            out[c] = (col.to_numpy() if col.dtype in (np.int64, np.float64, np.bool_)
                      else col.to_numpy(dtype=object))
        return out
    return {c: df[c].to_numpy().astype(dt) for c in cols}


def factor_strs(values):
    """(codes, keys): ``str(values[i]) == keys[codes[i]]``, with ``str()``
    run once per distinct value.  Numeric arrays and object arrays of one
    Python type are factorised (equal values print alike); mixed object
    arrays are str()-ed element by element first, because 1, 1.0 and True
    hash equal but print differently."""
    a = np.asarray(values) if not isinstance(values, np.ndarray) else values
    if a.dtype == object and pd.api.types.infer_dtype(a, skipna=False) not in ("string", "integer", "floating",
                                                                                  "boolean", "bytes"):
        a = np.array([str(v) for v in a], dtype=object)  # mixed Python types
    codes, uniq = pd.factorize(a)
    keys = [str(u) for u in uniq]
    if (codes < 0).any():  # NaN / None (factorize's sentinel)
        na = a[np.argmax(codes < 0)]
        codes = np.where(codes < 0, len(keys), codes)
        keys.append(str(na))
    out = np.empty(len(keys), dtype=object)
    out[:] = keys
    return codes, out


def str_keys(values):
    """``[str(v) for v in values]`` (see ``factor_strs``)."""
    codes, keys = factor_strs(values)
    return keys[codes]


class Codebook:
    """One LabelEncoder: str(class) -> class index + 1 (DIN.py:330-342);
    duplicated str forms keep the last index, as the dict comprehension
    does."""

    def __init__(self, classes):
        keys = [str(c) for c in classes]
        s = pd.Series(np.arange(1, len(keys) + 1, dtype=np.int64), index=pd.Index(keys, dtype=object))
        self._s = s[~s.index.duplicated(keep="last")]

    def encode_strs(self, strs):
        """codes of already-str()-ed keys (0 = unknown)."""
        idx = self._s.index.get_indexer(pd.Index(strs, dtype=object))
        vals = self._s.to_numpy()
        return np.where(idx >= 0, vals[np.maximum(idx, 0)], 0).astype(np.int64)

    def encode(self, values):
        codes, keys = factor_strs(values)
        return self.encode_strs(keys)[codes]


def _raw_codes(book, values):
    """A feature column through ``_encode_feature_fast``: the codebook, or
    the raw value itself when the feature has no encoder (collate_fn then
    makes it an int64 tensor)."""
    if book is None:
        return np.asarray(values).astype(np.int64)
    return book.encode(values)


def _key_index(keys):
    """The dict's keys as a hash index with dict semantics (``x in d``:
    equal-and-same-hash, so 1 == 1.0 but "1" != 1)."""
    idx = np.empty(len(keys), dtype=object)
    idx[:] = keys
    return pd.Index(idx, dtype=object)


class DinEncoder:
    """Encoded DIN lookup tables for one data set (see the module doc)."""

    def __init__(self, user_profile_dict, item_features_dict, user_history_dict, user_features, item_features,
                 ctx_features, label_encoders, seq_max_len):
        self.user_features = list(user_features)
        self.item_features = list(item_features)
        self.ctx_features = list(ctx_features)
        self.T = int(seq_max_len)
        encs = label_encoders or {}
        self.books = {f: Codebook(e.classes_) for f, e in encs.items()}
        Fu, Fi, T = len(self.user_features), len(self.item_features), self.T

        # user profile table: profile dict order, .get(feat, 0) like :374
        ukeys = list(user_profile_dict.keys())
        self.user_index = _key_index(ukeys)
        self.user_table = np.zeros((len(ukeys), Fu), np.int32)
        profs = list(user_profile_dict.values())
        for j, f in enumerate(self.user_features):
            raw = np.empty(len(profs), dtype=object)
            raw[:] = [p.get(f, 0) for p in profs]
            self.user_table[:, j] = _raw_codes(self.books.get(f), raw)

        # item feature table (:385-391)
        ikeys = list(item_features_dict.keys())
        self.item_index = _key_index(ikeys)
        self.item_table = np.zeros((len(ikeys), Fi), np.int32)
        feats = list(item_features_dict.values())
        for j, f in enumerate(self.item_features):
            raw = np.empty(len(feats), dtype=object)
            raw[:] = [p.get(f, 0) for p in feats]
            self.item_table[:, j] = _raw_codes(self.books.get(f), raw)

        # history table: each user's LAST T items (:481-485), encoded through
        # item_features_dict (unknown item -> all-zero features, :397-401)
        hkeys = list(user_history_dict.keys())
        self.hist_index = _key_index(hkeys)
        lists = list(user_history_dict.values())
        lens = np.fromiter((len(v) for v in lists), dtype=np.int64, count=len(lists))
        flat = np.empty(int(lens.sum()), dtype=object)
        flat[:] = list(chain.from_iterable(lists))
        # the dict test is ``hist_item_id in item_features_dict`` on the raw
        # stored value (no str(): :397)
        rows = self.item_index.get_indexer(pd.Index(flat, dtype=object)) if len(flat) else np.zeros(0, np.int64)
        keep = np.minimum(lens, T)
        off = np.concatenate([[0], np.cumsum(lens)])
        start = off[:-1] + lens - keep
        t = np.arange(T)
        valid = t[None, :] < keep[:, None]
        pos = np.where(valid, start[:, None] + t[None, :], 0)
        hrow = np.where(valid, rows[pos] if len(rows) else -1, -1)
        ext = np.concatenate([self.item_table, np.zeros((1, Fi), np.int32)])  # row -1 -> zeros
        self.hist_table = ext[hrow]                                  # [H, T, Fi]
        self.mask_table = valid.astype(np.float32)                   # [H, T]

    # ------------------------------------------------------------ per call --
    def rows(self, user_ids, item_ids, ctx_cols):
        """Row indices of every sample into the three tables (-1 = unknown)
        and the context codes [n, Fc]; every lookup runs once per distinct
        key."""
        n = len(user_ids)
        uc, uk = factor_strs(user_ids)
        ic, ik = factor_strs(item_ids)
        uidx = pd.Index(uk, dtype=object)
        urow = self.user_index.get_indexer(uidx).astype(np.int32)[uc]
        hrow = self.hist_index.get_indexer(uidx).astype(np.int32)[uc]
        irow = self.item_index.get_indexer(pd.Index(ik, dtype=object)).astype(np.int32)[ic]
        ctx = np.zeros((n, len(self.ctx_features)), np.int32)
        for k, f in enumerate(self.ctx_features):
            ctx[:, k] = _raw_codes(self.books.get(f), ctx_cols[f])
        return urow, irow, hrow, ctx

    def encode_host(self, user_ids, item_ids, ctx_cols):
        """The collated batch tensors as numpy arrays (CPU path)."""
        urow, irow, hrow, ctx = self.rows(user_ids, item_ids, ctx_cols)

        def take(tab, r):
            ext = np.concatenate([tab, np.zeros((1,) + tab.shape[1:], tab.dtype)])
            return ext[np.where(r >= 0, r, len(tab))]

        return {"user": take(self.user_table, urow), "item": take(self.item_table, irow),
                "hist": take(self.hist_table, hrow), "ctx": ctx, "mask": take(self.mask_table, hrow)}

    def device_tables(self, device):
        """Upload the encoded tables once (int32 / f32 rows)."""
        import torch

        d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
        return {"user": d(self.user_table), "item": d(self.item_table), "hist": d(self.hist_table),
                "mask": d(self.mask_table)}

    def encode_device(self, tables, user_ids, item_ids, ctx_cols):
        """The collated batch as device tensors: the lookups gathered on the
        GPU (nrk_gather_rows) from ``device_tables``."""
        import torch

        from .. import ops

        urow, irow, hrow, ctx = self.rows(user_ids, item_ids, ctx_cols)
        dev = tables["user"].device
        d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        tu, ti, th = d(urow), d(irow), d(hrow)
        return {"user": ops.gather_rows(tables["user"], tu), "item": ops.gather_rows(tables["item"], ti),
                "hist": ops.gather_rows(tables["hist"], th), "ctx": d(ctx),
                "mask": ops.gather_rows(tables["mask"], th)}
