"""Ranker context features on the GPU.

Restates the context part of the reference's feature pipeline for the rows
the ranker scores:
  * FeatureExtractor._extract_context_features
    (src/features/feature_extractor.py:440-723) -- computed on the device by
    ``nrk_ctx_features`` (csrc/ctxfeat.hip) from resident tables;
  * FeatureExtractor._apply_binning (:838-898) + the context LabelEncoders of
    DINRanker._prepare_vocab_dicts (src/rank/DIN.py:603-613) -- FITTED on the
    host (``CtxSpec.fit``, sklearn's KBinsDiscretizer exactly as the reference
    calls it; fitting is offline ETL) and APPLIED on the device in the same
    kernel, giving the int codes DINDataset feeds the model (DIN.py:330-353).

``CtxTables`` holds the lookup tables in HBM, built from the dicts the
reference keeps (str item / user ids): article-id Word2Vec vectors,
250-d content embeddings (float64), MinMax created times, categories,
YouTubeDNN user / item vectors, and each user's history (last N items, the
distinct categories of the whole history).
"""
from __future__ import annotations

import ctypes
from itertools import chain

import numpy as np
import pandas as pd
import torch

from . import _lib, ops

P = ctypes.c_void_p


def ctx_feature_names(last_n=3):
    """feature_extractor.py:470-481 (the feature_lists.pkl order)."""
    names = ["score"]
    for i in range(1, last_n + 1):
        names += [f"sim_{i}", f"time_diff_{i}", f"word_diff_{i}"]
    return names + ["sim_max", "sim_mean", "sim_min", "sim_std", "item_user_sim", "recall_in_user_cat"]


class CtxTablesC(ctypes.Structure):
    """include/nrk.h nrk_ctx_tables."""
    _fields_ = [("n_groups", ctypes.c_int64), ("group_off", P), ("group_user", P), ("pair_pos", P),
                ("pair_item", P), ("pair_score", P), ("last_n", ctypes.c_int32), ("code_stride", ctypes.c_int32),
                ("hist_last", P), ("hist_n", P), ("ucat_off", P), ("ucat", P), ("user_yt", P), ("user_yt_ok", P),
                ("n_items", ctypes.c_int64), ("w2v", P), ("w2v_ok", P), ("dw", ctypes.c_int32), ("content", P),
                ("content_flags", P), ("dc", ctypes.c_int32), ("created", P), ("category", P), ("item_yt", P),
                ("item_yt_ok", P), ("dy", ctypes.c_int32)]


class CtxSpecC(ctypes.Structure):
    """include/nrk.h nrk_ctx_spec."""
    _fields_ = [("kind", ctypes.c_int32), ("n_edges", ctypes.c_int32), ("n_lut", ctypes.c_int32),
                ("n_vals", ctypes.c_int32), ("fill", ctypes.c_double), ("edges", ctypes.c_double * 16),
                ("vals", ctypes.c_double * 32), ("lut", ctypes.c_int32 * 32), ("codes", ctypes.c_int32 * 32)]


def _stack(d, keys, dim, dtype):
    """rows of dict ``d`` for ``keys`` (zeros + ok=0 when absent)."""
    out = np.zeros((len(keys), dim), dtype)
    ok = np.zeros(len(keys), np.uint8)
    for n, k in enumerate(keys):
        v = d.get(k)
        if v is not None:
            out[n] = v
            ok[n] = 1
    return out, ok


class CtxTables:
    """Device tables for nrk_ctx_features.  ``item_ids`` / ``user_ids`` fix
    the dense rows (str ids, as the reference's dicts key them)."""

    def __init__(self, item_ids, user_ids, w2v, content, created, category, user_history, user_yt=None,
                 item_yt=None, last_n=3, device="cuda"):
        self.device = torch.device(device)
        self.last_n = int(last_n)
        self.item_ids = list(item_ids)
        self.user_ids = list(user_ids)
        self.item_index = pd.Index(_obj(self.item_ids), dtype=object)
        self.user_index = pd.Index(_obj(self.user_ids), dtype=object)
        I = len(self.item_ids)
        dw = len(next(iter(w2v.values()))) if w2v else 1
        dc = len(next(iter(content.values()))) if content else 1
        w, w_ok = _stack(w2v, self.item_ids, dw, np.float32)
        c, c_ok = _stack(content, self.item_ids, dc, np.float64)
        flags = c_ok | ((c.astype(np.float32) != 0).any(1).astype(np.uint8) << 1)  # :641-643 on the f32 rows
        cre = np.array([created.get(i, np.nan) for i in self.item_ids], np.float64)
        cat = np.array([category.get(i, -1) if category.get(i) is not None else -1 for i in self.item_ids], np.int32)
        # per user: the last N history items (:519) and the categories of the
        # whole history (:497-506); history item ids not in the item table
        # (no vector, no content, no created time, no category) -> -1
        N = self.last_n
        hl = np.full((len(self.user_ids), N), -1, np.int32)
        hn = np.full(len(self.user_ids), -1, np.int32)
        cats = []
        for n, u in enumerate(self.user_ids):
            h = user_history.get(u)
            if h is None:
                cats.append([])
                continue
            last = h[-N:]
            r = self.item_index.get_indexer(_obj(last)) if len(last) else np.zeros(0, np.int64)
            hl[n, :len(last)] = r
            hn[n] = len(last)
            seen = []
            for it in h:
                cc = category.get(it)
                if cc is not None and cc not in seen:
                    seen.append(cc)
            cats.append(seen)
        co = np.concatenate([[0], np.cumsum([len(x) for x in cats])]).astype(np.int64)
        cv = np.array(list(chain.from_iterable(cats)), np.int32) if co[-1] else np.zeros(1, np.int32)
        d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(self.device)  # noqa: E731
        self.t = {"w2v": d(w), "w2v_ok": d(w_ok), "content": d(c), "flags": d(flags), "created": d(cre),
                  "category": d(cat), "hist_last": d(hl), "hist_n": d(hn), "ucat_off": d(co), "ucat": d(cv)}
        self.dw, self.dc, self.dy = dw, dc, 0
        if user_yt is not None and item_yt is not None and len(item_yt):
            dy = len(next(iter(item_yt.values())))
            uy, uy_ok = _stack(user_yt, self.user_ids, dy, np.float32)
            iy, iy_ok = _stack(item_yt, self.item_ids, dy, np.float32)
            self.t.update(user_yt=d(uy), user_yt_ok=d(uy_ok), item_yt=d(iy), item_yt_ok=d(iy_ok))
            self.dy = dy
        self.n_items = I

    @classmethod
    def from_device(cls, tensors, last_n=3):
        """Wrap device tensors laid out as in __init__ (the fused pipeline
        builds them on the GPU directly)."""
        self = cls.__new__(cls)
        self.device = tensors["w2v"].device
        self.last_n = int(last_n)
        self.t = dict(tensors)
        self.dw = tensors["w2v"].shape[1]
        self.dc = tensors["content"].shape[1]
        self.dy = tensors["item_yt"].shape[1] if "item_yt" in tensors else 0
        self.n_items = tensors["w2v"].shape[0]
        return self

    def struct(self, group_off, group_user, pair_item, pair_score, pair_pos=None, code_stride=None):
        t = self.t
        p = lambda x: P(x.data_ptr()) if x is not None else None  # noqa: E731
        F = 1 + 3 * self.last_n + 6
        return CtxTablesC(group_user.numel(), p(group_off), p(group_user), p(pair_pos), p(pair_item),
                          p(pair_score), self.last_n, code_stride or F, p(t["hist_last"]), p(t["hist_n"]),
                          p(t["ucat_off"]), p(t["ucat"]), p(t.get("user_yt")), p(t.get("user_yt_ok")),
                          self.n_items, p(t["w2v"]), p(t["w2v_ok"]), self.dw, p(t["content"]), p(t["flags"]),
                          self.dc, p(t["created"]), p(t["category"]), p(t.get("item_yt")), p(t.get("item_yt_ok")),
                          self.dy)


class CtxSpec:
    """The fitted binning + label encoding of every context feature."""

    def __init__(self, specs, names):
        self.names = list(names)
        self.specs = specs
        arr = (CtxSpecC * len(specs))(*specs)
        raw = np.frombuffer(bytes(arr), dtype=np.uint8)
        self._host = raw
        self._dev = {}

    def device(self, device):
        key = str(device)
        if key not in self._dev:
            self._dev[key] = torch.from_numpy(self._host.copy()).to(device)
        return self._dev[key]

    @classmethod
    def fit(cls, columns, names, n_bins=10, strategy="quantile"):
        """``columns``: feature -> raw column (numpy, the main_df dtype) over
        the rows the reference fits on.  _apply_binning (:838-898): numeric
        columns with > 20 distinct values are NaN-filled with their median and
        KBins-binned (n_bins = min(10, distinct)); then one LabelEncoder per
        feature over str(column.fillna(0)) (DIN.py:603-613)."""
        from sklearn.preprocessing import KBinsDiscretizer, LabelEncoder

        specs = []
        for f in names:
            col = pd.Series(columns[f])
            sp = CtxSpecC()
            binned = None
            if pd.api.types.is_numeric_dtype(col) and col.nunique() > 20 and not col.isna().all():
                med = col.median()
                fill = 0 if pd.isna(med) else med
                col = col.fillna(fill)
                nb = min(n_bins, col.nunique())
                if nb >= 2:
                    disc = KBinsDiscretizer(n_bins=nb, encode="ordinal", strategy=strategy)
                    binned = np.asarray(disc.fit_transform(col.to_frame())).astype(int).flatten()
                    edges = np.asarray(disc.bin_edges_[0], np.float64)[1:-1]
                    if len(edges) > 16:
                        raise NotImplementedError("more than 17 bins")
                    sp.kind = 0
                    sp.fill = float(np.asarray(fill, dtype=col.dtype))  # fillna casts to the column dtype
                    sp.n_edges = len(edges)
                    sp.edges[:len(edges)] = edges.tolist()
            elif pd.api.types.is_numeric_dtype(col) and col.isna().all():
                col = pd.Series(np.zeros(len(col), np.int64))  # all-NaN column -> 0 (:860-864)
            if binned is not None:
                le = LabelEncoder().fit(pd.Series(binned).astype(str))
                classes = list(le.classes_)
                sp.n_lut = len(edges) + 1
                for b in range(sp.n_lut):
                    sp.lut[b] = classes.index(str(b)) + 1 if str(b) in classes else 0
            else:
                le = LabelEncoder().fit(col.fillna(0).astype(str))
                classes = list(le.classes_)
                vals = pd.unique(col.dropna())
                if len(vals) > 32:
                    raise NotImplementedError(f"{f}: more than 32 distinct unbinned values")
                sp.kind = 1
                sp.n_vals = len(vals)
                for k, v in enumerate(vals):
                    sp.vals[k] = float(v)
                    sp.codes[k] = classes.index(str(v)) + 1 if str(v) in classes else 0
            specs.append(sp)
        return cls(specs, names)


def ctx_features(tables: CtxTables, user_rows, item_rows, scores, spec: CtxSpec | None = None, raw=True,
                 groups=None, out_codes=None):
    """Context features of n rows (device tensors: user_rows int32 [n] dense
    user row, item_rows int32 [n] (-1 unknown), scores f64 [n]).  Rows are
    grouped by user here (stable), or pass ``groups`` = (group_off int64,
    group_user int32, pair_pos int64 | None).  Returns (raw f64 [n, F] | None,
    codes int32 [n, F] | None)."""
    ops._dev(item_rows, scores)
    n = item_rows.numel()
    F = 1 + 3 * tables.last_n + 6
    dev = item_rows.device
    if groups is None:
        order = torch.sort(user_rows.long(), stable=True).indices
        us = user_rows.long()[order]
        uniq, counts = torch.unique_consecutive(us, return_counts=True)
        group_off = torch.zeros(uniq.numel() + 1, dtype=torch.int64, device=dev)
        group_off[1:] = torch.cumsum(counts, 0)
        groups = (group_off, uniq.to(torch.int32).contiguous(), order.contiguous())
    group_off, group_user, pair_pos = groups
    out_raw = torch.empty((n, F), dtype=torch.float64, device=dev) if raw else None
    if spec is not None and out_codes is None:
        out_codes = torch.empty((n, F), dtype=torch.int32, device=dev)
    if out_codes is not None and (tuple(out_codes.shape) != (n, F) or out_codes.dtype != torch.int32):
        raise ValueError(f"out_codes must be int32 [{n}, {F}]")
    st = tables.struct(group_off, group_user, item_rows, scores, pair_pos)
    sp = spec.device(dev) if spec is not None else None
    _lib.call("nrk_ctx_features", P(ctypes.addressof(st)), P(sp.data_ptr()) if sp is not None else None,
              P(out_raw.data_ptr()) if out_raw is not None else None,
              P(out_codes.data_ptr()) if out_codes is not None else None, ops._stream())
    return out_raw, out_codes


def _obj(seq):
    a = np.empty(len(seq), dtype=object)
    a[:] = list(seq)
    return a
