"""GPU RecallFusion: drop-in for src/recall/fusion.py.

Same plugin surface as the reference's ``RecallFusion`` (fusion.py:10-375):
``add_recall_result(name, result, weight)``, ``fuse(topk, user_history,
remove_seen)`` -> ``{user_id: [(item_id, score), ...]}``, ``save(path)`` (the
``all_recall_results.pkl`` wire format RecallPipeline writes,
recall_pipeline.py:276-294), the six fusion strategies and the three
normalisations.  Underneath, every user's merge runs on the GPU in one launch
(``nrk_fuse``, csrc/fusion.hip); the host side only flattens the result dicts
into arrays and builds the output dict.

Exactness: global / local min-max and every strategy run the reference's
float64 operations in the reference's order (bit-identical scores, identical
lists and tie order).  The z-score normalisation (:155-175) runs on the host
exactly as the reference does -- numpy mean / std of the method's scores and
numpy's exp for the sigmoid, so those scores are the reference's to the bit --
and the device takes them as pre-normalised.
"""
from __future__ import annotations

import os
import pickle
from itertools import chain
from typing import Dict, List, Optional, Tuple

import numpy as np
import pandas as pd
import torch

from .. import ops
from .._lib import P, call

STRATEGIES = {"weighted_sum": 0, "weighted_avg": 1, "max_score": 2, "harmonic_mean": 3,
              "diversity_weighted": 4, "rrf": 5}
NORMS = {"local": 0, "global": 1, "z-score": 2}
FUSE_MAX = 256        # entries per user (and topk) of nrk_fuse (4 per lane, registers)
FUSE_WIDE_MAX = 2048  # entries per user of nrk_fuse_wide (LDS)


class RecallFusion:
    def __init__(self, config=None, fusion_strategy: str = "weighted_avg", normalize_method: str = "local",
                 device="cuda"):
        self.config = config
        self.recall_results: Dict[str, Dict] = {}
        self.weights: Dict[str, float] = {}
        self.fusion_strategy = fusion_strategy
        self.normalize_method = normalize_method
        self.device = torch.device(device)
        self.fused_results = None

    def add_recall_result(self, name: str, result: Dict[int, List[Tuple[int, float]]], weight: float = 1.0):
        """fusion.py:55-69."""
        self.recall_results[name] = result
        self.weights[name] = weight

    # ------------------------------------------------------------------ fuse --
    def fuse(self, topk: int = 30, user_history: Optional[Dict[int, set]] = None,
             remove_seen: bool = True) -> Dict[int, List[Tuple[int, float]]]:
        """fusion.py:267-342 on the device."""
        if not self.recall_results:
            raise ValueError("No recall results added. Use add_recall_result() first.")
        names = list(self.recall_results)
        # the reference's user order: a set updated method by method (:306-309)
        all_users = set()
        for nm in names:
            all_users.update(self.recall_results[nm].keys())
        users = list(all_users)
        if not users:
            self.fused_results = {}
            return {}
        uidx = pd.Index(_obj(users), dtype=object)

        # flatten every (method, user, position) entry, method by method
        us, it, sc, mt, rk = [], [], [], [], []
        zmean = np.zeros(len(names))
        zstd = np.zeros(len(names))
        for m, nm in enumerate(names):
            res = self.recall_results[nm]
            lens = np.fromiter((len(v) for v in res.values()), np.int64, count=len(res))
            n = int(lens.sum())
            flat = list(chain.from_iterable(res.values()))
            items = _obj([t[0] for t in flat])
            scores = np.array([t[1] for t in flat], dtype=np.float64) if n else np.zeros(0)
            us.append(np.repeat(uidx.get_indexer(_obj(list(res.keys()))), lens))
            it.append(items)
            sc.append(scores)
            mt.append(np.full(n, m, np.int32))
            rk.append((np.arange(n) - np.repeat(np.cumsum(lens) - lens, lens)).astype(np.int32))
            if NORMS.get(self.normalize_method, 0) == 2 and n:
                # fusion.py:155-175 with numpy on the host: the same mean / std
                # of the Python list and the same np.exp, so the sigmoid is the
                # reference's to the bit; the device then takes the scores as
                # pre-normalised (norm 3)
                all_scores = [t[1] for t in flat]
                mean_score = np.mean(all_scores)
                std_score = np.std(all_scores)
                if std_score > 0:
                    z = (scores - mean_score) / std_score
                    sc[-1] = 1.0 / (1.0 + np.exp(-z))
                else:
                    sc[-1] = np.full(n, 0.5)
        us = np.concatenate(us)
        if len(us) == 0:  # every list empty: {user: []} as the reference (:311-333)
            self.fused_results = {u: [] for u in users}
            return self.fused_results
        order = np.argsort(us, kind="stable")  # by user; method order, then list order inside
        item_codes, item_keys = pd.factorize(np.concatenate(it)) if len(us) else (np.zeros(0, np.int64), [])
        score = np.concatenate(sc)[order]
        counts = np.bincount(us, minlength=len(users))
        max_entries = int(counts.max(initial=0))
        if max_entries > FUSE_WIDE_MAX:
            raise NotImplementedError(f"more than {FUSE_WIDE_MAX} recalled entries for one user")
        offsets = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        dev = self.device
        d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        t_off, t_item = d(offsets), d(item_codes[order].astype(np.int32))
        t_score, t_m = d(score), d(np.concatenate(mt)[order])
        t_rank, t_w = d(np.concatenate(rk)[order]), d(np.array([self.weights[n] for n in names], np.float64))
        norm = NORMS.get(self.normalize_method, 0)
        if norm == 2:
            norm = 3  # normalised on the host above
        gmin = gmax = 0.0
        if norm == 1 and len(score):
            mm = torch.empty(2, dtype=torch.float64, device=dev)
            call("nrk_fuse_minmax", P(t_score.data_ptr()), len(score), P(mm.data_ptr()), ops._stream())
            gmin, gmax = mm.tolist()
        seen_off = seen = None
        if remove_seen and user_history:
            code_of = pd.Index(item_keys, dtype=object) if len(item_keys) else None
            lists = [list(user_history.get(u, ())) for u in users]
            lens = np.fromiter((len(x) for x in lists), np.int64, count=len(lists))
            flat = _obj(list(chain.from_iterable(lists)))
            codes = code_of.get_indexer(flat) if code_of is not None and len(flat) else np.full(len(flat), -1)
            if len(flat):  # no history item at all (e.g. cold-start users): nothing to remove
                seen_off = d(np.concatenate([[0], np.cumsum(lens)]).astype(np.int64))
                seen = d(np.where(codes >= 0, codes, -2).astype(np.int32))  # -2 never matches an item code
        strat = STRATEGIES.get(self.fusion_strategy, 1)
        nu = len(users)
        o_item = torch.empty((nu, topk), dtype=torch.int32, device=dev)
        o_score = torch.empty((nu, topk), dtype=torch.float64, device=dev)
        o_cnt = torch.empty(nu, dtype=torch.int32, device=dev)
        zm, zs = d(zmean), d(zstd)
        p = lambda t: P(t.data_ptr()) if t is not None else None  # noqa: E731
        if max_entries <= FUSE_MAX and topk <= FUSE_MAX:
            call("nrk_fuse", p(t_off), nu, p(t_item), p(t_score), p(t_m), p(t_rank), len(names), p(t_w), strat,
                 norm, float(gmin), float(gmax), p(zm), p(zs), p(seen_off), p(seen), int(topk), p(o_item),
                 p(o_score), p(o_cnt), ops._stream())
        else:
            call("nrk_fuse_wide", p(t_off), nu, p(t_item), p(t_score), p(t_m), p(t_rank), len(names), p(t_w),
                 strat, norm, float(gmin), float(gmax), p(zm), p(zs), p(seen_off), p(seen), max_entries, int(topk),
                 p(o_item), p(o_score), p(o_cnt), ops._stream())
        oi, os_, oc = o_item.cpu().numpy(), o_score.cpu().numpy(), o_cnt.cpu().numpy()
        keys = np.asarray(item_keys, dtype=object)
        raw = keys[np.maximum(oi, 0)] if len(keys) else np.zeros(oi.shape, dtype=object)
        it_l, sc_l = raw.tolist(), os_.tolist()
        out = {}
        for n_, u in enumerate(users):
            c = int(oc[n_])
            out[u] = list(zip(it_l[n_][:c], sc_l[n_][:c]))
        self.fused_results = out
        return out

    # ------------------------------------------------------------------ save --
    def save(self, path: Optional[str] = None):
        """The fused dict as the pickle RecallPipeline writes
        (``all_recall_results.pkl``, recall_pipeline.py:290-294)."""
        if self.fused_results is None:
            raise ValueError("No fused results. Call fuse() first.")
        if path is None:
            path = getattr(self.config, "all_recall_results_path", None) or "all_recall_results.pkl"
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "wb") as fh:
            pickle.dump(self.fused_results, fh)
        return path


def _obj(seq):
    a = np.empty(len(seq), dtype=object)
    a[:] = seq
    return a
