"""ItemCF recaller: drop-in for src/recall/itemcf_recaller.py:11-129.

``_precompute_topk_similar_items`` (A9, :41-54) runs on the GPU
(nrk_itemcf_topn: per item, stable top-``itemcf_sim_item_topk`` by score,
ties in dict insertion order).  ``recall`` / ``batch_recall`` (A10,
:56-129) run on the GPU too (nrk_itemcf_recall: every query user of a batch
in one call -- candidate weights, ordered per-(user, item) sums through a
stable radix sort, hot-item fill and the stable top-k).  The neighbour
lists, the user histories and the embedding content weights are laid out
once, at construction, over one dense id space.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np
import torch

from .. import ops
from .base import BaseRecaller


class ItemCFRecaller(BaseRecaller):
    def __init__(self, config, similarity_matrix: Dict, item_created_time_dict: Dict,
                 user_item_time_dict: Dict, item_topk_click: List, emb_similarity_matrix: Dict = None,
                 device="cuda", sim_result=None):
        super().__init__(config)
        self.i2i_sim = similarity_matrix
        self.item_created_time_dict = item_created_time_dict
        self.user_item_time_dict = user_item_time_dict
        self.item_topk_click = item_topk_click
        self.emb_i2i_sim = emb_similarity_matrix or {}
        self.device = torch.device(device)
        self._sim_result = sim_result
        self._precompute_topk_similar_items()

    @classmethod
    def from_result(cls, config, sim_result, item_created_time_dict, user_item_time_dict, item_topk_click,
                    emb_similarity_matrix=None, device="cuda"):
        """Build straight from ItemCFSimilarity.compute()'s device CSR (no dict
        round trip for the top-n step)."""
        return cls(config, None, item_created_time_dict, user_item_time_dict, item_topk_click,
                   emb_similarity_matrix, device, sim_result)

    def _precompute_topk_similar_items(self):
        topn = self.config.itemcf_sim_item_topk
        d = self.device
        self.topk_sim_items = {}
        if self._sim_result is not None:
            r = self._sim_result
            sim = r.sim
            oc, ov, cnt = ops.itemcf_topn(sim.row_offsets(), sim.j, sim.v, sim.first, topn)
            oc, ov, cnt = oc.cpu().numpy(), ov.cpu().numpy(), cnt.cpu().numpy()
            ids = r.item_ids
            for row in r.row_order.tolist():
                m = int(cnt[row])
                self.topk_sim_items[int(ids[row])] = list(zip(ids[oc[row, :m]].tolist(), ov[row, :m].tolist()))
            self._build_device(np.asarray(ids, np.int64), np.asarray(ids, np.int64)[np.maximum(oc, 0)], ov, cnt)
            return
        rows = list(self.i2i_sim.keys())
        lens = np.array([len(self.i2i_sim[i]) for i in rows], np.int64)
        off = np.zeros(len(rows) + 1, np.int64)
        off[1:] = np.cumsum(lens)
        n = int(off[-1])
        if n >= 2**31:
            raise ValueError("similarity has >= 2^31 entries")
        js = np.empty(n, np.int64)
        vs = np.empty(n, np.float64)
        k = 0
        for i in rows:
            sd = self.i2i_sim[i]
            m = len(sd)
            js[k:k + m] = list(sd.keys())
            vs[k:k + m] = list(sd.values())
            k += m
        pos = torch.arange(n, dtype=torch.int32, device=d)
        oc, ov, cnt = ops.itemcf_topn(torch.from_numpy(off).to(d), pos, torch.from_numpy(vs).to(d),
                                      pos.to(torch.int64), topn)
        oc, cnt = oc.cpu().numpy(), cnt.cpu().numpy()
        for r, i in enumerate(rows):
            m = int(cnt[r])
            sel = oc[r, :m]
            self.topk_sim_items[i] = list(zip(js[sel].tolist(), vs[sel].tolist()))
        sel = np.maximum(oc, 0)
        self._build_device(np.asarray(rows, np.int64).reshape(-1), js[sel] if n else np.zeros(oc.shape, np.int64),
                           vs[sel] if n else np.zeros(oc.shape), cnt)

    # ----------------------------------------------------------- device --
    def _build_device(self, rows_raw, cols_raw, vals, cnt):
        """Dense id space over every item the recall can touch (neighbour rows
        and columns, histories, hot items) and the device arrays of A10."""
        d = self.device
        users = list(self.user_item_time_dict.keys())
        lens = np.fromiter((len(self.user_item_time_dict[u]) for u in users), np.int64, len(users))
        offs = np.zeros(len(users) + 1, np.int64)
        offs[1:] = np.cumsum(lens)
        hist = np.fromiter((it for u in users for it, _ in self.user_item_time_dict[u]), np.int64, int(offs[-1]))
        hot = np.asarray(list(self.item_topk_click), np.int64)
        valid = np.arange(cols_raw.shape[1])[None, :] < cnt[:, None]
        ids = np.unique(np.concatenate([rows_raw, cols_raw[valid], hist, hot]))
        n = max(len(ids), 1)
        topn = max(cols_raw.shape[1], 1)
        nb_cols = np.full((n, topn), -1, np.int32)
        nb_vals = np.zeros((n, topn), np.float64)
        nb_cnt = np.zeros(n, np.int32)
        if len(rows_raw):
            rp = np.searchsorted(ids, rows_raw)
            cc = np.where(valid, np.searchsorted(ids, np.where(valid, cols_raw, ids[0])), -1)
            nb_cols[rp, :cols_raw.shape[1]] = cc
            nb_vals[rp, :cols_raw.shape[1]] = np.where(valid, vals, 0.0)
            nb_cnt[rp] = cnt
        ct = self.item_created_time_dict
        created = np.fromiter((float(ct.get(int(x), np.nan)) for x in ids), np.float64, len(ids))
        # recall() reads created[i] and created[j] for every history item i with
        # a neighbour j (itemcf_recaller.py:92-96): those must exist, as there
        hist_rows = np.searchsorted(ids, hist) if len(hist) else np.zeros(0, np.int64)
        looked = np.zeros(len(ids), bool)
        hr = hist_rows[nb_cnt[hist_rows] > 0] if len(hist_rows) else hist_rows
        looked[hr] = True
        nbr = nb_cols[hr][nb_cols[hr] >= 0] if len(hr) else np.zeros(0, np.int64)
        looked[nbr] = True
        missing = looked & np.isnan(created)
        if missing.any():
            raise KeyError(int(ids[np.argmax(missing)]))
        created = np.where(np.isnan(created), 0.0, created)  # hot-fill only items: never read
        self._ids = ids
        self._slot = {u: k for k, u in enumerate(users)}
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(d)  # noqa: E731
        self._dev = {
            "offsets": t(offs), "items": t(np.searchsorted(ids, hist).astype(np.int32)),
            "nbr_cols": t(nb_cols), "nbr_vals": t(nb_vals), "nbr_cnt": t(nb_cnt),
            "created": t(created if len(ids) else np.zeros(1)), "hot": t(np.searchsorted(ids, hot).astype(np.int32)),
        }
        self._emb = None
        if self.emb_i2i_sim:
            pos = {int(x): k for k, x in enumerate(ids)}
            rows = {}
            for i, dd in self.emb_i2i_sim.items():
                pi = pos.get(i)
                if pi is None:
                    continue
                rows[pi] = [(pos[j], v) for j, v in dd.items() if j in pos]
            ke = max([len(r) for r in rows.values()] + [1])
            ec = np.full((n, ke), -1, np.int32)
            ev = np.zeros((n, ke), np.float64)
            en = np.zeros(n, np.int32)
            for pi, r in rows.items():
                en[pi] = len(r)
                if r:
                    ec[pi, :len(r)] = [a for a, _ in r]
                    ev[pi, :len(r)] = [b for _, b in r]
            self._emb = (t(ec), t(ev), t(en))

    def batch_recall(self, user_ids: List[int], topk: int = 10) -> Dict[int, List[Tuple[int, float]]]:
        """Every user of the batch in one nrk_itemcf_recall call (recall/base.py:24-40)."""
        user_ids = list(user_ids)
        if not user_ids:
            return {}
        dv = self._dev
        q = torch.tensor([self._slot.get(u, -1) for u in user_ids], dtype=torch.int64, device=self.device)
        e = self._emb or (None, None, None)
        oi, osc, osrc, ocnt = ops.itemcf_recall(q, dv["offsets"], dv["items"], dv["nbr_cols"], dv["nbr_vals"],
                                                dv["nbr_cnt"], dv["created"], dv["hot"], topk,
                                                self.config.loc_beta, self.config.created_time_alpha, *e)
        oi, osc, osrc, ocnt = (x.cpu().numpy() for x in (oi, osc, osrc, ocnt))
        ids = self._ids
        out = {}
        for n, u in enumerate(user_ids):
            m = int(ocnt[n])
            raw = ids[oi[n, :m]].tolist()
            sc = osc[n, :m].tolist()
            src = osrc[n, :m].tolist()
            # hot-fill / cold-start scores are Python ints in the reference (:70, :120)
            out[u] = [(it, float(v) if k == 0 else int(v)) for it, v, k in zip(raw, sc, src)]
        return out

    def recall(self, user_id: int, topk: int = 10) -> List[Tuple[int, float]]:
        """itemcf_recaller.py:56-129 on the GPU (a batch of one)."""
        return self.batch_recall([user_id], topk)[user_id]
