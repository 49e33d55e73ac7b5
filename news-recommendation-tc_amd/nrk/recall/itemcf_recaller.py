"""ItemCF recaller: drop-in for src/recall/itemcf_recaller.py:11-129.

``_precompute_topk_similar_items`` (A9, :41-54) runs on the GPU
(nrk_itemcf_topn: per item, stable top-``itemcf_sim_item_topk`` by score,
ties in dict insertion order).  ``recall`` (A10, :56-129) is the
reference's per-user host loop over the precomputed neighbour lists (the GPU
version of A10 is the next row).
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

    def recall(self, user_id: int, topk: int = 10) -> List[Tuple[int, float]]:
        """itemcf_recaller.py:56-129, same arithmetic order."""
        if user_id not in self.user_item_time_dict:
            return [(item, -i) for i, item in enumerate(self.item_topk_click[:topk])]
        hist = self.user_item_time_dict[user_id]
        hist_set = {it for it, _ in hist}
        beta = self.config.loc_beta
        calpha = self.config.created_time_alpha
        ct = self.item_created_time_dict
        item_rank: Dict[int, float] = {}
        for loc, (i, _) in enumerate(hist):
            sims = self.topk_sim_items.get(i)
            if sims is None:
                continue
            for j, wij in sims:
                if j in hist_set:
                    continue
                created_w = np.exp(calpha ** np.abs(ct[i] - ct[j]))
                loc_w = beta ** (len(hist) - loc)
                content = 1.0
                if self.emb_i2i_sim:
                    if i in self.emb_i2i_sim and j in self.emb_i2i_sim[i]:
                        content += self.emb_i2i_sim[i][j]
                    if j in self.emb_i2i_sim and i in self.emb_i2i_sim[j]:
                        content += self.emb_i2i_sim[j][i]
                item_rank.setdefault(j, 0)
                item_rank[j] += created_w * loc_w * content * wij
        if len(item_rank) < topk:
            for i, item in enumerate(self.item_topk_click):
                if item in item_rank or item in hist_set:
                    continue
                item_rank[item] = -i - 100
                if len(item_rank) == topk:
                    break
        return sorted(item_rank.items(), key=lambda x: x[1], reverse=True)[:topk]
