"""GPU ItemCF similarity: drop-in for src/similarity/item_cf.py:12-108.

``ItemCFSimilarity.calculate(click_df, item_created_time_dict)`` returns the
reference's ``{item_i: {item_j: sim}}`` with the same dict order (rows in
first-click order, entries in first-encounter order) and the same fp64
values up to the last-ulp differences of exp/pow between libm and the
device.  The work runs in nrk_itemcf_sim (csrc/itemcf.hip);
``compute()`` returns the device CSR without materialising the dict.
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch

from .. import ops
from ..config import RecallConfig
from ..data.extractors import user_item_time_csr
from .base import BaseSimilarityCalculator


class ItemCFResult:
    """Device similarity over dense item ids + the raw-id map."""

    def __init__(self, sim: ops.ItemCFSim, item_ids: np.ndarray, row_order: np.ndarray):
        self.sim = sim
        self.item_ids = item_ids      # dense -> raw
        self.row_order = row_order    # dense ids in the reference's row (first click) order

    def to_dict(self) -> Dict[int, Dict[int, float]]:
        i = self.sim.i.cpu().numpy()
        j = self.sim.j.cpu().numpy()
        v = self.sim.v.cpu().numpy()
        f = self.sim.first.cpu().numpy()
        order = np.argsort(f, kind="stable")  # global first-encounter order
        ids = self.item_ids
        out: Dict[int, Dict[int, float]] = {int(ids[r]): {} for r in self.row_order}
        ri, rj, rv = ids[i[order]].tolist(), ids[j[order]].tolist(), v[order].tolist()
        for a, b, s in zip(ri, rj, rv):
            out[a][b] = s
        return out


class ItemCFSimilarity(BaseSimilarityCalculator):
    def __init__(self, config: RecallConfig = None, device="cuda"):
        super().__init__(config or RecallConfig())
        self.device = torch.device(device)

    def compute(self, users, offsets, items_raw, ts, item_created_time_dict) -> ItemCFResult:
        """Similarity from the user-item-time CSR (extractors.user_item_time_csr)."""
        c = self.config
        ids, dense = np.unique(items_raw, return_inverse=True)
        L = np.diff(offsets)
        # item_created_time_dict[i] is read only for pairs i != j (item_cf.py:47-64):
        # an item needs a created time iff its user's list holds >= 2 distinct items
        uid = np.repeat(np.arange(len(L)), L)
        distinct = np.zeros(len(L), np.int64)
        if len(dense):
            up = np.unique(uid.astype(np.int64) * (len(ids) + 1) + dense)
            distinct = np.bincount(up // (len(ids) + 1), minlength=len(L))
        needs = np.zeros(len(ids), bool)
        needs[dense[np.repeat(distinct >= 2, L)]] = True
        created = np.array([item_created_time_dict.get(raw, np.nan) for raw in ids.tolist()], np.float64)
        missing = needs & np.isnan(created)
        if missing.any():
            raise KeyError(ids[np.argmax(missing)].item())  # the reference's dict lookup fails too
        created = np.where(np.isnan(created), 0.0, created)  # never read by any pair
        # row order: first click of each item in the CSR walk (i2i_sim.setdefault, item_cf.py:44)
        _, first_pos = np.unique(dense, return_index=True)
        row_order = np.argsort(first_pos, kind="stable")
        d = self.device
        sim = ops.itemcf_sim(torch.from_numpy(np.ascontiguousarray(offsets, np.int64)).to(d),
                             torch.from_numpy(dense.astype(np.int32)).to(d),
                             torch.from_numpy(np.ascontiguousarray(ts, np.int64)).to(d),
                             torch.from_numpy(created).to(d), len(ids),
                             c.loc_alpha, c.loc_alpha_reverse, c.loc_beta, c.time_decay_alpha,
                             c.created_time_alpha)
        return ItemCFResult(sim, ids, row_order)

    def calculate(self, click_df, item_created_time_dict) -> Dict:
        users, offsets, items, ts = user_item_time_csr(click_df)
        self.result = self.compute(users, offsets, items, ts, item_created_time_dict)
        self.similarity_matrix = self.result.to_dict()
        return self.similarity_matrix

    def get_similar_items(self, item_id: int, topk: int = 20):
        """item_cf.py:91-115."""
        if not self.is_calculated():
            raise ValueError("Similarity matrix not calculated. Call calculate() first.")
        if item_id not in self.similarity_matrix:
            return []
        return sorted(self.similarity_matrix[item_id].items(), key=lambda x: x[1], reverse=True)[:topk]
