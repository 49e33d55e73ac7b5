"""GPU YouTubeDNN recaller: drop-in for src/recall/youtubednn_recaller.py.

Same plugin contract as the reference's ``YoutubeDNNRecaller``
(youtubednn_recaller.py:191-569): raw user ids in, ``[(raw_item_id, score)]``
out, rank 0 of the (topk+1) search dropped (:524), Faiss row r mapped through
``item_index_2_rawid[r]`` (:528-529 -- the reference's row->id quirk is kept
on purpose), unknown users -> ``[]`` (:513-514), not
ready -> ``ValueError`` (:508-509).

What changes is underneath: the user/item towers run as HIP kernels
(nrk_tt_user_fwd / nrk_tt_item_fwd), the Faiss IndexFlatIP becomes a device
catalog (nrk_ip_catalog_build) and ``batch_recall`` is ONE device top-k call
for the whole user list (nrk_ip_topk) instead of one Faiss search per user.
Training (:211-423) is outside the hot path: load trained weights with
``load_model`` or precomputed embeddings with ``from_embeddings``.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np
import pandas as pd
import torch

from .. import ops
from ..config import RecallConfig
from ..data import extractors
from .base import BaseRecaller


def _as_mapping_array(m, n=None):
    if isinstance(m, dict):
        n = len(m) if n is None else n
        return np.array([m[i] for i in range(n)], dtype=np.int64)
    return np.asarray(m, dtype=np.int64)


class YoutubeDNNRecaller(BaseRecaller):
    def __init__(self, config: RecallConfig | None = None, device: str | torch.device = "cuda"):
        super().__init__(config or RecallConfig())
        self.seq_max_len = getattr(self.config, "youtubednn_seq_max_len", 30)
        self.embedding_dim = getattr(self.config, "youtubednn_embedding_dim", 16)
        self.hidden_units = getattr(self.config, "youtubednn_hidden_units", [64, 16])
        self.device = torch.device(device)
        self.user_index_2_rawid: Dict[int, int] = {}
        self.user_rawid_2_index: Dict[int, int] = {}
        self.item_index_2_rawid: Dict[int, int] = {}
        self.item_rawid_2_index: Dict[int, int] = {}
        self.user_embeddings = None  # torch [U, D] on device
        self.item_embeddings = None  # torch [I, D] on device
        self.catalog = None          # ops.Catalog = the Faiss index
        self._item_raw = None        # np [I] row -> raw id (quirk mapping)

    # -------------------------------------------------------------- setup --
    @classmethod
    def from_embeddings(cls, user_embeddings, item_embeddings, user_index_2_rawid,
                        item_index_2_rawid, config=None, device="cuda"):
        """Wrap already-extracted embeddings (the state after
        _extract_embeddings, youtubednn_recaller.py:425-495)."""
        self = cls(config, device)
        dev = lambda x: (x.to(self.device, torch.float32) if torch.is_tensor(x)  # noqa: E731
                         else torch.as_tensor(np.asarray(x, np.float32)).to(self.device)).contiguous()
        ue, ie = dev(user_embeddings), dev(item_embeddings)
        self._set_state(ue, ie, _as_mapping_array(user_index_2_rawid),
                        _as_mapping_array(item_index_2_rawid))
        return self

    def load_model(self, state_dict, click_df):
        """Build mappings exactly as train() does (label encoding :324-353),
        then run both towers on the GPU for every user / item
        (_extract_embeddings :425-495).  ``state_dict`` holds the reference
        module's parameters (user_embedding.weight, item_embedding.weight,
        user_tower.0.*, user_tower.3.*)."""
        sd = {k: (v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v))
              for k, v in state_dict.items()}
        # user_tower = [Linear, ReLU, Dropout] per hidden unit: Linear l at index 3 l (:105-112)
        n_layers = len([k for k in sd if k.startswith("user_tower.") and k.endswith(".weight")])
        user_col = np.asarray(click_df["user_id"], np.int64)
        uid, hist, hlen, item_raw, profile = extractors.youtubednn_histories(
            user_col, np.asarray(click_df["click_article_id"], np.int64), self.seq_max_len)
        user_raw = np.unique(user_col)
        dev = self.device
        f = lambda a: torch.as_tensor(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        tabs = (f(sd["user_embedding.weight"].astype(np.float32)), f(sd["item_embedding.weight"].astype(np.float32)),
                f(uid.astype(np.int32)), f(hist.astype(np.int32)), f(hlen.astype(np.int32)))
        layers = [(f(sd[f"user_tower.{3 * l}.weight"].astype(np.float32)),
                   f(sd[f"user_tower.{3 * l}.bias"].astype(np.float32))) for l in range(n_layers)]
        if n_layers == 2 and layers[0][0].shape[0] <= 128:  # the tuned two-layer kernel (LDS-resident weights)
            ue = ops.tt_user_fwd(*tabs, *layers[0], *layers[1])
        else:
            ue = ops.tt_user_fwd_layers(*tabs, layers)
        ie = ops.tt_item_fwd(f(sd["item_embedding.weight"].astype(np.float32)),
                             f(profile.astype(np.int32)))
        self._set_state(ue, ie, user_raw, item_raw)
        return self

    def _set_state(self, ue, ie, user_raw, item_raw):
        self.user_embeddings = ue
        self.item_embeddings = ie
        self.user_index_2_rawid = {i: int(r) for i, r in enumerate(user_raw)}
        self.user_rawid_2_index = {int(r): i for i, r in enumerate(user_raw)}
        self.item_index_2_rawid = {i: int(r) for i, r in enumerate(item_raw)}
        self.item_rawid_2_index = {int(r): i for i, r in enumerate(item_raw)}
        self._item_raw = np.asarray(item_raw, np.int64)
        self._user_index = pd.Index(np.asarray(user_raw, np.int64))
        self.catalog = ops.Catalog(ie)

    # ------------------------------------------------------------- recall --
    def recall(self, user_id: int, topk: int = 20) -> List[Tuple[int, float]]:
        return self.batch_recall([user_id], topk)[user_id]

    def batch_recall(self, user_ids: List[int], topk: int = 20) -> Dict[int, List[Tuple[int, float]]]:
        """BaseRecaller.batch_recall (recall/base.py:24-40) as ONE device
        top-(k+1) search; the result dict is built with vectorised id mapping
        (row r -> item_index_2_rawid[r], the reference's quirk) and one
        zip per user instead of a per-item Python loop."""
        if self.user_embeddings is None or self.catalog is None:
            raise ValueError("Model not trained. Call train() first.")
        n_users = self.user_embeddings.shape[0]
        arr = np.asarray(user_ids)
        # the int64 index path only where the cast is value-preserving: signed
        # ids, or unsigned ids below 2^63 (a larger uint64 would wrap onto
        # another user); everything else takes the dict lookup
        fits = arr.dtype.kind == "i" or (arr.dtype.kind == "u" and (arr.size == 0 or int(arr.max()) < 2 ** 63))
        if fits and arr.ndim == 1 and self._user_index.is_unique:
            idx = self._user_index.get_indexer(arr.astype(np.int64))
        else:  # str / float / mixed ids: the reference's own dict lookup (user_rawid_2_index.get, :511)
            idx = np.array([self.user_rawid_2_index.get(u, -1) for u in user_ids], np.int64)
        known = (idx >= 0) & (idx < n_users)
        results: Dict[int, List[Tuple[int, float]]] = dict.fromkeys(user_ids)
        for u in results:
            results[u] = []
        if not known.any():
            return results
        rows_needed = torch.as_tensor(idx[known], device=self.device)
        q = self.user_embeddings.index_select(0, rows_needed).contiguous()
        s, r = ops.ip_topk(q, self.catalog, topk + 1)
        s = s[:, 1:].cpu().numpy()  # rank 0 dropped (youtubednn_recaller.py:524)
        r = r[:, 1:].cpu().numpy().astype(np.int64)
        n_map = len(self._item_raw)
        ok = (r >= 0) & (r < n_map)
        items = self._item_raw[np.where(ok, r, 0)]
        kn = [u for u, k in zip(user_ids, known) if k]
        full = ok.all(1)
        it_l, sc_l = items.tolist(), s.tolist()
        if full.all():
            results.update(zip(kn, map(list, map(zip, it_l, sc_l))))
        else:
            for n, u in enumerate(kn):
                if full[n]:
                    results[u] = list(zip(it_l[n], sc_l[n]))
                else:  # -1 padding (fewer than topk + 1 items): skipped like :528
                    results[u] = [(it_l[n][i], sc_l[n][i]) for i in range(topk) if ok[n, i]]
        return results

    def construct_embedding_dict(self, save: bool = False):
        if self.user_embeddings is None or self.item_embeddings is None:
            raise ValueError("Embeddings not extracted. Call train() first.")
        ue = self.user_embeddings.cpu().numpy()
        ie = self.item_embeddings.cpu().numpy()
        user_emb_dict = {self.user_index_2_rawid[i]: ue[i] for i in range(len(ue))}
        item_emb_dict = {self.item_index_2_rawid[i]: ie[i] for i in range(len(ie))}
        if save:
            import os
            import pickle

            os.makedirs(self.config.save_path, exist_ok=True)
            for name, obj in (("user_youtubednn_emb.pkl", user_emb_dict),
                              ("article_youtubednn_emb.pkl", item_emb_dict)):
                with open(os.path.join(self.config.save_path, name), "wb") as fh:
                    pickle.dump(obj, fh)
        return user_emb_dict, item_emb_dict
