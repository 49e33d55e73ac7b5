"""GPU embedding similarity: drop-in for src/similarity/embedding.py:10-95.

``EmbeddingSimilarity.calculate(item_emb_df)`` returns the reference's
``{raw_item: {raw_item: float(sim)}}`` for the ``embedding_topk`` nearest
articles of every article (the second Faiss ``IndexFlatIP`` site).  The rows
are L2-normalised by nrk_row_normalize (bit-identical to the reference's
numpy float32 ``item_emb_np / np.linalg.norm(...)``, :41) and searched by
nrk_ip_topk with users == items (:46-50), so scores and neighbour order follow
the same exact contract as the YouTubeDNN recall (ties -> lower row).  Column
0 of each result row is dropped whatever it holds (:60): with duplicated
embeddings "self" can sit at column 1 and survive, exactly as in the
reference.

Deliberate divergence: a zero-norm row makes the reference divide by zero
and hand NaN rows to Faiss (undefined order); here it raises ValueError.
``compute()`` keeps everything on the device and skips the dict.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np
import torch

from .. import ops
from ..config import RecallConfig
from .base import BaseSimilarityCalculator


class EmbeddingSimilarity(BaseSimilarityCalculator):
    def __init__(self, config: RecallConfig = None, device="cuda"):
        super().__init__(config or RecallConfig())
        self.embedding_dim = getattr(self.config, "embedding_dim", None)
        self.device = torch.device(device)

    def compute(self, emb: torch.Tensor, topk: int = None):
        """Device path: fp32 [n, d] rows -> (scores f32 [n, topk+1], rows i32
        [n, topk+1]) of the self-search, column 0 included."""
        topk = self.config.embedding_topk if topk is None else int(topk)
        if topk + 1 > ops.IP_KMAX:
            raise NotImplementedError(f"embedding_topk + 1 > {ops.IP_KMAX} is not compiled")
        xn, nr = ops.row_normalize(emb.contiguous(), norms=True)
        if emb.shape[0] and not bool(torch.isfinite(nr).all() and (nr > 0).all()):
            raise ValueError("item embeddings must be finite with non-zero norm")
        cat = ops.Catalog(xn)
        return ops.ip_topk(xn, cat, topk + 1)

    def calculate(self, item_emb_df) -> Dict:
        df = item_emb_df.reset_index(drop=True)
        ids = df["article_id"].tolist()
        cols = [c for c in df.columns if "emb" in c]
        x = np.ascontiguousarray(df[cols].values, dtype=np.float32)
        if self.embedding_dim is None:
            self.embedding_dim = x.shape[1]
        s, r = self.compute(torch.from_numpy(x).to(self.device))
        s = s[:, 1:].cpu().numpy().tolist()
        r = r[:, 1:].cpu().numpy().tolist()
        # row -> raw id; a -1 label (topk + 1 > n) raises KeyError(-1) as in the reference
        i2r = dict(enumerate(ids))
        out: Dict[int, Dict[int, float]] = {}
        for t, (rows, vals) in enumerate(zip(r, s)):
            d = out.setdefault(i2r[t], {})
            for rr, v in zip(rows, vals):
                d[i2r[rr]] = v
        self.similarity_matrix = out
        return self.similarity_matrix

    def get_similar_items(self, item_id: int, topk: int = 20) -> List[Tuple[int, float]]:
        """embedding.py:69-92."""
        if not self.is_calculated():
            raise ValueError("Similarity matrix not calculated. Call calculate() first.")
        if item_id not in self.similarity_matrix:
            return []
        return sorted(self.similarity_matrix[item_id].items(), key=lambda x: x[1], reverse=True)[:topk]

    def get_embedding_dimension(self):
        return self.embedding_dim
