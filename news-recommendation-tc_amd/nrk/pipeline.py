"""Fused recall -> rank on one GPU (BASELINE config 5, one rank's share).

The reference runs recall and rank as separate host pipelines joined by
pickles and CSVs (recall_pipeline.py -> feature_pipeline -> rank_pipeline.py).
Here the recalled pairs never leave HBM:

1. exact top-(k+1) inner-product recall of the rank's users over the
   replicated catalog (nrk_ip_topk, the YoutubeDNN recall of config 2), rank
   0 dropped as youtubednn_recaller.py:524 does;
2. per chunk of users, the DIN inputs of every recalled pair are assembled on
   the device (nrk_din_assemble: profile / candidate / last-T history indices
   and binned context features);
3. DIN scores the pairs in Dice batches of ``batch_size`` (nrk_din_forward_
   segments, the DINRanker.predict batching of DIN.py:1245-1283).

Chunks hold a multiple of ``batch_size`` pairs, so the Dice batches are
exactly those of one pass over all pairs in user-major order.
"""
from __future__ import annotations

import torch

from . import ops


class FusedRecallRank:
    def __init__(self, catalog: ops.Catalog, din: ops.DinParams, user_feat, item_feat, user_hist, hist_len,
                 k: int = 30, batch_size: int = 4096, chunk_users: int = 4096, n_ctx: int = 16,
                 ctx_bins: int = 10, seed: int = 23):
        if (chunk_users * k) % batch_size:
            raise ValueError("chunk_users * k must be a multiple of batch_size")
        self.cat, self.din = catalog, din
        self.user_feat, self.item_feat = user_feat, item_feat
        self.user_hist, self.hist_len = user_hist, hist_len
        self.k, self.bs, self.chunk = k, batch_size, chunk_users
        self.n_ctx, self.ctx_bins, self.seed = n_ctx, ctx_bins, seed
        dev = user_feat.device
        T = user_hist.shape[1]
        P = chunk_users * k
        self._ws = ops.din_workspace(din, P, T, dev, batch_size=batch_size)
        self._buf = None
        self._topk_ws = None
        self._validated = False

    def recall(self, users):
        """Exact top-(k+1) rows / scores of every user (rank 0 included)."""
        n = users.shape[0]
        nb = ops._lib.lib().nrk_ip_topk_workspace_bytes(n, self.cat.n, self.cat.d, self.k + 1)
        if self._topk_ws is None or self._topk_ws.numel() < nb:
            self._topk_ws = torch.empty(nb, dtype=torch.uint8, device=users.device)
        return ops.ip_topk(users, self.cat, self.k + 1, workspace=self._topk_ws)

    def rank(self, rec_scores, rec_rows, probs=None):
        """DIN probabilities of the k recalled pairs per user ([n_users * k],
        user-major) and their candidate rows."""
        n = rec_rows.shape[0]
        dev = rec_rows.device
        if probs is None:
            probs = torch.empty(n * self.k, dtype=torch.float32, device=dev)
        cand = torch.empty(n * self.k, dtype=torch.int32, device=dev)
        for u0 in range(0, n, self.chunk):
            nu = min(self.chunk, n - u0)
            a = ops.din_assemble(rec_rows, rec_scores, self.user_feat, self.item_feat, self.user_hist,
                                 self.hist_len, u0, nu, k_use=self.k, skip=1, n_ctx=self.n_ctx,
                                 ctx_bins=self.ctx_bins, seed=self.seed,
                                 out=self._buf if nu == self.chunk else None)
            if nu == self.chunk:
                self._buf = a
            P = nu * self.k
            sl = slice(u0 * self.k, u0 * self.k + P)
            if not self._validated:
                ops.din_validate(self.din, a["user"][:P], a["item"][:P], a["hist"][:P], a["ctx"][:P])
                self._validated = True
            ops.din_forward(self.din, a["user"][:P], a["item"][:P], a["hist"][:P], a["ctx"][:P], a["mask"][:P],
                            workspace=self._ws, out=probs[sl], validate=False,
                            batch_size=self.bs if P > self.bs else None)
            cand[sl] = a["cand"][:P]
        return probs, cand

    def __call__(self, users):
        s, r = self.recall(users)
        return self.rank(s, r)
