"""Fused recall -> rank on one GPU (BASELINE config 5, one rank's share).

The reference runs recall and rank as separate host pipelines joined by
pickles and CSVs (recall_pipeline.py -> feature_pipeline -> rank_pipeline.py).
Here the recalled pairs never leave HBM:

1. exact top-(k+1) inner-product recall of the rank's users over the
   replicated catalog (nrk_ip_topk, the YoutubeDNN recall of config 2), rank
   0 dropped as youtubednn_recaller.py:524 does;
2. per chunk of users, the DIN inputs of every recalled pair are assembled on
   the device (nrk_din_assemble: profile / candidate / last-T history
   indices) and the 16 context features are computed and encoded there too
   (nrk_ctx_features: the reference's feature_extractor.py:440-723 columns
   through the fitted binning + label codes; without ``ctx`` tables the
   synthetic score / hash bins of nrk_din_assemble stand in);
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
                 ctx_bins: int = 10, seed: int = 23, ctx=None):
        """``ctx`` = (features.CtxTables, features.CtxSpec) for the real
        context features (tables indexed by user row / catalog row)."""
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
        self.ctx = ctx
        if ctx is not None:
            self.n_ctx = 1 + 3 * ctx[0].last_n + 6
        self._validate_tables()

    def _validate_tables(self):
        """Every index the assembly / DIN kernels will gather, checked once
        here against the DIN vocabularies and table sizes (the kernels do not
        bounds-check), so no chunk needs a per-call check."""
        p = self.din
        if self.n_ctx != p.n_ctx or self.user_feat.shape[1] != p.n_user or self.item_feat.shape[1] != p.n_item:
            raise ValueError("feature tables do not match the DIN feature lists")
        if self.item_feat.shape[0] != self.cat.n:
            raise ValueError("item_feat needs one row per catalog row")
        for t, off in ((self.user_feat, 0), (self.item_feat, p.n_user)):
            if t.numel():
                mx = t.amax(0).cpu().tolist()
                if int(t.min()) < 0 or any(m >= p.vocab[off + f] for f, m in enumerate(mx)):
                    raise ValueError("feature table index out of its embedding table")
        T = self.user_hist.shape[1]
        if self.user_hist.numel() and (int(self.user_hist.min()) < 0 or
                                       int(self.user_hist.max()) >= self.item_feat.shape[0]):
            raise ValueError("user_hist rows out of [0, n_items)")
        if self.hist_len.numel() and (int(self.hist_len.min()) < 0 or int(self.hist_len.max()) > T):
            raise ValueError("hist_len out of [0, T]")
        cv = p.vocab[p.n_user + p.n_item:]
        if self.ctx is not None:
            spec = self.ctx[1]
            for f, sp in enumerate(spec.specs):
                codes = list(sp.lut[:sp.n_lut]) if sp.kind == 0 else list(sp.codes[:sp.n_vals])
                if max(codes + [0]) >= cv[f]:
                    raise ValueError(f"context spec code out of the {spec.names[f]} embedding table")
        elif any(self.ctx_bins + 1 > v for v in cv):
            raise ValueError("ctx_bins + 1 exceeds a context vocabulary")

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
                                 self.hist_len, u0, nu, k_use=self.k, skip=1,
                                 n_ctx=0 if self.ctx is not None else self.n_ctx,
                                 ctx_bins=self.ctx_bins, seed=self.seed,
                                 out=self._buf if nu == self.chunk else None, validate=False,
                                 ctx_width=self.n_ctx)
            if nu == self.chunk:
                self._buf = a
            P = nu * self.k
            sl = slice(u0 * self.k, u0 * self.k + P)
            if self.ctx is not None:
                self._context(a, rec_scores, u0, nu)
            ops.din_forward(self.din, a["user"][:P], a["item"][:P], a["hist"][:P], a["ctx"][:P], a["mask"][:P],
                            workspace=self._ws, out=probs[sl], validate=False,
                            batch_size=self.bs if P > self.bs else None)
            cand[sl] = a["cand"][:P]
        return probs, cand

    def _context(self, a, rec_scores, u0, nu):
        """The 16 context codes of the chunk's pairs (nrk_ctx_features),
        written into the assembled ctx block: one group per user, the recall
        score of column c + 1 as the pair's score."""
        from .features import ctx_features

        tables, spec = self.ctx
        dev = rec_scores.device
        k = self.k
        goff = torch.arange(0, (nu + 1) * k, k, dtype=torch.int64, device=dev)
        guser = torch.arange(u0, u0 + nu, dtype=torch.int32, device=dev)
        score = rec_scores[u0:u0 + nu, 1:k + 1].to(torch.float64).reshape(-1).contiguous()
        P = nu * k
        _, codes = ctx_features(tables, None, a["cand"][:P], score, spec, raw=False, groups=(goff, guser, None),
                                out_codes=a["ctx"][:P])
        return codes

    def __call__(self, users):
        s, r = self.recall(users)
        return self.rank(s, r)
