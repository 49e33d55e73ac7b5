"""Final per-user ranking: drop-in for RankPipeline.rank_and_recommend
(src/pipeline/rank_pipeline.py:143-191).

The reference assigns the DIN probabilities to ``main_df["rank_score"]``
(a float32 column, :163-164), then for every user (``groupby("user_id")``,
ascending ids) keeps ``group.nlargest(top_k, "rank_score")``: score
descending, ties in row order (``keep="first"``), NaN scores after all
numbers (in row order), and
returns ``{str(user_id): [(str(item_id), float(score)), ...]}`` (:166-172),
optionally pickled (:182-184).  Quirk kept: the rows come from
``iterrows()``, whose Series takes the common dtype of item_id and the
float32 score, so integer item ids are formatted as floats ("123.0").

Tie order: for a user with more than top_k rows nlargest's selection path
orders exact score ties by row (mergesort) and so does this kernel; for a
user with at most top_k rows pandas falls back to
``sort_values(kind="quicksort")``, whose numpy SIMD argsort orders exact
ties in a CPU-dependent way -- here they stay in row order (same items and
scores, tie order unpinned).

Here the grouping is a stable host argsort of the user column (the data
prep the reference does in pandas); the per-user top-k by (score desc, row
asc) runs on the GPU through nrk_itemcf_topn (one wave per user, running
top-64 bitonic merge; top_k > 64: a running top-K in LDS).  top_k <= 2048.
"""
from __future__ import annotations

import pickle
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from .. import ops


def rank_topk(user_ids, probs, top_k: int = 10, device="cuda"):
    """Per-user top-k rows.  Returns (users [G] ascending, rows [G, top_k]
    int32 into the inputs (-1 padded), scores [G, top_k] float32, counts [G])."""
    if not (1 <= top_k <= ops.CF_TOPK_MAX):
        raise NotImplementedError(f"top_k must be in [1, {ops.CF_TOPK_MAX}]")
    user_ids = np.asarray(user_ids)
    p = probs.detach().float().cpu().numpy() if torch.is_tensor(probs) else np.asarray(probs, np.float32)
    if len(p) != len(user_ids):
        raise ValueError("probs must have one entry per main_df row")
    order = np.argsort(user_ids, kind="stable")
    users, start = np.unique(user_ids[order], return_index=True)
    off = np.append(start, len(order)).astype(np.int64)
    d = torch.device(device)
    rows = torch.from_numpy(order.astype(np.int32)).to(d)
    # nlargest ranks NaN after every number, in row order: NaN -> -inf (probabilities are never -inf)
    v = p[order].astype(np.float64)
    v[np.isnan(v)] = -np.inf
    oc, _, cnt = ops.itemcf_topn(torch.from_numpy(off).to(d), rows, torch.from_numpy(v).to(d),
                                 rows.to(torch.int64), top_k)
    oc, cnt = oc.cpu().numpy(), cnt.cpu().numpy()
    scores = np.where(oc >= 0, p[np.maximum(oc, 0)], np.float32(0)).astype(np.float32)
    return users, oc, scores, cnt


def rank_and_recommend(main_df, probs, top_k: int = 10,
                       save_path: Optional[str] = None, device="cuda") -> Dict[str, List[Tuple[str, float]]]:
    """rank_pipeline.py:143-191 over ``main_df`` (user_id, item_id columns)
    and the ranker's probabilities, positional to main_df's rows."""
    users, rows, scores, cnt = rank_topk(main_df["user_id"].to_numpy(), probs, top_k, device)
    items = main_df["item_id"].to_numpy()
    # iterrows() row dtype = common type of (item_id, float32 rank_score)
    as_float = np.issubdtype(np.result_type(items.dtype, np.float32), np.floating)
    fmt = (lambda it: str(float(it))) if as_float else str
    rec: Dict[str, List[Tuple[str, float]]] = {}
    for g, u in enumerate(users.tolist()):
        m = int(cnt[g])
        rec[str(u)] = [(fmt(it), float(s)) for it, s in zip(items[rows[g, :m]].tolist(), scores[g, :m].tolist())]
    if save_path:
        with open(save_path, "wb") as f:
            pickle.dump(rec, f)
    return rec
