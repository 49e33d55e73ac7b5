"""Synthetic Tianchi-shaped data.

The real Tianchi CSVs are not available offline (README.md:11-16 of the
reference), so every test, fixture and benchmark runs on click logs and
article tables generated here with the shape the reference's README quotes
(README.md:20-29): 250,000 users (200k train with >= 2 clicks, 50k test with
>= 1 click), 364,047 articles, Zipf(1.1) item popularity, strictly increasing
per-user millisecond timestamps (so the reference's non-stable
``sort_values("click_timestamp")`` in extractors.py:20 is deterministic).

Everything is plain numpy and seeded; nothing here imports the reference.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

N_USERS = 250_000
N_TRAIN_USERS = 200_000
N_ITEMS = 364_047
TS_BASE = 1_507_029_570_190  # ms, README-era click timestamps
CREATED_MAX = 1_506_600_000_000


@dataclass
class ClickLog:
    """Columns of ``train_click_log.csv`` that the hot path reads.

    Rows are grouped by user (ascending raw user id) and, inside a user, in
    click-time order -- i.e. ``click_df`` row order as the loaders hand it
    over (loaders.py:36-78).
    """

    user_id: np.ndarray          # int64 [n_clicks]
    click_article_id: np.ndarray  # int64 [n_clicks]
    click_timestamp: np.ndarray   # int64 [n_clicks] ms

    def __len__(self) -> int:
        return int(self.user_id.shape[0])

    def to_pandas(self):
        import pandas as pd

        return pd.DataFrame(
            {
                "user_id": self.user_id,
                "click_article_id": self.click_article_id,
                "click_timestamp": self.click_timestamp,
            }
        )


@dataclass
class Articles:
    """Columns of ``articles.csv`` (README.md:14)."""

    article_id: np.ndarray     # int64 [n_items]
    category_id: np.ndarray    # int64
    created_at_ts: np.ndarray  # int64 ms
    words_count: np.ndarray    # int64


def make_articles(n_items: int = N_ITEMS, seed: int = 23) -> Articles:
    rng = np.random.default_rng(seed)
    created = CREATED_MAX - rng.integers(0, 50_000_000_000, size=n_items, dtype=np.int64)
    return Articles(
        article_id=np.arange(n_items, dtype=np.int64),
        category_id=rng.integers(0, 461, size=n_items, dtype=np.int64),
        created_at_ts=created,
        words_count=rng.integers(0, 6691, size=n_items, dtype=np.int64),
    )


def make_click_log(
    n_users: int = N_USERS,
    n_items: int = N_ITEMS,
    n_train_users: int | None = None,
    seed: int = 23,
    max_len: int = 250,
    zipf_a: float = 1.1,
) -> ClickLog:
    """Tianchi-shaped click log.

    Train users: L = 1 + Geometric(p) (mean 5.56, >= 2); test users:
    L = Geometric(p) (mean 10.36, >= 1); capped at ``max_len``.  Items are
    Zipf(zipf_a) ranks mapped through a random permutation of article ids.
    """
    if n_train_users is None:
        n_train_users = int(round(n_users * N_TRAIN_USERS / N_USERS))
    rng = np.random.default_rng(seed)
    n_test = n_users - n_train_users
    len_tr = 1 + rng.geometric(1.0 / 4.56, size=n_train_users)
    len_te = rng.geometric(1.0 / 10.36, size=n_test)
    lens = np.minimum(np.concatenate([len_tr, len_te]), max_len).astype(np.int64)
    n = int(lens.sum())
    users = np.repeat(np.arange(n_users, dtype=np.int64), lens)
    perm = rng.permutation(n_items).astype(np.int64)
    ranks = (rng.zipf(zipf_a, size=n).astype(np.int64) - 1) % n_items
    items = perm[ranks]
    # strictly increasing per-user timestamps: user start in a 16-day window,
    # Exp(30 min) gaps, at least 1 ms apart.
    start = TS_BASE + rng.integers(0, 16 * 86_400_000, size=n_users, dtype=np.int64)
    gaps = np.maximum(1, rng.exponential(1_800_000.0, size=n).astype(np.int64))
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    csum = np.cumsum(gaps)
    first = csum[offs]
    ts = np.repeat(start, lens) + csum - np.repeat(first, lens)
    return ClickLog(users, items, ts.astype(np.int64))


def user_lists(log: ClickLog):
    """CSR view of a click log: (user ids, offsets, items, timestamps).

    Equivalent to ``UserFeatureExtractor.get_user_item_time_dict``
    (extractors.py:10-36) for a log whose per-user timestamps are strictly
    increasing: users in ascending id order, each list in click-time order.
    """
    order = np.lexsort((log.click_timestamp, log.user_id))
    u = log.user_id[order]
    it = log.click_article_id[order]
    ts = log.click_timestamp[order]
    uniq, starts = np.unique(u, return_index=True)
    offsets = np.append(starts, len(u)).astype(np.int64)
    return uniq.astype(np.int64), offsets, it.astype(np.int64), ts.astype(np.int64)


def minmax_created(art: Articles) -> np.ndarray:
    """``created_at_ts`` MinMax-scaled exactly as sklearn does it
    (extractors.py:136-164): ``X * scale_ + min_`` in float64."""
    x = art.created_at_ts.astype(np.float64)
    lo, hi = x.min(), x.max()
    rng_ = hi - lo
    scale = 1.0 / (rng_ if rng_ != 0 else 1.0)
    min_ = 0.0 - lo * scale
    out = x * scale
    out += min_
    return out


def youtubednn_histories(log: ClickLog, seq_max_len: int = 30):
    """extractors.youtubednn_histories over a ClickLog (kept for the tests)."""
    from .extractors import youtubednn_histories as _h

    return _h(log.user_id, log.click_article_id, seq_max_len)


def din_batch(
    n: int,
    seq_len: int = 50,
    user_vocab=(200, 5000, 6, 200000, 3000),
    item_vocab=(462, 3000, 300000, 1500),
    ctx_vocab=(11,) * 16,
    pad_frac: float = 0.2,
    seed: int = 23,
):
    """DIN index tensors for config 3: uniform indices,
    ``hist_len ~ U[1, T]`` with ``pad_frac`` all-pad rows (test users),
    left-aligned prefix masks as collate_fn builds them (DIN.py:476-490)."""
    rng = np.random.default_rng(seed)
    user = np.stack([rng.integers(0, v, size=n) for v in user_vocab], 1).astype(np.int32)
    item = np.stack([rng.integers(0, v, size=n) for v in item_vocab], 1).astype(np.int32)
    ctx = np.stack([rng.integers(0, v, size=n) for v in ctx_vocab], 1).astype(np.int32)
    hl = rng.integers(1, seq_len + 1, size=n)
    hl[rng.random(n) < pad_frac] = 0
    hist = np.stack(
        [rng.integers(0, v, size=(n, seq_len)) for v in item_vocab], 2
    ).astype(np.int32)
    mask = (np.arange(seq_len)[None, :] < hl[:, None]).astype(np.float32)
    hist = hist * (mask[:, :, None] > 0)  # padded positions carry index 0
    return {
        "user": user,
        "item": item,
        "hist": hist.astype(np.int32),
        "ctx": ctx,
        "mask": mask,
        "hist_len": hl.astype(np.int32),
    }
