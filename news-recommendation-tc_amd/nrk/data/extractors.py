"""Host-side input contracts of the ItemCF path, restating
src/data/extractors.py (the reference's pandas code) in array form.

``user_item_time_csr`` == UserFeatureExtractor.get_user_item_time_dict
(extractors.py:10-36): ``click_df.sort_values("click_timestamp")`` (pandas'
default quicksort -- NOT stable, so equal timestamps keep whatever order that
sort produces; we call the same sort) then ``groupby("user_id")`` (ascending
user ids, group rows in sorted-frame order).

``item_created_time`` == ItemFeatureExtractor.get_item_info_dict's
created-time dict (extractors.py:136-164): sklearn MinMaxScaler over the
whole article table.
"""
from __future__ import annotations

import numpy as np


def user_item_time_csr(click_df):
    """-> (user ids [U] asc, offsets [U+1], raw item ids [N], ts [N])."""
    df = click_df.sort_values("click_timestamp")
    u = df["user_id"].to_numpy()
    order = np.argsort(u, kind="stable")  # groupby keeps the sorted frame's row order
    u = u[order]
    items = df["click_article_id"].to_numpy()[order]
    ts = df["click_timestamp"].to_numpy()[order]
    users, starts = np.unique(u, return_index=True)
    offsets = np.append(starts, len(u)).astype(np.int64)
    return users.astype(np.int64), offsets, items.astype(np.int64), ts.astype(np.int64)


def csr_to_dict(users, offsets, items, ts):
    """The reference's ``{user: [(item, ts), ...]}`` view of the CSR."""
    return {int(u): list(zip(items[offsets[n]:offsets[n + 1]].tolist(), ts[offsets[n]:offsets[n + 1]].tolist()))
            for n, u in enumerate(users)}


def item_created_time(item_info_df):
    """{item_id: MinMax-scaled created_at_ts} (extractors.py:149-163)."""
    from sklearn.preprocessing import MinMaxScaler

    x = MinMaxScaler().fit_transform(item_info_df[["created_at_ts"]])[:, 0]
    return dict(zip(item_info_df["click_article_id"], x))


def item_topk_click(click_df, k=50):
    """ItemFeatureExtractor.get_item_topk_click (extractors.py:166-168)."""
    return click_df["click_article_id"].value_counts().index[:k].tolist()


def youtubednn_histories(user_id, click_article_id, seq_max_len: int = 30):
    """User-tower inputs exactly as youtubednn_recaller.py:425-443 builds them.

    Users are label-encoded (sorted raw ids -> 0..U-1); each user's history is
    their rows in ``click_df`` row order (groupby, not time-sorted, :432-436)
    with item ids label-encoded; the FIRST ``seq_max_len`` are kept and the
    rest zero-padded (collate_fn :63-70).  Returns (uid[U], hist[U,T],
    hist_len[U], item_raw_ids (encoded -> raw), first_occurrence item order).
    """
    u_raw = np.asarray(user_id, np.int64)
    i_raw = np.asarray(click_article_id, np.int64)
    u_classes, u_enc = np.unique(u_raw, return_inverse=True)
    i_classes, i_enc = np.unique(i_raw, return_inverse=True)
    # stable sort by encoded user keeps click_df row order inside a user
    order = np.argsort(u_enc, kind="stable")
    ue = u_enc[order]
    ie = i_enc[order]
    n_u = len(u_classes)
    counts = np.bincount(ue, minlength=n_u)
    offs = np.concatenate([[0], np.cumsum(counts)[:-1]])
    pos = np.arange(len(ue)) - np.repeat(offs, counts)
    keep = pos < seq_max_len
    hist = np.zeros((n_u, seq_max_len), dtype=np.int64)
    hist[ue[keep], pos[keep]] = ie[keep]
    hist_len = np.minimum(counts, seq_max_len).astype(np.int64)
    _, first_idx = np.unique(i_enc, return_index=True)
    item_profile = i_enc[np.sort(first_idx)]  # encoded ids, first-occurrence order
    return (
        np.arange(n_u, dtype=np.int64),
        hist,
        hist_len,
        i_classes.astype(np.int64),
        item_profile.astype(np.int64),
    )
