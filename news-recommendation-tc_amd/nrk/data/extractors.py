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
