"""CPU: the host-side input contracts (nrk/data/extractors.py) against the
dicts the reference's own extractors produced for the ItemCF fixture
(tests/golden/itemcf_small.npz, written by executing
src/data/extractors.py:136-169 in tests/golden/make_golden.py):
created-time MinMax dict and the top-50 hot items."""
import numpy as np
import pandas as pd


def _articles():
    from nrk.data import synth

    art = synth.make_articles(5000, seed=7)  # the fixture's article table (make_golden.gen_itemcf)
    return pd.DataFrame({"click_article_id": art.article_id * 7 + 11, "category_id": art.category_id,
                         "words_count": art.words_count, "created_at_ts": art.created_at_ts})


def test_item_created_time_matches_reference(golden):
    from nrk.data.extractors import item_created_time

    g = golden("itemcf_small")
    d = item_created_time(_articles())
    assert sorted(d) == g["created_ids"].tolist()
    assert [d[i] for i in g["created_ids"].tolist()] == g["created_vals"].tolist()


def test_item_topk_click_matches_reference(golden):
    from nrk.data.extractors import item_topk_click

    g = golden("itemcf_small")
    click_df = pd.DataFrame({"user_id": g["click_user"], "click_article_id": g["click_item"],
                             "click_timestamp": g["click_ts"]})
    assert item_topk_click(click_df, k=50) == g["hot"].tolist()


def test_user_item_time_csr_matches_reference(golden):
    from nrk.data.extractors import user_item_time_csr

    g = golden("itemcf_small")
    click_df = pd.DataFrame({"user_id": g["click_user"], "click_article_id": g["click_item"],
                             "click_timestamp": g["click_ts"]})
    users, offs, items, ts = user_item_time_csr(click_df)
    assert np.array_equal(users, g["uit_users"]) and np.array_equal(offs, g["uit_offsets"])
    assert np.array_equal(items, g["uit_items"]) and np.array_equal(ts, g["uit_ts"])
