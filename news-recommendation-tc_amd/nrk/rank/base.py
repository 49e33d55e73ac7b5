"""Ranker plugin contract: a restatement of src/rank/base.py:10-117.

``BaseRanker(config)`` with ``load()``, ``train()`` and ``predict()``.  The
reference's generic ``load`` reads train / test feature sets and history
dicts from ``config.train_set_path`` etc. -- fields ``RankConfig`` does not
define, so it raises there; ``DINRanker``
overrides it (DIN.py:529-558), as the reference's does.  Training is out of
scope for this hot path: ``train()`` stays the reference's no-op.
"""
from __future__ import annotations

import os
import pickle
from abc import ABC


def load_pickle(path):
    """PersistenceManager.load_pickle (src/utils/persistence.py): the
    pipeline's own artifacts (the feature step's and save_model's outputs),
    read with the reference's loader and trust model."""
    with open(path, "rb") as f:
        return pickle.load(f)


class BaseRanker(ABC):
    def __init__(self, config) -> None:
        self.config = config

    def load(self, load_din_specific: bool = True):
        """rank/base.py:14-61: train / test sets and history dicts (+ the DIN
        feature groups)."""
        import pandas as pd

        for attr, path_attr, reader in (("train_set", "train_set_path", pd.read_csv),
                                        ("test_set", "test_set_path", pd.read_csv),
                                        ("train_history_dict", "train_history_dict_path", load_pickle),
                                        ("test_history_dict", "test_history_dict_path", load_pickle)):
            path = getattr(self.config, path_attr)  # AttributeError on RankConfig, as in the reference
            if not os.path.exists(path):
                raise FileNotFoundError(f"{attr} not found at {path}")
            setattr(self, attr, reader(path))
        if load_din_specific:
            self._load_din_specific_data()

    def _load_din_specific_data(self):
        """rank/base.py:63-111: missing files give empty lists / dict."""
        for attr, path_attr, empty in (("user_profile_features", "user_profile_features_path", []),
                                       ("item_features", "item_features_path", []),
                                       ("context_features", "context_features_path", []),
                                       ("article_info_dict", "article_info_dict_path", {})):
            path = getattr(self.config, path_attr)
            setattr(self, attr, load_pickle(path) if os.path.exists(path) else empty)

    def train(self):
        pass

    def predict(self):
        pass
