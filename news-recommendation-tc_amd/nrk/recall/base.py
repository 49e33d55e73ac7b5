"""Recaller plugin interface -- same contract as the reference's
src/recall/base.py:6-57 (raw ids in/out, scores as Python floats sorted desc)."""
from abc import ABC, abstractmethod
from typing import Dict, List, Tuple


class BaseRecaller(ABC):
    def __init__(self, config):
        self.config = config

    @abstractmethod
    def recall(self, user_id: int, topk: int = 10) -> List[Tuple[int, float]]:
        """Recall top-k items for one user: [(item_id, score), ...]."""

    def batch_recall(self, user_ids: List[int], topk: int = 10) -> Dict[int, List[Tuple[int, float]]]:
        """Recall for many users (reference: a per-user loop, recall/base.py:37-40;
        GPU recallers override this with one batched device call)."""
        return {u: self.recall(u, topk) for u in user_ids}

    def _filter_history(self, candidates, history_items: set):
        return [(item, score) for item, score in candidates if item not in history_items]
