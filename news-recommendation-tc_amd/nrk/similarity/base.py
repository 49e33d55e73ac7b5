"""Similarity plugin interface -- reference src/similarity/base.py:8-40."""
import os
import pickle
from abc import ABC, abstractmethod
from typing import Any, Dict


class BaseSimilarityCalculator(ABC):
    def __init__(self, config):
        self.config = config
        self.save_path = getattr(config, "save_path", ".")
        self.similarity_matrix = {}

    @abstractmethod
    def calculate(self, data: Any) -> Dict:
        pass

    def save(self, filename: str) -> None:
        if not self.similarity_matrix:
            raise ValueError("Similarity matrix is empty. Call calculate() first.")
        with open(os.path.join(self.save_path, filename), "wb") as f:
            pickle.dump(self.similarity_matrix, f)

    def get_similarity_matrix(self) -> Dict:
        return self.similarity_matrix

    def is_calculated(self) -> bool:
        return len(self.similarity_matrix) > 0
