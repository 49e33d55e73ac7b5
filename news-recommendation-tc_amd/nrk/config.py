"""Hyper-parameters of the hot path, with the reference's field names and
defaults (src/utils/config.py:7-168).  Unlike the reference, constructing a
config has no side effects: the reference makes ``data/raw`` and ``temp``
under the project root in __post_init__ (config.py:60-71, :141-161); here the
paths are only derived, and the caller's pipeline owns the directories.

``RankConfig`` carries the artifact paths DINRanker.load / load_model read
(config.py:106-112, :146-158): ``save_path`` = <_project_root>/temp unless
given, every feature file under it."""
import os
from dataclasses import dataclass, field
from typing import List, Optional


@dataclass
class RecallConfig:
    save_path: str = field(default_factory=lambda: os.path.join(os.getcwd(), "temp"))
    itemcf_sim_item_topk: int = 20
    itemcf_recall_num: int = 20
    itemcf_hot_topk: int = 20
    embedding_topk: int = 20
    embedding_dim: int = 64
    youtubednn_seq_max_len: int = 30
    youtubednn_embedding_dim: int = 16
    youtubednn_hidden_units: List[int] = field(default_factory=lambda: [64, 16])
    youtubednn_topk: int = 20
    fuse_topk: int = 30
    loc_alpha: float = 1.0
    loc_alpha_reverse: float = 0.7
    loc_beta: float = 0.9
    time_decay_alpha: float = 0.7
    created_time_alpha: float = 0.8
    random_seed: int = 23


@dataclass
class RankConfig:
    # general settings (config.py:95-97)
    debug_mode: bool = False
    offline: bool = True
    random_seed: int = 23
    # paths (config.py:100-112): derived from _project_root / save_path
    _project_root: str = field(default_factory=os.getcwd)
    save_path: Optional[str] = None
    # DIN model hyperparameters (config.py:115-119)
    din_embedding_dim: int = 32
    din_attention_hidden_units: List[int] = field(default_factory=lambda: [36])
    din_mlp_hidden_units: List[int] = field(default_factory=lambda: [200, 80])
    din_activation: str = "dice"
    din_seq_max_len: int = 30
    # training / loader settings (config.py:122-136; training is out of scope,
    # the fields keep a reference config dict loadable)
    batch_size: int = 256
    learning_rate: float = 0.001
    epochs: int = 4
    num_workers: int = 4
    pin_memory: bool = True
    enable_negative_sampling: bool = True
    negative_positive_ratio: float = 10.0

    def __post_init__(self):
        """The reference's path layout (config.py:141-158), without makedirs."""
        self.data_path = os.path.join(self._project_root, "data", "raw")
        if self.save_path is None:
            self.save_path = os.path.join(self._project_root, "temp")
        self.main_features_path = os.path.join(self.save_path, "main_features.csv")
        self.user_profile_dict_path = os.path.join(self.save_path, "user_profile_dict.pkl")
        self.item_features_dict_path = os.path.join(self.save_path, "item_features_dict.pkl")
        self.user_history_dict_path = os.path.join(self.save_path, "user_history_dict.pkl")
        self.feature_lists_path = os.path.join(self.save_path, "feature_lists.pkl")
        self.discretizers_path = os.path.join(self.save_path, "discretizers.pkl")

    @classmethod
    def from_dict(cls, config_dict: dict) -> "RankConfig":
        return cls(**{k: v for k, v in config_dict.items() if k in cls.__annotations__})

    def to_dict(self) -> dict:
        return self.__dict__
