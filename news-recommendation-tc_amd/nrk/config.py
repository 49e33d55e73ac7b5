"""Hyper-parameters of the hot path, with the reference's field names and
defaults (src/utils/config.py:7-168).  Unlike the reference, constructing a
config has no side effects (the reference makes directories in
__post_init__, config.py:60-71)."""
import os
from dataclasses import dataclass, field
from typing import List


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
    save_path: str = field(default_factory=lambda: os.path.join(os.getcwd(), "temp"))
    din_embedding_dim: int = 32
    din_attention_hidden_units: List[int] = field(default_factory=lambda: [36])
    din_mlp_hidden_units: List[int] = field(default_factory=lambda: [200, 80])
    din_activation: str = "dice"
    din_seq_max_len: int = 30
    batch_size: int = 256
    random_seed: int = 23
