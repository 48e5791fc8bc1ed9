"""Sparse parameter-server configuration.

The BoxPS config file format is closed (``InitializeGPUAndLoadModel(conf, ...)``
at reference ``paddle/fluid/framework/fleet/box_wrapper.cc:1201-1242``); the
knobs it carries are visible through the HeterPS analogue
(``heter_ps/optimizer_conf.h:20-124``) and the PSCore CTR accessor
(``distributed/ps/table/ctr_accessor.{h,cc}``).  We expose them as one typed
config that serialises to YAML/JSON.
"""
from __future__ import annotations

import dataclasses
import json
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import yaml


@dataclass
class SparseSGDConfig:
    """Adagrad-family sparse optimizer (defaults: heter_ps/optimizer_conf.h:20-45)."""

    nonclk_coeff: float = 0.1
    clk_coeff: float = 1.0
    min_bound: float = -10.0
    max_bound: float = 10.0
    learning_rate: float = 0.05
    initial_g2sum: float = 3.0
    initial_range: float = 0.0
    mf_create_thresholds: float = 10.0
    mf_learning_rate: float = 0.05
    mf_initial_g2sum: float = 3.0
    mf_initial_range: float = 1e-4
    mf_min_bound: float = -10.0
    mf_max_bound: float = 10.0
    nodeid_slot: float = 9008.0
    feature_learning_rate: float = 0.05
    use_feature_lr: int = 0

    def to_native(self, mod):
        c = mod.SparseSGDConfig()
        for f in dataclasses.fields(self):
            setattr(c, f.name, getattr(self, f.name))
        return c


@dataclass
class ShrinkConfig:
    """Decay / eviction (ctr_accessor.cc:63-80)."""

    show_click_decay_rate: float = 0.98
    delete_threshold: float = 0.8
    delete_after_unseen_days: float = 30.0
    nonclk_coeff: float = 0.1
    clk_coeff: float = 1.0

    def to_native(self, mod):
        c = mod.ShrinkConfig()
        for f in dataclasses.fields(self):
            setattr(c, f.name, getattr(self, f.name))
        return c


@dataclass
class SaveConfig:
    """xbox base/delta filters (ctr_accessor.cc:102-144)."""

    base_threshold: float = 1.5
    delta_threshold: float = 0.25
    delta_keep_days: float = 16.0
    embedx_threshold: float = 10.0


@dataclass
class TierConfig:
    """Embedding cache tiers: HBM working set -> pinned host -> SSD."""

    hbm_capacity: int = 0  # feature slots in HBM per GPU (0 = auto)
    load_factor: float = 0.8
    host_enabled: bool = True
    ssd_path: Optional[str] = None
    ssd_spill_threshold: int = 0  # host-tier row cap: rows of the oldest passes spill to SSD beyond it (0 = off)
    spill_unseen_days: float = 1.0  # host rows unseen this long move to the SSD tier at EndPass


@dataclass
class PSConfig:
    embedx_dim: int = 8
    expand_embed_dim: int = 0
    feature_type: int = 0  # 0 normal, 1 quant int16 embedx, 2 variable/expand
    pull_embedx_scale: float = 1.0
    # sparse optimizer of the GPU PS rows: "adagrad" (default) or "adam"
    # (SparseAdam, heter_ps/optimizer.cuh.h:147-330)
    sparse_optimizer: str = "adagrad"
    adam_beta1: float = 0.9
    adam_beta2: float = 0.999
    adam_epsilon: float = 1e-8
    # route fp32 Adagrad through the row-codec kernels too (testing)
    force_codec: bool = False
    sgd: SparseSGDConfig = field(default_factory=SparseSGDConfig)
    shrink: ShrinkConfig = field(default_factory=ShrinkConfig)
    save: SaveConfig = field(default_factory=SaveConfig)
    tier: TierConfig = field(default_factory=TierConfig)
    slot_lr: Dict[str, float] = field(default_factory=dict)

    @staticmethod
    def from_dict(d: dict) -> "PSConfig":
        d = dict(d or {})
        sub = {
            "sgd": SparseSGDConfig,
            "shrink": ShrinkConfig,
            "save": SaveConfig,
            "tier": TierConfig,
        }
        kw = {}
        for k, v in d.items():
            if k in sub and isinstance(v, dict):
                kw[k] = sub[k](**v)
            else:
                kw[k] = v
        return PSConfig(**kw)

    @staticmethod
    def load(path: str) -> "PSConfig":
        with open(path) as f:
            text = f.read()
        if path.endswith(".json"):
            return PSConfig.from_dict(json.loads(text))
        return PSConfig.from_dict(yaml.safe_load(text))

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)


def feature_pull_offsets(embedx_dim: int, expand_dim: int = 0) -> Dict[str, int]:
    """FeaturePullOffset equivalent (box_wrapper.cc:1140-1181)."""
    return {
        "show": 0,
        "clk": 1,
        "embed_w": 2,
        "embedx": 3,
        "embedx_size": embedx_dim,
        "expand": 3 + embedx_dim,
        "expand_size": expand_dim,
        "cvm_offset": 3,
        "pull_size": 3 + embedx_dim + expand_dim,
    }


def feature_push_offsets(embedx_dim: int, expand_dim: int = 0) -> Dict[str, int]:
    """FeaturePushOffset equivalent."""
    return {
        "slot": 0,
        "show": 1,
        "clk": 2,
        "embed_g": 3,
        "embedx_g": 4,
        "expand_g": 4 + embedx_dim,
        "push_size": 4 + embedx_dim + expand_dim,
    }


def row_layout(dim: int) -> Dict[str, int]:
    """Mirror of pbx::make_row_layout (csrc/common/pbx_common.h)."""
    eg = 3 + dim
    l = {
        "show": 0,
        "click": 1,
        "embed_w": 2,
        "embedx": 3,
        "embed_g2sum": eg,
        "embedx_g2sum": eg + 1,
        "delta_score": eg + 2,
        "slot": eg + 3,
        "unseen_days": eg + 4,
        "mf_size": eg + 5,
    }
    used = l["mf_size"] + 1
    l["stride"] = (used + 3) & ~3
    return l


PULL_HEAD = 3


def pull_width(dim: int) -> int:
    return 3 + dim


def push_width(dim: int) -> int:
    return 4 + dim


def padded(n: int, m: int = 4) -> int:
    return (n + m - 1) // m * m


__all__: List[str] = [
    "SparseSGDConfig",
    "ShrinkConfig",
    "SaveConfig",
    "TierConfig",
    "PSConfig",
    "feature_pull_offsets",
    "feature_push_offsets",
    "row_layout",
    "pull_width",
    "push_width",
    "padded",
]
