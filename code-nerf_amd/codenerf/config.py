"""The reference's YAML configs (config/*.yml) as attribute access, for the build's drivers.

train.py:198-201 builds ``CfgNode(vars(args), new_allowed=True)`` and merges the YAML file into
it; the drivers then read ``cfg.experiment.*``, ``cfg.dataset.*``, ``cfg.models.*``,
``cfg.optimizer.*``, ``cfg.nerf.*`` and the CLI keys ``gpus`` / ``is_distributed`` /
``load_checkpoint``.  ``load_config`` reads the same file with ``yaml.safe_load`` into nested
attribute dicts holding exactly those keys (the yacs machinery -- freezing, key validation,
``dump`` -- is not rebuilt; SURVEY.md section 2 marks it out of scope).
"""
from __future__ import annotations

from typing import Any, Dict, Optional

import yaml


class Cfg(dict):
    """A dict whose keys are also attributes (nested dicts become Cfg)."""

    def __init__(self, d: Optional[Dict[str, Any]] = None, **kw):
        super().__init__()
        for k, v in dict(d or {}, **kw).items():
            self[k] = Cfg(v) if isinstance(v, dict) and not isinstance(v, Cfg) else v

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def __or__(self, other):
        return merge(Cfg(self.to_dict()), dict(other))

    def to_dict(self) -> Dict[str, Any]:
        return {k: v.to_dict() if isinstance(v, Cfg) else v for k, v in self.items()}


def merge(base: Cfg, other: Dict[str, Any]) -> Cfg:
    """Recursive merge of ``other`` into ``base`` (CfgNode.merge_from_file with new_allowed)."""
    for k, v in other.items():
        if isinstance(v, dict) and isinstance(base.get(k), dict):
            merge(base[k], v)
        else:
            base[k] = Cfg(v) if isinstance(v, dict) else v
    return base


def load_config(path: str, gpus: int = 1, is_distributed: bool = False, load_checkpoint: str = "",
                **overrides) -> Cfg:
    """train.py:182-201 / eval.py:245-266: the CLI keys, then the YAML file merged in, then
    ``overrides`` (nested dicts merge)."""
    cfg = Cfg(config=path, gpus=gpus, is_distributed=is_distributed, load_checkpoint=load_checkpoint)
    with open(path) as f:
        merge(cfg, yaml.safe_load(f) or {})
    return merge(cfg, overrides)
