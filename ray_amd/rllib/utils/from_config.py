"""``ray.rllib.utils.from_config`` (reference path): build an object from a config dict
with a ``type`` key (a class, an import path, or a name in ``cls``'s module)."""

from __future__ import annotations

import copy
import importlib


def from_config(cls, config=None, **kwargs):
    if config is None:
        return None
    if not isinstance(config, dict):
        if isinstance(config, type):
            return config(**kwargs)
        if isinstance(config, str):
            config = {"type": config}
        else:
            return config
    cfg = copy.deepcopy(config)
    cfg.update(kwargs)
    typ = cfg.pop("type", cls)
    if isinstance(typ, str):
        if "." in typ:
            mod, _, name = typ.rpartition(".")
            typ = getattr(importlib.import_module(mod), name)
        else:
            typ = getattr(importlib.import_module(cls.__module__), typ)
    return typ(**cfg)
