"""Minimal plugin contract of the reference core (nemo/core/classes/common.py), re-designed.

* `typecheck` — the reference decorator (common.py:795-918) validates neural types and requires
  keyword-only calls (common.py:891-892).  Here: the keyword-only rule is enforced (same
  TypeError), type annotation is a no-op.
* `Serialization.from_config_dict` — resolves a config's `_target_` to a class and instantiates it
  with the remaining keys (common.py:426-487, which goes through hydra.utils.instantiate).
* `Typing` — input_types / output_types properties.
"""
from __future__ import annotations

import functools
import importlib
from typing import Any, Mapping


class typecheck:
    """Keyword-only enforcement for typed methods (reference common.py:891-892)."""

    def __init__(self, input_types=None, output_types=None, ignore_collections: bool = False):
        self.input_types = input_types
        self.output_types = output_types

    def __call__(self, fn):
        @functools.wraps(fn)
        def wrapper(instance, *args, **kwargs):
            if args:
                raise TypeError("All arguments must be passed by kwargs only for typed methods")
            return fn(instance, **kwargs)

        return wrapper


class Typing:
    @property
    def input_types(self):
        return None

    @property
    def output_types(self):
        return None


def _locate(path: str):
    module, _, name = path.rpartition(".")
    obj = importlib.import_module(module)
    return getattr(obj, name)


class Serialization:
    @classmethod
    def from_config_dict(cls, config: Mapping[str, Any], trainer=None):
        """Instantiate `config['_target_']` (or `cls`) with the other keys as kwargs."""
        cfg = dict(config)
        target = cfg.pop("_target_", None)
        cfg.pop("_convert_", None)
        klass = _locate(target) if target else cls
        return klass(**cfg)

    def to_config_dict(self):
        return getattr(self, "_cfg", None)
