"""Model configs as the reference's yamls write them, without OmegaConf/Hydra (absent here).

The reference builds models from `configs/conformer_ctc_bpe.yaml` / `conformer_transducer_bpe.yaml`
through OmegaConf (`ModelPT.__init__`, nemo/core/classes/modelPT.py; `hydra.main` in the example
scripts).  What those configs use, and what this module reproduces:

* YAML anchors / aliases (`sample_rate: &sample_rate 16000`, `*sample_rate`) — plain YAML;
  `yaml.safe_load` resolves them (and executes nothing from the file);
* `${a.b.c}` node interpolation against the document root (`${model.preprocessor.features}`,
  `${name}`) — resolved once, after overrides are applied;
* `???` mandatory-missing markers (`manifest_filepath: ???`, `tokenizer.dir: ???`) — kept as the
  MISSING sentinel; reading one raises `MissingMandatoryValue` (OmegaConf's behaviour) so a field
  nobody reads (a data manifest) never matters, and one that is read must be overridden;
* attribute access (`cfg.decoder.feat_in`), `in`, `.get()`, item assignment (`open_dict` is not
  needed: configs here are always writable).
"""
from __future__ import annotations

import copy
from typing import Any, Dict, Mapping, Optional

import yaml

from nemo.core.connectors.save_restore_connector import resolve_interpolations

MISSING = "???"


class MissingMandatoryValue(KeyError):
    """OmegaConf's MissingMandatoryValue: a `???` field was read before being set."""


class Config(dict):
    """A dict with attribute access whose nested mappings are Configs (DictConfig stand-in)."""

    def __init__(self, data: Optional[Mapping[str, Any]] = None, _path: str = ""):
        super().__init__()
        object.__setattr__(self, "_path", _path)
        for k, v in (data or {}).items():
            dict.__setitem__(self, k, _wrap(v, f"{_path}.{k}" if _path else str(k)))

    def _check(self, key, v):
        if isinstance(v, str) and v == MISSING:
            raise MissingMandatoryValue(f"Missing mandatory value: {self._path + '.' if self._path else ''}{key}")
        return v

    def __getitem__(self, key):
        return self._check(key, dict.__getitem__(self, key))

    def __getattr__(self, key):
        if key.startswith("__"):
            raise AttributeError(key)
        try:
            return self[key]
        except MissingMandatoryValue:
            raise
        except KeyError:
            raise AttributeError(f"config {self._path or '<root>'} has no key {key!r}") from None

    def __setattr__(self, key, value):
        self[key] = value

    def __setitem__(self, key, value):
        dict.__setitem__(self, key, _wrap(value, f"{self._path}.{key}" if self._path else str(key)))

    def get(self, key, default=None):
        if key not in self:
            return default
        return self[key]

    def is_missing(self, key) -> bool:
        return key in self and isinstance(dict.__getitem__(self, key), str) and dict.__getitem__(self, key) == MISSING

    def to_dict(self) -> Dict[str, Any]:
        return _unwrap(self)

    def __deepcopy__(self, memo):
        return Config(copy.deepcopy(_unwrap(self), memo), self._path)


def _wrap(v, path):
    if isinstance(v, Config):
        return v
    if isinstance(v, Mapping):
        return Config(v, path)
    if isinstance(v, list):
        return [_wrap(x, f"{path}[{i}]") for i, x in enumerate(v)]
    return v


def _unwrap(v):
    if isinstance(v, Mapping):
        return {k: _unwrap(dict.__getitem__(v, k) if isinstance(v, Config) else v[k]) for k in v}
    if isinstance(v, list):
        return [_unwrap(x) for x in v]
    return v


def _set_dotted(root: Dict[str, Any], dotted: str, value: Any) -> None:
    node = root
    parts = dotted.split(".")
    for p in parts[:-1]:
        if p not in node or not isinstance(node[p], dict):
            node[p] = {}
        node = node[p]
    node[parts[-1]] = value


def load_config(source: Any, overrides: Optional[Mapping[str, Any]] = None) -> Config:
    """A reference yaml (path, yaml text or dict) -> Config, `${}` resolved against the document root.

    overrides: {"model.train_ds.manifest_filepath": "...", ...} applied before resolution, the way a
    Hydra command line (`model.tokenizer.dir=...`) would."""
    if isinstance(source, Mapping):
        doc = copy.deepcopy(_unwrap(source))
    elif isinstance(source, str) and "\n" not in source and source.endswith((".yaml", ".yml")):
        with open(source, encoding="utf-8") as f:
            doc = yaml.safe_load(f)
    else:
        doc = yaml.safe_load(source)
    if not isinstance(doc, dict):
        raise ValueError("a model config must be a mapping")
    for k, v in (overrides or {}).items():
        _set_dotted(doc, k, v)
    # an interpolation of a `???` node yields `???` (still missing), as in OmegaConf
    return Config(resolve_interpolations(doc, doc))
