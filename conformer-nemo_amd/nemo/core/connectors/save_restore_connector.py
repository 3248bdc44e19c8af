"""`.nemo` checkpoint import/export (reference nemo/core/connectors/save_restore_connector.py:23-470),
SURVEY §8 row f4: load real NeMo checkpoints into the MI355X-native modules.

A `.nemo` file is a tar archive (uncompressed since NeMo 1.7, gzip before; `_unpack_nemo_file`
:440-456 tries "r:" then "r:gz") holding `model_config.yaml` (the model's resolved OmegaConf config,
common.py:556-569) and `model_weights.ckpt` (torch.save of the model's state_dict, :458-460).

Differences by design (safety and the absent Lightning/OmegaConf stack):
* members are read in memory — nothing is extracted to disk, so archive paths cannot escape;
* the config is parsed with `yaml.safe_load` and the weights with
  `torch.load(..., weights_only=True)`: nothing in the file is executed;
* `${a.b.c}` interpolations left in a config are resolved against its root (OmegaConf semantics
  for plain node references);
* there is no Lightning `ModelPT`: `restore_modules` instantiates the drop-in sub-modules the
  config names (preprocessor, spec_augment, encoder, decoder, joint) under the attribute names
  EncDecCTCModel / EncDecRNNTModel give them (ctc_models.py:168-199, rnnt_models.py:69-95) and
  loads each one's slice of the checkpoint (strict by default).
"""
from __future__ import annotations

import copy
import io
import os
import re
import tarfile
from typing import Any, Dict, Optional, Tuple

import torch
import yaml

MODEL_CONFIG_YAML = "model_config.yaml"
MODEL_WEIGHTS_CKPT = "model_weights.ckpt"
_INTERP = re.compile(r"\$\{([^}]+)\}")


def _lookup(root: Dict[str, Any], dotted: str):
    node: Any = root
    for part in dotted.strip().split("."):
        if isinstance(node, dict) and part in node:
            node = node[part]
        else:
            raise KeyError(f"interpolation ${{{dotted}}} does not resolve")
    return node


def resolve_interpolations(cfg: Any, root: Optional[Dict[str, Any]] = None, _depth: int = 0) -> Any:
    """Replace `${node.path}` references by the referenced values (whole-string references keep the
    referenced type; embedded references are substituted as text)."""
    if _depth > 32:
        raise ValueError("interpolation cycle")
    root = cfg if root is None else root
    if isinstance(cfg, dict):
        return {k: resolve_interpolations(v, root, _depth) for k, v in cfg.items()}
    if isinstance(cfg, list):
        return [resolve_interpolations(v, root, _depth) for v in cfg]
    if isinstance(cfg, str):
        m = _INTERP.fullmatch(cfg.strip())
        if m:
            return resolve_interpolations(_lookup(root, m.group(1)), root, _depth + 1)
        if _INTERP.search(cfg):
            return _INTERP.sub(lambda mm: str(resolve_interpolations(_lookup(root, mm.group(1)), root, _depth + 1)),
                               cfg)
    return cfg


def _member_name(name: str) -> str:
    return name[2:] if name.startswith("./") else name


class SaveRestoreConnector:
    """save_restore_connector.py:23-470 (config + weights handling; artifacts are carried as bytes)."""

    def __init__(self) -> None:
        self._model_config_yaml = MODEL_CONFIG_YAML
        self._model_weights_ckpt = MODEL_WEIGHTS_CKPT

    # --- archive I/O -------------------------------------------------------------------------
    @staticmethod
    def _read_nemo_members(path2file: str) -> Dict[str, bytes]:
        """`_unpack_nemo_file` (:440-456) without touching the filesystem: regular-file members by
        name (leading './' stripped)."""
        if not os.path.exists(path2file):
            raise FileNotFoundError(f"{path2file} does not exist")
        try:
            tar = tarfile.open(path2file, "r:")
        except tarfile.ReadError:
            tar = tarfile.open(path2file, "r:gz")   # older checkpoints
        out: Dict[str, bytes] = {}
        with tar:
            for m in tar.getmembers():
                if m.isfile():
                    f = tar.extractfile(m)
                    out[_member_name(m.name)] = f.read() if f is not None else b""
        return out

    @staticmethod
    def _make_nemo_file_from_members(filename: str, members: Dict[str, bytes]) -> None:
        """`_make_nemo_file_from_folder` (:434-438): an uncompressed tar with members under './'."""
        d = os.path.dirname(filename)
        if d:
            os.makedirs(d, exist_ok=True)
        with tarfile.open(filename, "w:") as tar:
            for name, data in members.items():
                info = tarfile.TarInfo("./" + name)
                info.size = len(data)
                tar.addfile(info, io.BytesIO(data))

    @staticmethod
    def _load_state_dict_from_bytes(data: bytes, map_location=None) -> Dict[str, torch.Tensor]:
        """`_load_state_dict_from_disk` (:462-464) with the safe loader."""
        return torch.load(io.BytesIO(data), map_location=map_location, weights_only=True)

    # --- public API ----------------------------------------------------------------------------
    def save_to(self, cfg: Dict[str, Any], state_dict: Dict[str, torch.Tensor], save_path: str,
                artifacts: Optional[Dict[str, bytes]] = None) -> None:
        """`save_to` (:31-55) for a (config, state_dict) pair: config yaml + torch.save'd weights."""
        buf = io.BytesIO()
        torch.save({k: v.detach().cpu() for k, v in state_dict.items()}, buf)
        members = {self.model_config_yaml: yaml.safe_dump(cfg, sort_keys=False).encode(),
                   self.model_weights_ckpt: buf.getvalue()}
        members.update(artifacts or {})
        self._make_nemo_file_from_members(save_path, members)

    def load_config_and_state_dict(self, restore_path: str, override_config_path=None, map_location=None,
                                   return_config: bool = False):
        """`load_config_and_state_dict` (:57-145): (conf, state_dict) with `model:` unwrapped
        (:111-112); only conf when return_config."""
        members = self._read_nemo_members(restore_path)
        if override_config_path is None:
            if self.model_config_yaml not in members:
                raise FileNotFoundError(f"{restore_path}: no {self.model_config_yaml}")
            conf = yaml.safe_load(members[self.model_config_yaml].decode())
        elif isinstance(override_config_path, dict):
            conf = copy.deepcopy(override_config_path)
        else:
            with open(override_config_path, encoding="utf-8") as f:
                conf = yaml.safe_load(f)
        conf = resolve_interpolations(conf)
        if isinstance(conf, dict) and "model" in conf:
            conf = conf["model"]
        if return_config:
            return conf
        if self.model_weights_ckpt not in members:
            raise FileNotFoundError(f"{restore_path}: no {self.model_weights_ckpt}")
        state_dict = self._load_state_dict_from_bytes(members[self.model_weights_ckpt], map_location)
        return conf, state_dict

    def artifact_members(self, restore_path: str) -> Dict[str, bytes]:
        """The archive's artifact files (every member but the config and the weights) whose names are plain
        file names - what `nemo:<name>` config paths refer to (:333-336); anything with a directory
        part or '..' is ignored, so nothing is written outside the caller's folder."""
        out = {}
        for name, data in self._read_nemo_members(restore_path).items():
            if name in (self.model_config_yaml, self.model_weights_ckpt):
                continue
            if name and name == os.path.basename(name) and name not in (".", ".."):
                out[name] = data
        return out

    def extract_state_dict_from(self, restore_path: str, save_dir: str, split_by_module: bool = False):
        """`extract_state_dict_from` (:212-285): model_weights.ckpt, or one `<module>.ckpt` per
        top-level prefix when split_by_module; returns the full state dict."""
        _, state_dict = self.load_config_and_state_dict(restore_path, map_location="cpu")
        save_dir = os.path.abspath(save_dir)
        os.makedirs(save_dir, exist_ok=True)
        if not split_by_module:
            torch.save(state_dict, os.path.join(save_dir, self.model_weights_ckpt))
        else:
            for prefix in sorted({k.split(".", 1)[0] for k in state_dict}):
                sub = {k.split(".", 1)[1]: v for k, v in state_dict.items() if k.startswith(prefix + ".")}
                torch.save(sub, os.path.join(save_dir, f"{prefix}.ckpt"))
        return state_dict

    @property
    def model_config_yaml(self) -> str:
        return self._model_config_yaml

    @model_config_yaml.setter
    def model_config_yaml(self, path: str):
        self._model_config_yaml = path

    @property
    def model_weights_ckpt(self) -> str:
        return self._model_weights_ckpt

    @model_weights_ckpt.setter
    def model_weights_ckpt(self, path: str):
        self._model_weights_ckpt = path


# model attribute <- config block (ctc_models.py:168-199, rnnt_models.py:69-95)
_BLOCKS = (("preprocessor", "preprocessor"), ("spec_augmentation", "spec_augment"), ("encoder", "encoder"),
           ("decoder", "decoder"), ("joint", "joint"))


# `_target_` values restore_modules will instantiate: the drop-in modules this package provides
# under the reference's import paths (and nothing else — a .nemo config is untrusted input).
RESTORABLE_TARGETS = frozenset({
    "nemo.collections.asr.modules.ConformerEncoder",
    "nemo.collections.asr.modules.conformer_encoder.ConformerEncoder",
    "nemo.collections.asr.modules.AudioToMelSpectrogramPreprocessor",
    "nemo.collections.asr.modules.audio_preprocessing.AudioToMelSpectrogramPreprocessor",
    "nemo.collections.asr.modules.SpectrogramAugmentation",
    "nemo.collections.asr.modules.audio_preprocessing.SpectrogramAugmentation",
    "nemo.collections.asr.modules.ConvASRDecoder",
    "nemo.collections.asr.modules.conv_asr.ConvASRDecoder",
    "nemo.collections.asr.modules.RNNTDecoder",
    "nemo.collections.asr.modules.rnnt.RNNTDecoder",
    "nemo.collections.asr.modules.RNNTJoint",
    "nemo.collections.asr.modules.rnnt.RNNTJoint",
})


def _subdict(sd: Dict[str, torch.Tensor], prefix: str) -> Dict[str, torch.Tensor]:
    p = prefix + "."
    return {k[len(p):]: v for k, v in sd.items() if k.startswith(p)}


def restore_modules(restore_path: str, map_location=None, strict: bool = True,
                    connector: Optional[SaveRestoreConnector] = None) -> Tuple[Dict[str, Any], Dict[str, torch.nn.Module]]:
    """Instantiate the drop-in modules a `.nemo` config names and load their weights.

    Returns (conf, modules) with modules keyed by the reference model's attribute names.  Blocks
    whose `_target_` this package does not provide (e.g. an LSTM `RNNTDecoder`) are skipped, and
    their weights stay in the checkpoint untouched."""
    from nemo.core.classes.common import Serialization, _locate

    conn = connector or SaveRestoreConnector()
    conf, sd = conn.load_config_and_state_dict(restore_path, map_location="cpu")
    mods: Dict[str, torch.nn.Module] = {}
    for attr, key in _BLOCKS:
        block = conf.get(key) if isinstance(conf, dict) else None
        if not isinstance(block, dict) or "_target_" not in block:
            continue
        block = dict(block)
        if attr == "decoder" and "encoder" in mods and "joint" not in conf:
            # EncDecCTCModel fills decoder.feat_in / num_classes (ctc_models.py:171-184)
            if not block.get("feat_in"):
                block["feat_in"] = mods["encoder"]._feat_out
            if block.get("num_classes", 0) < 1 and block.get("vocabulary") is not None:
                block["num_classes"] = len(block["vocabulary"])
        target = block.get("_target_")
        if target not in RESTORABLE_TARGETS:
            # Only this package's drop-in classes are ever instantiated from a checkpoint's config:
            # an arbitrary `_target_` (e.g. a function of the standard library) is never resolved.
            if strict and target is not None and str(target).split(".")[0] != "nemo":
                raise ValueError(f"refusing to instantiate {attr}._target_={target!r} from {restore_path}: "
                                 f"not one of this package's drop-in modules")
            continue
        try:
            klass = _locate(target)
        except (ImportError, AttributeError, ModuleNotFoundError):
            continue                                   # not a drop-in of this package
        if not (isinstance(klass, type) and issubclass(klass, torch.nn.Module)):
            raise ValueError(f"{attr}._target_={target!r} does not name an nn.Module")
        m = Serialization.from_config_dict(block)
        sub = _subdict(sd, attr)
        if sub or strict:
            m.load_state_dict(sub, strict=strict)
        if map_location is not None:
            m = m.to(map_location)
        mods[attr] = m
    return conf, mods
