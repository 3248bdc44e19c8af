"""`ModelPT` (reference nemo/core/classes/modelPT.py), the model shell the ASR models derive from,
without PyTorch Lightning (absent here and out of scope): a `NeuralModule` that keeps its
config (`cfg` / `_cfg`), builds sub-modules with `from_config_dict`, saves / restores `.nemo` files
through the SaveRestoreConnector, and sets up the optimizer + scheduler its `optim:` block names
(`setup_optimization`, modelPT.py; `NoamAnnealing`, nemo/core/optim/lr_scheduler.py:444-490).
"""
from __future__ import annotations

import math
import os
import shutil
import tempfile
import threading
import uuid
import weakref
from typing import Any, Dict, Mapping, Optional

import torch

from nemo.core.classes.module import NeuralModule
from nemo.core.config import Config, load_config


class NoamAnnealing(torch.optim.lr_scheduler.LambdaLR):
    """lr_scheduler.py:444-490: lr = base * d_model^-0.5 * min(step^-0.5, step * warmup^-1.5),
    floored at min_lr after warm-up (and min_lr past max_steps)."""

    def __init__(self, optimizer, *, d_model, warmup_steps=None, warmup_ratio=None, max_steps=None, min_lr=0.0,
                 last_epoch=-1):
        if warmup_steps is not None and warmup_ratio is not None:
            raise ValueError("Either use particular number of step or ratio")
        if warmup_ratio is not None and max_steps is None:
            raise ValueError("If there is a ratio, there should be a total steps")
        self.max_steps = max_steps
        self.warmup_steps = warmup_steps if warmup_steps is not None else (
            int(warmup_ratio * max_steps) if warmup_ratio is not None else 0)
        self.min_lr = min_lr
        norm = d_model ** (-0.5)
        bases = [g["lr"] for g in optimizer.param_groups]
        for b in bases:
            if b < min_lr:
                raise ValueError(f"{self} received an initial learning rate that was lower than the minimum learning rate.")

        def factor(i):
            def f(epoch):
                step = max(1, epoch)
                if self.max_steps is not None and step > self.max_steps:
                    return self.min_lr / bases[i]
                w = self.warmup_steps
                mult = norm * (min(step ** (-0.5), step * (w ** (-1.5))) if w > 0 else step ** (-0.5))
                lr = bases[i] * mult
                if step > w:                  # the floor applies after warm-up (lr_scheduler.py:490-491)
                    lr = max(lr, self.min_lr)
                return lr / bases[i]
            return f

        super().__init__(optimizer, [factor(i) for i in range(len(bases))], last_epoch)


def _check_targets(conf: Any, where: str, path: str = "model") -> None:
    """A `.nemo` config is untrusted input: every `_target_` in it must name one of this package's
    drop-in modules (save_restore_connector.RESTORABLE_TARGETS) before any of it is instantiated."""
    from nemo.core.connectors.save_restore_connector import RESTORABLE_TARGETS
    if isinstance(conf, Mapping):
        t = conf.get("_target_")
        if t is not None and t not in RESTORABLE_TARGETS:
            raise ValueError(f"refusing to instantiate {path}._target_={t!r} from {where}: "
                             f"not one of this package's drop-in modules")
        for k, v in conf.items():
            _check_targets(v, where, f"{path}.{k}")
    elif isinstance(conf, (list, tuple)):
        for i, v in enumerate(conf):
            _check_targets(v, where, f"{path}[{i}]")


# The artifact folder of the .nemo being restored (thread-local, set while restore_from builds the model):
# `nemo:<name>` artifact paths in its config resolve there (save_restore_connector.py:333-336).
_RESTORE = threading.local()


def _restored_member(name: str) -> str:
    """Path of archive member `name` of the .nemo being restored; only plain member names resolve (no
    directories, no '..'), so a config cannot point outside the extraction folder."""
    folder = getattr(_RESTORE, "folder", None)
    if folder is None:
        raise FileNotFoundError(f"nemo:{name}: artifact paths resolve only while restoring a .nemo file")
    if not name or name != os.path.basename(name) or name in (".", ".."):
        raise FileNotFoundError(f"nemo:{name}: not a plain archive member name")
    path = os.path.join(folder, name)
    if not os.path.isfile(path):
        raise FileNotFoundError(f"nemo:{name}: no such member in the archive")
    return path


def _set_path(cfg: Dict[str, Any], dotted: str, value: Any) -> None:
    node = cfg
    keys = dotted.split(".")
    for k in keys[:-1]:
        node = node.setdefault(k, {})
    node[keys[-1]] = value


class ModelPT(NeuralModule):
    def __init__(self, cfg: Any, trainer=None):
        super().__init__()
        self.__dict__.setdefault("_artifacts", {})   # config path -> local file (register_artifact)
        if isinstance(cfg, Mapping) and not isinstance(cfg, Config):
            cfg = Config(cfg)
        if isinstance(cfg, Config) and "model" in cfg and "encoder" not in cfg:
            cfg = cfg.model        # a whole experiment yaml was passed
        self._cfg = cfg
        self._trainer = trainer
        self._optimizer = None
        self._scheduler = None

    @property
    def cfg(self) -> Config:
        return self._cfg

    @classmethod
    def from_config_file(cls, path: str, overrides: Optional[Mapping[str, Any]] = None, trainer=None):
        """Build from a reference experiment yaml (`model:` block), `${}` resolved, `???` kept."""
        return cls(load_config(path, overrides).model, trainer=trainer)

    # --- artifacts (modelPT.py register_artifact -> save_restore_connector.py:304-358) -----------
    def register_artifact(self, config_path: str, src: Optional[str], verify_src_exists: bool = True) -> Optional[str]:
        """A file the model needs (tokenizer model / vocabulary) that its .nemo carries: `src` is a local
        path, or `nemo:<member>` while restoring.  Returns the local path to use (None for a missing
        optional artifact); save_to packs the file and writes `nemo:<uuid>_<name>` at `config_path`."""
        src = "" if src is None else str(src)
        if src.startswith("nemo:"):
            path = _restored_member(src[5:])
        elif src and os.path.exists(os.path.abspath(src)):
            path = os.path.abspath(src)
        elif verify_src_exists:
            raise FileNotFoundError(f"src path does not exist or it is not a path in nemo file. src value I got "
                                    f"was: {src}. Absolute: {os.path.abspath(src)}")
        else:
            return None
        self.__dict__.setdefault("_artifacts", {})[config_path] = path
        return path

    @property
    def artifacts(self) -> Dict[str, str]:
        return dict(self.__dict__.get("_artifacts", {}))

    # --- .nemo I/O (modelPT.py save_to / restore_from through the connector) -----------------
    def save_to(self, save_path: str) -> None:
        from nemo.core.connectors.save_restore_connector import SaveRestoreConnector
        cfg = self._cfg.to_dict() if isinstance(self._cfg, Config) else dict(self._cfg)
        packed: Dict[str, bytes] = {}
        for config_path, local in self.artifacts.items():   # _handle_artifacts (:360-396): copy into the archive
            with open(local, "rb") as f:
                data = f.read()
            name = f"{uuid.uuid4().hex}_{os.path.basename(local)}"
            packed[name] = data
            _set_path(cfg, config_path, "nemo:" + name)
        SaveRestoreConnector().save_to({"model": cfg}, self.state_dict(), save_path, artifacts=packed)

    @classmethod
    def restore_from(cls, restore_path: str, map_location=None, strict: bool = True, override_config_path=None):
        from nemo.core.connectors.save_restore_connector import SaveRestoreConnector
        conn = SaveRestoreConnector()
        conf, sd = conn.load_config_and_state_dict(restore_path, override_config_path=override_config_path,
                                                   map_location="cpu")
        _check_targets(conf, restore_path)
        # the archive's artifact members, written under plain names into a private folder that lives as
        # long as the model (nemo: paths in the config resolve there while the model is built)
        folder = tempfile.mkdtemp(prefix="nemo_artifacts_")
        for name, data in conn.artifact_members(restore_path).items():
            with open(os.path.join(folder, name), "wb") as f:
                f.write(data)
        prev = getattr(_RESTORE, "folder", None)
        _RESTORE.folder = folder
        try:
            model = cls(Config(conf))
        except BaseException:
            shutil.rmtree(folder, ignore_errors=True)
            raise
        finally:
            _RESTORE.folder = prev
        weakref.finalize(model, shutil.rmtree, folder, True)
        model.load_state_dict(sd, strict=strict)
        if map_location is not None:
            model = model.to(map_location)
        return model

    # --- optimisation (optim: block of the yamls) ----------------------------------------------
    def setup_optimization(self, optim_config: Optional[Mapping[str, Any]] = None, max_steps: Optional[int] = None):
        """The `optim:` block -> torch optimizer (+ NoamAnnealing when `sched.name` says so)."""
        oc = dict(optim_config if optim_config is not None else self._cfg.get("optim", {}) or {})
        name = str(oc.pop("name", "adamw")).lower()
        sched = oc.pop("sched", None)
        lr = float(oc.pop("lr", 1e-3))
        params = [p for p in self.parameters() if p.requires_grad]
        kw = {k: (tuple(v) if isinstance(v, list) else v) for k, v in oc.items()}
        if "weight_decay" in kw:
            kw["weight_decay"] = float(kw["weight_decay"])
        if name == "adamw":
            opt = torch.optim.AdamW(params, lr=lr, **kw)
        elif name == "adam":
            opt = torch.optim.Adam(params, lr=lr, **kw)
        elif name == "sgd":
            opt = torch.optim.SGD(params, lr=lr, **kw)
        else:
            raise ValueError(f"optimizer {name!r} is not provided (adamw | adam | sgd)")
        self._optimizer = opt
        self._scheduler = None
        if sched:
            sched = dict(sched)
            sname = sched.pop("name", None)
            if sname != "NoamAnnealing":
                raise ValueError(f"scheduler {sname!r} is not provided (NoamAnnealing)")
            for k in ("min_lr",):
                if k in sched:
                    sched[k] = float(sched[k])
            self._scheduler = NoamAnnealing(opt, max_steps=sched.pop("max_steps", max_steps), **sched)
        return opt, self._scheduler

    @property
    def num_weights(self) -> int:
        return sum(p.numel() for p in self.parameters() if p.requires_grad)

    def _current_lr(self) -> float:
        if self._optimizer is None:
            return math.nan
        return float(self._optimizer.param_groups[0]["lr"])
