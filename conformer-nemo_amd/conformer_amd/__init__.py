"""MI355X-native Conformer encoder forward: host runtime over the libcfm.so C-ABI.

The drop-in plugin class lives at `nemo.collections.asr.modules.ConformerEncoder` (this directory's
sibling `nemo/` namespace mirror), so reference yaml `_target_` strings resolve unchanged.
"""
from . import _lib  # noqa: F401
from .runtime import NativeEncoder, encoded_length, make_cfg  # noqa: F401

__all__ = ["NativeEncoder", "encoded_length", "make_cfg"]
