from .common import Serialization, Typing, typecheck  # noqa: F401
from .module import NeuralModule  # noqa: F401


class Exportable:
    """Export mixin placeholder (reference nemo/core/classes/exportable.py:37): export is out of scope."""
