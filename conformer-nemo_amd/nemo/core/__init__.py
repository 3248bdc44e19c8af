"""Core plugin contract (thin mirror of the reference's nemo.core)."""
from .classes import NeuralModule, Serialization, Typing, typecheck  # noqa: F401
