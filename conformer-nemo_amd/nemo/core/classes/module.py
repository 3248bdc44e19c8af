"""NeuralModule (reference nemo/core/classes/module.py:24-77): nn.Module + typing + serialization
+ freeze/unfreeze."""
from __future__ import annotations

import torch

from .common import Serialization, Typing


class NeuralModule(torch.nn.Module, Typing, Serialization):
    @property
    def num_weights(self) -> int:
        return sum(p.numel() for p in self.parameters() if p.requires_grad)

    def input_example(self, max_batch=None, max_dim=None):
        return None

    def freeze(self) -> None:
        for p in self.parameters():
            p.requires_grad = False
        self.eval()

    def unfreeze(self) -> None:
        for p in self.parameters():
            p.requires_grad = True
        self.train()
