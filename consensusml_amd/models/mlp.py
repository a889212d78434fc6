"""2-layer MLP — BASELINE.json config 1 ("2-layer MLP on synthetic data, world_size=2
CPU/gloo, coordinate-wise median aggregation")."""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class MLP(nn.Module):
    def __init__(self, in_features: int = 32, hidden: int = 64, classes: int = 2):
        super().__init__()
        self.fc1 = nn.Linear(in_features, hidden)
        self.fc2 = nn.Linear(hidden, classes)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.fc2(F.relu(self.fc1(x)))
