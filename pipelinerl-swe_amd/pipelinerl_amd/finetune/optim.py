"""Optimizer with decay / no-decay parameter groups (contract of pipelinerl/finetune/optim.py:8-45).

adamw_torch uses torch's fused AdamW on the device (one multi-tensor kernel per step);
adafactor comes from transformers.  DeepSpeed's cpuadam and Lion are out of scope.
"""

from __future__ import annotations

import torch

NO_DECAY = ("bias", "LayerNorm.weight")


def get_grouped_params(model, weight_decay: float, no_decay=NO_DECAY):
    with_wd, without_wd = [], []
    for n, p in model.named_parameters():
        if not p.requires_grad:
            continue
        (without_wd if any(nd in n for nd in no_decay) else with_wd).append(p)
    return [{"params": with_wd, "weight_decay": weight_decay}, {"params": without_wd, "weight_decay": 0.0}]


def get_optimizer(name: str, model, learning_rate: float, weight_decay: float):
    groups = get_grouped_params(model, weight_decay)
    if name == "adamw_torch":
        on_gpu = all(p.is_cuda for g in groups for p in g["params"])
        return torch.optim.AdamW(groups, lr=learning_rate, fused=on_gpu or None)
    if name == "adafactor":
        from transformers import Adafactor

        return Adafactor(groups, lr=learning_rate, relative_step=False, scale_parameter=False)
    raise ValueError(f"Unknown optimizer: {name}")
