"""Masked reductions and metric aggregation (mirror of pipelinerl/finetune/rl/utils.py).

The trainer hot path does not use these (the fused kernel computes its sums); they are the
host-side helpers the reference's callers import, with the same semantics.
"""

from __future__ import annotations

import torch


def aggregate_rl_stats(rl_stats: dict, num_samples: int) -> dict[str, float]:
    """utils.py:8-22: keys with 'min'/'max' reduce by min/max, 'loss' and '*sum*' by sum,
    everything else by sum / num_samples.  Keys get an 'rl/' prefix."""
    out: dict[str, float] = {}
    for k, v in rl_stats.items():
        t = torch.tensor(v, dtype=torch.float32)
        if "min" in k:
            r = torch.min(t)
        elif "max" in k:
            r = torch.max(t)
        elif k == "loss" or "sum" in k:
            r = torch.sum(t)
        else:
            r = torch.sum(t) / num_samples
        out["rl/" + k] = r.item()
    return out


def mask_sum(values: torch.Tensor, mask: torch.Tensor, axis: int | None = None) -> torch.Tensor:
    x = (values * mask).nan_to_num(0)
    return x.sum() if axis is None else x.sum(axis=axis)


def mask_mean(values: torch.Tensor, mask: torch.Tensor, axis: int | None = None) -> torch.Tensor:
    x = (values * mask).nan_to_num(0)
    return x.sum() / mask.sum() if axis is None else x.sum(axis=axis) / mask.sum(axis=axis)


def mean_sum(values: torch.Tensor, masks: torch.Tensor, segments: list | None) -> torch.Tensor:
    if segments and values.shape[-1] != 1:
        assert values.shape[0] == 1, "seq packed samples must have dimension 0 of 1"
        sums = torch.stack([mask_sum(values[0, a:b], masks[0, a:b]) for a, b in segments])
        counts = torch.stack([masks[0, a:b].sum() for a, b in segments])
        return (sums / counts).sum()
    return mask_mean(values, masks, -1).sum()


def sum_sum(values: torch.Tensor, masks: torch.Tensor, segments: list | None) -> torch.Tensor:
    if segments and values.shape[-1] != 1:
        assert values.shape[0] == 1, "seq packed samples must have dimension 0 of 1"
        return torch.stack([mask_sum(values[0, a:b], masks[0, a:b]) for a, b in segments]).sum()
    return mask_sum(values, masks)
