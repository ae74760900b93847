"""Helpers shared by the GPU parity tests, smoke() and bench.py (test infrastructure)."""

from __future__ import annotations

import types

import numpy as np
import torch

BATCH_KEYS = ("input_ids", "labels", "attention_mask", "position_ids", "rewards", "advantages", "ref_logprobs",
              "old_logprobs", "group_tokens", "num_labels", "overflow", "seq_boundaries")


class LogitsModel(torch.nn.Module):
    """Stub causal LM: forward returns fixed logits (and value-head outputs) as parameters."""

    def __init__(self, logits: torch.Tensor, values: torch.Tensor | None = None):
        super().__init__()
        self.logits = torch.nn.Parameter(logits)
        if values is not None:
            self.value_head = torch.nn.Parameter(values)

    def forward(self, **kw):
        return types.SimpleNamespace(logits=self.logits, value=getattr(self, "value_head", None))


def to_batch(b: dict, device="cuda"):
    from pipelinerl_amd.finetune.types import PipelineBatchEncoding

    kw = {k: torch.as_tensor(np.asarray(b[k])) for k in BATCH_KEYS if k in b}
    kw["is_packed"] = bool(b.get("is_packed", False))
    kw["model_version"] = int(b.get("model_version", 0))
    return PipelineBatchEncoding(**kw).to_device(device)


def rel_close(a, b, rtol, atol):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    err = np.abs(a - b)
    ok = err <= atol + rtol * np.abs(b)
    return bool(ok.all()), float(err.max()) if err.size else 0.0
