"""Micro-batch collation (mirror of pipelinerl/finetune/data.py:163-279).

collate_packed concatenates rollouts into one [1, T] row — the layout the fused loss kernel
consumes directly (row t scored against token t+1; the first label of every sequence after
the first is masked so no token is predicted across a sequence boundary).
"""

from __future__ import annotations

from typing import Any

import numpy as np
import torch

from .rl import RL_DATA_COLUMNS
from .types import PipelineBatchEncoding
from .utils import create_sentinel_example

MASKED_TOKEN_ID = -100


def collate_packed(examples: list[dict[str, Any]], tokenizer, seq_parallel: int,
                   label_pad_value: int = MASKED_TOKEN_ID) -> PipelineBatchEncoding:
    """data.py:215-279.  Pads with a sentinel example to a multiple of seq_parallel tokens."""
    total = sum(len(e["input_ids"]) for e in examples)
    padding = 0
    if total % seq_parallel:
        padding = seq_parallel - total % seq_parallel
        version = max(e["model_version"] for e in examples)
        examples = examples + [create_sentinel_example(padding, tokenizer=tokenizer, model_version=version)]
        total += padding
    lens = np.array([len(e["input_ids"]) for e in examples], dtype=np.int64)
    bounds = np.zeros(len(examples) + 1, dtype=np.int32)
    bounds[1:] = np.cumsum(lens)
    ids = np.empty(total, dtype=np.int64)
    labels = np.empty(total, dtype=np.int64)
    pos = np.empty(total, dtype=np.int64)
    for i, e in enumerate(examples):
        a, b = int(bounds[i]), int(bounds[i + 1])
        ids[a:b] = e["input_ids"]
        pos[a:b] = np.arange(b - a)
        labels[a:b] = e["labels"]
        if i > 0 and b > a:
            labels[a] = label_pad_value
    extra = [c for c in RL_DATA_COLUMNS if c in examples[0]]
    fields: dict[str, Any] = {}
    for k in extra:
        vals = []
        for e in examples:
            v = e[k]
            vals.extend(v) if isinstance(v, (list, tuple)) else vals.append(v)
        fields[k] = torch.tensor([vals], dtype=torch.float32)
    return PipelineBatchEncoding(
        input_ids=torch.from_numpy(ids)[None], labels=torch.from_numpy(labels)[None],
        attention_mask=torch.ones(1, total, dtype=torch.long), position_ids=torch.from_numpy(pos)[None],
        model_version=min(e.get("model_version", 0) for e in examples), is_packed=True,
        seq_boundaries=torch.from_numpy(bounds), padding=padding, **fields)


def collate(examples: list[dict[str, Any]], tokenizer, label_mask_value: int = MASKED_TOKEN_ID,
            pad_to_multiple_of: int = 16) -> PipelineBatchEncoding:
    """data.py:163-212: right/left padding to a multiple of pad_to_multiple_of ([B, L] batch)."""
    L = max(len(e["input_ids"]) for e in examples)
    if L % pad_to_multiple_of:
        L += pad_to_multiple_of - L % pad_to_multiple_of
    right = getattr(tokenizer, "padding_side", "right") == "right"
    out: dict[str, Any] = {}
    for k in examples[0]:
        if k == "model_version":
            continue
        seqs = [e[k] for e in examples]
        if any(isinstance(s, (str, dict)) for s in seqs):
            continue
        if any(isinstance(x, (str, dict)) for s in seqs if isinstance(s, list) for x in s):
            continue
        pad = label_mask_value if k == "labels" else (0.0 if k in RL_DATA_COLUMNS else 0)
        rows = []
        for s in seqs:
            if s is None:
                continue
            s = s if isinstance(s, list) else [s]
            p = [pad] * (L - len(s))
            rows.append(s + p if right else p + s)
        out[k] = torch.tensor(rows)
    out["model_version"] = min(e.get("model_version", 0) for e in examples)
    out["is_packed"] = False
    return PipelineBatchEncoding(**out)
