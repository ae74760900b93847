"""Micro-batch collation (mirror of pipelinerl/finetune/data.py:163-279).

collate_packed concatenates rollouts into one [1, T] row — the layout the fused loss kernel
consumes directly (row t scored against token t+1; the first label of every sequence after
the first is masked so no token is predicted across a sequence boundary).
"""

from __future__ import annotations

import array
from typing import Any

import numpy as np
import torch

from .. import native_data
from .rl import RL_DATA_COLUMNS
from .types import PipelineBatchEncoding
from .utils import create_sentinel_example

MASKED_TOKEN_ID = -100


def _concat(seqs, code: str, dtype) -> np.ndarray:
    """Concatenate lists / arrays into one flat array: libprl_data's list loop (2-5 ns per
    element) for plain int / float lists, else array.array's."""
    total = sum(len(s) if isinstance(s, (list, tuple, np.ndarray)) else 1 for s in seqs)
    fast = native_data.concat_lists(seqs, native_data.DT_I64 if code == "q" else native_data.DT_F64, total)
    if fast is not None:
        return fast
    buf = array.array(code)
    for s in seqs:
        if isinstance(s, (list, tuple)):
            buf.extend(s)
        else:
            buf.extend(np.atleast_1d(np.asarray(s, dtype=dtype)).tolist())
    return np.frombuffer(buf, dtype=dtype) if len(buf) else np.empty(0, dtype)


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
    lens = np.fromiter((len(e["input_ids"]) for e in examples), np.int64, len(examples))
    ids, labels, pos, bounds = native_data.collate_arrays(
        lens, _concat([e["input_ids"] for e in examples], "q", np.int64),
        _concat([e["labels"] for e in examples], "q", np.int64), label_pad_value)
    extra = [c for c in RL_DATA_COLUMNS if c in examples[0]]
    fields: dict[str, Any] = {}
    for k in extra:
        fields[k] = torch.from_numpy(_concat([e[k] for e in examples], "d", np.float64).astype(np.float32))[None]
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
