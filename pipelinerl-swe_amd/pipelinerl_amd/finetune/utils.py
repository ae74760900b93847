"""Sentinel batches (mirror of pipelinerl/finetune/utils.py:16-75).

A rank that has already processed its share of a step's samples still has to join every
lockstep pass of the data-parallel loop; it is fed a sentinel batch (8 EOS tokens, every
label masked), whose loss the trainer multiplies by 0 (finetune_loop.py:664-666).
"""

from __future__ import annotations

import torch

from .types import PipelineBatchEncoding

SENTINEL_LENGTH = 8


def create_sentinel_batch(device=None, tokenizer=None, model_version: int = 0) -> PipelineBatchEncoding:
    eos = getattr(tokenizer, "eos_token_id", 2) if tokenizer else 2
    n = SENTINEL_LENGTH
    z = torch.zeros(1, n)
    o = torch.ones(1, n)
    b = PipelineBatchEncoding(
        input_ids=torch.full((1, n), eos, dtype=torch.long), attention_mask=torch.ones(1, n, dtype=torch.long),
        labels=torch.full((1, n), -100, dtype=torch.long), position_ids=torch.arange(n)[None],
        rewards=z, advantages=z.clone(), ref_logprobs=z.clone(), old_logprobs=z.clone(), group_tokens=o,
        num_labels=o.clone(), overflow=z.clone(), seq_boundaries=torch.tensor([0, n], dtype=torch.int),
        model_version=model_version, sentinel=True, is_packed=True)
    return b.to_device(device) if device is not None else b


def create_sentinel_example(n_tokens: int, tokenizer=None, model_version: int = 0) -> dict:
    eos = tokenizer.eos_token_id
    return {
        "input_ids": [eos] * n_tokens, "attention_mask": [1] * n_tokens, "labels": [-100] * n_tokens,
        "position_ids": list(range(n_tokens)), "rewards": [0.0] * n_tokens, "advantages": [0.0] * n_tokens,
        "ref_logprobs": [0.0] * n_tokens, "old_logprobs": [0.0] * n_tokens, "group_tokens": [1.0] * n_tokens,
        "num_labels": [1.0] * n_tokens, "overflow": [0.0] * n_tokens, "model_version": model_version,
    }
