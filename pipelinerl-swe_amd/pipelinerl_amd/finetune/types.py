"""Batch schema of the trainer's input (mirror of pipelinerl/finetune/types.py:28-178).

``PipelineBatchEncoding`` is the packed micro-batch the preprocessor writes to the
``training_data`` stream and the trainer feeds to ``rl_step``: [1, T] (packed) or [B, L]
(padded) token tensors, per-token RL fields as float32, and packing metadata.
Lists / numpy arrays are converted to tensors on construction, as in the reference.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Union

import numpy as np
import torch
from pydantic import PrivateAttr, BaseModel, ConfigDict, field_validator

LONG_FIELDS = ("input_ids", "attention_mask", "labels", "position_ids", "image_grid_thw")
FLOAT_FIELDS = ("rewards", "advantages", "ref_logprobs", "old_logprobs", "group_tokens", "num_labels",
                "overflow", "pixel_values")
TOKEN_FIELDS = ("input_ids", "attention_mask", "labels", "position_ids", "rewards", "advantages",
                "ref_logprobs", "old_logprobs", "group_tokens", "overflow", "num_labels")


@dataclass
class TrainingMetrics:
    """types.py:28-45 — counters persisted in training_state and summary.json."""
    epoch: int = 0
    passes: int = 0
    completed_steps: int = 0
    samples: int = 0
    tokens: int = 0
    samples_too_old_to_queue: int = 0
    samples_too_old_to_train: int = 0
    last_broadcasted_version: int = 0
    train_loss: float = 1e9
    eval_loss: float = 1e9
    dev_loss: float = 1e9
    grad_norm: float = 0.0
    best_eval_loss: float = 1e9
    best_completed_steps: int = 0
    lr: float = 0.0
    time_waiting_for_data: float = 0.0


def _as_tensor(v, dtype):
    if v is None:
        return None
    if isinstance(v, torch.Tensor):
        return v.to(dtype)
    if isinstance(v, (list, tuple, np.ndarray)):
        return torch.as_tensor(np.asarray(v), dtype=dtype)
    raise ValueError(f"Unsupported type for {dtype} tensor: {type(v)}")


class PipelineBatchEncoding(BaseModel):
    """types.py:48-178."""

    model_config = ConfigDict(arbitrary_types_allowed=True)

    input_ids: torch.Tensor
    attention_mask: torch.Tensor
    labels: torch.Tensor
    position_ids: torch.Tensor | None = None

    rewards: torch.Tensor
    advantages: torch.Tensor
    ref_logprobs: torch.Tensor
    old_logprobs: torch.Tensor
    group_tokens: torch.Tensor
    num_labels: torch.Tensor
    overflow: torch.Tensor

    model_version: int
    sentinel: bool = False
    padding: int = 0
    is_packed: bool = False
    seq_boundaries: torch.Tensor | None = None

    pixel_values: torch.Tensor | None = None
    image_grid_thw: torch.Tensor | None = None
    # build-only, not part of the stream format: the loss rows q = b*(L-1)+t whose label is not
    # -100, computed on the host by the trainer's loader (the label-row lm_head needs their count
    # on the host: without this it reads it back from the device, a sync per micro-batch)
    _label_rows: torch.Tensor | None = PrivateAttr(default=None)

    @field_validator(*LONG_FIELDS, mode="before")
    @classmethod
    def _long(cls, v):
        return _as_tensor(v, torch.long)

    @field_validator("seq_boundaries", mode="before")
    @classmethod
    def _int(cls, v):
        return _as_tensor(v, torch.int)

    @field_validator(*FLOAT_FIELDS, mode="before")
    @classmethod
    def _float(cls, v):
        return _as_tensor(v, torch.float)

    def to_device(self, device: Union[str, torch.device], non_blocking: bool = False) -> "PipelineBatchEncoding":
        for name in type(self).model_fields:
            val = getattr(self, name)
            if isinstance(val, torch.Tensor):
                setattr(self, name, val.to(device, non_blocking=non_blocking))
        if self._label_rows is not None:
            self._label_rows = self._label_rows.to(device, non_blocking=non_blocking)
        return self

    def label_rows_from_host(self) -> torch.Tensor:
        """Record (and return) the label rows of this batch from its host-side labels."""
        lab = self.labels
        rows = torch.nonzero((lab[:, 1:] != -100).reshape(-1)).reshape(-1)
        self._label_rows = rows
        return rows

    @classmethod
    def from_dict(cls, data: dict[str, Any], **defaults) -> "PipelineBatchEncoding":
        merged = {**defaults, **data}
        known = {k: v for k, v in merged.items() if k in cls.model_fields}
        inst = cls(**known)
        extra = {k: v for k, v in merged.items() if k not in cls.model_fields}
        if extra:
            object.__setattr__(inst, "__pydantic_extra__", {**(inst.model_extra or {}), **extra})
        return inst

    def make_slices(self, num_slices: int) -> list["PipelineBatchEncoding"]:
        """Split a packed [1, T] batch into num_slices contiguous sequence-parallel slices."""
        if self.position_ids is None or self.input_ids.shape[0] > 1:
            raise ValueError("Cannot a batch that is not properly packed")
        T = self.input_ids.shape[1]
        if T < num_slices:
            raise ValueError(f"Cannot slice batch of size {T} into {num_slices} slices")
        if T % num_slices:
            raise ValueError(f"Sequence length {T} is not divisible by number of slices {num_slices}")
        step = T // num_slices
        out = []
        for i in range(num_slices):
            sl = slice(i * step, (i + 1) * step)
            fields = {k: getattr(self, k)[:, sl] for k in TOKEN_FIELDS}
            fields.update(model_version=self.model_version, sentinel=self.sentinel, is_packed=self.is_packed,
                          padding=self.padding, seq_boundaries=self.seq_boundaries,
                          pixel_values=self.pixel_values, image_grid_thw=self.image_grid_thw)
            out.append(PipelineBatchEncoding(**fields))
        return out
