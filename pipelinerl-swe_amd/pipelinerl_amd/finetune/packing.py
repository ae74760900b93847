"""Per-trainer micro-batch packing with exact per-step sample quotas and sentinel batches —
the preprocessor's write loop (pipelinerl/preprocess.py:557-626, seq_packing branch),
restated as a deterministic state machine so the trainer's input contract can be produced
(stream replay, tests, benchmarks) without the preprocessor process.

For every optimizer step each lead trainer gets exactly ``samples_per_lead_per_step``
samples, packed greedily into micro-batches of at most ``seq_length`` tokens; a trainer
whose quota for the step is full receives sentinel batches until the step's global sample
count is reached; trainers are served round-robin (stride = seq_parallel).
"""

from __future__ import annotations

from collections import deque
from typing import Any, Iterable

from .data import collate_packed
from .types import PipelineBatchEncoding
from .utils import create_sentinel_batch


def filter_zero_advantage_groups(dataset: list[dict[str, Any]], epsilon: float = 1e-6) -> tuple[list[dict[str, Any]], int]:
    """Drop every group whose rollouts all have |advantage| <= epsilon on every token
    (pipelinerl/preprocess.py:287-324; applied to each populated chunk before packing when
    ``rl.filter_zero_advantage_groups`` is set, :509-513).  Kept groups come out in order of
    their first appearance, each group's entries in input order; returns (kept, number dropped).
    A NaN advantage counts as zero (``abs(nan) > epsilon`` is false), as in the reference."""
    groups: dict[Any, list[dict[str, Any]]] = {}
    for entry in dataset:
        groups.setdefault(entry["group_id"], []).append(entry)
    kept: list[dict[str, Any]] = []
    dropped = 0
    for entries in groups.values():
        if any(abs(a) > epsilon for e in entries for a in e["advantages"]):
            kept.extend(entries)
        else:
            dropped += len(entries)
    return kept, dropped


class MicroBatchPacker:
    def __init__(self, num_trainers: int, seq_length: int, samples_per_lead_per_step: int, tokenizer,
                 seq_parallel: int = 1):
        if num_trainers % seq_parallel:
            raise ValueError("num_trainers must be divisible by seq_parallel")
        self.num_trainers = num_trainers
        self.seq_length = seq_length
        self.seq_parallel = seq_parallel
        self.per_lead = samples_per_lead_per_step
        self.tokenizer = tokenizer
        self.train_batch_size = samples_per_lead_per_step * (num_trainers // seq_parallel)
        self.queue: deque[dict[str, Any]] = deque()
        self.trainer_id = 0
        self.samples_per_trainer = [0] * num_trainers
        self.target = samples_per_lead_per_step
        self.published = 0
        self.batch_boundary = self.train_batch_size
        self.current: list[dict[str, Any]] = []
        self.current_length = 0
        self.max_model_version = 0

    def _advance(self):
        self.trainer_id = (self.trainer_id + self.seq_parallel) % self.num_trainers

    def feed(self, entries: Iterable[dict[str, Any]]) -> list[tuple[int, PipelineBatchEncoding]]:
        """Queue processed samples; return the (trainer_id, micro_batch) writes now possible."""
        appended = False
        for e in entries:
            self.queue.append(e)
            appended = True
        if appended:  # preprocess.py:542-546: the max over the entries still queued, after the appends
            self.max_model_version = max(int(e.get("model_version", 0)) for e in self.queue)
        out: list[tuple[int, PipelineBatchEncoding]] = []
        while self.queue:  # the reference's outer loop re-enters the write loop after each step
            out.extend(self._write_step())
        return out

    def _write_step(self) -> list[tuple[int, PipelineBatchEncoding]]:
        out: list[tuple[int, PipelineBatchEncoding]] = []
        batch_done = False
        while self.queue and not batch_done:
            tid = self.trainer_id
            if self.samples_per_trainer[tid] == self.target:
                out.append((tid, create_sentinel_batch(None, self.tokenizer, self.max_model_version)))
                self._advance()
            else:
                write = False
                while self.queue:
                    n = len(self.queue[0]["input_ids"])
                    if self.current_length + n > self.seq_length:
                        write = True
                        break
                    self.current.append(self.queue.popleft())
                    self.current_length += n
                    if len(self.current) + self.samples_per_trainer[tid] == self.target:
                        write = True
                        break
                if write:
                    if not self.current:
                        raise AssertionError("Current batch should not be empty when writing "
                                             f"(a sample is longer than seq_length={self.seq_length})")
                    out.append((tid, collate_packed(self.current, self.tokenizer, self.seq_parallel)))
                    self.published += len(self.current)
                    self.samples_per_trainer[tid] += len(self.current)
                    self._advance()
                    self.current = []
                    self.current_length = 0
            batch_done = self.published == self.batch_boundary and self.trainer_id == 0
            if batch_done:
                self.batch_boundary += self.train_batch_size
                self.target += self.per_lead
        return out
