"""GPU phase timing of the trainer step (SURVEY.md §5 tracing row: the reference has only wall-clock
stamps, logging_.py:78-81 and finetune_loop.py:598/:677).

``PhaseTrace.mark(name)`` records a HIP event on the current stream at the END of phase ``name``
(the phase runs from the previous mark); nothing is read back until ``collect()``, which the loop
calls where it already waits for the device (the grad-norm read after the optimizer step), so the
trace adds no host synchronisation.  Per optimizer step it reports ``trace/<phase>_ms`` summed
over the step's micro-batches and ``trace/gpu_step_ms`` (first to last mark).  On a CPU device the
marks are wall-clock stamps.  Enabled by ``finetune.trace_gpu_phases`` or ``PRL_TRACE_GPU=1``.
"""

from __future__ import annotations

import time
from collections import defaultdict

import torch


class PhaseTrace:
    def __init__(self, device: torch.device, enabled: bool = True):
        self.device = torch.device(device)
        self.enabled = enabled
        self.on_gpu = self.device.type == "cuda"
        self._marks: list[tuple[str, object]] = []

    def _stamp(self):
        if self.on_gpu:
            e = torch.cuda.Event(enable_timing=True)
            e.record(torch.cuda.current_stream(self.device))
            return e
        return time.perf_counter()

    def start(self) -> None:
        """The step's first mark (the start of its first phase)."""
        if self.enabled:
            self._marks = [("", self._stamp())]

    def mark(self, name: str) -> None:
        if not self.enabled:
            return
        if not self._marks:
            self.start()
        self._marks.append((name, self._stamp()))

    def collect(self) -> dict[str, float]:
        """Phase totals (ms) of the marks since start(); waits for the last event only."""
        if not self.enabled or len(self._marks) < 2:
            self._marks = []
            return {}
        marks, self._marks = self._marks, []
        if self.on_gpu:
            marks[-1][1].synchronize()
            dt = lambda a, b: a.elapsed_time(b)  # noqa: E731
        else:
            dt = lambda a, b: (b - a) * 1e3  # noqa: E731
        out: dict[str, float] = defaultdict(float)
        for (_, a), (name, b) in zip(marks, marks[1:]):
            out[f"trace/{name}_ms"] += dt(a, b)
        out["trace/gpu_step_ms"] = dt(marks[0][1], marks[-1][1])
        return dict(out)
