"""Diagnostic: bench.py with GradBuckets' side stream at normal priority (the round-5 setting), for
the one-GPU multi-rank rehearsal A/B.  Usage as bench.py (torch.distributed.run … this file …)."""
import runpy
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]

import torch  # noqa: E402

from pipelinerl_amd.finetune import grad_sync  # noqa: E402

_orig_init = grad_sync.GradBuckets.__init__


def _init(self, *a, **k):
    _orig_init(self, *a, **k)
    if self.stream is not None:
        self.stream = torch.cuda.Stream(device=self.stream.device)


grad_sync.GradBuckets.__init__ = _init
sys.argv[0] = str(ROOT / "bench.py")
runpy.run_path(str(ROOT / "bench.py"), run_name="__main__")
