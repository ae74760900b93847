"""Test infrastructure for tests/test_launcher_cpu.py (never on the product path).

Put on PYTHONPATH of the reference launcher's command, it makes each trainer rank (a process
that has LOCAL_RANK set by the launcher) train with the CPU torch restatement of rl_step
(tests/cpu_rl_step.py) instead of the HIP loss head, which needs a GPU: the only thing it
changes is ``run_finetuning_loop``'s default ``step_fn``.  The launcher, the entry script run by
path, the config loader and the loop itself are the product's."""

import os
import sys
from pathlib import Path

if os.environ.get("PRL_TEST_CPU_STEP") == "1" and "LOCAL_RANK" in os.environ:
    _root = Path(__file__).resolve().parents[2]
    sys.path[:0] = [str(_root / "tests"), str(_root / "pipelinerl-swe_amd")]
    from cpu_rl_step import cpu_rl_step  # noqa: E402

    import pipelinerl_amd.finetune_loop as _fl  # noqa: E402

    _d = list(_fl.run_finetuning_loop.__defaults__)
    _d[0] = cpu_rl_step
    _fl.run_finetuning_loop.__defaults__ = tuple(_d)
