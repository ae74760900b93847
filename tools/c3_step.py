"""One GPU's share of BASELINE configs[2] (C3): the Qwen2.5-7B trainer step on C3's packed math
rollouts (trainer_probe.dp_step_probe), for kernel profiles of that workload:

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run -- python3 tools/c3_step.py

Prints the probe's JSON line.
"""

from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--micro-batches", type=int, default=4)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--layers", type=int, default=None)
    a = ap.parse_args()
    import torch

    from pipelinerl_amd.trainer_probe import dp_step_probe

    torch.cuda.set_device(0)

    r = dp_step_probe(a.config, micro_batches=a.micro_batches, steps=a.steps, warmup=a.warmup,
                      device=torch.device("cuda", 0), layers=a.layers)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
