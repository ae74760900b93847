"""One GPU's share of BASELINE configs[2] (C3): the Qwen2.5-7B trainer step on C3's packed math
rollouts (trainer_probe.dp_step_probe), for kernel profiles of that workload:

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run -- python3 tools/c3_step.py

``--snapshot`` also times the step with WeightUpdateManager's snapshot in flight
(trainer_probe.snapshot_overlap; its kernel trace shows prl_flatten_bf16 beside the step's kernels,
tools/kernel_overlap.py).  Prints the probe's JSON line.
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
    ap.add_argument("--snapshot", action="store_true")
    ap.add_argument("--paced-arms", default=None,
                    help="with --snapshot: the emulated broadcast-read arms as GBps:workgroups[:asleep][:one],... "
                         "(default trainer_probe.PACED_ARMS)")
    ap.add_argument("--grad-ckpt", action="store_true", help="gradient checkpointing (the reference config's)")
    ap.add_argument("--keep-layers", type=int, default=0, help="with --grad-ckpt: the last K layers keep activations")
    a = ap.parse_args()
    import gc
    import time

    import torch

    # host garbage collections inside the timed steps (TrainerStep.timed), by generation: count
    # and total ms (the stalls pipelinerl_amd/hostgc.py removes)
    gcs = {g: [0, 0.0] for g in range(3)}
    t_gc = [0.0]
    window = [False]

    def on_gc(phase, info):
        if phase == "start":
            t_gc[0] = time.perf_counter()
        elif window[0]:
            gcs[info["generation"]][0] += 1
            gcs[info["generation"]][1] += (time.perf_counter() - t_gc[0]) * 1e3

    from pipelinerl_amd import trainer_probe
    from pipelinerl_amd.trainer_probe import TrainerStep

    if a.paced_arms:
        # GBps:workgroups[:asleep][:one] (asleep: the workgroups held as long, two 64 KiB reads each per
        # bucket; one: a single launch for the whole buffer instead of one per 256 MiB bucket)
        trainer_probe.PACED_ARMS = {f"paced_{x[0]}GBps_{x[1]}wg" + "".join("_" + f for f in x[2:]):
                                    (float(x[0]), int(x[1]), *x[2:])
                                    for x in (y.split(":") for y in a.paced_arms.split(","))}

    timed = TrainerStep.timed

    def timed_window(self, *args, **kw):
        window[0] = True
        try:
            return timed(self, *args, **kw)
        finally:
            window[0] = False

    TrainerStep.timed = timed_window
    gc.callbacks.append(on_gc)

    from pipelinerl_amd.trainer_probe import dp_step_probe

    torch.cuda.set_device(0)

    r = dp_step_probe(a.config, micro_batches=a.micro_batches, steps=a.steps, warmup=a.warmup,
                      device=torch.device("cuda", 0), layers=a.layers, snapshot=a.snapshot, grad_ckpt=a.grad_ckpt,
                      keep_layers=a.keep_layers)
    r["grad_ckpt"], r["keep_layers"] = a.grad_ckpt, a.keep_layers
    r["host_gc"] = {f"gen{g}": {"n": n, "ms": round(ms, 1)} for g, (n, ms) in gcs.items()}
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
