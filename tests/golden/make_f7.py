"""F7 fixture: the trainer's per-step ``stats/*`` and ``throughput/*`` metrics
(pipelinerl/finetune_loop.py:725-764) at world size 2, from the reference's own expression.

Run in the build container only (reads /root/reference; writes data):

    PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_f7.py

finetune_loop.py does not import here (deepspeed, ring_flash_attn): the dict literal passed to
``metrics_dict.update`` that holds ``throughput/real_tokens_per_sec`` is taken from the file's
syntax tree and evaluated in a namespace holding the names it reads (training metrics, lag stats,
the batch queue, this worker's token counts and pass times, the accelerator's process count, ...).
Only inputs and the evaluated values are stored.
"""

from __future__ import annotations

import ast
import json
import types
from pathlib import Path

HERE = Path(__file__).resolve().parent
REF = Path("/root/reference/pipelinerl/finetune_loop.py")


def metrics_expr():
    tree = ast.parse(REF.read_text())
    for node in ast.walk(tree):
        if isinstance(node, ast.Dict) and any(isinstance(k, ast.Constant) and k.value == "throughput/real_tokens_per_sec"
                                              for k in node.keys):
            return compile(ast.Expression(body=node), str(REF), "eval")
    raise RuntimeError("metrics dict not found")


CASES = [
    dict(world=2, tokens=[4096, 3000, 4000, 1200], passes=[0.31, 0.27, 0.30, 0.12], mbs=[7, 5, 6, 2],
         samples_per_step=40, step_took=1.37, lag={"min_version": 96, "max_version": 128}, qsize=1,
         metrics=dict(lr=3e-6, grad_norm=0.71, samples=160, tokens=2 * 24592, samples_too_old_to_queue=0,
                      samples_too_old_to_train=3, passes=16, completed_steps=4, epoch=0, time_waiting_for_data=0.52,
                      last_broadcasted_version=160)),
    dict(world=2, tokens=[12000], passes=[2.5], mbs=[11], samples_per_step=22, step_took=2.9,
         lag={"min_version": 0, "max_version": 0}, qsize=0,
         metrics=dict(lr=1e-6, grad_norm=0.0, samples=22, tokens=24000, samples_too_old_to_queue=2,
                      samples_too_old_to_train=0, passes=1, completed_steps=1, epoch=1, time_waiting_for_data=0.0,
                      last_broadcasted_version=0)),
]


def main():
    code = metrics_expr()
    out = []
    for c in CASES:
        acc = types.SimpleNamespace(state=types.SimpleNamespace(num_processes=c["world"]))
        q = types.SimpleNamespace(qsize=lambda n=c["qsize"]: n)
        ns = dict(training_metrics=types.SimpleNamespace(**c["metrics"]), lag_stats=dict(c["lag"]), batch_queue=q,
                  this_worker_tokens=sum(c["tokens"]), tokens_processed=list(c["tokens"]),
                  passes_took=list(c["passes"]), micro_batches_size=list(c["mbs"]),
                  samples_per_step=c["samples_per_step"], step_took=c["step_took"], get_accelerator=lambda: acc)
        values = eval(code, ns)  # the reference's expression over stand-in values only
        out.append({"inputs": c, "expected": values})
    (HERE / "f7_step_metrics.json").write_text(json.dumps(out, indent=1, sort_keys=True) + "\n")


if __name__ == "__main__":
    main()
