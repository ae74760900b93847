"""Fused gate/up vs separate projections over three optimizer steps of a 2-layer Qwen2.5-0.5B-shaped
model (native AdamW, lr 1e-3): relative difference of the MLP weights' total updates.  With
``--stale`` the native AdamW's version-counter bump is disabled (the pre-fix behaviour), to show
the check discriminates.  Prints one JSON line."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "pipelinerl-swe_amd"))
from pipelinerl_amd.finetune import model_ops, optim  # noqa: E402
from pipelinerl_amd.trainer_probe import TrainerStep  # noqa: E402


def updates(fused: bool, steps: int = 3, lr: float = 1e-3) -> dict:
    model_ops._FUSED_GATE_UP = fused
    ts = TrainerStep("0.5b", tokens=2048, seq=1024, prompt=128, micro_batches=2, device="cuda", layers=2)
    for g in ts.opt.param_groups:
        g["lr"] = lr
    w0 = {n: p.detach().clone() for n, p in ts.model.named_parameters() if ".mlp." in n}
    for _ in range(steps):
        ts.step()
    torch.cuda.synchronize()
    out = {n: (p.detach().float() - w0[n].float()) for n, p in ts.model.named_parameters() if ".mlp." in n}
    ts.close()
    return out


def main():
    if "--stale" in sys.argv:
        optim.increment_version = lambda *a, **k: None
    a, b = updates(True), updates(False)
    rel = {n: float((a[n] - b[n]).norm() / b[n].norm()) for n in a}
    print(json.dumps({"stale": "--stale" in sys.argv, "max_rel": max(rel.values()), "rel": rel}))


if __name__ == "__main__":
    main()
