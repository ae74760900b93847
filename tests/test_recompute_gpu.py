"""Partial recompute on the GPU (finetune/recompute.py, checkpoints.keep_activations): a
patched-op Qwen2 (HIP RMSNorm / SwiGLU / RoPE, HIP attention, label-row lm_head + HIP loss head)
with every layer recomputed, the last 2 of 4 recomputing nothing, and all 4 kept, against the same
model without checkpointing: the gradients agree (the recomputed forward runs the same kernels on
the same inputs) and the peak memory grows with the layers kept."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _run(keep):
    from pipelinerl_amd.finetune.rl import rl_step
    from pipelinerl_amd.trainer_probe import packed_batch, qwen2_model, rl_config

    torch.cuda.empty_cache()
    model = qwen2_model("tiny", DEV, grad_ckpt=keep is not None, layers=4, keep_layers=keep or 0)
    b = packed_batch(8192, 1024, 128, 512, DEV, seed=3)
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated(DEV)
    torch.cuda.reset_peak_memory_stats(DEV)
    loss, _ = rl_step(model, b, 0, 10, rl_config(8))
    loss.backward()
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated(DEV) - base
    flags = [bool(getattr(m, "gradient_checkpointing", False)) for m in model.model.layers]
    return {n: p.grad.float().clone() for n, p in model.named_parameters()}, peak, flags


def test_partial_recompute_gradients_and_memory():
    ref, peak_none, _ = _run(None)
    peaks = {}
    for keep in (0, 2, 4):
        g, peaks[keep], flags = _run(keep)
        assert flags == [True] * (4 - keep) + [False] * keep
        worst = max(float((g[n] - r).norm() / (r.norm() + 1e-30)) for n, r in ref.items())
        assert worst <= 1e-2, (keep, worst)
    assert peaks[0] < peaks[2] < peaks[4], peaks
    print({"peak_mb": {k: round(v / 2**20, 1) for k, v in peaks.items()}, "no_ckpt_mb": round(peak_none / 2**20, 1)})
