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


def test_plan_bounds_the_measured_peak_per_kept_layers():
    """The plan's estimate (finetune/recompute.py, without its fixed headroom) against the measured
    peak of the C3 step on an 8-layer 7B-shaped model (2 of C3's packed micro-batches, AdamW) with
    0, 4 and 8 layers keeping their activations: an upper bound within 1.3 x at every K."""
    import gc

    from transformers import AutoModelForCausalLM, Qwen2Config

    from pipelinerl_amd import workloads
    from pipelinerl_amd.finetune.recompute import HEADROOM_BYTES, HEADROOM_FRAC, plan_gradient_checkpointing
    from pipelinerl_amd.trainer_probe import QWEN, dp_step_probe

    batches = workloads.micro_batches("c3", 2, seed=1234)
    T = max(int(b.attention_mask.sum()) for b in batches)
    with torch.device("meta"):
        meta = AutoModelForCausalLM.from_config(Qwen2Config(**dict(QWEN["7b"], num_hidden_layers=8)),
                                                dtype=torch.bfloat16)
    dev_bytes = torch.cuda.get_device_properties(DEV).total_memory
    out = {}
    for keep in (0, 4, 8):
        gc.unfreeze()  # the probe freezes the heap it sets up (as the loop does): release the last one
        gc.collect()
        torch.cuda.empty_cache()
        base = torch.cuda.memory_allocated(DEV)  # the probe's peak counts from here
        r = dp_step_probe("c3", steps=1, warmup=1, device=DEV, layers=8, batches=batches, grad_ckpt=True,
                          keep_layers=keep)
        peak = r["peak_mem_gb"] * 1e9 - base
        args = {"gradient_checkpointing": True, "seq_length": T, "gradient_checkpointing_keep_layers": keep}
        p = plan_gradient_checkpointing(args, meta, DEV, device_bytes=dev_bytes)
        est = p.need_bytes - int(HEADROOM_FRAC * dev_bytes) - HEADROOM_BYTES
        out[keep] = (round(peak / 1e9, 2), round(est / 1e9, 2))
        assert peak <= est <= 1.3 * peak, (keep, out)
    print({"peak_vs_estimate_gb": out, "tokens": T})
