"""patch_model on a CPU model: every patched path (RMSNorm, SwiGLU MLP, the q/k/v group, the
decoder-layer forward with the fused residual adds) must fall back to the eager HF code off the
GPU and leave the model's outputs and gradients bit-identical (no HIP call is made: the kernels'
preconditions fail on CPU tensors).  The GPU tests cover the fused paths themselves."""

import copy

import torch


def test_patched_cpu_model_equals_eager(tmp_path):
    from loop_helpers import tiny_model_dir
    from transformers import AutoConfig, AutoModelForCausalLM

    from pipelinerl_amd.finetune.model_ops import patch_model

    cfg = AutoConfig.from_pretrained(tiny_model_dir(tmp_path, vocab=128))
    torch.manual_seed(0)
    eager = AutoModelForCausalLM.from_config(cfg, dtype=torch.float32)
    patched = copy.deepcopy(eager)
    counts = patch_model(patched)
    n = cfg.num_hidden_layers
    assert counts["rmsnorm"] == 2 * n + 1 and counts["swiglu_mlp"] == n
    assert counts["qkv_groups"] == n and counts["add_norm_layers"] == n
    ids = torch.randint(0, 128, (1, 24))
    outs = []
    for m in (eager, patched):
        lg = m(input_ids=ids, use_cache=False).logits
        lg.pow(2).mean().backward()
        outs.append(lg.detach())
    assert torch.equal(outs[0], outs[1])
    for (name, p), (_, q) in zip(eager.named_parameters(), patched.named_parameters()):
        assert torch.equal(p.grad, q.grad), name
    # no hand-over left pending on any norm after a full forward
    assert all(m.__dict__.get("_prl_pending") is None for m in patched.modules())
