"""FSDP2 resharding with the build's patched model ops on the GPU: two ranks share cuda:0 over
gloo (RCCL needs one GPU per rank), so FSDP really frees each layer's unsharded parameters after
the forward and all-gathers them again for the backward — the case where PrlLinearFn / RMSNorm /
SwiGLU / RoPE autograd functions must find their saved parameters re-gathered in place.  The
sharded gradients (mean over the two ranks' batches) must equal one unsharded model's gradients
of the mean loss — also with gradient checkpointing on the first layer and the second keeping its
activations (checkpoints.keep_activations, the plan's partial recompute), where the recomputed
layer's forward runs inside FSDP's backward."""

import os
import sys
from pathlib import Path

import pytest
import torch
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu


def _model(tmp):
    from loop_helpers import tiny_model_dir
    from transformers import AutoConfig, AutoModelForCausalLM

    from pipelinerl_amd.finetune.attention import register
    from pipelinerl_amd.finetune.model_ops import patch_model

    cfg = AutoConfig.from_pretrained(tiny_model_dir(Path(tmp), vocab=512))
    cfg.hidden_size, cfg.intermediate_size, cfg.num_attention_heads, cfg.num_key_value_heads = 256, 512, 2, 1
    torch.manual_seed(0)
    m = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16, attn_implementation=register()).to("cuda:0")
    patch_model(m)
    return m


def _loss(m, ids, pos, kw):
    return m(input_ids=ids, position_ids=pos, use_cache=False, **kw).logits.float().pow(2).mean()


def _batch(rank):
    from pipelinerl_amd.finetune.attention import packed_kwargs

    g = torch.Generator().manual_seed(100 + rank)
    ids = torch.randint(0, 512, (1, 192), generator=g).to("cuda:0")
    pos = torch.cat([torch.arange(128), torch.arange(64)])[None].to("cuda:0")
    b = type("B", (), {"seq_boundaries": torch.tensor([0, 128, 192]), "position_ids": pos})()
    return ids, pos, packed_kwargs(b, "cuda:0")


def _run(rank, port, tmp, keep):
    sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd"), str(ROOT / "tests")]
    os.environ["OMP_NUM_THREADS"] = "1"
    import torch.distributed as dist

    from pipelinerl_amd.finetune.sharding import shard_model

    torch.cuda.set_device(0)
    # gloo for CUDA tensors too: FSDP's device mesh would otherwise open an RCCL group, which
    # cannot span two ranks on one GPU
    dist.init_process_group("cpu:gloo,cuda:gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    m = _model(tmp)
    if keep is not None:
        from pipelinerl_amd.finetune.checkpoints import keep_activations

        m.gradient_checkpointing_enable(gradient_checkpointing_kwargs={"use_reentrant": False})
        assert keep_activations(m, keep) == keep
    m = shard_model(m)
    ids, pos, kw = _batch(rank)
    _loss(m, ids, pos, kw).backward()
    grads = {n: p.grad.full_tensor().float().cpu() for n, p in m.named_parameters()}
    if rank == 0:
        ref = _model(tmp)  # unsharded, same init: gradient of the mean of both ranks' losses
        (0.5 * sum(_loss(ref, *_batch(r)) for r in range(2))).backward()
        torch.save({"fsdp": grads, "ref": {n: p.grad.float().cpu() for n, p in ref.named_parameters()}},
                   Path(tmp) / "grads.pt")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("keep", [None, 1])
def test_fsdp_resharding_with_patched_ops(tmp_path, keep):
    from test_weight_update_cpu import free_port

    mp.spawn(_run, args=(free_port(), str(tmp_path), keep), nprocs=2, join=True)
    d = torch.load(tmp_path / "grads.pt")
    for n, r in d["ref"].items():
        g = d["fsdp"][n]
        err = float((g - r).abs().max())
        assert err <= 3e-2 * float(r.abs().max()) + 1e-6, (n, err)
