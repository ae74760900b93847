"""GPU integration: rl_step (HIP loss head) through a real HF Qwen2 forward/backward, and the
trainer loop end to end on one MI355X."""

import json
import os
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.gpu


def _tiny_model(tmp, dtype):
    from loop_helpers import tiny_model_dir
    from transformers import AutoConfig, AutoModelForCausalLM

    d = tiny_model_dir(tmp)
    torch.manual_seed(0)
    from pipelinerl_amd.finetune.attention import register

    return AutoModelForCausalLM.from_config(AutoConfig.from_pretrained(d), dtype=dtype,
                                            attn_implementation=register()).cuda()


def test_rl_step_through_hf_model_matches_torch_reference(tmp_path):
    import copy
    import types

    from cpu_rl_step import cpu_rl_step
    from loop_helpers import EOS, rollouts
    from pipelinerl_amd.finetune.data import collate_packed
    from pipelinerl_amd.finetune.rl import RLConfig, rl_step

    model = _tiny_model(tmp_path, torch.float32)
    twin = copy.deepcopy(model)
    data = rollouts(2, 4)
    batch = collate_packed(data, types.SimpleNamespace(eos_token_id=EOS), 1).to_device("cuda")
    cfg = RLConfig(policy_loss="ppo", epsilon=0.2, kl_coef=0.05, final_kl_coef=0.05, entropy_bonus=0.01,
                   final_entropy_bonus=0.01, batch_size=8, clamp_log_ratio_ref_new_value=5)
    loss, stats = rl_step(model, batch, 0, 10, cfg)
    loss.backward()
    ref_loss, ref_stats = cpu_rl_step(twin, batch, 0, 10, cfg)
    ref_loss.backward()
    assert abs(float(loss) - float(ref_loss)) <= 1e-4 * max(1, abs(float(ref_loss)))
    assert abs(stats["entropy"] - ref_stats["entropy"]) <= 1e-4 * max(1, abs(ref_stats["entropy"]))
    for (n, p), (_, q) in zip(model.named_parameters(), twin.named_parameters()):
        err = float((p.grad - q.grad).abs().max())
        assert err <= 1e-5 + 1e-3 * float(q.grad.abs().max()), (n, err)


def test_trainer_loop_one_gpu(tmp_path):
    from loop_helpers import loop_cfg, rollouts, tiny_model_dir, write_training_data
    from pipelinerl_amd.finetune_loop import run_finetuning_loop
    from pipelinerl_amd.streams import reset_streams_backend, set_streams_backend

    reset_streams_backend()
    set_streams_backend("files")
    tiny_model_dir(tmp_path)
    data = rollouts(4, 4)
    write_training_data(tmp_path, data, 1, 28, 8)
    reset_streams_backend()
    for k in ("RANK", "WORLD_SIZE", "MASTER_ADDR"):
        os.environ.pop(k, None)
    cfg = loop_cfg(tmp_path, tmp_path / "tiny_qwen2", 1, 8, 2, load_as_bf16=True, dist_backend=None,
                   trace_gpu_phases=True)
    m = run_finetuning_loop(cfg)
    assert m.completed_steps == 2 and m.samples == 16
    lines = [json.loads(x) for x in (tmp_path / "finetune" / "logs" / "metrics.jsonl").read_text().splitlines()]
    assert all(np.isfinite(line["rl/loss"]) for line in lines)
    # HIP-event phase times (finetune/trace.py): every phase measured, within the step's span
    for line in lines:
        phases = [line[f"trace/{p}_ms"] for p in ("forward", "backward", "allreduce_wait", "clip", "optimizer")]
        assert all(v >= 0 for v in phases) and line["trace/forward_ms"] > 0 and line["trace/backward_ms"] > 0
        assert sum(phases) <= line["trace/gpu_step_ms"] * (1 + 1e-4) + 1e-3
    assert (tmp_path / "finetune" / "current" / "model.safetensors").exists()


def test_varlen_attention_gpu(tmp_path):
    from test_attention_cpu import check

    check(tmp_path, "cuda")


def _fsdp_rank(rank, port, exp):
    sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "pipelinerl-swe_amd")]
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from loop_helpers import loop_cfg
    from pipelinerl_amd.finetune_loop import run_finetuning_loop
    from pipelinerl_amd.streams import reset_streams_backend

    reset_streams_backend()
    exp = Path(exp)
    cfg = loop_cfg(exp, exp / "tiny_qwen2", 1, 8, 2, load_as_bf16=True, dist_backend=None, sharding="fsdp",
                   grad_reduce="mean")
    m = run_finetuning_loop(cfg)
    (exp / "fsdp_metrics.json").write_text(json.dumps({"steps": m.completed_steps, "samples": m.samples,
                                                       "backend": dist.get_backend()}))
    dist.destroy_process_group()


def test_trainer_loop_one_gpu_fsdp(tmp_path):
    """The FSDP2 path on the GPU (RCCL process group of one rank, HIP loss head): two steps,
    full-weight checkpoint and sharded optimizer state."""
    import torch.multiprocessing as mp
    from loop_helpers import rollouts, tiny_model_dir, write_training_data
    from pipelinerl_amd.streams import reset_streams_backend, set_streams_backend
    from test_weight_update_cpu import free_port

    reset_streams_backend()
    set_streams_backend("files")
    tiny_model_dir(tmp_path)
    write_training_data(tmp_path, rollouts(4, 4), 1, 28, 8)
    reset_streams_backend()
    mp.spawn(_fsdp_rank, args=(free_port(), str(tmp_path)), nprocs=1, join=True)
    m = json.loads((tmp_path / "fsdp_metrics.json").read_text())
    assert m == {"steps": 2, "samples": 16, "backend": "nccl"}
    lines = [json.loads(x) for x in (tmp_path / "finetune" / "logs" / "metrics.jsonl").read_text().splitlines()]
    assert all(np.isfinite(line["rl/loss"]) for line in lines)
    assert (tmp_path / "finetune" / "current" / "model.safetensors").exists()
    assert (tmp_path / "finetune" / "training_state" / "optim").is_dir()
