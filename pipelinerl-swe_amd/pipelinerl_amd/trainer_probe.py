"""Trainer-step throughput probe: the full packed-GRPO optimizer step on Qwen2.5-shaped models
(random init — no checkpoints offline), as ``rl_finetuning_worker`` runs it
(finetune_loop.py; reference finetune_loop.py:567-719):

  per optimizer step and rank: ``micro_batches`` packed micro-batches of ``tokens`` tokens
  (forward with varlen attention, fused HIP loss head, backward); the last one is armed so the
  bucketed RCCL gradient all-reduce (GradBuckets) overlaps its backward; clip 0.3; fused AdamW.

Used by bench.py (key ``trainer_step``) and tools/trainer_step_bench.py.
"""

from __future__ import annotations

import time

import torch
import torch.distributed as dist

QWEN = {  # published Qwen2.5 shapes (config.json of each checkpoint)
    "0.5b": dict(hidden_size=896, intermediate_size=4864, num_hidden_layers=24, num_attention_heads=14,
                 num_key_value_heads=2, vocab_size=151936, tie_word_embeddings=True),
    "1.5b": dict(hidden_size=1536, intermediate_size=8960, num_hidden_layers=28, num_attention_heads=12,
                 num_key_value_heads=2, vocab_size=151936, tie_word_embeddings=True),
    "7b": dict(hidden_size=3584, intermediate_size=18944, num_hidden_layers=28, num_attention_heads=28,
               num_key_value_heads=4, vocab_size=152064, tie_word_embeddings=False),
}


def qwen2_model(name: str, device: torch.device, grad_ckpt: bool = False, fused_ops: bool = True):
    from transformers import AutoModelForCausalLM, Qwen2Config

    from .finetune.attention import register

    cfg = Qwen2Config(max_position_embeddings=32768, rope_theta=1e6, rms_norm_eps=1e-6, **QWEN[name])
    torch.manual_seed(0)
    with torch.device(device):  # initialise on the GPU (a CPU init of 1.5B+ params takes minutes)
        model = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16, attn_implementation=register())
    if fused_ops:
        from .finetune.model_ops import patch_model

        patch_model(model)
    if grad_ckpt:
        model.gradient_checkpointing_enable(gradient_checkpointing_kwargs={"use_reentrant": False})
    model.train()
    return model


def packed_batch(T: int, seq: int, prompt: int, V: int, device, seed: int = 0):
    """One packed micro-batch: T // seq rollouts of ``seq`` tokens (``prompt`` of them prompt)."""
    from .finetune.types import PipelineBatchEncoding

    g = torch.Generator().manual_seed(seed)
    nseq = T // seq
    pos = torch.arange(T) % seq
    ids = torch.randint(0, min(V, 151643), (1, T), generator=g)
    labels = torch.where(pos[None] >= prompt, ids, torch.full_like(ids, -100))
    rewards = torch.repeat_interleave(torch.randint(0, 2, (nseq,), generator=g).float(), seq)[None]
    lab = (labels != -100).float()
    old = (torch.randn((1, T), generator=g) - 12.0) * lab
    b = PipelineBatchEncoding(
        input_ids=ids, labels=labels, attention_mask=torch.ones_like(ids), position_ids=pos[None],
        rewards=rewards, advantages=rewards - rewards.mean(), ref_logprobs=old.clone(), old_logprobs=old,
        group_tokens=torch.full((1, T), float(seq)), num_labels=torch.full((1, T), float(seq - prompt)),
        overflow=torch.zeros((1, T)), seq_boundaries=torch.arange(0, T + 1, seq, dtype=torch.int32),
        model_version=0, is_packed=True)
    sb = b.seq_boundaries
    b.to_device(device)
    b.seq_boundaries = sb  # host metadata, as the trainer's loader keeps it
    return b


def rl_config(samples_per_step: int, fused_head: bool = False):
    from .finetune.rl import RLConfig

    # GRPO defaults (conf/finetune/base.yaml + grpo.yaml): ppo, eps 4, kl 0, C 5
    return RLConfig(policy_loss="ppo", epsilon=4.0, kl_coef=0.0, final_kl_coef=0.0, clamp_log_ratio_ref_new_value=5,
                    batch_size=samples_per_step, fused_lm_head=fused_head)


def trainer_step_probe(name: str = "1.5b", tokens: int = 16384, seq: int = 2048, prompt: int = 256,
                       micro_batches: int = 4, steps: int = 3, warmup: int = 1, device=None,
                       fused_head: bool = False, grad_ckpt: bool = False, fused_ops: bool = True) -> dict:
    from .finetune.grad_sync import GradBuckets
    from .finetune.optim import get_optimizer
    from .finetune.rl import rl_step

    device = device or torch.device("cuda", torch.cuda.current_device())
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    torch.cuda.reset_peak_memory_stats(device)
    model = qwen2_model(name, device, grad_ckpt, fused_ops)
    opt = get_optimizer("adamw_torch", model, 1e-6, 0.01)
    grads = GradBuckets(list(model.parameters())) if world > 1 else None
    batches = [packed_batch(tokens, seq, prompt, QWEN[name]["vocab_size"], device, seed=rank * 97 + i)
               for i in range(micro_batches)]
    cfg = rl_config(micro_batches * (tokens // seq) * world, fused_head)

    def one_step():
        for i, b in enumerate(batches):
            if grads is not None and i == len(batches) - 1:
                grads.arm()
            loss, _ = rl_step(model, b, 0, 100, cfg)
            loss.backward()
        if grads is not None:
            grads.finish()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 0.3)
        opt.step()
        if grads is not None:
            grads.zero_()
        else:
            opt.zero_grad(set_to_none=True)

    for _ in range(warmup):
        one_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        one_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    sec = float(dt) / steps
    peak = torch.cuda.max_memory_allocated(device) / 1e9
    if grads is not None:
        grads.remove()
    del model, opt, grads, batches
    torch.cuda.empty_cache()
    total = tokens * micro_batches * world
    return {"model": f"Qwen2.5-{name} shapes (random init, bf16)", "tokens_per_micro_batch": tokens,
            "micro_batches_per_step": micro_batches, "seq_len": seq, "prompt_len": prompt,
            "loss_head": "fused_lm_head" if fused_head else "fused", "fused_model_ops": fused_ops,
            "ms_per_optimizer_step": round(sec * 1e3, 2),
            "tokens_per_s": round(total / sec, 1), "tokens_per_s_per_gpu": round(total / sec / world, 1),
            "peak_mem_gb": round(peak, 2), "steps": steps, "warmup": warmup}
