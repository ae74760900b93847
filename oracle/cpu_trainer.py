"""CPU baseline of one finetune micro-batch step (TEST / BASELINE INFRASTRUCTURE — never the product
path; only ``bench.py``'s ``cpu_baseline`` leg and tests may import it).

Restates what the reference's CPU finetune path (BASELINE.json configs[0], C1: Qwen2.5-0.5B,
world_size 1, no actor) does per micro-batch, ``pipelinerl/finetune_loop.py:620-719``:
HF Qwen2 forward (eager torch on CPU, ``attn_implementation="sdpa"``), ``rl_step``'s loss head
(``rl/__init__.py:199-377``) — here the pinned numpy oracle (``grpo_oracle.rl_step_oracle``, which
also yields d loss / d logits) — the model backward from those logit gradients, gradient clipping
at 0.3 and AdamW.  Random-init weights of the published 0.5B shapes (no checkpoints offline),
bf16 as on the GPU.  Timed on the host cores of the GPU box, so the GPU trainer step has a CPU
number beside it (a reported baseline, not a target).
"""

from __future__ import annotations

import time

import numpy as np
import torch

from . import grpo_oracle, synth

QWEN05 = dict(hidden_size=896, intermediate_size=4864, num_hidden_layers=24, num_attention_heads=14,
              num_key_value_heads=2, vocab_size=151936, tie_word_embeddings=True, max_position_embeddings=4096,
              rope_theta=1e6, rms_norm_eps=1e-6)
GRPO = dict(policy_loss="ppo", epsilon=4.0, kl_coef=0.0, final_kl_coef=0.0, clamp_log_ratio_ref_new_value=5)


def qwen05_cpu(dtype=torch.bfloat16, layers: int | None = None):
    """The 0.5B architecture on CPU with cheap deterministic weights (meta init + normal_: an HF
    random init of 0.5B parameters takes ~40 s on 8 cores and the values do not matter here)."""
    from transformers import AutoModelForCausalLM, Qwen2Config

    cfg = Qwen2Config(**dict(QWEN05, **({"num_hidden_layers": layers} if layers else {})))
    with torch.device("meta"):
        model = AutoModelForCausalLM.from_config(cfg, dtype=dtype, attn_implementation="sdpa")
    model.to_empty(device="cpu")
    g = torch.Generator().manual_seed(0)
    with torch.no_grad():
        for name, p in model.named_parameters():
            if name.endswith("norm.weight"):
                p.fill_(1.0)
            elif name.endswith(".bias"):
                p.zero_()
            else:
                p.copy_(torch.randn(p.shape, generator=g, dtype=torch.float32).mul_(0.02).to(dtype))
    rot = type(model.model.rotary_emb)(config=cfg)  # to_empty dropped the non-persistent inv_freq
    model.model.rotary_emb = rot
    model.tie_weights()
    return model.train()


def micro_batch(n_seq: int, seq: int, prompt: int, V: int, seed: int = 11) -> dict:
    """n_seq rollouts of ``seq`` tokens as an unpacked [n_seq, seq] batch (rl_step's non-packed
    path), RL fields as populate_rl_data would give them (oracle/synth.py)."""
    b = synth.packed_rl_batch(seed, [seq] * n_seq, [prompt] * n_seq, id_range=min(V, 151643), eos=151643,
                              rewards=[float(i % 2) for i in range(n_seq)])  # nonzero advantages
    m = b["labels"] != -100
    rng = np.random.default_rng(seed)
    b["old_logprobs"] = np.where(m, rng.normal(-3, 1, m.shape), 0).astype(np.float32)
    b["ref_logprobs"] = b["old_logprobs"].copy()
    out = {k: (v.reshape(n_seq, seq) if isinstance(v, np.ndarray) and v.ndim == 2 else v) for k, v in b.items()}
    out["is_packed"] = False
    out["position_ids"] = np.tile(np.arange(seq), (n_seq, 1))
    return out


def cpu_trainer_step(n_seq: int = 2, seq: int = 512, prompt: int = 128, threads: int = 16, layers: int | None = None,
                     steps: int = 1) -> dict:
    """Tokens/s of ``steps`` timed micro-batch steps (after one short untimed warm-up step)."""
    torch.set_num_threads(threads)
    model = qwen05_cpu(layers=layers)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-6, weight_decay=0.01)
    V = QWEN05["vocab_size"]

    def step(b):
        ids = torch.from_numpy(b["input_ids"])
        out = model(input_ids=ids, attention_mask=torch.ones_like(ids), use_cache=False)
        lg = out.logits.detach().float().numpy()
        o = grpo_oracle.rl_step_oracle(lg, b, dict(GRPO, batch_size=b["input_ids"].shape[0]), 0, 100,
                                       dtype=np.float32, threads=threads, row_chunk=16)
        out.logits.backward(torch.from_numpy(o["dlogits"]).to(out.logits.dtype))
        torch.nn.utils.clip_grad_norm_(model.parameters(), 0.3)
        opt.step()
        opt.zero_grad(set_to_none=True)
        return o["loss"]

    step(micro_batch(1, 64, 16, V))
    b = micro_batch(n_seq, seq, prompt, V)
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step(b)
    dt = (time.perf_counter() - t0) / steps
    tokens = n_seq * seq
    return {"value": round(tokens / dt, 1), "unit": "tokens/s", "cores": threads, "kind": "port",
            "sample": f"{steps} x Qwen2.5-0.5B-shaped (random init, bf16) micro-batch step of {n_seq} x {seq} tokens "
                      f"on CPU: HF forward, numpy-oracle loss head + dlogits, backward, clip, AdamW; {dt:.2f} s/step",
            "loss": float(loss)}


def cpu_c1_step(threads: int, sample_micro_batches: int = 2) -> dict:
    """BASELINE.json configs[0] (C1) on CPU, as BASELINE.md §3 / SURVEY.md §8(d) describe it:
    Qwen2.5-0.5B shapes, 256 rollouts (32 groups x 8, prompt U{32..128} + completion U{16..384})
    packed at seq_length 4096 by the preprocessor's packer, ONE optimizer step (every micro-batch:
    HF forward with packed-sequence attention, the oracle's loss head + d loss / d logits,
    backward; then clip 0.3 and AdamW).  Bounded sample: the first ``sample_micro_batches``
    micro-batches are run and timed, the optimizer tail once; the step time is their per-token
    time x the step's tokens (Σ attention_mask, finetune_loop.py:259-263) + the tail."""
    from pipelinerl_amd import workloads
    from pipelinerl_amd.finetune.attention import packed_kwargs, register
    from transformers import AutoModelForCausalLM, Qwen2Config

    torch.set_num_threads(threads)
    data = workloads.rollouts("c1", 256)
    mbs = [b for _, b in workloads.pack(data, 4096, 256) if not b.sentinel]
    step_tokens = sum(int(b.attention_mask.sum()) for b in mbs)
    model = qwen05_cpu()
    cfg = Qwen2Config(**QWEN05)
    cfg._attn_implementation = register()  # packed rollouts: attention stays inside each one
    model.config._attn_implementation = cfg._attn_implementation
    for layer in model.model.layers:
        layer.self_attn.config._attn_implementation = cfg._attn_implementation
    opt = torch.optim.AdamW(model.parameters(), lr=1e-6, weight_decay=0.01)
    rl = dict(GRPO, batch_size=256)

    def micro(b):
        ids = b.input_ids
        out = model(input_ids=ids, position_ids=b.position_ids, use_cache=False, **packed_kwargs(b, ids.device))
        lg = out.logits.detach().float().numpy()
        host = {k: getattr(b, k).numpy() for k in ("input_ids", "labels", "position_ids", "rewards", "advantages",
                                                   "ref_logprobs", "old_logprobs", "group_tokens", "num_labels",
                                                   "overflow")}
        host["is_packed"] = True
        o = grpo_oracle.rl_step_oracle(lg, host, rl, 0, 1, dtype=np.float32, threads=threads, row_chunk=16)
        out.logits.backward(torch.from_numpy(o["dlogits"]).to(out.logits.dtype))
        return int(b.attention_mask.sum())

    micro(mbs[-1])  # untimed warm-up on the shortest (tail) micro-batch
    opt.zero_grad(set_to_none=True)
    t0 = time.perf_counter()
    sampled = sum(micro(b) for b in mbs[:sample_micro_batches])
    t_mb = time.perf_counter() - t0
    t1 = time.perf_counter()
    torch.nn.utils.clip_grad_norm_(model.parameters(), 0.3)
    opt.step()
    opt.zero_grad(set_to_none=True)
    t_tail = time.perf_counter() - t1
    t_step = t_mb / sampled * step_tokens + t_tail
    return {"value": round(step_tokens / t_step, 1), "unit": "tokens/s", "cores": threads, "kind": "port",
            "sample": f"C1: Qwen2.5-0.5B-shaped (random init, bf16) optimizer step over 256 rollouts = "
                      f"{len(mbs)} packed micro-batches, {step_tokens} tokens; {sample_micro_batches} micro-batches "
                      f"({sampled} tokens, {t_mb:.1f} s) + clip/AdamW ({t_tail:.1f} s) timed, step = per-token time "
                      f"x step tokens + tail = {t_step:.1f} s; HF forward, numpy-oracle loss head, backward",
            "step_tokens": step_tokens, "micro_batches": len(mbs), "step_s": round(t_step, 2)}
