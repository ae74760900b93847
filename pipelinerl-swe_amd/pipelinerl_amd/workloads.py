"""Synthetic packed-GRPO workloads of BASELINE.json's configs, shared by
bench.py, the GPU parity tests and the CPU baseline (measurement infrastructure: no product code
path imports this module).

Generator: numpy ``Generator(PCG64(seed))``, seed 1234; token ids uniform in
[0, 151643); EOS 151643 appended to 75 % of the rollouts ("finished"); rewards Bernoulli(0.5) per
rollout; groups of ``attempts`` rollouts share a prompt length; per-token fields from the build's
``prepare_rl_fields`` / ``populate_rl_data`` (the reference's rl/__init__.py:380-525, pinned to
the F3 fixture) with GRPO defaults (advantage = reward − group mean, no std division).
``old_logprobs`` are −|N(0, 1.5²)| on completion tokens (a trained policy's log-probs are not
available without its logits); ``ref_logprobs`` = old (the fork's default) or
old + N(0, 0.05²) for C5 (KL-to-reference on).

  c1  Qwen2.5-0.5B, 32 groups x 8, prompt U{32..128} + completion U{16..384} (<= 512 tokens),
      packed at seq_length 4096, 256 samples per optimizer step (conf/finetune/base.yaml:61 with
      the C1 cap)
  c3  Qwen2.5-7B math: prompt U{64..512} + completion U{256..8192} (max_tokens 8192,
      conf/base.yaml:47), packed at seq_length 12000 (conf/finetune/base.yaml:61)
  c5  Qwen2.5-32B: the c3 rollouts with ref = old + N(0, 0.05²) and kl_coef 0.001
      (conf/deepscaler15b.yaml:34)
"""

from __future__ import annotations

import copy
import types
from dataclasses import dataclass

import numpy as np

EOS = 151643  # Qwen2.5 <|endoftext|>
ID_RANGE = 151643


@dataclass(frozen=True)
class Spec:
    model: str
    prompt: tuple[int, int]
    completion: tuple[int, int]
    max_total: int | None
    attempts: int
    seq_length: int
    kl_coef: float = 0.0
    ref_noise: float = 0.0


SPECS = {
    "c1": Spec("0.5b", (32, 128), (16, 384), 512, 8, 4096),
    "c3": Spec("7b", (64, 512), (256, 8192), None, 8, 12000),
    "c5": Spec("32b", (64, 512), (256, 8192), None, 8, 12000, kl_coef=0.001, ref_noise=0.05),
}


def rollouts(config: str, n: int, seed: int = 1234, max_completion: int | None = None) -> list[dict]:
    """``n`` processed rollouts (dicts in the preprocessor's output format) of ``config``."""
    from .finetune.rl import RLConfig, populate_rl_data, prepare_rl_fields

    spec = SPECS[config]
    rng = np.random.Generator(np.random.PCG64(seed))
    data = []
    prompt = 0
    for i in range(n):
        if i % spec.attempts == 0:
            prompt = int(rng.integers(spec.prompt[0], spec.prompt[1] + 1))
        hi = spec.completion[1] if max_completion is None else min(spec.completion[1], max_completion)
        comp = int(rng.integers(spec.completion[0], hi + 1))
        if spec.max_total is not None:
            comp = min(comp, spec.max_total - prompt)
        L = prompt + comp
        ids = rng.integers(0, ID_RANGE, L).tolist()
        if rng.random() < 0.75:
            ids[-1] = EOS
        old = (-np.abs(rng.normal(0.0, 1.5, comp))).astype(np.float32)
        ref = old + rng.normal(0.0, spec.ref_noise, comp).astype(np.float32) if spec.ref_noise else old
        enc = prepare_rl_fields({"input_ids": ids, "labels": [-100] * prompt + ids[prompt:], "attention_mask": [1] * L},
                                float(rng.random() < 0.5), old.tolist(), ref.tolist())
        enc.update(group_id=f"g{i // spec.attempts}", rollout_index=i % spec.attempts, step_index=0, model_version=0)
        data.append(enc)
    return populate_rl_data(data, EOS, RLConfig(divide_advantage_by_std=False))


def pack(data: list[dict], seq_length: int, samples_per_step: int, num_trainers: int = 1,
         filter_zero_advantage_groups: bool = False) -> list[tuple[int, object]]:
    """(trainer_id, PipelineBatchEncoding) writes of the preprocessor's packer (quota + sentinel
    protocol, preprocess.py:557-626) for ``data``; with ``filter_zero_advantage_groups`` the
    chunk first loses its all-zero-advantage groups, as rl.filter_zero_advantage_groups does
    (preprocess.py:509-513)."""
    from .finetune import packing

    data = copy.deepcopy(data)
    if filter_zero_advantage_groups:
        data, _ = packing.filter_zero_advantage_groups(data)
    packer = packing.MicroBatchPacker(num_trainers, seq_length, samples_per_step // num_trainers,
                                      types.SimpleNamespace(eos_token_id=EOS))
    return packer.feed(data)


def micro_batches(config: str, count: int, seed: int = 1234, seq_length: int | None = None) -> list:
    """``count`` non-sentinel packed micro-batches of ``config`` (one trainer), greedy-packed up to
    ``seq_length`` tokens (default: the config's)."""
    spec = SPECS[config]
    cap = seq_length or spec.seq_length
    out: list = []
    n = max(8, count * 4)
    while True:
        data = rollouts(config, n, seed=seed, max_completion=cap - spec.prompt[1] if cap < 9000 else None)
        writes = pack(data, cap, len(data))
        out = [b for _, b in writes if not b.sentinel]
        if len(out) > count:  # the last one may be a partial tail: keep only full-ish ones
            return out[:count]
        n *= 2


def rl_config(config: str, samples_per_step: int):
    """GRPO defaults (conf/finetune/base.yaml:92-105 + grpo.yaml: ppo, eps 4, C 5), the config's KL."""
    from .finetune.rl import RLConfig

    spec = SPECS[config]
    return RLConfig(policy_loss="ppo", epsilon=4.0, kl_coef=spec.kl_coef, final_kl_coef=spec.kl_coef,
                    clamp_log_ratio_ref_new_value=5, divide_advantage_by_std=False, batch_size=samples_per_step)


# lockstep_cost(config, N, 4096 // N)["efficiency"]["loop"]: the protocol's efficiency of one C3
# optimizer step (4096 samples) at N data-parallel ranks, on the preprocessor's packing of C3's
# rollouts (seed 7).  Minutes of CPU per N, so tabled: regenerate with tools/lockstep_table.py.
LOCKSTEP_EFFICIENCY = {"c3": {1: 1.0, 2: 0.9786, 4: 0.9669, 8: 0.949}}


def lockstep_cost(config: str, ranks: int, samples_per_rank: int, seed: int = 7, seq_length: int | None = None,
                  ms_fixed: float = 30.0, ms_per_token: float = (350.0 - 30.0) / 11425,
                  forward_share: float = 1 / 3) -> dict:
    """A timing model of one optimizer step under the reference's lockstep protocol
    (finetune_loop.py:577-617: every pass exchanges the sample counts on the host; ranks past their
    quota run sentinel passes) on the preprocessor's own assignment of ``config``'s rollouts to
    ``ranks`` trainers (preprocess.py:557-626, ``samples_per_rank`` each).  A micro-batch costs
    ms_fixed + ms_per_token x tokens on the device (defaults: the C3 7B step in DESIGN.md, 350 ms at
    11 425 tokens; a sentinel 30 ms), ``forward_share`` of it in the forward.  A host reaches pass
    p's exchange once its forward(p-1) statistics are read back, so the exchange ends when the
    slowest rank's forward(p-1) has.  Step times (ms): ``full_pass`` (every pass waits for every
    rank's whole previous pass: the naive bound), ``exchange_then_forward`` (forward(p) enqueued
    after the exchange: the reference's order and this build's through round 4),
    ``forward_then_exchange`` (forward(p) enqueued before it, backward(p) after), ``loop`` (this
    loop: in addition a rank below its quota queues backward(p) before the exchange too), ``free``
    (no per-pass coupling; sentinels skipped) and ``balanced`` (the mean rank's
    work); efficiencies = balanced / each."""
    spec = SPECS[config]
    data = rollouts(config, ranks * samples_per_rank, seed=seed)
    writes = pack(data, seq_length or spec.seq_length, ranks * samples_per_rank, num_trainers=ranks)
    tok: dict[int, list[int]] = {r: [] for r in range(ranks)}
    for r, b in writes:
        tok[r].append(0 if b.sentinel else int(b.attention_mask.sum()))
    t = {r: [ms_fixed + ms_per_token * x for x in v] for r, v in tok.items()}
    passes = max(len(v) for v in t.values())

    def cost(r: int, p: int) -> float:
        return t[r][p] if p < len(t[r]) else 0.0

    def coupled(forward_first: bool) -> float:
        end, fwd = [0.0] * ranks, [0.0] * ranks
        for p in range(passes):
            barrier = max(fwd)
            for r in range(ranks):
                f, b = cost(r, p) * forward_share, cost(r, p) * (1 - forward_share)
                if forward_first:
                    fwd[r] = end[r] + f
                    end[r] = max(fwd[r], barrier) + b
                else:
                    fwd[r] = max(end[r], barrier) + f
                    end[r] = fwd[r] + b
        return max(end)

    last_real = {r: max((i for i, x in enumerate(tok[r]) if x), default=-1) for r in range(ranks)}

    def loop_order() -> float:
        # this loop: forward(p); below the rank's quota backward(p) then the exchange, at the quota
        # the exchange then backward(p); the host moves on once the exchange is done and its
        # forward(p) statistics are read back
        end, host = [0.0] * ranks, [0.0] * ranks
        for p in range(passes):
            fwd = [max(end[r], host[r]) + cost(r, p) * forward_share for r in range(ranks)]
            x = max(host)  # every host reaches the exchange right after queueing its pass
            for r in range(ranks):
                b = cost(r, p) * (1 - forward_share)
                end[r] = (fwd[r] if p < last_real[r] else max(fwd[r], x)) + b
                host[r] = max(x, fwd[r])
        return max(end)

    times = {"full_pass": sum(max(cost(r, p) for r in range(ranks)) for p in range(passes)),
             "exchange_then_forward": coupled(False), "forward_then_exchange": coupled(True), "loop": loop_order(),
             "free": max(sum(x for x, n in zip(t[r], tok[r]) if n) for r in range(ranks))}
    balanced = sum(sum(x for x, n in zip(t[r], tok[r]) if n) for r in range(ranks)) / ranks
    return {"config": config, "ranks": ranks, "samples_per_step": ranks * samples_per_rank, "passes": passes,
            "sentinels_per_rank": [v.count(0) for v in tok.values()], "tokens_per_rank": [sum(v) for v in tok.values()],
            "ms": {k: round(v, 1) for k, v in times.items()} | {"balanced": round(balanced, 1)},
            "efficiency": {k: round(balanced / v, 4) for k, v in times.items()}}
