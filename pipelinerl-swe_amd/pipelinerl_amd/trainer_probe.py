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

import numpy as np
import torch
import torch.distributed as dist

QWEN = {  # published Qwen2.5 shapes (config.json of each checkpoint)
    "0.5b": dict(hidden_size=896, intermediate_size=4864, num_hidden_layers=24, num_attention_heads=14,
                 num_key_value_heads=2, vocab_size=151936, tie_word_embeddings=True),
    "1.5b": dict(hidden_size=1536, intermediate_size=8960, num_hidden_layers=28, num_attention_heads=12,
                 num_key_value_heads=2, vocab_size=151936, tie_word_embeddings=True),
    "7b": dict(hidden_size=3584, intermediate_size=18944, num_hidden_layers=28, num_attention_heads=28,
               num_key_value_heads=4, vocab_size=152064, tie_word_embeddings=False),
    "32b": dict(hidden_size=5120, intermediate_size=27648, num_hidden_layers=64, num_attention_heads=40,
                num_key_value_heads=8, vocab_size=152064, tie_word_embeddings=False),
    # tests: the product path (patched ops, HIP attention at head dim 128) on a two-layer model
    "tiny": dict(hidden_size=512, intermediate_size=1024, num_hidden_layers=2, num_attention_heads=4,
                 num_key_value_heads=2, vocab_size=512, tie_word_embeddings=True),
}


def qwen2_model(name: str, device: torch.device, grad_ckpt: bool = False, fused_ops: bool = True,
                layers: int | None = None, keep_layers: int = 0):
    """``grad_ckpt``: HF gradient checkpointing, except the last ``keep_layers`` decoder layers
    (finetune/checkpoints.keep_activations, the plan's partial recompute)."""
    from transformers import AutoModelForCausalLM, Qwen2Config

    from .finetune.attention import register

    shapes = dict(QWEN[name], **({"num_hidden_layers": layers} if layers else {}))
    cfg = Qwen2Config(max_position_embeddings=32768, rope_theta=1e6, rms_norm_eps=1e-6, **shapes)
    torch.manual_seed(0)
    with torch.device(device):  # initialise on the GPU (a CPU init of 1.5B+ params takes minutes)
        model = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16, attn_implementation=register())
    if fused_ops:
        from .finetune.model_ops import patch_model

        patch_model(model)
    if grad_ckpt:
        from .finetune.checkpoints import keep_activations

        model.gradient_checkpointing_enable(gradient_checkpointing_kwargs={"use_reentrant": False})
        keep_activations(model, keep_layers)
    model.train()
    return model


def packed_batch(T: int, seq: int, prompt: int, V: int, device, seed: int = 0, ref_noise: bool = False):
    """One packed micro-batch: T // seq rollouts of ``seq`` tokens (``prompt`` of them prompt);
    ``ref_noise``: reference log-probs = old + N(0, 0.05^2) on label tokens."""
    from .finetune.types import PipelineBatchEncoding

    g = torch.Generator().manual_seed(seed)
    nseq = T // seq
    pos = torch.arange(T) % seq
    ids = torch.randint(0, min(V, 151643), (1, T), generator=g)
    labels = torch.where(pos[None] >= prompt, ids, torch.full_like(ids, -100))
    rewards = torch.repeat_interleave(torch.randint(0, 2, (nseq,), generator=g).float(), seq)[None]
    lab = (labels != -100).float()
    old = (torch.randn((1, T), generator=g) - 12.0) * lab
    ref = old + 0.05 * torch.randn((1, T), generator=g) * lab if ref_noise else old.clone()
    b = PipelineBatchEncoding(
        input_ids=ids, labels=labels, attention_mask=torch.ones_like(ids), position_ids=pos[None],
        rewards=rewards, advantages=rewards - rewards.mean(), ref_logprobs=ref, old_logprobs=old,
        group_tokens=torch.full((1, T), float(seq)), num_labels=torch.full((1, T), float(seq - prompt)),
        overflow=torch.zeros((1, T)), seq_boundaries=torch.arange(0, T + 1, seq, dtype=torch.int32),
        model_version=0, is_packed=True)
    sb = b.seq_boundaries
    b.to_device(device)
    b.seq_boundaries = sb  # host metadata, as the trainer's loader keeps it
    return b


def rl_config(samples_per_step: int, fused_head: bool = True, kl_coef: float = 0.0):
    from .finetune.rl import RLConfig

    # GRPO defaults (conf/finetune/base.yaml + grpo.yaml): ppo, eps 4, kl 0, C 5; C5 turns KL on
    # (kl_coef 0.001, conf/deepscaler15b.yaml:34)
    return RLConfig(policy_loss="ppo", epsilon=4.0, kl_coef=kl_coef, final_kl_coef=kl_coef,
                    clamp_log_ratio_ref_new_value=5, batch_size=samples_per_step, fused_lm_head=fused_head)


def _sync(device) -> None:
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)


def _sync_compute(device) -> None:
    """Wait for the trainer's compute stream only: a weight update's broadcast still running on its
    side stream belongs to the steps after it, not to the ones just timed."""
    if torch.device(device).type == "cuda":
        torch.cuda.current_stream(device).synchronize()


class TrainerStep:
    """One rank's optimizer step as the trainer loop runs it (finetune_loop.py rl_finetuning_worker):
    ``micro_batches`` packed micro-batches (the last one armed so the bucketed gradient all-reduce
    over ``group`` overlaps its backward), clip 0.3, the weight manager's snapshot fence, AdamW.

    ``model`` / ``step_fn`` default to the product path (Qwen2 shapes on the device, rl_step with
    the HIP loss head); tests inject a CPU model and loss to exercise the control flow on gloo.
    """

    def __init__(self, name: str = "1.5b", tokens: int = 16384, seq: int = 2048, prompt: int = 256,
                 micro_batches: int = 4, device=None, fused_head: bool = True, grad_ckpt: bool = False,
                 fused_ops: bool = True, group=None, model=None, step_fn=None, vocab: int | None = None,
                 fsdp: bool = False, kl_coef: float = 0.0, layers: int | None = None, batches: list | None = None,
                 samples_per_step: int | None = None, local: bool = False, flat_params: bool = True,
                 keep_layers: int = 0, master_weights: bool = True, value_head: bool = False):
        """``batches``: the packed micro-batches to train on (host PipelineBatchEncodings, e.g. from
        workloads.micro_batches), ``samples_per_step`` their global sample count (RLConfig.batch_size);
        default: ``micro_batches`` synthetic batches of ``tokens`` tokens.  ``local``: no gradient
        all-reduce even under a multi-rank group (the replica's compute alone, for the DP overhead).
        ``master_weights``: fp32 master weights + moments, the trainer's default (finetune/optim.py).
        ``value_head``: the model wrapped with a value head (finetune/value_model.py; the reference's
        default actor_critic fine-tune config), value_loss_coef 0.1 (conf/finetune/actor_critic.yaml)."""
        from .finetune.grad_sync import GradBuckets
        from .finetune.optim import get_optimizer
        from .finetune.sharding import shard_model

        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.group = group
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world, self.tokens, self.micro_batches = world, tokens, micro_batches
        self.model = model if model is not None else qwen2_model(name, self.device, grad_ckpt, fused_ops, layers,
                                                                 keep_layers)
        if value_head:
            from .finetune.value_model import AutoModelForCausalLMWithValueHead

            self.model = AutoModelForCausalLMWithValueHead(self.model).to(self.device)
        self.fsdp = fsdp
        if fsdp:  # FSDP2 over the default group (finetune/sharding.py): it reduce-scatters the grads
            if group is not None:
                raise ValueError("fsdp shards over the default process group")
            self.model = shard_model(self.model, master_weights=master_weights)
        elif flat_params:  # as the loop does at load (finetune.flat_parameters, weight_update.py)
            from .weight_update import rehome_parameters

            rehome_parameters(self.model)
        from .finetune.rl import rl_step

        self.native_step = step_fn is None or step_fn is rl_step
        self._tail_events: list = []
        self._tail_cpu: list[float] = []
        self.step_fn = step_fn if step_fn is not None else rl_step
        self.opt = get_optimizer("adamw_torch", self.model, 1e-6, 0.01, master_weights=master_weights)
        self.grads = GradBuckets(list(self.model.parameters()), group=group) \
            if world > 1 and not fsdp and not local else None
        V = vocab or QWEN[name]["vocab_size"]
        if batches is not None:
            self.batches = []
            for b in batches:
                sb = b.seq_boundaries
                b = b.to_device(self.device)
                b.seq_boundaries = sb  # host metadata, as the trainer's loader keeps it
                self.batches.append(b)
            self.micro_batches = len(self.batches)
            self.tokens = sum(int(b.attention_mask.sum()) for b in self.batches) / max(1, len(self.batches))
            self.cfg = rl_config(samples_per_step or 1, fused_head, kl_coef)
        else:
            self.batches = [packed_batch(tokens, seq, prompt, V, self.device, seed=rank * 97 + i,
                                         ref_noise=kl_coef > 0) for i in range(micro_batches)]
            self.cfg = rl_config(micro_batches * (tokens // seq) * world, fused_head, kl_coef)
        if value_head:
            self.cfg.value_loss_coef = 0.1
        from .hostgc import freeze_setup_heap

        freeze_setup_heap()  # as the loop does before its first step

    def step(self, wum=None, version: int = 0) -> None:
        from .finetune.optim import clip_grad_norm
        from .finetune.sharding import set_gradient_sync

        for i, b in enumerate(self.batches):
            if self.grads is not None and i == len(self.batches) - 1:
                self.grads.arm()
            if self.fsdp:  # reduce-scatter on the boundary micro-batch only (the reference's no_sync)
                set_gradient_sync(self.model, i == len(self.batches) - 1)
            if self.native_step:  # as the loop runs it: statistics read after the backward is queued
                loss, stats = self.step_fn(self.model, b, 0, 100, self.cfg, defer_stats=True)
                loss.backward()
                stats.resolve()  # the reference's non-finite assertions
            else:
                loss, _ = self.step_fn(self.model, b, 0, 100, self.cfg)
                loss.backward()
        if self.grads is not None:
            self.grads.finish()
        on_gpu = self.device.type == "cuda"
        if on_gpu:  # the optimizer tail (clip, AdamW, zero) on the device, end of backward -> done
            t0 = torch.cuda.Event(enable_timing=True)
            t0.record()
        else:
            c0 = time.perf_counter()
        clip_grad_norm(self.model.parameters(), 0.3, self.opt)
        if wum is not None:
            wum.before_optimizer_step()  # the previous snapshot is read before params change
        self.opt.step()
        if self.grads is not None:
            self.grads.zero_()
        else:
            self.opt.zero_grad(set_to_none=True)
        if on_gpu:
            t1 = torch.cuda.Event(enable_timing=True)
            t1.record()
            self._tail_events.append((t0, t1))
        else:
            self._tail_cpu.append(time.perf_counter() - c0)
        if wum is not None:
            wum.send_weight_update(version)  # returns at once: overlapped with the next step

    def timed(self, steps: int, warmup: int, wum=None, version0: int = 0) -> float:
        """Seconds per optimizer step (max over the group's ranks).  With a weight manager ``wum``
        every step sends an update that overlaps the NEXT step, as in the trainer loop: the timed
        region starts with the last warm-up step's update in flight and ends when the compute stream
        is done (the last update's broadcast tail runs on, outside it: it would overlap the next
        step), then the whole device is waited for."""
        v = version0
        for _ in range(warmup):
            v += 1
            self.step(wum, v)
        _sync_compute(self.device)
        self._tail_events, self._tail_cpu = [], []
        if self.world > 1:
            dist.barrier(self.group)
        t0 = time.perf_counter()
        for _ in range(steps):
            v += 1
            self.step(wum, v)
        _sync_compute(self.device)
        if self.world > 1:
            dist.barrier(self.group)
        dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=self.device)
        _sync(self.device)
        if self.world > 1:
            dist.all_reduce(dt, op=dist.ReduceOp.MAX, group=self.group)
        return float(dt) / steps

    def optimizer_tail(self) -> float:
        """Seconds of the last ``timed`` run's optimizer tail (clip_grad_norm, AdamW, zeroing) per
        step, mean over its steps, max over the group's ranks."""
        if self._tail_events:
            _sync(self.device)
            t = sum(a.elapsed_time(b) for a, b in self._tail_events) / len(self._tail_events) / 1e3
        else:
            t = sum(self._tail_cpu) / max(1, len(self._tail_cpu))
        dt = torch.tensor([t], dtype=torch.float64, device=self.device)
        if self.world > 1:
            dist.all_reduce(dt, op=dist.ReduceOp.MAX, group=self.group)
        return float(dt)

    def allreduce_alone(self, iters: int = 3, group_sync: bool = True) -> float:
        """Seconds of the bucketed gradient all-reduce over the model's real buckets with no
        backward to hide behind (max over the group's ranks; ``group_sync`` False: this rank alone,
        an emulated all-reduce at N = 1)."""
        if self.grads is None:
            return 0.0
        params = [p for p in self.model.parameters() if p.requires_grad]
        times = []
        for it in range(iters + 1):
            _sync(self.device)
            if group_sync:
                dist.barrier(self.group)
            t0 = time.perf_counter()
            self.grads.arm()
            for p in reversed(params):  # the order backward produces gradients
                self.grads._hook(p)
            self.grads.finish()
            _sync(self.device)
            if it:
                times.append(time.perf_counter() - t0)
        self.grads.zero_()
        dt = torch.tensor([sum(times) / len(times)], dtype=torch.float64, device=self.device)
        if group_sync:
            dist.all_reduce(dt, op=dist.ReduceOp.MAX, group=self.group)
        return float(dt)

    def close(self) -> None:
        if self.grads is not None:
            self.grads.remove()
        self.model = self.opt = self.grads = self.batches = None
        if self.device.type == "cuda":
            torch.cuda.empty_cache()


def step_roofline(ts: "TrainerStep", seconds: float, breakdown: bool = True) -> dict | None:
    """The step's MFMA roofline (step_flops.py): model FLOPs of this rank's micro-batches, summed over
    the ranks, per GPU over ``seconds`` (the step time, max over ranks), against the dense bf16 peak;
    with ``breakdown`` one more step runs under torch.profiler for its GEMM / attention kernel time
    (every rank runs it: the step's collectives stay matched).  None for a model without a config."""
    from .step_flops import kernel_breakdown, mfma_roofline, shape_of, step_flops

    cfg = getattr(getattr(ts.model, "module", ts.model), "config", None)
    if cfg is None or not hasattr(cfg, "num_hidden_layers"):
        return None
    flops = step_flops(cfg, [shape_of(b) for b in ts.batches], label_row_head=ts.cfg.fused_lm_head)
    world = ts.world
    if world > 1:
        tot = torch.tensor([float(flops[k]) for k in ("linear", "lm_head", "attention", "total")], dtype=torch.float64,
                           device=ts.device)
        dist.all_reduce(tot, group=ts.group)
        flops = dict(flops, **{k: float(v) / world for k, v in zip(("linear", "lm_head", "attention", "total"),
                                                                     tot.cpu().tolist())})
    kb = None
    if breakdown and ts.device.type == "cuda":
        try:
            kb = kernel_breakdown(ts.step, ts.device)
        except Exception as e:  # noqa: BLE001 - the profiler is measurement only
            kb = {"error": f"{type(e).__name__}: {e}"[:200]}
    r = mfma_roofline(flops, seconds, kb if kb and "error" not in kb else None)
    if kb and "error" in kb:
        r["kernel_breakdown"] = kb
    r["per"] = "GPU (this world's model FLOPs per rank, mean over ranks) / step time (max over ranks)"
    return r


def trainer_step_probe(name: str = "1.5b", tokens: int = 16384, seq: int = 2048, prompt: int = 256,
                       micro_batches: int = 4, steps: int = 3, warmup: int = 1, device=None,
                       fused_head: bool = True, grad_ckpt: bool = False, fused_ops: bool = True,
                       layers: int | None = None) -> dict:
    """The optimizer step at this world size.  With several ranks the same replica is also timed
    without the gradient all-reduce first (``local_tokens_per_s_per_gpu``: what one GPU does on its
    own, on this node at this moment), so ``dp_efficiency`` = DP / local tokens/s per GPU is the
    trainer-step scaling fraction of this N, measured beside it."""
    device = device or torch.device("cuda", torch.cuda.current_device())
    torch.cuda.reset_peak_memory_stats(device)
    multi = dist.is_initialized() and dist.get_world_size() > 1
    ts = TrainerStep(name, tokens, seq, prompt, micro_batches, device, fused_head, grad_ckpt, fused_ops, local=multi,
                     layers=layers)
    world = dist.get_world_size() if dist.is_initialized() else 1
    local = None
    if multi:
        from .finetune.grad_sync import GradBuckets

        local = ts.timed(steps, warmup)
        ts.grads = GradBuckets(list(ts.model.parameters()))
    sec = ts.timed(steps, warmup)
    peak = torch.cuda.max_memory_allocated(device) / 1e9
    roof = step_roofline(ts, sec)
    ts.close()
    total = tokens * micro_batches * world
    out = {"model": f"Qwen2.5-{name} shapes{f' ({layers} layers)' if layers else ''} (random init, bf16)",
           "tokens_per_micro_batch": tokens,
           "micro_batches_per_step": micro_batches, "seq_len": seq, "prompt_len": prompt,
           "loss_head": "fused_lm_head" if fused_head else "fused", "fused_model_ops": fused_ops,
           "ms_per_optimizer_step": round(sec * 1e3, 2),
           "tokens_per_s": round(total / sec, 1), "tokens_per_s_per_gpu": round(total / sec / world, 1),
           "peak_mem_gb": round(peak, 2), "steps": steps, "warmup": warmup, "world": world}
    if roof is not None:
        out["roofline"] = roof
    if local is not None:
        out["local_tokens_per_s_per_gpu"] = round(total / world / local, 1)
        out["ms_per_optimizer_step_local"] = round(local * 1e3, 2)
        out["dp_efficiency"] = round(local / sec, 4)
    return out


def _snapshot_only_group():
    """An actor group with no receivers (measurement only): WeightUpdateManager takes its snapshot
    exactly as for real actors (stream-ordered, as with an RcclComm); the broadcasts are no-ops."""
    from .comm import RcclComm

    class SnapshotOnlyGroup(RcclComm):
        def __init__(self):
            super().__init__(None, 0, 1, None)

        def broadcast(self, t: torch.Tensor, src: int = 0, bucket_bytes: int = 0) -> None:
            return None

    return SnapshotOnlyGroup()


def _paced_read_group(gbps: float, blocks: int, device, asleep: bool = False):
    """An actor group with no receivers whose broadcast READS what it would send, as an RCCL root
    does, at a link rate: ``blocks`` workgroups (the channels) stream each bucket paced to ``gbps``
    (prl_paced_read, stream-ordered on the broadcast's side stream).  One xGMI link ~153 GB/s
    (SURVEY.md §5).  ``asleep`` (a control): the same workgroups resident for the same time per
    bucket, reading two 64 KiB turns each — the CUs held without the memory traffic."""
    import ctypes

    from . import _native
    from .comm import RcclComm

    lib = _native.load()
    sink = torch.zeros(max(1, blocks), dtype=torch.int32, device=device)

    class PacedReadGroup(RcclComm):
        def __init__(self):
            super().__init__(None, 0, 1, None)

        def broadcast(self, t: torch.Tensor, src: int = 0, bucket_bytes: int = 0) -> None:
            st = torch.cuda.current_stream(t.device).cuda_stream
            nbytes, rate = t.numel() * t.element_size(), float(gbps)
            if asleep:
                small = min(nbytes, 2 * int(blocks) * 65536)
                nbytes, rate = small, rate * small / max(1, nbytes)
            _native.check(lib.prl_paced_read(ctypes.c_void_p(t.data_ptr()), nbytes, rate, int(blocks),
                                             ctypes.c_void_p(sink.data_ptr()), st), "prl_paced_read")

    return PacedReadGroup()


# the broadcast's reads of the parameters emulated at N = 1: (GB/s, channels) of one xGMI link and of
# four (a 1 -> 4 actors broadcast spread over several rings)
PACED_ARMS = {"zero_copy_1link": (153.0, 16), "zero_copy_4link": (612.0, 32)}


def snapshot_overlap(ts: "TrainerStep", t_ref: float, steps: int, warmup: int, flatten_iters: int = 3,
                     rounds: int = 3) -> dict:
    """The trainer-side half of "weight broadcast fully overlapped" (north_star), on this rank's GPU.

    First the staging copy alone: prl_flatten_bf16 over every parameter into a bf16 buffer on a side
    stream, HIP events, nothing else running (``snapshot_ms``).  Then the same optimizer step as
    ``t_ref`` (seconds per step, measured just before on ``ts``) in three arms, ``rounds`` rounds of
    ``steps`` steps each, the arms' order rotating every round (medians reported): no weight update; WeightUpdateManager (weight_update.py, rank 0)
    with ``snapshot="copy"`` (the staging copy on its side stream after each optimizer step); and with
    ``snapshot="zero_copy"`` (the default: parameters re-homed once into the broadcast layout, read in
    place; re-homed at load by TrainerStep, as the loop does, so every arm runs the same step).  No receiver: the broadcasts are no-ops, so the arms price the trainer-side snapshot alone
    (the broadcast's own cost needs actors: ``split_pipeline`` at N > 1).  ``exposed_ms`` = median step
    time of an arm − the no-update arm's (the no-update arm's own spread is the noise floor); ``hidden_frac`` = 1 − exposed / snapshot_ms.  The
    reference blocks the trainer for the whole update instead (finetune_loop.py:174-215).

    The zero-copy arm does no device work at all with no receiver, so its hidden_frac is null.  The
    ``zero_copy_1link`` / ``zero_copy_4link`` arms give it a real number: the same in-place update whose
    broadcast READS the 15.23 GB of parameters as an RCCL root sending them would — paced to one xGMI
    link (153 GB/s, 16 channel workgroups) and to four (612 GB/s, 32) — on the side stream while the
    next step runs; ``device_work_ms`` is those reads alone (HIP events, nothing else running)."""
    from .weight_update import FlatLayout, HipFlatPacker, WeightUpdateManager, parameters_info

    rank = dist.get_rank() if dist.is_initialized() else 0
    mk = lambda mode: WeightUpdateManager([], ts.model, None, _snapshot_only_group(), transport="bucketed",  # noqa: E731
                                          overlap=True, is_main=rank == 0, write_message=lambda s, m: None,
                                          snapshot=mode)
    named = list(ts.model.named_parameters())
    layout = FlatLayout.from_infos(parameters_info(named))
    flat = torch.empty(layout.total, dtype=torch.bfloat16, device=ts.device)
    params = [p.detach() for _, p in named]
    side = torch.cuda.Stream(device=ts.device)
    side.wait_stream(torch.cuda.current_stream(ts.device))
    evs = []
    with torch.cuda.stream(side):
        for _ in range(flatten_iters + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(side)
            HipFlatPacker().flatten(params, layout.offsets, flat)
            e1.record(side)
            evs.append((e0, e1))
    _sync(ts.device)
    snap_ms = sum(a.elapsed_time(b) for a, b in evs[1:]) / flatten_iters
    del flat, params
    nbytes = sum(p.numel() * p.element_size() for _, p in named) + 2 * sum(p.numel() for _, p in named)
    managers = {"no_update": None, "copy": mk("copy"), "zero_copy": mk("zero_copy")}
    # the parameters are re-homed at load (TrainerStep, as the loop does; or here, before any arm
    # runs): every arm runs the same step, the fused gate/up weight a view of them
    in_place = managers["zero_copy"]._zero_copy_flat(named, layout) is not None if rank == 0 else False
    paced_ms = {}
    if in_place:
        flat_p = managers["zero_copy"]._flat_params
        for name, (gbps, blocks, *mode) in PACED_ARMS.items():
            # mode flags (measurement controls): "asleep" (the workgroups held, almost no reads),
            # "one" (one launch for the whole buffer instead of one per 256 MiB bucket)
            grp = _paced_read_group(gbps, blocks, ts.device, asleep="asleep" in mode)
            bucket = (1 << 40) if "one" in mode else (256 << 20)
            managers[name] = WeightUpdateManager([], ts.model, None, grp, transport="bucketed", overlap=True,
                                                 is_main=rank == 0, write_message=lambda s, m: None,
                                                 snapshot="zero_copy", bucket_bytes=bucket)
            with torch.cuda.stream(side):  # the reads alone, nothing else running
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(side)
                for a, b in layout.buckets(bucket // 2):  # buckets of bf16
                    grp.broadcast(flat_p[a:b])
                e1.record(side)
            _sync(ts.device)
            paced_ms[name] = e0.elapsed_time(e1)
    arms = {m: [] for m in managers}
    arms["no_update"] = [t_ref]
    order = list(managers)
    for r in range(rounds):  # the order rotates every round, so a drift of the clocks hits every arm
        k = r % len(order)
        for mode in order[k:] + order[:k]:
            # one warm-up step per arm and round: the first timed step runs with an update in flight
            wu = max(1, warmup) if mode != "no_update" else (warmup if r == 0 else 0)
            arms[mode].append(ts.timed(steps, wu, wum=managers[mode]))
            if managers[mode] is not None:
                managers[mode].wait()
    for m in managers.values():
        if m is not None:
            m.close()
            m._staging = None
    mean = {k: float(np.median(v)) for k, v in arms.items()}

    spread = (max(arms["no_update"]) - min(arms["no_update"])) * 1e3

    def arm(mode: str, cost_ms: float) -> dict:
        delta = (mean[mode] - mean["no_update"]) * 1e3
        exposed = max(0.0, delta)
        return {"ms_per_step": round(mean[mode] * 1e3, 2), "step_delta_ms": round(delta, 3),
                "exposed_ms": round(exposed, 3), "within_noise": abs(delta) <= spread, "device_work_ms": cost_ms,
                "hidden_frac": (round(1.0 - min(1.0, exposed / cost_ms), 4) if cost_ms > 0 else None)}

    zc = arm("zero_copy", 0.0 if in_place else round(snap_ms, 3))
    if in_place:
        zc["hidden_frac_note"] = "unmeasured at N=1: no receiver, the broadcast reads nothing (see zero_copy_1link/4link)"
    paced = {}
    for name, (gbps, blocks, *mode) in PACED_ARMS.items():
        if name in paced_ms:
            paced[name] = dict(arm(name, round(paced_ms[name], 3)), link_GBps=gbps, channel_workgroups=blocks,
                               reads="the 15.23 GB flat parameter buffer in 256 MiB buckets, prl_paced_read")

    return {"params": len(named), "snapshot_bytes": 2 * layout.total, "snapshot_ms": round(snap_ms, 3),
            "snapshot_GBps": round(nbytes / (snap_ms * 1e-3) / 1e9, 1),
            "ms_per_step_no_update": round(mean["no_update"] * 1e3, 2),
            "no_update_spread_ms": round(spread, 3),
            "copy": arm("copy", round(snap_ms, 3)),
            # in place with no receiver there is no device work on the trainer: step_delta_ms is the
            # run's noise (compare no_update_spread_ms); the paced arms price the broadcast's reads
            "zero_copy": dict(zc, in_place=in_place), **paced,
            "arms_ms": {k: [round(x * 1e3, 2) for x in v] for k, v in arms.items()},
            "steps_per_arm": steps, "rounds": rounds}


class EmulatedRingBuckets:
    """GradBuckets whose bucket all-reduce, at N = 1, makes the HBM reads and holds the CUs a ring
    all-reduce over ``ranks`` GPUs would on this one (a ring moves 2(N−1)/N x S bytes
    per GPU, per-link bound at ~153 GB/s per xGMI link): ``prl_paced_read`` over each bucket,
    2(N−1)/N x its bytes, paced to ``gbps`` with ``channels`` workgroups, launched from the same
    post-accumulate-grad hooks on GradBuckets' own stream the moment the bucket's last gradient lands
    in the boundary micro-batch's backward.  What it prices: the all-reduce's contention with the
    backward (CUs, HBM) and the tail no backward is left to hide (the embedding's gradient lands
    last).  What it does not: the links' own latency and the peers' skew."""

    def __new__(cls, params, ranks: int, gbps: float, channels: int, bucket_bytes: int = 256 << 20):
        import ctypes

        from . import _native
        from .finetune.grad_sync import GradBuckets

        lib = _native.load()

        class _Done:
            def wait(self):
                return None

        class _Emulated(GradBuckets):
            def _launch(self, b):
                b.launched = True
                self.stream.wait_stream(torch.cuda.current_stream(b.flat.device))
                nbytes = b.flat.numel() * b.flat.element_size() // 16 * 16
                todo = int(2 * (ranks - 1) / ranks * nbytes) // 16 * 16
                with torch.cuda.stream(self.stream):
                    while todo > 0:  # the ring's 2(N-1)/N passes over the bucket
                        n = min(todo, nbytes)
                        _native.check(lib.prl_paced_read(ctypes.c_void_p(b.flat.data_ptr()), n, float(gbps),
                                                         int(channels), ctypes.c_void_p(self._sink.data_ptr()),
                                                         self.stream.cuda_stream), "prl_paced_read")
                        todo -= n
                b.work = _Done()

        inst = _Emulated(params, bucket_bytes=bucket_bytes, world=1)
        inst._sink = torch.zeros(max(1, int(channels)), dtype=torch.int32, device=inst.buckets[0].flat.device)
        inst.bytes_per_gpu = int(2 * (ranks - 1) / ranks * sum(b.flat.numel() * b.flat.element_size()
                                                               for b in inst.buckets))
        return inst


# emulated ring all-reduce arms at N = 1 (dp_step_probe ``emulate``): ranks, GB/s, channel workgroups.
# One ring over one 153 GB/s xGMI link (the conservative case) at the SCALE run's N = 4
# and 8; and N = 8 over the 7 direct links at once.
RING_ARMS = {"n4_1link": (4, 153.0, 16), "n8_1link": (8, 153.0, 16), "n8_7links": (8, 7 * 153.0, 32)}


def projected_dp_efficiency(lockstep_eff: float, exposed_ms: float, ms_per_micro_batch: float,
                            micro_batches_per_rank: float, tail_ms: float) -> dict:
    """C3's data-parallel efficiency at N from its two losses: the lockstep protocol's
    (workloads.LOCKSTEP_EFFICIENCY: sentinel passes and the per-pass coupling of the ranks, the
    loop's order) and the all-reduce's exposed time in one optimizer step, ``exposed_ms`` against
    the step it ends (``micro_batches_per_rank`` x ``ms_per_micro_batch`` + the optimizer tail +
    itself)."""
    step = micro_batches_per_rank * ms_per_micro_batch + tail_ms + exposed_ms
    ar = 1.0 - exposed_ms / step if step > 0 else 1.0
    return {"lockstep_efficiency": round(lockstep_eff, 4), "allreduce_efficiency": round(ar, 6),
            "projected_efficiency": round(lockstep_eff * ar, 4), "step_ms": round(step, 1)}


def dp_step_probe(config: str = "c3", micro_batches: int = 4, steps: int = 2, warmup: int = 1, device=None,
                  samples_per_step: int = 4096, layers: int | None = None, batches: list | None = None,
                  model=None, step_fn=None, snapshot: bool = False, grad_ckpt: bool = False,
                  keep_layers: int = 0, emulate: dict | None = None, value_head: bool = False) -> dict:
    """BASELINE.json configs[2] (C3) data-parallel trainer step on this rank's GPU: the config's
    model shapes (Qwen2.5-7B), ``micro_batches`` packed micro-batches per rank from the config's
    rollout distribution (workloads.py: prompt U{64..512} + completion U{256..8192}, packing cap
    12 000, a different sample per rank), label-row lm_head + fused loss head, the bucketed RCCL
    gradient all-reduce of the whole model (15.23 GB bf16 for 7B) launched from the last
    micro-batch's backward, clip 0.3, AdamW.

    Measured on the same ranks, same batches: the replica's step without any all-reduce
    (``local``), the DP step, and the all-reduce alone over the same buckets.  ``overlap`` = 1 −
    (DP − local) / all-reduce alone.  The real C3 step trains ``samples_per_step`` (4096) samples,
    i.e. ~``samples_per_step / world / samples_per_micro_batch`` micro-batches per rank for ONE
    all-reduce: ``extrapolated_tokens_per_s_per_gpu`` prices that step as (its micro-batches x the
    measured per-micro-batch time, the optimizer tail taken out) + the exposed all-reduce + one
    optimizer tail (clip + AdamW + zeroing, timed with device events: ``optimizer_tail_ms``).
    Collective over the default group (every rank calls it).  ``batches`` / ``model`` /
    ``step_fn`` are injectable (gloo tests on CPU).  ``snapshot``: also time the same step with the
    weight-update snapshot in flight (``snapshot_overlap``, HIP devices only).  ``emulate`` (N = 1,
    HIP): {name: (ranks, GB/s, channels)} — the same step with each emulated ring all-reduce
    (EmulatedRingBuckets) launched from the boundary backward's hooks: ``allreduce_emulated``, each
    arm's exposed time and its projection to C3's real step at its N.  ``value_head``: the model
    wrapped with a value head (the reference's default actor_critic config, value_loss_coef 0.1)."""
    from . import workloads

    device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    on_gpu = device.type == "cuda"
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    spec = workloads.SPECS[config]
    if batches is None:
        batches = workloads.micro_batches(config, micro_batches, seed=1234 + 7919 * rank)
    micro_batches = len(batches)
    n_samples = sum(int((b.position_ids[0] == 0).sum()) for b in batches)
    n_tokens = sum(int(b.attention_mask.sum()) for b in batches)
    if on_gpu:
        torch.cuda.reset_peak_memory_stats(device)
    ts = TrainerStep(spec.model, device=device, fused_head=True, kl_coef=spec.kl_coef, layers=layers,
                     batches=batches, samples_per_step=samples_per_step, local=True, model=model, step_fn=step_fn,
                     grad_ckpt=grad_ckpt, keep_layers=keep_layers, value_head=value_head)
    t_local = ts.timed(steps, warmup)
    t_tail = ts.optimizer_tail()
    t_dp, t_ar = t_local, 0.0
    emulated = {}
    if emulate and world == 1 and on_gpu:
        for name, (ranks, gbps, channels) in emulate.items():
            ts.grads = EmulatedRingBuckets(list(ts.model.parameters()), ranks, gbps, channels)
            t_e = ts.timed(steps, warmup)
            t_alone = ts.allreduce_alone(group_sync=False)  # the reads alone, no backward to hide behind
            emulated[name] = {"ranks": ranks, "link_GBps": gbps, "channel_workgroups": channels,
                              "bytes_per_gpu": ts.grads.bytes_per_gpu, "ms_per_step": round(t_e * 1e3, 2),
                              "alone_ms": round(t_alone * 1e3, 2),
                              "exposed_ms": round(max(0.0, t_e - t_local) * 1e3, 2)}
            ts.grads.remove()
            ts.grads = None
    if world > 1:
        from .finetune.grad_sync import GradBuckets

        ts.grads = GradBuckets(list(ts.model.parameters()))
        ts.world = world
        t_dp = ts.timed(steps, warmup)
        t_ar = ts.allreduce_alone()
    nbytes = sum(p.numel() * p.element_size() for p in ts.model.parameters())
    peak = torch.cuda.max_memory_allocated(device) / 1e9 if on_gpu else 0.0  # before the staging buffer
    roof = step_roofline(ts, t_dp, breakdown=on_gpu)
    snap = snapshot_overlap(ts, t_dp, steps, warmup) if snapshot and on_gpu else None
    ts.close()
    stats = torch.tensor([n_tokens, n_samples, t_local], dtype=torch.float64, device=device)
    if world > 1:  # ranks drew different samples: sum tokens / samples, slowest replica's time
        tot = stats[:2].clone()
        dist.all_reduce(tot)
        tmax = stats[2:].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        stats = torch.cat([tot, tmax])
    else:
        stats = stats.clone()
    tok_all, samp_all, t_local_max = (float(x) for x in stats.cpu())
    exposed = max(0.0, t_dp - t_local_max)
    # the real step: samples_per_step samples over all ranks, one all-reduce, ONE optimizer tail
    # (finetune_loop.py:700-719 runs clip + AdamW once per samples_per_step, not per micro-batch)
    mb_real = samples_per_step / (samp_all / (micro_batches * world))
    t_tail = min(t_tail, t_local_max)
    per_mb = (t_local_max - t_tail) / micro_batches
    tok_per_mb = tok_all / (micro_batches * world)
    t_real = (mb_real / world) * per_mb + t_tail + exposed
    from .workloads import LOCKSTEP_EFFICIENCY

    for arm in emulated.values():  # projected to C3's real step at the arm's N
        n = arm["ranks"]
        arm["projection"] = projected_dp_efficiency(LOCKSTEP_EFFICIENCY[config][n], arm["exposed_ms"], per_mb * 1e3,
                                                    mb_real / n, t_tail * 1e3)
    return {"config": f"C3: Qwen2.5-{spec.model} shapes{f' ({layers} layers)' if layers else ''} (random init, bf16), "
                      f"math rollouts packed at {spec.seq_length}, label-row lm_head",
            "micro_batches_per_rank": micro_batches, "tokens_per_rank_step": round(tok_all / world, 1),
            "samples_per_rank_step": round(samp_all / world, 1),
            "ms_per_step_local": round(t_local_max * 1e3, 2), "ms_per_step_dp": round(t_dp * 1e3, 2),
            "allreduce_bytes": nbytes, "allreduce_alone_ms": round(t_ar * 1e3, 2),
            "allreduce_exposed_ms": round(exposed * 1e3, 2),
            "optimizer_tail_ms": round(t_tail * 1e3, 2),
            "overlap": round(1.0 - min(1.0, exposed / t_ar), 4) if t_ar > 0 else None,
            "tokens_per_s_per_gpu": round(tok_all / world / t_dp, 1),
            "tokens_per_s": round(tok_all / t_dp, 1),
            "local_tokens_per_s_per_gpu": round(tok_all / world / t_local_max, 1),
            "extrapolated": {"samples_per_step": samples_per_step, "micro_batches_per_rank": round(mb_real / world, 1),
                             "ms_per_micro_batch": round(per_mb * 1e3, 2),
                             "tokens_per_s_per_gpu": round(tok_per_mb * (mb_real / world) / t_real, 1),
                             "allreduce_share": round(exposed / t_real, 5)},
            "peak_mem_gb": round(peak, 2), "steps": steps, "warmup": warmup, "world": world,
            **({"roofline": roof} if roof is not None else {}),
            **({"allreduce_emulated": emulated} if emulated else {}),
            **({"value_head": True} if value_head else {}),
            **({"snapshot_overlap": snap} if snap is not None else {})}


def fsdp_step_probe(name: str = "32b", tokens: int = 4096, seq: int = 2048, prompt: int = 256,
                    micro_batches: int = 1, steps: int = 2, warmup: int = 1, device=None, kl_coef: float = 0.001,
                    layers: int | None = None, keep_gathered: int | str = 0) -> dict:
    """BASELINE.json configs[4] (C5): Qwen2.5-32B shapes sharded with FSDP2 over every rank (RCCL
    all-gather / reduce-scatter), KL-to-reference on, packed micro-batches; the whole optimizer
    step as the trainer runs it with ``sharding: fsdp``.  Collective over the default group.

    ``keep_gathered``: how many of the last decoder layers stay gathered from forward to backward
    (0: FSDP2's default, every layer resharded after its forward and gathered again for its
    backward); "plan": as many as the loop's memory plan gives for this micro-batch size
    (finetune/recompute.py plan_fsdp_gathering, gradient checkpointing as the reference config sets
    it, policy auto) — one all-gather per kept layer and step fewer."""
    from .finetune.recompute import plan_gradient_checkpointing
    from .finetune.sharding import set_kept_gathered

    device = device or torch.device("cuda", torch.cuda.current_device())
    torch.cuda.reset_peak_memory_stats(device)
    ts = TrainerStep(name, tokens, seq, prompt, micro_batches, device, fsdp=True, kl_coef=kl_coef, layers=layers)
    world = ts.world
    plan = None
    if keep_gathered == "plan":
        plan = plan_gradient_checkpointing({"gradient_checkpointing": True, "seq_length": tokens}, ts.model, device,
                                           shard_world=world)
        keep_gathered = 0 if plan.checkpoint else plan.gathered_layers
    kept = set_kept_gathered(ts.model, int(keep_gathered))
    sec = ts.timed(steps, warmup)
    peak = torch.cuda.max_memory_allocated(device) / 1e9
    ts.close()
    total = tokens * micro_batches * world
    n_layers = layers or QWEN[name]["num_hidden_layers"]
    out = {"model": f"Qwen2.5-{name} shapes ({n_layers} layers, random init, bf16), FSDP2 over {world} ranks",
           "kl_coef": kl_coef, "tokens_per_micro_batch": tokens, "micro_batches_per_step": micro_batches,
           "seq_len": seq, "ms_per_optimizer_step": round(sec * 1e3, 2), "tokens_per_s": round(total / sec, 1),
           "tokens_per_s_per_gpu": round(total / sec / world, 1), "peak_mem_gb": round(peak, 2),
           "steps": steps, "warmup": warmup, "kept_gathered_layers": kept}
    if plan is not None:
        out["plan"] = {k: v for k, v in plan.as_dict().items() if k in ("reason", "need_gb", "device_gb",
                                                                        "gathered_layers", "gathered_gb")}
    return out


def split_pipeline_probe(actors: int, steps: int = 2, warmup: int = 1, device=None, transport: str = "bucketed",
                         bucket_bytes: int = 256 << 20, make_trainer=None, make_actor_module=None,
                         packer=None) -> dict:
    """BASELINE.json configs[3] (C4) on one node: ranks [0, W-actors) train data-parallel, ranks
    [W-actors, W) are actors.  Trainer rank 0 broadcasts every optimizer step's weights to the
    actors over their own group (WeightUpdateManager -> WorkerExtension.receive_weight_update,
    finetune_loop.py:174-256 / vllm1.py:81-94) while the trainers run the next step.

    The trainers' step is timed twice: without weight updates, then with one update per step in
    flight.  ``hidden_frac`` = 1 - (extra step time) / (broadcast latency): 1.0 means the
    broadcast is fully overlapped (north_star), 0 means it is serialised as in the reference.

    make_trainer(dp_group) -> TrainerStep; make_actor_module() -> a module whose
    named_parameters() match the trainer model's (actors hold the inference copy).
    All ranks must call this collectively.  Returns the same dict on every rank.
    """
    from .actor import StandaloneWorker
    from .weight_update import ParameterInfo, WeightUpdateManager, WeightUpdateRequest

    world, rank = dist.get_world_size(), dist.get_rank()
    if not 1 <= actors < world:
        raise ValueError(f"need 1 <= actors < world ({actors}, {world})")
    n_tr = world - actors
    trainer_ranks = list(range(n_tr))
    # every rank creates every group, in the same order (torch.distributed requirement)
    from .torch_utils import collective_options

    opts = collective_options(dist.get_backend())  # as the trainer creates its DP and actor groups
    dp_group = dist.new_group(trainer_ranks, pg_options=opts)
    bc_group = dist.new_group([0] + list(range(n_tr, world)), pg_options=opts)
    is_trainer = rank < n_tr
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    from .comm_probe import group_census

    # both groups report (and carry) exactly the ranks the split intends, before any traffic
    mine = {}
    if is_trainer:
        mine["split_dp"] = (dp_group, n_tr)
    if rank == 0 or not is_trainer:
        mine["actor"] = (bc_group, 1 + actors)  # world.py:184: 1 + actor GPUs
    census = group_census(mine, dev)
    result = {}
    nupdates = warmup + steps
    if is_trainer:
        ts = make_trainer(dp_group)
        infos = [ParameterInfo(name=n, shape=list(p.shape), dtype=str(torch.bfloat16))
                 for n, p in ts.model.named_parameters()]
        sec_plain = ts.timed(steps, warmup)
        wum = None
        if rank == 0:
            wum = WeightUpdateManager([], ts.model, None, bc_group, transport=transport, bucket_bytes=bucket_bytes,
                                      overlap=True, packer=packer, write_message=lambda s, m: None)
            dist.broadcast_object_list([[i.model_dump() for i in infos]], src=0, group=bc_group)
        lat = []
        sec_bcast = ts.timed(steps, warmup, wum=wum)
        if wum is not None:
            wum.wait()
            lat = [wum.last_latency_s]
            wum.close()
        ts.close()
        result = {"plain_s": sec_plain, "bcast_s": sec_bcast, "latency_s": lat[0] if lat else 0.0, "groups": census}
    else:
        holder = [None]
        dist.broadcast_object_list(holder, src=0, group=bc_group)
        infos = [ParameterInfo(**d) for d in holder[0]]
        module = make_actor_module()
        worker = StandaloneWorker(module, rank=0, device=dev)
        worker.process_group = bc_group
        for v in range(nupdates):
            worker.receive_weight_update(WeightUpdateRequest(
                version=v + 1, parameters_info=infos, transport=transport,
                bucket_bytes=bucket_bytes if transport == "bucketed" else 0))
        _sync(dev)
        result = {"received": nupdates}
    # rank 0's view to everyone (object collective on the default group)
    out = [result]
    dist.broadcast_object_list(out, src=0)
    r0 = out[0]
    extra = max(0.0, r0["bcast_s"] - r0["plain_s"])
    lat = r0["latency_s"]
    nbytes = sum(2 * int(torch.Size(i.shape).numel()) for i in infos)
    return {"trainers": n_tr, "actors": actors, "transport": transport, "updates": nupdates,
            "ms_per_step_no_broadcast": round(r0["plain_s"] * 1e3, 2),
            "ms_per_step_with_broadcast": round(r0["bcast_s"] * 1e3, 2),
            "broadcast_latency_ms": round(lat * 1e3, 2), "broadcast_bytes": nbytes,
            "hidden_frac": round(1.0 - min(1.0, extra / lat), 4) if lat > 0 else None,
            "groups": r0.get("groups")}
