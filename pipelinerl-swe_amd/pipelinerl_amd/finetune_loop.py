"""The RL trainer process on MI355X (drop-in for pipelinerl/finetune_loop.py).

Same entry (``run_finetuning_loop(cfg)``, launched per rank by
``entrypoints/run_finetune.py --config-dir exp/conf --config-name exp_config +me.*=...``), same
inputs (the rank's ``training_data`` stream partition) and outputs (``weight_update_request``
topic messages, ``finetune/{current,intermediate,training_state,logs}``, summary.json,
rl_summary.json, the stats/throughput/rl metric keys), same protocol:

  * every pass is a lockstep exchange of sample counts across the data-parallel ranks; a rank
    whose share of the step is done gets sentinel batches (loss x 0) until the global count
    reaches ``samples_per_step`` (finetune_loop.py:567-617);
  * loss normalisation uses ``rl.batch_size = samples_per_step`` (:564-566);
  * the optimizer steps when the global count hits the step target; version = cumulative
    samples; weights are broadcast to the actors every ``weight_update_interval`` samples.

MI355X-first differences: the loss head is the fused HIP kernel (rl_step); the per-pass
count exchange runs on a CPU (gloo) control group, so the host never drains the GPU queue for
it; gradients are reduced in 256 MiB flat buckets overlapped with the boundary backward
(grad_sync.py), or sharded with FSDP2 (``use_fsdp`` / ``finetune.sharding: fsdp``,
finetune/sharding.py); the weight broadcast is snapshotted by a HIP kernel and overlapped with the
next step on a side stream (weight_update.py); no per-pass empty_cache; no HF-internal CE pass.
"""

from __future__ import annotations

import json
import logging
import math
import os
import threading
import time
from collections import defaultdict
from dataclasses import asdict
from pathlib import Path
from queue import Empty, Queue
from typing import Any, Callable

import numpy as np
import torch
import torch.distributed as dist

from .finetune.checkpoints import (load_model, load_tokenizer, load_training_state, remove_results,
                                   save_model_and_tokenizer, save_training_state)
from .finetune.grad_sync import GradBuckets
from .finetune.optim import clip_grad_norm, get_optimizer, master_weights_requested
from .finetune.rl import RLConfig, RLStats, rl_step
from .finetune.rl.utils import aggregate_rl_stats
from .finetune.sharding import decide_sharding, is_sharded, set_gradient_sync, shard_model
from .finetune.trace import PhaseTrace
from . import native_data
from .devalloc import DEFAULT_SETTINGS, configure_device_allocator
from .hostgc import freeze_setup_heap
from .finetune.types import PipelineBatchEncoding, TrainingMetrics
from .streams import SingleStreamSpec, read_stream, set_streams_backend, write_to_streams
from .weight_update import (TRAINER_TOPIC, ParameterInfo, SamplesProcessed, WeightUpdateManager,  # noqa: F401
                            WeightUpdateRequest, WeightUpdateSuccess)

logger = logging.getLogger(__name__)


# ------------------------------------------------------------------------------------------
# distributed context

class Dist:
    """rank / world / device + the CPU control group used for lockstep bookkeeping."""

    def __init__(self, backend: str | None = None, high_priority_collectives: bool = True):
        """``high_priority_collectives``: the RCCL data-parallel group runs its collectives on
        high-priority streams (torch_utils.collective_options), off the compute stream's queue."""
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        use_gpu = torch.cuda.is_available() and backend != "gloo"
        self.device = torch.device("cuda", self.local_rank) if use_gpu else torch.device("cpu")
        if use_gpu:
            torch.cuda.set_device(self.device)
        self.pg_options = None
        if not dist.is_initialized() and (self.world > 1 or "MASTER_ADDR" in os.environ):
            from .torch_utils import collective_options

            be = backend or ("nccl" if use_gpu else "gloo")
            self.pg_options = collective_options(be, high_priority_collectives)
            dist.init_process_group(be, device_id=self.device if use_gpu else None, pg_options=self.pg_options)
        self.initialized = dist.is_initialized()
        if self.initialized:
            self.world = dist.get_world_size()
            self.rank = dist.get_rank()
        self.ctrl = dist.new_group(backend="gloo") if self.initialized and dist.get_backend() != "gloo" else None

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    def barrier(self) -> None:
        if self.initialized:
            dist.barrier(group=self.ctrl)

    def sum_int(self, x: int) -> int:
        if not self.initialized:
            return int(x)
        t = torch.tensor([int(x)], dtype=torch.int64)
        dist.all_reduce(t, group=self.ctrl)
        return int(t.item())

    def gather_object(self, obj: Any) -> list[Any]:
        if not self.initialized:
            return [obj]
        out: list[Any] = [None] * self.world
        dist.all_gather_object(out, obj, group=self.ctrl)
        return out


# ------------------------------------------------------------------------------------------
# data loading

def run_data_loader(data_stream: SingleStreamSpec, batch_queue: Queue, device: torch.device,
                    stop: threading.Event | None = None, timeout: float | None = None) -> None:
    """Reads PipelineBatchEncoding micro-batches (finetune_loop.py:92-115); token counts are
    taken on the host before the pinned, non-blocking H2D copy."""
    native = os.environ.get("PRL_NATIVE_DECODE", "1") != "0"  # 0: json + validators (A/B)
    pin = device.type == "cuda"
    try:
        with read_stream(data_stream, timeout=timeout) as reader:
            for line in reader.read_lines():
                if stop is not None and stop.is_set():
                    return
                # libprl_data decodes the numeric fields into pinned tensors without the GIL
                b = native_data.decode_batch(line, pin=pin) if native else PipelineBatchEncoding(**json.loads(line))
                ntok = int(b.attention_mask.sum())
                nseq = batch_sequence_count(b)
                if device.type == "cuda":
                    rows = b.label_rows_from_host()  # the label-row lm_head's count, known on the host
                    for name in type(b).model_fields:
                        v = getattr(b, name)
                        if isinstance(v, torch.Tensor) and name != "seq_boundaries":  # host metadata
                            setattr(b, name, (v if v.is_pinned() else v.pin_memory()).to(device, non_blocking=True))
                    if rows is not None:
                        b._label_rows = rows.pin_memory().to(device, non_blocking=True)
                batch_queue.put((b, ntok, nseq))
        if stop is None or not stop.is_set():  # the reader went idle for `timeout` s: fail, not hang
            batch_queue.put(TimeoutError(f"no training data on {data_stream} for {timeout} s"))
    except Exception as e:
        batch_queue.put(e)


def batch_sequence_count(batch: PipelineBatchEncoding) -> int:
    """finetune_loop.py:266-276."""
    if batch.position_ids is not None:
        assert batch.seq_boundaries is not None
        n = len(batch.seq_boundaries) - 1
        return n if batch.padding == 0 else n - 1
    return int(batch.input_ids.size(0))


def calculate_train_steps(args, interrupt_train_steps: int) -> int:
    if interrupt_train_steps == -1:
        assert args.interrupt_train_steps <= args.max_train_steps
        return args.max_train_steps if args.interrupt_train_steps < 0 else args.interrupt_train_steps
    assert interrupt_train_steps <= args.max_train_steps
    return interrupt_train_steps


def write_message(stream: SingleStreamSpec, msg) -> None:
    with write_to_streams(stream) as w:
        w.write(msg)


def wait_for_inference_servers(urls: list[str], timeout: float = 3600.0) -> None:
    import requests

    t0 = time.time()
    for url in urls:
        while True:
            try:
                if requests.get(url + "/health", timeout=5).status_code == 200:
                    break
            except requests.RequestException:
                pass
            if time.time() - t0 > timeout:
                raise TimeoutError(f"inference server {url} not healthy")
            time.sleep(1.0)


# ------------------------------------------------------------------------------------------

def run_finetuning_loop(cfg, step_fn: Callable = rl_step, model=None, tokenizer=None,
                        weight_update_manager_factory: Callable | None = None) -> TrainingMetrics:
    """Trainer process main (finetune_loop.py:290-486).  ``step_fn``/``model`` are injectable
    for tests; production uses rl_step and the HF model named by cfg.finetune.config_name."""
    set_streams_backend(**cfg.streams)
    high_prio = str(cfg.finetune.get("collective_stream_priority", "high")) == "high"
    ctx = Dist(cfg.finetune.get("dist_backend"), high_prio)
    args = cfg.finetune if "finetune" in cfg else cfg
    grad_mode = grad_scale_convention(cfg)
    if args.gradient_accumulation_passes % ctx.world:
        raise ValueError("gradient_accumulation_passes must be divisible by num_processes")
    torch.manual_seed(args.seed)
    np.random.seed(args.seed)
    # variable-length micro-batches: cached blocks reusable across nearby sizes (devalloc.py)
    configure_device_allocator(args.get("allocator_settings", DEFAULT_SETTINGS))

    exp_root = Path(cfg.output_dir)
    output_dir = Path(args.output_dir)
    current_dir, inter_dir = output_dir / "current", output_dir / "intermediate"
    state_dir, log_dir = output_dir / "training_state", output_dir / "logs"
    if args.get("force_restart", False) and ctx.is_main:
        remove_results(current_dir, inter_dir, state_dir, log_dir)
    ctx.barrier()
    setup_logging(log_dir, ctx.rank)
    update_stream = SingleStreamSpec(exp_path=exp_root, topic=TRAINER_TOPIC)

    master = master_weights_requested(cfg)  # fp32 masters + moments: the reference default's optimizer state
    world = ctx.world if ctx.initialized else 1
    layout: dict[str, Any] = {}

    def choose_shard_world(m) -> int:
        """The model state's layout over the DP ranks (finetune/sharding.py decide_sharding)."""
        shard, reason = decide_sharding(cfg, args, m, ctx.device, world, master)
        layout.update(shard=shard, reason=reason)
        if ctx.is_main:
            logger.info(f"model state layout: {'FSDP' if shard else 'replicas'} ({reason}); "
                        f"optimizer state: {'fp32 master weights + fp32 AdamW moments' if master else 'bf16'}")
        return world if shard else 1

    snapshot = weight_snapshot_mode(args)
    if model is None:
        model = load_model(args, args.model_class, current_dir, ctx.device, shard_world=choose_shard_world,
                           master_weights=master)
    else:
        choose_shard_world(model)
    sharded = layout["shard"] and ctx.initialized  # FSDP2 needs a process group (one rank included)
    if tokenizer is None:
        tokenizer = load_tokenizer(args.config_name, getattr(getattr(model, "config", None), "eos_token_id", None))
    if sharded:  # before the optimizer: it must see the sharded parameters
        plan = getattr(model, "prl_memory_plan", None)  # load_model's (finetune/recompute.py)
        model = shard_model(model, cfg.get("fsdp"), grad_reduce=args.get("grad_reduce", "mean"),
                            keep_gathered=plan.gathered_layers if plan is not None else 0, master_weights=master)
    elif args.get("flat_parameters", True):
        # every bf16 parameter into one buffer in the weight broadcast's layout (weight_update.py):
        # in-place broadcasts, the gate / up projections one tensor without a concatenation copy
        from .weight_update import rehome_parameters

        rehome_parameters(model)
    data_stream = SingleStreamSpec(exp_path=exp_root, topic=args.input, instance=0, partition=ctx.rank)
    optimizer = get_optimizer(args.optim, model, args.learning_rate, args.weight_decay, master_weights=master)
    from transformers import get_scheduler

    lr_scheduler = get_scheduler(args.lr_scheduler_type, optimizer, args.num_warmup_steps, args.max_train_steps)
    grads = None
    if ctx.initialized and ctx.world > 1 and not sharded:
        grads = GradBuckets(list(model.parameters()), bucket_bytes=int(args.get("grad_bucket_mb", 256)) << 20,
                            reduce=args.get("grad_reduce", "mean"))

    actor_group = None
    if ctx.is_main and args.send_weight_updates:
        from .torch_utils import init_extra_process_group

        backend = args.get("actor_group_backend", "nccl")
        if backend == "prl_comm":  # RCCL communicator of the prl_comm C ABI (comm.py)
            from .comm import RcclComm

            actor_group = RcclComm.create(cfg.me.weight_update_group_init_method, 0,
                                          cfg.me.weight_update_group_world_size, ctx.device)
        else:
            from .torch_utils import collective_options

            actor_group = init_extra_process_group(
                group_name="actor", backend=backend, init_method=cfg.me.weight_update_group_init_method, rank=0,
                world_size=cfg.me.weight_update_group_world_size, pg_options=collective_options(backend, high_prio))
    ctx.barrier()

    metrics = TrainingMetrics()
    if state_dir.exists():  # finetune_loop.py:416-418: resume whenever the directory exists
        check_training_state_layout(state_dir)
        metrics = load_training_state(state_dir, model, optimizer, lr_scheduler, metrics)
        metrics.lr = optimizer.param_groups[0]["lr"]
    if ctx.is_main:
        write_message(update_stream, SamplesProcessed(samples_processed=metrics.samples))

    wum = None
    if args.send_weight_updates:
        urls = cfg.me.llm_urls.split("+")
        if ctx.is_main and args.get("wait_for_inference_servers", True):
            wait_for_inference_servers(urls)
        ctx.barrier()
        factory = weight_update_manager_factory or WeightUpdateManager
        wum = factory(urls, model, update_stream, actor_group, transport=args.get("weight_transport", "per_tensor"),
                      bucket_bytes=int(args.get("weight_bucket_mb", 256)) << 20,
                      overlap=bool(args.get("overlap_weight_updates", True)), is_main=ctx.is_main,
                      timeout_s=args.get("weight_update_timeout_s", 900.0),
                      http_timeout_s=args.get("weight_update_http_timeout_s", 600.0),
                      snapshot=snapshot)
        wum.send_weight_update(metrics.samples)

    batch_queue: Queue = Queue(maxsize=1)
    stop = threading.Event()
    loader = threading.Thread(target=run_data_loader,
                              args=(data_stream, batch_queue, ctx.device, stop, args.get("data_timeout_s")),
                              daemon=True)
    model.train()
    freeze_setup_heap()  # no generation-2 walks over the set-up heap mid-step (hostgc.py)
    loader.start()
    try:
        return rl_finetuning_worker(args, ctx, model, optimizer, lr_scheduler, grads, wum, tokenizer, metrics,
                                    batch_queue, update_stream, step_fn, grad_scale_mode=grad_mode)
    finally:
        stop.set()
        if wum is not None:
            wum.close()
        if actor_group is not None:
            if hasattr(actor_group, "close"):
                actor_group.close()
            else:
                dist.destroy_process_group(actor_group)


def weight_snapshot_mode(args) -> str:
    """``finetune.weight_snapshot``: "zero_copy" broadcasts the parameters in place, which needs them
    re-homed into one flat buffer at load (``finetune.flat_parameters``, the default); with
    ``flat_parameters: false`` the default is the staging copy, and an explicit "zero_copy" falls
    back to it (with a warning) rather than re-homing the parameters after the optimizer exists."""
    flat = bool(args.get("flat_parameters", True))
    mode = args.get("weight_snapshot", "zero_copy" if flat else "copy")
    if mode == "zero_copy" and not flat:
        logger.warning("finetune.weight_snapshot=zero_copy needs finetune.flat_parameters=true; "
                       "using the staging copy (weight_snapshot=copy)")
        mode = "copy"
    return mode


class TrainingStateError(RuntimeError):
    """A training_state/ directory this trainer cannot resume from."""


def check_training_state_layout(state_dir: Path) -> None:
    """The reference resumes whenever ``training_state/`` exists (finetune_loop.py:416-418), in one
    of two layouts (finetune/checkpoints.py:169-180): Accelerate's ``training_state.pt`` (this
    trainer's own, loaded) or DeepSpeed's ``model.save_checkpoint(dir, tag="deepspeed")`` (a
    ``deepspeed/`` tag directory + ``latest``, the reference's default backend).  The DeepSpeed
    layout holds ZeRO-partitioned model and optimizer shards this trainer does not read: starting
    over at samples=0 would silently restart the weight versions the actors see, so raise."""
    if (state_dir / "training_state.pt").exists():
        return
    if (state_dir / "deepspeed").is_dir() or (state_dir / "latest").exists():
        raise TrainingStateError(
            f"{state_dir} holds a DeepSpeed checkpoint (tag 'deepspeed', finetune/checkpoints.py:169-180); this "
            "trainer resumes only from training_state.pt: convert it (DeepSpeed's zero_to_fp32 for the weights into "
            "finetune/current) or start from a fresh output_dir")
    raise TrainingStateError(f"{state_dir} exists but holds no training_state.pt (the reference would fail to "
                             "load it too, finetune/checkpoints.py:229)")


def grad_scale_convention(cfg) -> str:
    """Which engine's gradient-accumulation convention the run follows.  The reference's backend
    is DeepSpeed ZeRO-3 by default (conf/base.yaml ``use_deepspeed: true``), whose
    ``engine.backward`` divides every micro-batch loss by ``gradient_accumulation_steps``
    (injected at finetune_loop.py:307-312); with Accelerate (FSDP or plain DDP, GAS 1) the
    micro-batch gradients are summed.  ``finetune.grad_scale: accelerate | deepspeed`` overrides."""
    args = cfg.finetune if "finetune" in cfg else cfg
    mode = args.get("grad_scale")
    if mode is None:
        mode = "deepspeed" if cfg.get("use_deepspeed", False) and not cfg.get("use_fsdp", False) else "accelerate"
        if (mode == "accelerate" and not cfg.get("use_deepspeed", False) and not cfg.get("use_fsdp", False)
                and cfg.get("deepspeed_config")):
            # the documented way to launch without DeepSpeed (use_deepspeed=false, launch.py:272-277)
            # also flips this default: the clipped gradient becomes GAS x the reference default's
            logger.warning(
                f"use_deepspeed is false but the config still names deepspeed_config={cfg.get('deepspeed_config')}: "
                "the reference's default run uses DeepSpeed's gradient-accumulation scale (every micro-batch loss "
                "/ GAS) and fp32 master weights; this run sums micro-batch gradients (accelerate) and, unless "
                "finetune.master_weights=true, trains the bf16 weights directly. Set finetune.grad_scale=deepspeed "
                "and finetune.master_weights=true to keep the reference default's gradients and optimizer state, or "
                "finetune.grad_scale=accelerate to silence this warning")
    if mode not in ("accelerate", "deepspeed"):
        raise ValueError(f"finetune.grad_scale must be 'accelerate' or 'deepspeed', got {mode!r}")
    return mode


def micro_batch_loss_scale(args, world: int, mode: str) -> float:
    """1 / gradient_accumulation_steps under DeepSpeed, where GAS = seq_parallel *
    gradient_accumulation_passes / num_processes (finetune_loop.py:306-310); 1 otherwise."""
    if mode != "deepspeed":
        return 1.0
    gas = args.seq_parallel * (args.gradient_accumulation_passes // world)
    return 1.0 / gas


def rl_finetuning_worker(args, ctx: Dist, model, optimizer, lr_scheduler, grads: GradBuckets | None,
                         wum: WeightUpdateManager | None, tokenizer, metrics: TrainingMetrics, batch_queue: Queue,
                         update_stream: SingleStreamSpec, step_fn: Callable = rl_step,
                         grad_scale_mode: str = "accelerate") -> TrainingMetrics:
    """finetune_loop.py:488-867."""
    output_dir = Path(args.output_dir)
    current_dir, inter_dir, state_dir = output_dir / "current", output_dir / "intermediate", output_dir / "training_state"
    final_steps = calculate_train_steps(args, args.interrupt_train_steps)
    if metrics.completed_steps == final_steps:
        logger.info("Training is already completed")
        return metrics

    num_lead = ctx.world // args.seq_parallel
    per_lead_passes = args.gradient_accumulation_passes // num_lead
    samples_per_lead_per_step = per_lead_passes * args.train_batch_size
    samples_per_step = samples_per_lead_per_step * num_lead
    start_samples = metrics.samples
    rl_config = RLConfig(**dict(args.rl))
    rl_config.batch_size = samples_per_step
    target_per_lead, target = samples_per_lead_per_step, samples_per_step
    local_samples = 0
    first_pass = True
    rl_metrics: dict[str, list] = defaultdict(list)
    lag: dict[str, int] = {}
    tokens_processed: list[int] = []
    passes_took: list[float] = []
    mb_sizes: list[int] = []
    waiting = 0.0
    sync_every = bool(args.get("fsdp_sync_every_micro_batch", False))
    safe = bool(args.get("use_safetensors", False))  # checkpoints.py:285 default
    loss_scale = micro_batch_loss_scale(args, ctx.world, grad_scale_mode)
    native_step = step_fn is rl_step
    defer_stats = True  # statistics resolved after the backward is queued (rl_step(defer_stats=True))
    collective_backward = is_sharded(model)  # FSDP: every rank's backward joins all-gathers
    trace = PhaseTrace(ctx.device, bool(args.get("trace_gpu_phases", False)) or os.environ.get("PRL_TRACE_GPU") == "1")
    trace_md: dict[str, float] = {}

    def next_batch():
        timeout = 0.1
        while True:
            try:
                item = batch_queue.get(timeout=timeout)
                break
            except Empty:
                timeout = min(timeout * 1.5, 5.0)
        if isinstance(item, Exception):
            raise item
        return item

    while metrics.completed_steps < final_steps:
        if first_pass:
            first_pass = False
            step_start = time.time()
            trace.start()
        t_wait = time.time()
        batch, ntok, nseq = next_batch()
        sentinel = bool(batch.sentinel)
        if local_samples == target_per_lead:
            assert sentinel, "We should get a sentinel batch"
        waiting += time.time() - t_wait
        if args.get("max_lag") is not None and metrics.last_broadcasted_version - batch.model_version > args.max_lag:
            metrics.samples_too_old_to_train += args.train_batch_size
        lag["min_version"] = min(lag.get("min_version", batch.model_version), batch.model_version)
        lag["max_version"] = max(lag.get("max_version", batch.model_version), batch.model_version)
        if not sentinel:
            t_pass = time.time()
            metrics.passes += 1
            mb_sizes.append(nseq)
            local_samples += nseq
            tokens_processed.append(ntok)

        if native_step:  # stats read back after the backward is queued; gradients at loss_scale
            loss, stats = step_fn(model, batch, metrics.completed_steps, final_steps, rl_config,
                                  grad_scale=loss_scale, defer_stats=defer_stats)
        else:
            loss, stats = step_fn(model, batch, metrics.completed_steps, final_steps, rl_config)
        trace.mark("forward")
        # The lockstep count exchange (CPU control group) after the forward is queued: a host waiting
        # there for a slower rank leaves its device this pass's forward (and, below the quota, its
        # backward) to run instead of nothing.  Only the boundary pass needs the answer before its
        # backward (it arms the gradient all-reduce / FSDP's reduce-scatter); a rank still below
        # its own quota cannot be on it — every rank's count is at most its quota, so the total is
        # short of the target — and exchanges after queueing the backward, unless the backward
        # itself is collective (FSDP re-gathers parameters there: a rank at its quota would wait in
        # the exchange for one blocked in that all-gather).  Same values exchanged,
        # same messages as the reference (finetune_loop.py:577-617); workloads.lockstep_cost prices
        # the coupling.
        def exchange() -> int:
            total_over = ctx.sum_int(local_samples)
            assert total_over % args.seq_parallel == 0
            return total_over // args.seq_parallel

        early = args.seq_parallel == 1 and local_samples < target_per_lead and not collective_backward
        if early:
            do_step = False
        else:
            total = exchange()
            do_step = total == target
            if do_step and grads is not None:
                grads.arm()
        set_gradient_sync(model, do_step or sync_every)  # FSDP: reduce-scatter on the boundary only
        if sentinel:
            loss = loss * 0.0
        elif loss_scale != 1.0:
            loss = loss * loss_scale  # DeepSpeed's engine.backward: loss / gradient_accumulation_steps
        loss.backward()
        trace.mark("backward")
        if early:
            total = exchange()
            if total == target:
                raise RuntimeError(f"the global sample count reached the step's target ({target}) while this rank "
                                   f"was below its quota ({local_samples} < {target_per_lead}): the input streams "
                                   "do not follow the per-rank quota protocol")
        if isinstance(stats, RLStats):
            stats = stats.resolve()  # also raises the reference's non-finite assertions
        if not sentinel:
            for k, v in stats.items():
                rl_metrics[k].append(v)
            metrics.lr = optimizer.param_groups[0]["lr"]
        if not sentinel:
            passes_took.append(time.time() - t_pass)
        if ctx.is_main:
            write_message(update_stream, SamplesProcessed(samples_processed=start_samples + total))
        if not do_step:
            continue

        target_per_lead += samples_per_lead_per_step
        target += samples_per_step
        step_took = time.time() - step_start
        first_pass = True
        metrics.completed_steps += 1
        metrics.samples = start_samples + total
        worker_tokens = sum(tokens_processed)
        metrics.tokens += worker_tokens * ctx.world

        if grads is not None:
            grads.finish()
        trace.mark("allreduce_wait")
        clip = args.get("gradient_clipping_threshold")
        # torch's clip_grad_norm_; with the HIP AdamW the multiply runs inside its step (optim.py)
        gn = clip_grad_norm(model.parameters(), clip if clip else float("inf"), optimizer)
        trace.mark("clip")
        if wum is not None:
            wum.poll()  # a failed update (actor error / timeout) ends training here
            wum.before_optimizer_step()
        optimizer.step()
        if grads is not None:
            grads.zero_()
        else:
            optimizer.zero_grad(set_to_none=True)
        lr_scheduler.step()
        trace.mark("optimizer")
        metrics.grad_norm = float(gn)
        trace_md = trace.collect()  # the device has just been waited for (grad norm read)

        time_to_stop = metrics.completed_steps >= final_steps
        time_to_log = metrics.completed_steps % args.log_each_n_steps == 0
        also = list(args.get("also_save_steps", []) or [])
        time_to_save = (metrics.completed_steps % args.save_checkpoint_steps == 0 or
                        metrics.completed_steps in also) and not time_to_stop
        assert sum(mb_sizes) == samples_per_lead_per_step, (sum(mb_sizes), samples_per_lead_per_step)
        metrics.time_waiting_for_data += waiting
        md: dict[str, Any] = {}
        if time_to_log or time_to_save:
            md.update(step_metrics(metrics, lag, batch_queue, tokens_processed, passes_took, mb_sizes, ctx.world,
                                   samples_per_step, step_took))
            gathered = defaultdict(list)
            for per_rank in ctx.gather_object(dict(rl_metrics)):  # gather_rl_metrics, finetune_loop.py:62-89
                for k, vs in per_rank.items():
                    if vs:  # an empty list adds no key; non-finite values are dropped
                        gathered[k].extend(v for v in vs if np.isfinite(v))
            avg = aggregate_rl_stats(gathered, samples_per_step)
            if avg.get("rl/ratio_new_old_squared_sum") and avg.get("rl/num_output_tokens_sum"):
                avg["rl/ess"] = (avg["rl/ratio_new_old_sum"] ** 2 / avg["rl/ratio_new_old_squared_sum"]
                                 / avg["rl/num_output_tokens_sum"])
            md.update(avg)
            md.update(trace_md)
            rl_metrics = defaultdict(list)
            lag = {}
            tokens_processed, passes_took, mb_sizes = [], [], []
            waiting = 0.0
        if md and ctx.is_main:
            log_metrics(metrics.completed_steps, md, output_dir / "logs")
        if wum is not None and metrics.samples - metrics.last_broadcasted_version >= args.weight_update_interval:
            wum.send_weight_update(metrics.samples)  # overlapped with the next step
            metrics.last_broadcasted_version = metrics.samples
        if time_to_save:
            save_model_and_tokenizer(current_dir, model, tokenizer, safe_serialization=safe, group=ctx.ctrl)
            save_training_state(state_dir, model, optimizer, lr_scheduler, asdict(metrics), group=ctx.ctrl)
            if args.get("keep_intermediate_checkpoints", False):
                save_model_and_tokenizer(inter_dir / str(metrics.completed_steps), model, tokenizer,
                                         safe_serialization=safe, group=ctx.ctrl)
        if time_to_stop:
            break

    if wum is not None:
        wum.wait()
    save_model_and_tokenizer(current_dir, model, tokenizer, safe_serialization=safe, group=ctx.ctrl)
    if args.get("save_final_training_state", True):
        save_training_state(state_dir, model, optimizer, lr_scheduler, asdict(metrics), group=ctx.ctrl)
    if ctx.is_main:
        (output_dir / "summary.json").write_text(json.dumps(asdict(metrics), indent=4, sort_keys=True))
        (output_dir / "rl_summary.json").write_text(json.dumps(dict(rl_metrics), indent=4, sort_keys=True))
    return metrics


def step_metrics(m: TrainingMetrics, lag, q, tokens, passes, mbs, world, samples_per_step, step_took) -> dict:
    """The stats/* and throughput/* keys of finetune_loop.py:726-764, with the reference's values
    (``tokens``: this rank's micro-batch token counts; pinned by F7, tests/golden/make_f7.py).
    ``throughput/real_tokens_per_sec`` is this rank's tokens / step wall time as at :754; the
    whole job's rate is the added ``throughput/real_tokens_per_sec_all_ranks``."""
    wt = sum(tokens)
    sp = sum(passes)
    return {
        "stats/lr": m.lr, "stats/grad_norm": m.grad_norm, "stats/samples": m.samples, "stats/tokens": m.tokens,
        "stats/samples_too_old_to_queue": m.samples_too_old_to_queue,
        "stats/samples_too_old_to_train": m.samples_too_old_to_train, "stats/passes": m.passes,
        "stats/completed_steps": m.completed_steps, "stats/epoch": m.epoch,
        "stats/min_actor_version": lag.get("min_version", 0), "stats/max_actor_version": lag.get("max_version", 0),
        "stats/queue/batches": q.qsize(), "stats/time_waiting_for_data": m.time_waiting_for_data,
        "stats/lag": m.last_broadcasted_version - lag.get("min_version", 0),
        "throughput/tokens_perGPU_per_sec": wt / sp if sp else 0,
        "throughput/tokens_per_step": wt * world,
        "throughput/micro_batches_per_step": len(tokens),
        "throughput/min_tokens_per_micro_batch": min(tokens) if tokens else 0,
        "throughput/max_tokens_per_micro_batch": max(tokens) if tokens else 0,
        "throughput/tokens_per_micro_batch": wt / len(tokens) if tokens else 0,
        "throughput/tokens_per_sec": wt * world / sp if sp else 0,
        "throughput/real_tokens_per_sec": wt / step_took if step_took else 0,
        "throughput/real_tokens_per_sec_all_ranks": wt * world / step_took if step_took else 0,
        "throughput/sec_per_pass": sp / len(passes) if passes else 0,
        "throughput/steps_per_sec": 1 / step_took if step_took else 0,
        "throughput/samples_per_sec": samples_per_step / sp if sp else 0,
        "throughput/sec_per_step": step_took,
        "throughput/max_sequences_per_micro_batch": max(mbs) if mbs else 0,
        "throughput/min_sequences_per_micro_batch": min(mbs) if mbs else 0,
        "throughput/sequences_per_micro_batch": sum(mbs) / len(mbs) if mbs else 0,
    }


def setup_logging(log_dir: Path, rank: int) -> None:
    log_dir.mkdir(parents=True, exist_ok=True)
    fh = logging.FileHandler(log_dir / f"info_{rank}.log")
    fh.setFormatter(logging.Formatter("[%(asctime)s][%(name)s][%(levelname)s] - %(message)s"))
    root = logging.getLogger()
    if not any(isinstance(h, logging.FileHandler) and getattr(h, "baseFilename", "") == fh.baseFilename
               for h in root.handlers):
        root.addHandler(fh)
    root.setLevel(logging.INFO)


def log_metrics(step: int, md: dict, log_dir: Path) -> None:
    line = {"step": step, **{k: (float(v) if isinstance(v, (int, float)) and not isinstance(v, bool) else v)
                             for k, v in md.items()}}
    with open(Path(log_dir) / "metrics.jsonl", "a") as f:
        f.write(json.dumps(line) + "\n")
    logger.info(f"step {step}: " + ", ".join(f"{k}={v:.4g}" for k, v in md.items()
                                             if isinstance(v, (int, float)) and math.isfinite(float(v))))
