"""Trainer-step benchmark: fused packed-GRPO loss head on MI355X (BASELINE.json configs[1], C2).

Workload per rank (weak scaling): one packed micro-batch of T = 65536 tokens (32 rollouts x 2048,
prompt 256) of Qwen2.5-1.5B-shaped logits [1, T, 151936] bf16, synthetic, resident in HBM.
One step = what rl_step does for a micro-batch after the model forward (rl/__init__.py:199-377):
fused HIP forward (log-softmax + gather + entropy + PPO/KL loss + stats + dlogits), the
autograd backward (upstream-gradient check on device), the one D2H read of the statistics,
and for N > 1 the per-pass sample-count exchange of the DP loop (finetune_loop.py:613,
all-reduce of one int64 over RCCL).  The statistics are read back as the trainer loop reads them
(rl_step(defer_stats=True): an async copy into pinned memory, resolved later) so the GPU queue
does not drain between micro-batches: in the loop the model's backward is queued when a
micro-batch's statistics are resolved; here the loss head's backward is a few microseconds, so a
micro-batch's statistics are resolved once the next micro-batch is queued (every step's are read
inside the timed region; the last one's before the closing synchronize).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...     (one rank per GPU)

At N > 1, after the timed region, the trainer's exchange steps are measured on the real code
paths over the C2 model's parameter set (pipelinerl_amd/comm_probe.py) and reported under
"exchange": the bucketed DP gradient all-reduce (GradBuckets, RCCL) and the trainer -> actors
weight broadcast (WeightUpdateManager -> WorkerExtension, rank 0 -> ranks 1..N-1).

After that, at every N, the whole optimizer step the loss head sits in is measured and reported
under "trainer_step" (pipelinerl_amd/trainer_probe.py): Qwen2.5-1.5B shapes (random init, bf16),
2 packed micro-batches of 65 536 tokens per rank (C2's micro-batch; varlen attention, fused
RMSNorm / SwiGLU / RoPE, label-row lm_head + fused loss head, backward), the bucketed RCCL
gradient all-reduce overlapped with the last backward, clip, fused AdamW.

Then, at every N, "c3_dp": BASELINE.json configs[2] (C3), the Qwen2.5-7B data-parallel trainer step
on C3's packed math rollouts (prompt U{64..512} + completion U{256..8192}, packing cap 12 000), 4
micro-batches per rank, with the full bucketed 15.23 GB gradient all-reduce at N > 1: the replica's
step without the all-reduce, the DP step and the all-reduce alone, its exposed share and overlap,
and the tokens/s extrapolated to C3's 4096-sample step (one all-reduce per ~hundreds of
micro-batches).  trainer_step at N > 1 likewise times the replica alone first: dp_efficiency is
the trainer-step scaling fraction at this N.  At N = 1, c3_dp also times the step with an emulated
ring all-reduce of the gradients (trainer_probe.EmulatedRingBuckets: the reads a ring over N = 4 / 8
GPUs makes on each, paced to xGMI link rates, launched from the boundary backward's hooks) and
projects C3's DP efficiency at that N (dp_scaling.c3_projected_efficiency); "c3_dp_value_head" is
the same step with a value head (the reference's default actor_critic config).

At N > 1, last, BASELINE.json configs[3] (C4) is measured under "split_pipeline": ranks
[0, N/2) train Qwen2.5-7B shapes data-parallel while ranks [N/2, N) act as actors; trainer rank 0
broadcasts each step's weights to them (WeightUpdateManager -> WorkerExtension) while the
trainers run the next step.  The trainers' step time with and without the broadcast in flight
gives hidden_frac (1.0 = the broadcast latency is fully overlapped).  At N >= 4, "fsdp_32b":
BASELINE.json configs[4] (C5), Qwen2.5-32B shapes sharded with FSDP2 over all ranks, KL on; last,
"fsdp_32b_kept_gathered": the same with the memory plan's decoder layers kept gathered from forward
to backward (one all-gather per layer fewer), and its speedup over "fsdp_32b".

At N = 1, "snapshot_overlap" prices the trainer-side half of "weight broadcast fully overlapped":
C3's 7B step with no weight update, with WeightUpdateManager's staging copy in flight after each
optimizer step, and with the in-place (zero-copy, default) snapshot, in rotating rounds, beside the
copy's own duration.  At N > 1, "communicators" first checks that every communicator reports (and
carries, by an all-reduce of ones) the intended rank count: the DP group, the CPU control group and a
prl_comm RCCL communicator (ncclCommCount); the split pipeline's DP and actor groups are checked in
its own probe ("split_pipeline.groups").  At N = 1, "loss_head_fp32": the same C2 micro-batch with
fp32 logits (Accelerate's upcast regime; grpo_fwd_pair_f32, each row resident over two CUs, with the
round-4 part-resident kernel alternated beside it), its kernel time and fraction of the HBM peak on
2 x 4 x T x V algorithmic bytes.

Prints ONE JSON line (rank 0).  roofline.achieved = algorithmic bytes per launch
(T*V*2 read + T*V*2 dlogits write + 37*T side data) / the average duration
of the prl_grpo_forward launch measured with HIP events on its stream; roofline.box_copy = the
same bytes through torch's device copy in the same run (box-to-box HBM rates differ by a few %).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
for _p in (str(ROOT), str(ROOT / "pipelinerl-swe_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md); measured float4 copy 6290 GB/s
SIDE_BYTES_PER_TOKEN = 37  # ids 8 + old 4 + ref 4 + adv 4 + w 4 + mask 1 + lp/H/tok_loss 12


def fp32_loss_head_probe(T: int, V: int, device, iters: int = 8, warmup: int = 2, rounds: int = 2) -> dict:
    """C2's micro-batch with fp32 logits (Accelerate's mixed precision upcasts them,
    finetune_loop.py:381-385): the fused loss head's forward + gradient, HIP events on its stream;
    algorithmic bytes = logits read once + dlogits written once + side data.
    At Qwen2.5 vocabularies the product kernel is grpo_fwd_pair_f32<19> (each row fully resident
    over a pair of CUs); the round-4 part-resident grpo_fwd_hybrid_f32<19, 9> (PrlGrpoParams.f32_rows
    = 1) is timed in alternation beside it, same process and buffers."""
    from pipelinerl_amd.finetune.rl.fused import GrpoParams, grpo_loss

    lb, fields = make_workload(T, V, seq=2048, prompt=256, seed=4321, device=device)
    logits = lb.detach().float().requires_grad_(True)
    del lb
    torch.cuda.empty_cache()
    params = GrpoParams(policy_loss="ppo", epsilon=4.0, kl_coef=0.0, entropy_coef=0.0, clamp_log_ratio=5.0,
                        temperature=1.0, batch_size=4096.0)
    times: dict[str, list[float]] = {"pair": [], "hybrid": []}
    import ctypes
    import dataclasses

    from pipelinerl_amd import _native
    from pipelinerl_amd.finetune.rl.fused import _workspace

    def fallbacks() -> int:  # row halves that computed their partner's partial themselves (read + reset)
        n = ctypes.c_uint64(0)
        ws = _workspace(device)
        _native.check(_native.load().prl_grpo_pair_fallbacks(ws.data_ptr(), ws.numel(),
                                                             torch.cuda.current_stream(device).cuda_stream,
                                                             ctypes.byref(n)), "prl_grpo_pair_fallbacks")
        return int(n.value)

    fallbacks()
    fb, pair_launches = 0, 0
    arm_params = {"pair": params, "hybrid": dataclasses.replace(params, f32_rows=1)}
    for _ in range(rounds):
        for arm in ("pair", "hybrid"):
            for i in range(warmup + iters):
                logits.grad = None
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                loss, stats, _ = grpo_loss(logits, fields, arm_params[arm])
                e1.record()
                loss.backward()
                stats.cpu()
                if i >= warmup:
                    times[arm].append(e0.elapsed_time(e1))
            if arm == "pair":
                fb += fallbacks()
                pair_launches += warmup + iters
    # beside 16 resident side workgroups reading at one xGMI link's rate (an RCCL collective's
    # channels beside the loss head): the pair kernel's time, and its extra HBM reads — every row
    # half that computed its partner's partial itself re-read that half row (V/2 x 4 B); PMC counting
    # serialises kernels, so the extra traffic comes from the kernel's own fallback counter
    side = torch.cuda.Stream(device=device)
    src = torch.empty(4 << 30, dtype=torch.uint8, device=device)
    sink = torch.zeros(16, dtype=torch.int32, device=device)
    lib = _native.load()
    fallbacks()
    side_ms: list[float] = []
    for i in range(warmup + iters):
        logits.grad = None
        side.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(side):  # ~26 ms of reads at 153 GB/s: covers the launch
            _native.check(lib.prl_paced_read(ctypes.c_void_p(src.data_ptr()), 4 << 30, 153.0, 16,
                                             ctypes.c_void_p(sink.data_ptr()), side.cuda_stream), "prl_paced_read")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        loss, stats, _ = grpo_loss(logits, fields, params)
        e1.record()
        loss.backward()
        stats.cpu()
        torch.cuda.synchronize(device)
        if i >= warmup:
            side_ms.append(e0.elapsed_time(e1))
    fb_side = fallbacks() / (warmup + iters)
    del src
    ms = float(np.median(times["pair"]))
    ms_h = float(np.median(times["hybrid"]))
    alg = 2.0 * T * V * 4 + SIDE_BYTES_PER_TOKEN * T
    del logits, fields
    torch.cuda.empty_cache()
    traffic = traffic_h = None  # HBM bytes per launch from the committed PMC passes (tools/profile_bench.sh)
    pmcs = sorted((ROOT / "profiles").glob("r*_fp32_pmc.json"))  # the newest round's passes
    src = pmcs[-1].name if pmcs else "r05_fp32_pmc.json"
    try:
        pmc = json.loads((ROOT / "profiles" / src).read_text())["per_launch_median"]
        if T == 65536 and V == 151936:
            for k, v in pmc.items():
                if "pair_f32" in k:
                    traffic = v["fetch_size_bytes"] + v["write_size_bytes"]
                elif "hybrid" in k:
                    traffic_h = v["fetch_size_bytes"] + v["write_size_bytes"]
    except (OSError, KeyError, ValueError):
        pass
    return {"kernel": "grpo_fwd_pair_f32<19> (+slot memset, stats/finalize) per prl_grpo_forward", "tokens": T,
            "vocab": V, "logits_dtype": "fp32", "kernel_ms": round(ms, 4), "algorithmic_bytes": alg,
            "achieved_GBps": round(alg / ms / 1e6, 1), "frac": round(alg / ms / 1e6 / HBM_PEAK_GBS, 4),
            "traffic": traffic, "traffic_over_algorithmic": round(traffic / alg, 4) if traffic else None,
            "traffic_source": src if traffic else None,
            "tokens_per_s": round(T / ms * 1e3, 1), "iters": iters * rounds,
            "pair_fallbacks_per_launch": round(fb / max(1, pair_launches), 3),
            "pair_row_halves_per_launch": 2 * T,
            "beside_16_side_workgroups": {
                "side": "prl_paced_read, 16 workgroups at 153 GB/s on another stream, launched with each call",
                "kernel_ms": round(float(np.median(side_ms)), 4),
                "fallbacks_per_launch": round(fb_side, 2),
                "traffic_over_algorithmic": (round((traffic + fb_side * (V // 2) * 4) / alg, 4) if traffic else None),
                "traffic_basis": "PMC per-launch traffic (serialised) + fallback half rows x V/2 x 4 B re-read"},
            "hybrid": {"kernel": "grpo_fwd_hybrid_f32<19, 9> (f32_rows=1, alternated)", "kernel_ms": round(ms_h, 4),
                       "frac": round(alg / ms_h / 1e6 / HBM_PEAK_GBS, 4),
                       "traffic_over_algorithmic": round(traffic_h / alg, 4) if traffic_h else None}}


def make_workload(T: int, V: int, seq: int, prompt: int, seed: int, device):
    g = torch.Generator(device=device).manual_seed(seed)
    logits = torch.empty((1, T, V), dtype=torch.bfloat16, device=device)
    chunk = 4096
    for a in range(0, T, chunk):  # chunked generation keeps the fp32 temporary small
        b = min(T, a + chunk)
        logits[0, a:b] = (torch.randn((b - a, V), generator=g, device=device) * 3.0).to(torch.bfloat16)
    nseq = T // seq
    pos = torch.arange(T, device=device) % seq
    ids = torch.randint(0, 151643, (1, T), generator=g, device=device)
    labels = torch.where(pos[None] >= prompt, ids, torch.full_like(ids, -100))
    rewards = torch.repeat_interleave(torch.randint(0, 2, (nseq,), generator=g, device=device).float(), seq)[None]
    lab = (labels != -100).float()
    old = (torch.randn((1, T), generator=g, device=device) - 12.0) * lab
    fields = {
        "input_ids": ids, "labels": labels, "rewards": rewards, "advantages": rewards - rewards.mean(),
        "ref_logprobs": old.clone(), "old_logprobs": old,
        "group_tokens": torch.full((1, T), float(seq), device=device),
        "num_labels": torch.full((1, T), float(seq - prompt), device=device),
        "overflow": torch.zeros((1, T), device=device),
    }
    return logits.requires_grad_(True), {k: v.contiguous() for k, v in fields.items()}


def cpu_baseline(rows: int, V: int, threads: int, min_seconds: float = 10.0, max_reps: int = 16) -> dict:
    """Oracle (numpy restatement of rl_step's loss head incl. gradient) on a bounded sample."""
    from oracle import grpo_oracle, synth

    T = rows + 1
    b = synth.packed_rl_batch(11, [T], [1], id_range=151643, eos=151643)
    lg = synth.to_bf16(np.random.default_rng(0).normal(0, 3.0, (1, T, V))).astype(np.float32)
    m = b["labels"] != -100
    b["old_logprobs"] = np.where(m, -12.0, 0).astype(np.float32)
    b["ref_logprobs"] = b["old_logprobs"].copy()
    cfg = dict(policy_loss="ppo", epsilon=4.0, kl_coef=0.0, final_kl_coef=0.0, batch_size=256,
               clamp_log_ratio_ref_new_value=5)
    # repeat the sample until ~min_seconds of CPU work (bounded: the bench stays within minutes)
    reps, t0 = 0, time.perf_counter()
    while reps < max_reps and (reps == 0 or time.perf_counter() - t0 < min_seconds):
        grpo_oracle.rl_step_oracle(lg, b, cfg, 0, 10, dtype=np.float32, threads=threads, row_chunk=16)
        reps += 1
    dt = time.perf_counter() - t0
    return {"value": round(rows * reps / dt, 1), "unit": "tokens/s", "cores": threads, "kind": "port",
            "sample": f"{reps} x {rows} packed rows x V={V}, fwd+grad, numpy float32 oracle, {threads} threads, "
                      f"{dt:.2f} s"}


def host_cpu() -> dict:
    """The host the CPU baseline ran on (record nproc and the CPU model)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "torch": torch.__version__}


def cpu_threads() -> int:
    """The CPU share this process is given: OMP_NUM_THREADS when the pool sets it (16 per GPU on
    the MI355X boxes, whose nproc counts the whole 256-CPU machine), else the affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS")
    return max(1, int(env)) if env and env.isdigit() else len(os.sched_getaffinity(0))


def load_traffic(T: int, V: int) -> tuple[float | None, str | None]:
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if one exists for this shape."""
    for p in sorted((ROOT / "profiles").glob("*pmc_traffic.json"), reverse=True):
        try:
            d = json.loads(p.read_text())
        except Exception:
            continue
        if d.get("T") == T and d.get("V") == V and d.get("bytes_per_launch"):
            return float(d["bytes_per_launch"]), p.name
    return None, None


def dp_scaling(world: int, c3: dict | None, trainer: dict | None) -> dict | None:
    """The north star's trainer-step scaling quantity beside `value` (which, at N > 1, is the loss
    head's weak scaling and linear by construction): C3's data-parallel 7B step tokens/s over N x
    what one replica does alone on its GPU in the same run (its `local` timing, no all-reduce), per
    measured 4-micro-batch step and extrapolated to C3's 4096-sample step (one all-reduce and one
    optimizer tail per ~hundreds of micro-batches); and the 1.5B trainer step's."""
    if not c3 or "tokens_per_s" not in c3:
        return None
    out = {"metric": "C3 DP trainer tokens/s / (N x one replica's local tokens/s)", "n_gpus": world,
           "c3_tokens_per_s": c3["tokens_per_s"], "c3_local_tokens_per_s_per_gpu": c3["local_tokens_per_s_per_gpu"],
           "c3_efficiency": round(c3["tokens_per_s"] / (world * c3["local_tokens_per_s_per_gpu"]), 4),
           "c3_speedup_vs_one_replica": round(c3["tokens_per_s"] / c3["local_tokens_per_s_per_gpu"], 3)}
    ex = c3.get("extrapolated") or {}
    if ex.get("allreduce_share") is not None:
        out["c3_extrapolated_efficiency"] = round(1.0 - ex["allreduce_share"], 5)
        out["c3_extrapolated_tokens_per_s"] = round(ex["tokens_per_s_per_gpu"] * world, 1)
    emu = c3.get("allreduce_emulated")
    if emu:
        # N = 1 bound on the scaling claim: the emulated ring all-reduce's exposed time per arm, and
        # C3's efficiency at that arm's N projected from it and the lockstep protocol's model
        out["allreduce_exposed_ms_emulated"] = {k: v["exposed_ms"] for k, v in emu.items()}
        out["c3_projected_efficiency"] = {k: v["projection"]["projected_efficiency"] for k, v in emu.items()
                                          if "projection" in v}
        out["c3_projected_efficiency_basis"] = (
            "lockstep model (workloads.LOCKSTEP_EFFICIENCY, the loop's order on C3's packing) x (1 - emulated "
            "all-reduce exposed ms / C3's 4096-sample step); arms: ranks, xGMI GB/s, channel workgroups in c3_dp")
    if trainer and trainer.get("dp_efficiency") is not None:
        out["trainer_step_1.5b_efficiency"] = trainer["dp_efficiency"]
    return out


def communicator_census(world: int, ctrl, device, prl_comm: bool = True) -> dict:
    """The N > 1 line's ``communicators`` object: the default (DP) group, the CPU control group and,
    with ``prl_comm``, an RCCL communicator of the prl_comm C ABI over all ranks (ncclCommCount), each
    checked against ``world`` (comm_probe.group_census raises on a mismatch).  The split pipeline's
    own DP and actor groups are checked inside its probe (``split_pipeline.groups``).  A prl_comm
    communicator needs one GPU per rank: the one-GPU rehearsal passes ``prl_comm=False``."""
    from pipelinerl_amd import comm_probe

    groups = {"dp": (None, world), "ctrl": (ctrl, world)}
    rc = None
    if prl_comm:
        from pipelinerl_amd.comm import RcclComm

        rc = RcclComm.from_group(ctrl, device)
        groups["prl_comm_dp"] = (rc, world)
    try:
        return comm_probe.group_census(groups, device)
    finally:
        if rc is not None:
            rc.close()


T_START = time.perf_counter()


class ProbeRunner:
    """Runs the bench's side probes independently: a probe that raises is reported as an error
    (its traceback on this rank's stderr); the ranks agree over the CPU control group ``ctrl``
    whether a probe failed anywhere (``error_on_another_rank``) BEFORE any of them synchronises the
    device; every result carries its wall time (``wall`` collects them).

    A failure on EVERY rank (the same probe failing the same way, e.g. out of memory) leaves the
    collectives matched and the next probe runs.  A failure on SOME ranks only may leave the other
    ranks' RCCL collectives without partners: those ranks then skip their device synchronise,
    abort the default RCCL group (so its queued collectives return instead of hanging), and every
    later probe is skipped with the reason.  An agreement that times out counts as such a failure.
    A device that no longer synchronises ends the probing (SystemExit).

    ``deadline_s`` (N > 1): a probe still running after that long is taken to be stuck in a
    collective that will never complete; a timer thread aborts this rank's RCCL communicators (the
    torch groups and prl_comm's), so the stuck collective returns with an error, the probe fails,
    and every later probe is skipped — the line with `value` (measured before the probes) is still
    printed, well before torch's own RCCL watchdog (10 min) would abort the process."""

    def __init__(self, rank: int, device, ctrl=None, deadline_s: float | None = None):
        self.rank, self.device, self.ctrl = rank, torch.device(device), ctrl
        self.wall: dict[str, float] = {}
        self.poisoned: str | None = None
        self.deadline_s = deadline_s
        self.expired: str | None = None

    def _agree(self, failed: int) -> tuple[int, int]:
        """(ranks that failed, ranks in ctrl); (-1, n) when the agreement itself failed."""
        if self.ctrl is None:
            return failed, 1
        n = dist.get_world_size(self.ctrl)
        try:
            flag = torch.tensor([failed], dtype=torch.int64)
            dist.all_reduce(flag, group=self.ctrl)
            return int(flag), n
        except Exception as e:  # noqa: BLE001 - a peer never arrived (stuck or dead)
            print(f"[rank {self.rank}] probe agreement failed: {type(e).__name__}: {e}", file=sys.stderr, flush=True)
            return -1, n

    def _abort_rccl(self) -> None:
        try:
            if dist.is_initialized() and "nccl" in str(dist.get_backend()):
                dist.distributed_c10d._abort_process_group()
        except Exception as e:  # noqa: BLE001
            print(f"[rank {self.rank}] aborting the RCCL group failed: {e}", file=sys.stderr, flush=True)
        try:
            from pipelinerl_amd import comm

            comm.abort_all()
        except Exception as e:  # noqa: BLE001
            print(f"[rank {self.rank}] aborting the prl_comm communicators failed: {e}", file=sys.stderr, flush=True)

    def _expire(self, name: str) -> None:
        self.expired = name
        print(f"[rank {self.rank}] probe {name} still running after its {self.deadline_s:.0f} s deadline: "
              "aborting the RCCL communicators", file=sys.stderr, flush=True)
        self._abort_rccl()

    def run(self, name: str, fn):
        t0 = time.perf_counter()
        if self.poisoned is not None:
            self.wall[name] = 0.0
            why = ("passed its deadline: the RCCL communicators were aborted" if self.expired
                   else "failed on some ranks only: its collectives may be unmatched")
            return {"skipped": f"probe {self.poisoned} {why}", "wall_s": 0.0}
        res, failed = None, 0
        done = threading.Event()
        if self.rank == 0:  # progress on stderr (a silent multi-minute probe looks hung to a watchdog)
            print(f"[bench] probe {name} started", file=sys.stderr, flush=True)

            def beat():
                while not done.wait(45.0):
                    print(f"[bench] probe {name} running {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)

            threading.Thread(target=beat, daemon=True).start()
        timer = None
        if self.deadline_s and self.ctrl is not None:
            timer = threading.Timer(self.deadline_s, self._expire, args=(name,))
            timer.daemon = True
            timer.start()
        try:
            res = fn()
        except Exception as e:  # noqa: BLE001
            import traceback

            failed = 1
            print(f"[rank {self.rank}] probe {name} failed:\n{traceback.format_exc()}", file=sys.stderr, flush=True)
            res = {"error": f"{type(e).__name__}: {e}"[:400]}
        finally:
            if timer is not None:  # after join() the abort either ran to completion or never will
                timer.cancel()
                timer.join()
        if self.expired == name:  # the communicators are gone: nothing after this may use them
            failed = 1
            res = dict(res or {}, deadline_s=self.deadline_s)
        nfail, n = self._agree(failed)  # before any device synchronise
        partial = nfail < 0 or 0 < nfail < n or self.expired is not None
        if nfail != 0 and not failed:
            res = dict(res or {}, error_on_another_rank=True)
        if partial:
            self.poisoned = name
            self._abort_rccl()
        ok = 1
        # the probe's memory back before the next one: Python garbage first (reference cycles can
        # hold a probe's model and optimizer state; the trainer probes freeze the heap they set up,
        # as the loop does, so it is unfrozen first or those cycles would never be collected — the
        # C3 probe's 15 GB parameter buffer stayed allocated through every later probe), then
        # torch's cached device blocks and pinned host buffers (gloo stages CUDA tensors through
        # pinned host memory in the one-GPU rehearsal, where every rank shares one card)
        import gc

        gc.unfreeze()
        gc.collect()
        if self.device.type == "cuda" and not partial:
            try:
                torch.cuda.synchronize(self.device)
                torch.cuda.empty_cache()
            except Exception as e:  # noqa: BLE001 - the device itself failed
                res, ok = {"error": f"device after {name}: {type(e).__name__}: {e}"[:400]}, -1
        if hasattr(torch._C, "_host_emptyCache"):
            torch._C._host_emptyCache()
        try:
            import psutil

            rss = round(psutil.Process().memory_info().rss / 2 ** 30, 2)
        except Exception:  # noqa: BLE001
            rss = None
        done.set()
        self.wall[name] = round(time.perf_counter() - t0, 1)
        if self.rank == 0:
            state = "ok" if nfail == 0 else ("failed on every rank" if nfail == n else "failed on some ranks")
            print(f"[bench] probe {name} done in {self.wall[name]} s ({state})", file=sys.stderr, flush=True)
        if isinstance(res, dict):
            res["wall_s"] = self.wall[name]
            res["host_rss_gib_after"] = rss
            if self.device.type == "cuda" and ok >= 0 and not partial:
                res["device_free_gib_after"] = round(torch.cuda.mem_get_info(self.device)[0] / 2 ** 30, 2)
        if ok < 0:
            raise SystemExit(f"device failure in probe {name}")
        return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--vocab", type=int, default=151936)
    ap.add_argument("--cpu-rows", type=int, default=4096)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-comm-probe", action="store_true", help="N > 1: skip the all-reduce / broadcast probes")
    ap.add_argument("--no-trainer-step", action="store_true", help="skip the full trainer-step probe")
    ap.add_argument("--no-c3", action="store_true", help="skip the configs[2] 7B DP trainer-step probe")
    ap.add_argument("--no-fsdp", action="store_true", help="N >= 4: skip the configs[4] FSDP 32B probe")
    ap.add_argument("--no-fp32", action="store_true", help="N = 1: skip the fp32-logits loss-head probe")
    ap.add_argument("--no-split-pipeline", action="store_true",
                    help="N > 1: skip the split trainer/actor probe (configs[3]: 7B, overlapped weight broadcast)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # PRL_BENCH_REHEARSE=gloo: rehearsal of the N > 1 control flow on ONE GPU (every rank on
    # cuda:0, gloo collectives); the measured multi-GPU runs use RCCL, one GPU per rank
    rehearse = os.environ.get("PRL_BENCH_REHEARSE") == "gloo"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if rehearse:  # gloo for CUDA tensors too (FSDP's device mesh would open RCCL groups)
            dist.init_process_group("cpu:gloo,cuda:gloo")
        else:
            from pipelinerl_amd.torch_utils import collective_options

            # the trainer's DP group (finetune_loop.Dist): collectives on high-priority streams
            dist.init_process_group("nccl", device_id=dev, pg_options=collective_options("nccl"))

    from pipelinerl_amd import _native
    from pipelinerl_amd.finetune.rl.fused import GrpoParams, grpo_loss

    _native.load()
    T, V = args.tokens, args.vocab
    logits, fields = make_workload(T, V, seq=2048, prompt=256, seed=1234 + rank, device=dev)
    # GRPO defaults: conf/finetune/base.yaml:92-105 + grpo.yaml (ppo, eps 4, kl 0, C 5)
    params = GrpoParams(policy_loss="ppo", epsilon=4.0, kl_coef=0.0, entropy_coef=0.0, clamp_log_ratio=5.0,
                        temperature=1.0, batch_size=4096.0)
    samples = torch.zeros(1, dtype=torch.int64, device=dev)
    fwd_ev = []
    # the statistics' read-back as rl_step(defer_stats=True) does it: one async D2H copy into pinned
    # memory per micro-batch (two slots: one resolving while the next is written), waited on later
    from pipelinerl_amd._native import NSTAT

    host_stats = [torch.empty(NSTAT, dtype=torch.float64, pin_memory=True) for _ in range(2)]
    resolved = []

    def step(timed: bool, i: int):
        logits.grad = None
        if timed:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        loss, stats, _ = grpo_loss(logits, fields, params)
        if timed:
            e1.record()
            fwd_ev.append((e0, e1))
        host_stats[i % 2].copy_(stats, non_blocking=True)  # the one statistics read-back per micro-batch
        copied = torch.cuda.Event()
        copied.record()
        loss.backward()
        if world > 1:
            samples.fill_(T // 2048)
            dist.all_reduce(samples)
        return copied, i % 2

    def resolve(pending):
        if pending is not None:
            pending[0].synchronize()
            resolved.append(float(host_stats[pending[1]][0]))  # (the loss term, kept as a use of the read)

    def run(n: int, timed: bool):
        pending = None
        for i in range(n):
            nxt = step(timed, i)
            resolve(pending)  # micro-batch i - 1's statistics, micro-batch i queued behind them
            pending = nxt
        resolve(pending)

    run(args.warmup, False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps, True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t_max = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in fwd_ev]))
    k_max = torch.tensor([kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        dist.all_reduce(k_max, op=dist.ReduceOp.MAX)
    elapsed = float(t_max)
    kern_ms = float(k_max)
    # the same bytes through a plain device copy on this box (torch's copy kernel, logits -> a second
    # buffer: one read + one write of T x V bf16), after the timed region: HBM rates vary a few %
    # from box to box, and this puts the loss head's rate beside a copy measured in the same run
    copy_ms = None
    if rank == 0:
        dst = torch.empty_like(logits)
        cts = []
        for i in range(8):
            c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            c0.record()
            dst.copy_(logits.detach())
            c1.record()
            c1.synchronize()
            if i >= 2:
                cts.append(c0.elapsed_time(c1))
        copy_ms = float(np.median(cts))
        del dst
    # The probes below are reported beside `value`, never in it.  Each one is independent: a probe
    # that raises is reported as an error (every rank's traceback on stderr), the ranks agree on its
    # outcome over a CPU control group, and the next probe still runs; each reports its wall time.
    # Order = what the north star needs first (C3 DP scaling, the 1.5B step, C5, C4, the exchange
    # microbenchmarks), so a driver lease that runs out loses the least important ones.
    import datetime

    ctrl = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=300)) if world > 1 else None
    # a probe stuck in a collective is cut off after this long (N > 1; torch's RCCL watchdog: 10 min)
    deadline = float(os.environ.get("PRL_BENCH_PROBE_DEADLINE_S", "480")) if world > 1 else None
    runner = ProbeRunner(rank, dev, ctrl, deadline_s=deadline)
    optional, probe_wall = runner.run, runner.wall

    logits = fields = None
    torch.cuda.empty_cache()
    census = None
    if world > 1:
        # every communicator of the run reports the size it was meant to have (and that many ranks
        # take part in an all-reduce over it) before any probe relies on it
        census = optional("communicators", lambda: communicator_census(world, ctrl, dev, prl_comm=not rehearse))
    c3 = None
    if not args.no_c3:
        # configs[2] (C3): Qwen2.5-7B DP trainer step on C3's packed math rollouts, with the full
        # bucketed 15.23 GB gradient all-reduce at N > 1 (local / DP / all-reduce-alone timings);
        # at N = 1 also the same step with the weight-update snapshot (staging copy / in place) in
        # flight (at N > 1 the split_pipeline probe prices the whole broadcast with real actors)
        from pipelinerl_amd.trainer_probe import RING_ARMS, dp_step_probe

        # at N = 1 also the same step with emulated ring all-reduces of the gradients (N = 4 / 8 at one
        # xGMI link's rate, N = 8 over seven) launched from the boundary backward's hooks
        c3 = optional("c3_dp", lambda: dp_step_probe("c3", micro_batches=4, steps=2, warmup=1, device=dev,
                                                      layers=4 if rehearse else None, snapshot=world == 1,
                                                      emulate=RING_ARMS if world == 1 else None))
    c3_vh = None
    if world == 1 and not args.no_c3:
        # the reference's default fine-tune config is actor_critic (conf/base.yaml:2): the same C3 step
        # with a value head, through the label-row lm_head as the GRPO step
        from pipelinerl_amd.trainer_probe import dp_step_probe

        c3_vh = optional("c3_dp_value_head", lambda: dp_step_probe("c3", micro_batches=4, steps=2, warmup=1,
                                                                    device=dev, value_head=True))
    trainer = None
    if not args.no_trainer_step:
        # the whole optimizer step the loss head sits in
        from pipelinerl_amd.trainer_probe import trainer_step_probe

        trainer = optional("trainer_step", lambda: trainer_step_probe("1.5b", tokens=T, micro_batches=2, steps=2,
                                                                      warmup=1, device=dev, fused_head=True,
                                                                      layers=4 if rehearse else None))
    fp32 = None
    if world == 1 and not args.no_fp32:
        # the loss head in the fp32-logits regime (Accelerate's upcast): the pair kernel (+ the hybrid A/B)
        fp32 = optional("loss_head_fp32", lambda: fp32_loss_head_probe(T, V, dev))
    fsdp = None
    if world >= 4 and not args.no_fsdp:
        # configs[4] (C5): Qwen2.5-32B shapes, FSDP2 over every rank, KL-to-reference on
        from pipelinerl_amd.trainer_probe import fsdp_step_probe

        fsdp = optional("fsdp_32b", lambda: fsdp_step_probe("32b", tokens=2048 if rehearse else 4096, micro_batches=1,
                                                             steps=2, warmup=1,
                                                             device=dev, kl_coef=0.001,
                                                             layers=2 if rehearse else None))
    split = None
    if world > 1 and not args.no_split_pipeline:
        # configs[3] (C4): half the ranks train Qwen2.5-7B shapes data-parallel, the other half are
        # actors receiving every step's weights from trainer rank 0 while the trainers run the next
        # step; reports the step time with and without the broadcast in flight (hidden_frac)
        from pipelinerl_amd import comm_probe
        from pipelinerl_amd.trainer_probe import TrainerStep, split_pipeline_probe

        # a rehearsal puts every rank on one GPU: 4 of the 7B's layers, 4 096-token micro-batches
        split_layers, split_tokens = (4, 4096) if rehearse else (None, 16384)

        def split_run():
            shapes = comm_probe.qwen2_param_shapes("7b", layers=split_layers)
            r = split_pipeline_probe(
                world // 2, steps=2, warmup=1, device=dev,
                make_trainer=lambda g: TrainerStep("7b", tokens=split_tokens, micro_batches=2, device=dev, group=g,
                                                   layers=split_layers),
                make_actor_module=lambda: comm_probe.ShapedModule(shapes, device=dev, fill=0.0))
            r["model"] = (f"Qwen2.5-7b shapes{f' ({split_layers} layers)' if split_layers else ''} (random init, "
                          f"bf16), 2 x {split_tokens}-token micro-batches per trainer rank")
            return r

        split = optional("split_pipeline", split_run)
    comm = None
    if world > 1 and not args.no_comm_probe:
        # the trainer's two exchange steps on the C2 model's parameter set: DP gradient all-reduce,
        # trainer -> actors broadcast
        from pipelinerl_amd import comm_probe

        def exchange():
            shapes = comm_probe.qwen2_param_shapes("1.5b")
            return {"model": "Qwen2.5-1.5B parameter shapes, bf16",
                    "grad_allreduce": comm_probe.grad_allreduce_probe(shapes, dev, iters=5),
                    "weight_broadcast": comm_probe.broadcast_probe(shapes, dev, iters=3)}

        comm = optional("exchange", exchange)
    fsdp_kept = None
    if world >= 4 and not args.no_fsdp and not rehearse:
        # C5 again with the loop's memory plan applied: the last R decoder layers kept gathered from
        # forward to backward (finetune.fsdp_keep_gathered_layers), beside fsdp_32b's FSDP2 default.
        # Last, as its own probe: it holds up to every layer unsharded, and a failure here costs no
        # other probe.  (Not in a one-GPU rehearsal: ~100 s per FSDP step over gloo.)
        from pipelinerl_amd.trainer_probe import fsdp_step_probe

        def kept_run():
            r = fsdp_step_probe("32b", tokens=4096, micro_batches=1, steps=2, warmup=1, device=dev, kl_coef=0.001,
                                keep_gathered="plan")
            if isinstance(fsdp, dict) and fsdp.get("ms_per_optimizer_step"):
                r["speedup_vs_fsdp_32b"] = round(fsdp["ms_per_optimizer_step"] / r["ms_per_optimizer_step"], 4)
            return r

        fsdp_kept = optional("fsdp_32b_kept_gathered", kept_run)

    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        tokens_total = T * world * args.steps
        alg_bytes = 2.0 * T * V * 2 + SIDE_BYTES_PER_TOKEN * T
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
        traffic, tsrc = load_traffic(T, V)
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            threads = cpu_threads()
            cpu = cpu_baseline(args.cpu_rows, V, threads)
            # the reference's CPU finetune path on configs[0] (C1: Qwen2.5-0.5B, 256 packed
            # rollouts, one optimizer step; a bounded sample of its micro-batches, extrapolated)
            from oracle import cpu_trainer

            cpu["c1"] = cpu_trainer.cpu_c1_step(threads)
            cpu["host"] = host_cpu()
        out = {
            "metric": "trainer tokens/s (packed GRPO) at 1/2/4/8 MI355X; loss-kernel HBM GB/s",
            "value": round(tokens_total / elapsed, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic packed rollouts (randn*3 bf16 logits, 32 x 2048-token sequences, 256-token prompts)",
            "config": {"workload": "C2: fused GRPO loss head fwd+grad, Qwen2.5-1.5B vocab, packed micro-batch",
                       "tokens_per_rank": T, "vocab": V, "logits_dtype": "bf16", "policy_loss": "ppo",
                       "parallelism": f"dp{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "kernel": "grpo_fwd_resident<19> (+stats/finalize) per prl_grpo_forward",
                         "kernel_ms": round(kern_ms, 4), "algorithmic_bytes": alg_bytes,
                         "traffic_source": tsrc,
                         "box_copy": None if copy_ms is None else {
                             "what": "torch copy_ of the T x V bf16 logits into a second buffer, same run",
                             "ms": round(copy_ms, 4), "GBps": round(2.0 * T * V * 2 / copy_ms / 1e6, 1),
                             "loss_head_vs_copy": round(copy_ms / kern_ms, 4)}},
            "cpu_baseline": cpu,
        }
        scaling = dp_scaling(world, c3, trainer)
        if scaling is not None:
            out["dp_scaling"] = scaling
        if isinstance(c3, dict) and "snapshot_overlap" in c3:
            # the trainer-side half of "weight broadcast fully overlapped": C3's 7B step with and
            # without WeightUpdateManager's snapshot in flight on its side stream
            out["snapshot_overlap"] = dict(c3.pop("snapshot_overlap"), step="c3_dp (Qwen2.5-7B, 4 micro-batches)")
        if isinstance(c3_vh, dict):  # beside the GRPO step: its rate, step time and roofline only
            c3_vh = {k: c3_vh[k] for k in ("config", "value_head", "ms_per_step_local", "tokens_per_s_per_gpu",
                                           "optimizer_tail_ms", "peak_mem_gb", "roofline", "extrapolated")
                     if k in c3_vh}
        for key, res in (("communicators", census), ("c3_dp", c3), ("c3_dp_value_head", c3_vh),
                         ("trainer_step", trainer),
                         ("loss_head_fp32", fp32), ("fsdp_32b", fsdp),
                         ("split_pipeline", split), ("exchange", comm), ("fsdp_32b_kept_gathered", fsdp_kept)):
            if res is not None:
                out[key] = res
        out["probe_wall_s"] = probe_wall
        out["wall_total_s"] = round(time.perf_counter() - T_START, 1)
        print(json.dumps(out), flush=True)
    if world > 1:
        try:
            dist.destroy_process_group()
        except Exception as e:  # noqa: BLE001 - an aborted RCCL group (see ProbeRunner)
            print(f"[rank {rank}] destroy_process_group: {e}", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
