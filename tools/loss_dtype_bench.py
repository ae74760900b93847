"""The fused loss head with bf16 logits (DeepSpeed regime, the resident kernel) and fp32 logits
(Accelerate mixed precision upcasts the logits: the streaming kernel, whose gradient pass
re-reads the row) at the same packed micro-batch; algorithmic bytes = logits read once + dlogits
written once (measurement tool).

With ``--f32-kernels``: the fp32 loss head's kernels alternated in one process at C2 (the row split
over a pair of workgroups, fully resident — the default —; PRL_F32_PAIR=0: the part-resident hybrid;
PRL_PAIR_SPIN_TICKS=0: the pair kernel whose halves never wait for each other's partial), medians
of HIP-event times per arm and round, one JSON line per arm.

With ``--inplace``: the bf16 loss head writing dlogits to its own buffer (the bench's form) vs over
the logits it has just read (dlogits aliasing batch->logits, allowed by include/prl_hip.h): same
bytes, same kernel, alternating arms, HIP events on the launch stream.

    python tools/loss_dtype_bench.py [--tokens 65536] [--vocab 151936] [--inplace]
"""

import argparse
import ctypes
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def f32_kernels_ab(a):
    import os

    from pipelinerl_amd.finetune.rl.fused import GrpoParams, grpo_loss

    dev = torch.device("cuda", 0)
    params = GrpoParams(policy_loss="ppo", epsilon=4.0, kl_coef=0.0, entropy_coef=0.0, clamp_log_ratio=5.0,
                        temperature=1.0, batch_size=4096.0)
    lb, fields = bench.make_workload(a.tokens, a.vocab, 2048, 256, 4321, dev)
    logits = lb.detach().float().requires_grad_(True)
    del lb
    arms = {"pair": {"PRL_F32_PAIR": "1"}, "hybrid": {"PRL_F32_PAIR": "0"},
            "pair_nowait": {"PRL_F32_PAIR": "1", "PRL_PAIR_SPIN_TICKS": "0"}}
    torch.cuda.empty_cache()
    alg = 2.0 * a.tokens * a.vocab * logits.element_size() + bench.SIDE_BYTES_PER_TOKEN * a.tokens
    res = {k: [] for k in arms}
    ref = None
    for r in range(a.rounds):
        for name, env in arms.items():
            os.environ.pop("PRL_PAIR_SPIN_TICKS", None)
            os.environ.update(env)
            times = []
            for i in range(8):
                logits.grad = None
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                loss, stats, _ = grpo_loss(logits, fields, params)
                e1.record()
                loss.backward()
                torch.cuda.synchronize()
                if i >= 2:
                    times.append(e0.elapsed_time(e1))
            out = (float(loss), logits.grad[0, ::997].float().clone())
            if ref is None:
                ref = out
            same = out[0] == ref[0] and torch.equal(out[1], ref[1])
            res[name].append(float(np.median(times)))
            print(json.dumps({"round": r, "arm": name, "ms": round(float(np.median(times)), 4),
                              "frac": round(alg / np.median(times) / 1e6 / bench.HBM_PEAK_GBS, 4),
                              "loss": out[0], "same_as_first_arm": bool(same)}), flush=True)
    for name, v in res.items():
        ms = float(np.median(v))
        print(json.dumps({"arm": name, "median_ms": round(ms, 4), "frac": round(alg / ms / 1e6 / bench.HBM_PEAK_GBS, 4),
                          "tokens": a.tokens, "vocab": a.vocab, "algorithmic_bytes": alg}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--vocab", type=int, default=151936)
    ap.add_argument("--inplace", action="store_true", help="separate vs aliased dlogits A/B (bf16)")
    ap.add_argument("--f32-kernels", action="store_true", help="pair vs hybrid fp32 kernels, alternated")

    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--dl-offsets", default=None,
                    help="comma-separated byte offsets of the dlogits buffer's start (bf16 A/B of HBM placement)")
    a = ap.parse_args()
    if a.inplace:
        return inplace_ab(a)
    if a.f32_kernels:
        return f32_kernels_ab(a)

    if a.dl_offsets:
        return offsets_ab(a, [int(x) for x in a.dl_offsets.split(",")])
    from pipelinerl_amd.finetune.rl.fused import GrpoParams, grpo_loss

    dev = torch.device("cuda", 0)
    params = GrpoParams(policy_loss="ppo", epsilon=4.0, kl_coef=0.0, entropy_coef=0.0, clamp_log_ratio=5.0,
                        temperature=1.0, batch_size=4096.0)
    for dt in (torch.bfloat16, torch.float32):
        logits, fields = bench.make_workload(a.tokens, a.vocab, 2048, 256, 1234, dev)
        if dt == torch.float32:
            logits = logits.detach().float().requires_grad_(True)
        times = []
        for i in range(8):
            logits.grad = None
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            loss, _, _ = grpo_loss(logits, fields, params)
            e1.record()
            loss.backward()
            torch.cuda.synchronize()
            if i >= 2:
                times.append(e0.elapsed_time(e1))
        ms = sum(times) / len(times)
        b = logits.element_size()
        alg = 2.0 * a.tokens * a.vocab * b + 37 * a.tokens
        print(json.dumps({"logits_dtype": str(dt).replace("torch.", ""), "T": a.tokens, "V": a.vocab, "ms": round(ms, 3),
                          "algorithmic_GBps": round(alg / ms / 1e6, 1), "tokens_per_s": round(a.tokens / ms * 1e3, 1)}),
              flush=True)
        del logits, fields, loss
        torch.cuda.empty_cache()


def inplace_ab(a, rounds: int = 5, iters: int = 10):
    from pipelinerl_amd import _native
    from pipelinerl_amd.finetune.rl.fused import GrpoParams, _c_batch, _workspace

    dev = torch.device("cuda", 0)
    lib = _native.load()
    params = GrpoParams(policy_loss="ppo", epsilon=4.0, kl_coef=0.0, entropy_coef=0.0, clamp_log_ratio=5.0,
                        temperature=1.0, batch_size=4096.0)
    logits, fields = bench.make_workload(a.tokens, a.vocab, 2048, 256, 1234, dev)
    x = logits.detach()
    master = x.clone()  # the in-place arm restores its logits from here before every launch
    sep = torch.empty_like(x)
    B, L, V = x.shape
    rows = torch.empty((8, B * (L - 1)), dtype=torch.float32, device=dev)
    stats = torch.empty(_native.NSTAT, dtype=torch.float64, device=dev)
    ws = _workspace(dev)
    cp = params.to_c(True)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def launch(out: torch.Tensor) -> float:
        cb = _c_batch(x, fields, None)
        co = _native.PrlGrpoOutputs(*[rows[i].data_ptr() for i in range(8)], None, out.data_ptr(), stats.data_ptr())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _native.check(lib.prl_grpo_forward(ctypes.byref(cb), ctypes.byref(cp), ctypes.byref(co), ws.data_ptr(),
                                           ws.numel(), stream), "prl_grpo_forward")
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1)

    # correctness first: the aliased launch writes exactly the separate launch's dlogits
    launch(sep)
    ref_rows = rows.clone()
    launch(x)
    same = bool(torch.equal(sep, x)) and bool(torch.equal(rows, ref_rows))
    times = {"separate": [], "in_place": []}
    for r in range(rounds):
        for arm in (("separate", "in_place") if r % 2 == 0 else ("in_place", "separate")):
            t = []
            for _ in range(iters):
                x.copy_(master)
                torch.cuda.synchronize()
                t.append(launch(sep if arm == "separate" else x))
            times[arm].append(float(np.median(t)))
    gb = 2.0 * x.numel() * x.element_size() + 37.0 * a.tokens
    out = {"tool": "loss_inplace_ab", "tokens": a.tokens, "vocab": a.vocab, "bit_identical": same}
    for arm, v in times.items():
        ms = float(np.median(v))
        out[arm] = {"ms": round(ms, 4), "rounds_ms": [round(t, 4) for t in v], "frac": round(gb / ms / 1e6 / 8000.0, 4)}
    print(json.dumps(out), flush=True)


def offsets_ab(a, offsets: list[int], rounds: int = 3, iters: int = 10):
    """The bf16 loss head writing dlogits into one spare buffer at several byte offsets of its start
    (16-B aligned): does the placement of the write stream relative to the read stream (HBM
    channels / banks) change the rate?  Alternating rounds; the outputs must be bit-identical."""
    from pipelinerl_amd import _native
    from pipelinerl_amd.finetune.rl.fused import GrpoParams, _c_batch, _workspace

    dev = torch.device("cuda", 0)
    lib = _native.load()
    params = GrpoParams(policy_loss="ppo", epsilon=4.0, kl_coef=0.0, entropy_coef=0.0, clamp_log_ratio=5.0,
                        temperature=1.0, batch_size=4096.0)
    logits, fields = bench.make_workload(a.tokens, a.vocab, 2048, 256, 1234, dev)
    x = logits.detach()
    nbytes = x.numel() * x.element_size()
    spare = torch.empty(nbytes + max(offsets) + 16, dtype=torch.uint8, device=dev)
    B, L, V = x.shape
    rows = torch.empty((8, B * (L - 1)), dtype=torch.float32, device=dev)
    stats = torch.empty(_native.NSTAT, dtype=torch.float64, device=dev)
    ws = _workspace(dev)
    cp = params.to_c(True)
    stream = torch.cuda.current_stream(dev).cuda_stream
    assert all(o % 16 == 0 for o in offsets)

    def launch(off: int) -> float:
        cb = _c_batch(x, fields, None)
        co = _native.PrlGrpoOutputs(*[rows[i].data_ptr() for i in range(8)], None, spare.data_ptr() + off,
                                    stats.data_ptr())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _native.check(lib.prl_grpo_forward(ctypes.byref(cb), ctypes.byref(cp), ctypes.byref(co), ws.data_ptr(),
                                           ws.numel(), stream), "prl_grpo_forward")
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1)

    launch(offsets[0])
    ref = spare[offsets[0]:offsets[0] + nbytes].clone()
    same = True
    for o in offsets[1:]:
        launch(o)
        same &= bool(torch.equal(spare[o:o + nbytes], ref))
    del ref
    times = {o: [] for o in offsets}
    for r in range(rounds):
        for o in (offsets if r % 2 == 0 else offsets[::-1]):
            times[o].append(float(np.median([launch(o) for _ in range(iters)])))
    gb = 2.0 * nbytes + 37.0 * a.tokens
    out = {"tool": "loss_dl_offsets_ab", "tokens": a.tokens, "vocab": a.vocab, "bit_identical": same,
           "base_mod_2MiB": spare.data_ptr() % (2 << 20), "logits_mod_2MiB": x.data_ptr() % (2 << 20)}
    for o, v in times.items():
        ms = float(np.median(v))
        out[str(o)] = {"ms": round(ms, 4), "rounds_ms": [round(t, 4) for t in v], "frac": round(gb / ms / 1e6 / 8000.0, 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
