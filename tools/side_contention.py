"""How much a side-stream kernel holding a few CUs slows the trainer step's own kernels (the
zero-copy weight broadcast's cost: its channels are workgroups that stay resident for the whole
transfer).  Each kernel under test is timed alone, then beside prl_paced_read on a side stream in
three forms: reading at one xGMI link's rate (153 GB/s, the emulated broadcast), nearly asleep
(0.01 GB/s: the same resident workgroups, almost no memory traffic) and ONE asleep workgroup, so CU
occupancy and memory contention separate.

    python tools/side_contention.py [--blocks 16] [--reps 30]

Kernels: the 7B gate/up GEMMs through libprl_gemm (forward, input and weight gradient) and
torch.matmul, the HIP attention forward at C3-like packing (7B heads 28 / 4, D 128; 12 000 tokens in
three sequences), the fused residual-add RMSNorm (12 000 x 3584) and, as a control, torch's copy of
the same bytes.  Prints one JSON line."""

from __future__ import annotations

import argparse
import ctypes
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pipelinerl-swe_amd"))

from pipelinerl_amd import _native  # noqa: E402
from pipelinerl_amd.finetune.attention import PackedCausalAttention  # noqa: E402
from pipelinerl_amd import gemm as prl_gemm  # noqa: E402
from pipelinerl_amd.finetune.model_ops import AddRMSNormFn  # noqa: E402


def med_ms(fn, reps: int) -> float:
    evs = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        evs.append((a, b))
    torch.cuda.current_stream().synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in evs)
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=16)
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = _native.load()
    g = torch.Generator(device=dev).manual_seed(0)
    T, H, HKV, D = 12000, 28, 4, 128
    lens = [5000, 4000, 3000]
    bounds = [sum(lens[:i]) for i in range(len(lens) + 1)]
    q = torch.randn((T, H, D), generator=g, device=dev).to(torch.bfloat16)
    k = torch.randn((T, HKV, D), generator=g, device=dev).to(torch.bfloat16)
    v = torch.randn((T, HKV, D), generator=g, device=dev).to(torch.bfloat16)
    cu = torch.tensor(bounds, dtype=torch.int32, device=dev)
    x = torch.randn((T, 3584), generator=g, device=dev).to(torch.bfloat16)
    r = torch.randn((T, 3584), generator=g, device=dev).to(torch.bfloat16)
    w = torch.ones(3584, device=dev, dtype=torch.bfloat16)
    big = torch.empty(2 * T * 3584, dtype=torch.bfloat16, device=dev)
    dst = torch.empty_like(big)
    # the 7B MLP's gate/up and down GEMMs at 12 000 tokens: forward, input and weight gradient
    wgu = torch.randn((2 * 18944, 3584), generator=g, device=dev).to(torch.bfloat16) * 0.02
    dy = torch.randn((T, 2 * 18944), generator=g, device=dev).to(torch.bfloat16)
    # the fused loss head on a C2-shaped micro-batch slice (8192 x 151936 bf16 logits; persistent
    # grid of one 1024-thread workgroup per CU)
    from pipelinerl_amd.finetune.rl.fused import GrpoParams, grpo_loss
    sys.path.insert(0, str(ROOT))
    from bench import make_workload

    lg, fields = make_workload(8192, 151936, seq=2048, prompt=256, seed=0, device=dev)
    params = GrpoParams(policy_loss="ppo", epsilon=4.0, kl_coef=0.0, entropy_coef=0.0, clamp_log_ratio=5.0,
                        temperature=1.0, batch_size=4096.0)
    lg.requires_grad_(True)
    sg, su = (torch.randn((65536, 8960), generator=g, device=dev).to(torch.bfloat16) for _ in range(2))
    sh, sdg, sdu = torch.empty_like(sg), torch.empty_like(sg), torch.empty_like(sg)
    ctr = torch.zeros(4, dtype=torch.int32, device=dev)  # the SwiGLU chunk counter (caller-owned)
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    kernels = {
        "loss_head_fwd_8192_rows": lambda: grpo_loss(lg, fields, params),
        # the phased SwiGLU kernels (one 1024-thread workgroup per CU) at the 1.5B step's C2 shape,
        # chunks claimed from the counter and with the static stride (no counter)
        "swiglu_fwd_65536x8960": lambda: lib.prl_swiglu_forward(sg.data_ptr(), su.data_ptr(), sh.data_ptr(),
                                                                sg.numel(), ctr.data_ptr(), st()),
        "swiglu_fwd_65536x8960_static": lambda: lib.prl_swiglu_forward(sg.data_ptr(), su.data_ptr(), sh.data_ptr(),
                                                                       sg.numel(), None, st()),
        "swiglu_bwd_65536x8960": lambda: lib.prl_swiglu_backward(sh.data_ptr(), sg.data_ptr(), su.data_ptr(),
                                                                 sdg.data_ptr(), sdu.data_ptr(), sg.numel(),
                                                                 ctr.data_ptr(), st()),
        "swiglu_bwd_65536x8960_static": lambda: lib.prl_swiglu_backward(sh.data_ptr(), sg.data_ptr(), su.data_ptr(),
                                                                        sdg.data_ptr(), sdu.data_ptr(), sg.numel(),
                                                                        None, st()),
        "gemm_fwd_gate_up": lambda: prl_gemm.linear_fwd(x, wgu),
        "gemm_dgrad_gate_up": lambda: prl_gemm.linear_dgrad(dy, wgu),
        "gemm_wgrad_gate_up": lambda: prl_gemm.linear_wgrad(dy, x),
        "torch_matmul_gate_up": lambda: torch.matmul(x, wgu.t()),
        "attn_fwd": lambda: PackedCausalAttention.apply(q, k, v, cu, max(lens), bounds),
        "add_rmsnorm_fwd": lambda: AddRMSNormFn.apply(r, x, w, 1e-6),
        "torch_copy_same_bytes": lambda: dst.copy_(big),
    }
    src = torch.empty(16 << 30, dtype=torch.uint8, device=dev)  # what the side kernel reads
    sink = torch.zeros(4096, dtype=torch.int32, device=dev)
    side = torch.cuda.Stream(device=dev)
    out = {"blocks": a.blocks, "reps": a.reps, "ms": {}}
    with torch.no_grad():
        for name, fn in kernels.items():
            for _ in range(3):
                fn()
            alone = med_ms(fn, a.reps)
            row = {"alone": round(alone, 4)}
            span_s = 3 * a.reps * alone / 1e3 + 0.05  # the side kernel outlasts the timed loop
            for arm, gbps, blocks in (("reading_153GBps", 153.0, a.blocks), ("asleep", 0.01, a.blocks),
                                      ("asleep_1wg", 0.01, 1)):
                nbytes = min(src.numel(), max(blocks * 65536, int(gbps * 1e9 * span_s)))
                if gbps < 1:  # two turns per workgroup, the second one due after span_s
                    nbytes = 2 * blocks * 65536
                    gbps_eff = nbytes / span_s / 1e9
                else:
                    gbps_eff = gbps
                torch.cuda.synchronize()
                with torch.cuda.stream(side):
                    _native.check(lib.prl_paced_read(ctypes.c_void_p(src.data_ptr()), nbytes, gbps_eff, blocks,
                                                     ctypes.c_void_p(sink.data_ptr()), side.cuda_stream),
                                  "prl_paced_read")
                torch.cuda._sleep(2_000_000)  # ~1 ms: the side kernel's workgroups are resident first
                row[arm] = round(med_ms(fn, a.reps), 4)
                torch.cuda.synchronize()
            row["ratio_reading"] = round(row["reading_153GBps"] / alone, 3)
            row["ratio_asleep"] = round(row["asleep"] / alone, 3)
            row["ratio_asleep_1wg"] = round(row["asleep_1wg"] / alone, 3)
            out["ms"][name] = row
    print(json.dumps(out))


if __name__ == "__main__":
    main()
