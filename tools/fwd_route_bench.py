"""Forward-GEMM routing check for C3's 7B layer shapes at the packed micro-batch sizes C3 actually
produces (4 096 - 12 000 tokens): torch's F.linear (torch's bundled hipBLASLt) vs prl_gemm with the
ROCm 7.2 library heuristic (solution -1) vs whatever gemm_solutions.json routes (the product path).
Events bracket 30 back-to-back launches on random operands; one JSON line per (shape, T).

    python tools/fwd_route_bench.py [T ...]
"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "pipelinerl-swe_amd"))
from pipelinerl_amd import gemm  # noqa: E402

H, I, KV = 3584, 18944, 512
SHAPES = {"q_proj": (H, H, True), "o_proj": (H, H, False), "k/v_proj": (H, KV, True),
          "down_proj": (I, H, False), "gate_up_fused": (H, 2 * I, False)}


def timed(fn, reps=30):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    Ts = [int(a) for a in sys.argv[1:]] or [4096, 5120, 6144, 7168, 8000, 9216, 12000]
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, (K, N, has_bias) in SHAPES.items():
        w = torch.randn((N, K), generator=g, device="cuda").to(torch.bfloat16)
        b = torch.randn((N,), generator=g, device="cuda").to(torch.bfloat16) if has_bias else None
        for T in Ts:
            x = torch.randn((T, K), generator=g, device="cuda").to(torch.bfloat16)
            routed = gemm.solution_for("fwd", T, N, K)
            ref = torch.nn.functional.linear(x, w, b)
            heur = gemm.linear_fwd(x, w, b, solution=-1)
            err = float((heur.float() - ref.float()).abs().max() / ref.float().abs().max())
            t_torch = timed(lambda: torch.nn.functional.linear(x, w, b))
            t_heur = timed(lambda: gemm.linear_fwd(x, w, b, solution=-1))
            rec = {"layer": name, "T": T, "N": N, "K": K, "bias": has_bias, "torch_ms": round(t_torch, 4),
                   "prl_heuristic_ms": round(t_heur, 4), "routed": routed, "rel_err_vs_torch": err}
            if routed is not None and routed >= 0:
                rec["prl_routed_ms"] = round(timed(lambda: gemm.linear_fwd(x, w, b, solution=routed)), 4)
            print(json.dumps(rec), flush=True)
            del x, ref, heur
        del w, b
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
