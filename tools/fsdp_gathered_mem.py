"""Where FSDP2's memory goes with decoder layers kept gathered (finetune.fsdp_keep_gathered_layers):
two ranks share cuda:0 through gloo (as tests/test_fsdp_gathered_gpu.py), Qwen2.5-32B layer shapes
with 4 decoder layers, one packed 4 096-token rl_step; for each R the device's allocated bytes after
every decoder layer's forward and backward and the step's peak.

    python tools/fsdp_gathered_mem.py [--keep 0 1 2 4] [--out gpurun_out/fsdp_gathered_mem.json]
"""

from __future__ import annotations

import argparse
import gc
import json
import os
import sys
from pathlib import Path

import torch
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
T, SEQ, PROMPT, LAYERS = 4096, 1024, 128, 4


def _run(rank: int, port: int, keeps: list[int], out_path: str):
    sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd"), str(ROOT / "tests")]
    os.environ["OMP_NUM_THREADS"] = "4"
    import torch.distributed as dist

    from pipelinerl_amd.finetune.rl import rl_step
    from pipelinerl_amd.finetune.sharding import decoder_layers, shard_model
    from pipelinerl_amd.trainer_probe import QWEN, packed_batch, qwen2_model, rl_config

    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    dist.init_process_group("cpu:gloo,cuda:gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    batch = packed_batch(T, SEQ, PROMPT, QWEN["32b"]["vocab_size"], dev, seed=100 + rank, ref_noise=True)
    cfg = rl_config(2 * (T // SEQ), kl_coef=0.001)
    res = {}
    for R in keeps:
        model = shard_model(qwen2_model("32b", dev, layers=LAYERS), keep_gathered=R)
        trace = []

        def mark(what):
            torch.cuda.synchronize()
            trace.append((what, round(torch.cuda.memory_allocated(dev) / 1e9, 3),
                          round(torch.cuda.max_memory_allocated(dev) / 1e9, 3)))

        for i, layer in enumerate(decoder_layers(model)):
            layer.register_forward_hook(lambda m, a, o, i=i: mark(f"fwd {i}"))
            layer.register_full_backward_hook(lambda m, gi, go, i=i: mark(f"bwd {i}"))
        for it in range(2):
            trace.clear()
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            torch.cuda.reset_peak_memory_stats(dev)
            mark("start")
            loss, stats = rl_step(model, batch, 0, 10, cfg, defer_stats=True)
            mark("loss")
            loss.backward()
            stats.resolve()
            mark("end")
            for p in model.parameters():
                p.grad = None
            del loss, stats  # the graph's AccumulateGrad nodes hold the parameters
        res[str(R)] = {"trace": list(trace), "peak_gb": round(torch.cuda.max_memory_allocated(dev) / 1e9, 3),
                       "memory_stats": {k: v for k, v in torch.cuda.memory_stats(dev).items()
                                        if k in ("num_alloc_retries", "num_device_alloc")}}
        del model, layer  # (the hook loop's last layer holds the FSDP tree too)
        gc.collect()  # FSDP's module <-> state cycles: else the previous model stays on the device
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    if rank == 0:
        Path(out_path).parent.mkdir(parents=True, exist_ok=True)
        Path(out_path).write_text(json.dumps(res, indent=1))
        print(json.dumps({R: (v["peak_gb"], v["trace"]) for R, v in res.items()}, indent=0))
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keep", type=int, nargs="+", default=[0, 1, 2, 4])
    ap.add_argument("--out", default="gpurun_out/fsdp_gathered_mem.json")
    a = ap.parse_args()
    sys.path[:0] = [str(ROOT / "tests")]
    from test_weight_update_cpu import free_port

    mp.spawn(_run, args=(free_port(), a.keep, a.out), nprocs=2, join=True)


if __name__ == "__main__":
    main()
