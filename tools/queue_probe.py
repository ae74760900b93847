"""Which hardware queue each of a trainer rank's streams lands on (VERDICT r05 "what's weak" 4).

Rank 0 of the split pipeline (C4) runs kernels from five streams: the compute stream, GradBuckets'
stream (finetune/grad_sync.py), the weight update's side stream (weight_update.py), and the two
process groups' own collective streams (ProcessGroupNCCL draws them from torch's stream pool:
high-priority pool streams with ``is_high_priority_stream``, torch_utils.collective_options, else
normal ones).  Kernels in one hardware queue run in order, so a collective stream that shares the
compute stream's queue would serialise behind the trainer's GEMMs instead of overlapping them.

This builds that stream set on one GPU in the trainer's creation order, runs C3-shaped GEMMs (7B
MLP up-projection, 12 000 rows) on the compute stream, and ``prl_paced_read`` (the reads an RCCL
kernel makes, paced to an xGMI link) on every other stream, each role with its own workgroup count
so the kernel trace tells them apart; plus real RCCL collectives on one-rank process groups created
as the trainer creates them.  ``--summarize DIR`` reads rocprofv3's kernel trace (Queue_Id column)
and writes, per role, the queues its kernels ran on.

    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/queue_probe.py
    python tools/queue_probe.py --summarize DIR > profiles/r06_queue_probe.json
"""

from __future__ import annotations

import argparse
import csv
import ctypes
import glob
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]

# role -> paced-read workgroups (the grid tells the roles apart in the trace)
ROLES = {"grad_buckets": 8, "wu_side": 12, "dp_collective": 20, "actor_collective": 28,
         "pool_normal_a": 36, "pool_normal_b": 44}


def run(iters: int) -> None:
    import torch
    import torch.distributed as dist

    from pipelinerl_amd import _native
    from pipelinerl_amd.torch_utils import collective_options, init_extra_process_group
    from pipelinerl_amd.weight_update import side_stream_priority

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    opts = collective_options("nccl")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev, pg_options=opts)  # the DP group
    actor = init_extra_process_group(backend="nccl", init_method="tcp://127.0.0.1:29562", rank=0, world_size=1,
                                     group_name="actor", pg_options=opts)
    compute = torch.cuda.current_stream(dev)
    from pipelinerl_amd.finetune.grad_sync import GradBuckets

    gb = GradBuckets([torch.nn.Parameter(torch.zeros(1 << 20, device=dev))])  # its own stream, as the trainer's
    streams = {  # the trainer's creation order: GradBuckets at set-up, the groups' streams at their
        # first collective, the weight update's side stream at the first update
        "grad_buckets": gb.stream,
        "dp_collective": torch.cuda.Stream(device=dev, priority=-1 if opts is not None else 0),
        "actor_collective": torch.cuda.Stream(device=dev, priority=-1 if opts is not None else 0),
        "wu_side": torch.cuda.Stream(device=dev, priority=side_stream_priority()),
        # two more normal-priority pool streams (what the collectives would get without the option)
        "pool_normal_a": torch.cuda.Stream(device=dev),
        "pool_normal_b": torch.cuda.Stream(device=dev),
    }
    lib = _native.load()
    buf = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
    sink = torch.zeros(64, dtype=torch.int32, device=dev)
    x = torch.randn(12000, 3584, dtype=torch.bfloat16, device=dev)
    w = torch.randn(3584, 18944, dtype=torch.bfloat16, device=dev)
    t = torch.ones(1 << 20, device=dev)
    for it in range(iters):
        for role, s in streams.items():
            s.wait_stream(compute)
            with torch.cuda.stream(s):
                _native.check(lib.prl_paced_read(ctypes.c_void_p(buf.data_ptr()), 64 << 20, 153.0, ROLES[role],
                                                 ctypes.c_void_p(sink.data_ptr()), s.cuda_stream), "prl_paced_read")
        for _ in range(8):
            torch.mm(x, w)
        # real RCCL calls issued as the trainer issues them (one rank: RCCL's one-rank kernels): the
        # bucket all-reduce async from GradBuckets' stream, the broadcast async from the side stream
        gb.stream.wait_stream(compute)
        with torch.cuda.stream(gb.stream):
            w1 = dist.all_reduce(t, op=dist.ReduceOp.AVG, async_op=True)
        streams["wu_side"].wait_stream(compute)
        with torch.cuda.stream(streams["wu_side"]):
            w2 = dist.broadcast(t, 0, group=actor, async_op=True)
        w1.wait()
        w2.wait()
    torch.cuda.synchronize()
    print(json.dumps({"iters": iters, "high_priority_collectives": opts is not None,
                      "wu_side_priority": side_stream_priority(),
                      "stream_priorities": {k: s.priority for k, s in streams.items()},
                      "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "unset (HIP default 4)")}))
    dist.destroy_process_group(actor)
    dist.destroy_process_group()


def summarize(d: str) -> dict:
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel_trace.csv under {d}")
    by_role: dict[str, set] = {}
    names: dict[str, set] = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                q = row.get("Queue_Id")
                grid = int(row.get("Grid_Size_X", row.get("Grid_Size", "0")) or 0)
                wg = int(row.get("Workgroup_Size_X", row.get("Workgroup_Size", "1")) or 1)
                if "paced_read" in name:
                    blocks = grid // max(1, wg)
                    role = next((r for r, b in ROLES.items() if b == blocks), f"paced_{blocks}")
                elif "Cijk" in name or "gemm" in name.lower() or "mm" in name.lower():
                    role = "compute"
                elif "nccl" in name.lower() or "rccl" in name.lower() or "onerank" in name.lower():
                    role = "rccl"
                else:
                    role = "other"
                by_role.setdefault(role, set()).add(q)
                names.setdefault(role, set()).add(name[:80])
    compute = by_role.get("compute", set())
    out = {"queues": {r: sorted(v) for r, v in sorted(by_role.items())},
           "kernel_names": {r: sorted(v)[:4] for r, v in sorted(names.items())},
           "shares_compute_queue": {r: bool(v & compute) for r, v in sorted(by_role.items()) if r != "compute"}}
    out["collective_streams_off_compute_queue"] = not any(
        out["shares_compute_queue"].get(r, False)
        for r in ("grad_buckets", "dp_collective", "actor_collective", "wu_side", "rccl"))
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--summarize", default=None)
    a = ap.parse_args()
    if a.summarize:
        print(json.dumps(summarize(a.summarize), indent=1))
    else:
        run(a.iters)
