"""BASELINE configs[4] (C5) probe outside bench.py: Qwen2.5-32B shapes under FSDP2 with KL on
(trainer_probe.fsdp_step_probe).  One rank per GPU (torchrun); on a one-GPU box it rehearses the
path with an RCCL group of one and fewer layers (the full 32B needs the 8-GPU node).

    python tools/fsdp_probe.py --layers 8 --tokens 4096
"""

import argparse
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="32b")
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--tokens", type=int, default=4096)
    ap.add_argument("--micro-batches", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    a = ap.parse_args()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group("nccl", device_id=dev)
    from pipelinerl_amd.trainer_probe import fsdp_step_probe

    r = fsdp_step_probe(a.model, tokens=a.tokens, micro_batches=a.micro_batches, steps=a.steps, warmup=a.warmup,
                        device=dev, layers=a.layers)
    if dist.get_rank() == 0:
        print(json.dumps(r), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
