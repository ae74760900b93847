"""Census of the ATen ops one trainer micro-batch step dispatches (forward + loss head + backward)
on a Qwen2.5-shaped model with the build's patches: op name x output shape -> count, and for
copies / cats / adds the Python stack frame that issued them (measurement tool, one GPU).

    python tools/op_census.py --model 1.5b --layers 2 --tokens 8192
"""

from __future__ import annotations

import argparse
import collections
import json
import sys
import traceback
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

WATCH = ("copy", "cat", "add", "fill", "zero", "clone", "contiguous", "_to_copy", "sum", "mul")


class Census(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.ops = collections.Counter()
        self.sites = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = str(func.overloadpacket.__name__)
        shape = tuple(out.shape) if isinstance(out, torch.Tensor) else None
        self.ops[(name, shape)] += 1
        if any(w in name for w in WATCH) and isinstance(out, torch.Tensor) and out.numel() >= 1 << 20:
            frames = [f for f in traceback.extract_stack()[:-1] if "torch/" not in f.filename
                      or "nn/modules" in f.filename]
            site = " <- ".join(f"{Path(f.filename).name}:{f.lineno}:{f.name}" for f in frames[-3:])
            self.sites[(name, shape, site)] += 1
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="1.5b")
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--tokens", type=int, default=8192)
    a = ap.parse_args()
    from pipelinerl_amd import trainer_probe
    from pipelinerl_amd.finetune.rl import rl_step

    trainer_probe.QWEN[a.model] = dict(trainer_probe.QWEN[a.model], num_hidden_layers=a.layers)
    dev = torch.device("cuda", 0)
    model = trainer_probe.qwen2_model(a.model, dev)
    batch = trainer_probe.packed_batch(a.tokens, 2048, 256, trainer_probe.QWEN[a.model]["vocab_size"], dev)
    cfg = trainer_probe.rl_config(a.tokens // 2048, fused_head=True)
    loss, _ = rl_step(model, batch, 0, 100, cfg)  # warm-up outside the census
    loss.backward()
    model.zero_grad(set_to_none=True)
    c = Census()
    with c:
        loss, _ = rl_step(model, batch, 0, 100, cfg)
        loss.backward()
    torch.cuda.synchronize()
    for (name, shape), n in sorted(c.ops.items(), key=lambda kv: -kv[1]):
        print(json.dumps({"op": name, "shape": shape, "count": n}))
    for (name, shape, site), n in sorted(c.sites.items(), key=lambda kv: -kv[1]):
        print(json.dumps({"watch": name, "shape": shape, "count": n, "site": site}))


if __name__ == "__main__":
    main()
