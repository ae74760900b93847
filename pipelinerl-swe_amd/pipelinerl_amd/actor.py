"""Actor-side receive of the trainer's weight broadcast (mirror of pipelinerl/vllm1.py:53-117).

``WorkerExtension`` is a mixin for an inference worker (vLLM's ``worker_extension_cls``) or any
object with: ``rank``, ``device``, ``model_runner.model.load_weights(weights=[(name, t)])`` and
``model_config.dtype``.  Methods, arguments and errors are the reference's:

  init_actor_update_group(actor_idx, actor_ngpus, weight_update_group_init_method,
                          weight_update_group_world_size)      -> joins the "actor" group as
                                                                  rank 1 + idx*ngpus + rank
  receive_weight_update(request)   -> receives every parameter, in parameters_info order:
      AssertionError on a dtype mismatch, ValueError if load_weights did not load exactly one.

Transport "bucketed" (both ends from this package) receives ~256 MiB chunks of the trainer's
flat bf16 snapshot into one staging buffer and loads each parameter from a view into it:
one receive per bucket instead of one receive + one allocation per tensor.

``python -m pipelinerl_amd.actor`` runs a small stand-alone actor (HTTP /health and
/receive_weight_update, a plain torch module as "model") used for integration tests and
broadcast benchmarks in place of a vLLM server.
"""

from __future__ import annotations

import argparse
import logging
import threading
import types
from typing import Any

import torch

from . import comm, torch_utils
from .weight_update import FlatLayout, WeightUpdateRequest

logger = logging.getLogger(__name__)


class WorkerExtension:
    actor_group_backend: str = "nccl"

    def init_actor_update_group(self, actor_idx: int, actor_ngpus: int, weight_update_group_init_method: str,
                                weight_update_group_world_size: int):
        self.pg_rank = 1 + actor_idx * actor_ngpus + self.rank
        logger.info(f"[INIT_ACTOR_UPDATE_GROUP]: actor {actor_idx}, ngpus {actor_ngpus}, rank {self.rank}, "
                    f"pg_rank {self.pg_rank}, init {weight_update_group_init_method}, "
                    f"world {weight_update_group_world_size}")
        if self.actor_group_backend == "prl_comm":  # RCCL communicator of the prl_comm C ABI
            from .comm import RcclComm

            self.process_group = RcclComm.create(weight_update_group_init_method, self.pg_rank,
                                                 weight_update_group_world_size, self.device)
            return
        self.process_group = torch_utils.init_extra_process_group(
            group_name="actor", backend=self.actor_group_backend, init_method=weight_update_group_init_method,
            rank=self.pg_rank, world_size=weight_update_group_world_size)

    def receive_weight_update(self, request: WeightUpdateRequest | dict):
        if isinstance(request, dict):
            request = WeightUpdateRequest(**request)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        logger.info("Start receiving weight update")
        model_dtype = self.model_config.dtype
        for info in request.parameters_info:
            assert info.dtype == str(model_dtype), f"mismatch dtype: src {info.dtype}, dst {model_dtype}"
        if getattr(request, "transport", "per_tensor") == "bucketed":
            self._receive_bucketed(request, model_dtype)
        else:
            for info in request.parameters_info:
                buf = torch.empty(tuple(info.shape), dtype=model_dtype, device=self.device)
                comm.broadcast(buf, self.process_group, src=0)
                self._load_one(info.name, buf)
        logger.info("Weight update received")

    def _receive_bucketed(self, request: WeightUpdateRequest, model_dtype: torch.dtype):
        layout = FlatLayout.from_infos(request.parameters_info)
        staging = getattr(self, "_staging", None)
        if staging is None or staging.numel() < layout.total or staging.device != self.device:
            staging = torch.empty(layout.total, dtype=torch.bfloat16, device=self.device)
            self._staging = staging
        flat = staging[:layout.total]
        elems = max(8, int(request.bucket_bytes) // 2)
        for a, b in layout.buckets(elems):
            comm.broadcast(flat[a:b], self.process_group, src=0)
        targets = self._direct_targets(layout)
        if targets is not None:  # parameters held directly: one HIP unflatten pass (32 tensors per launch)
            from .weight_update import HipFlatPacker

            HipFlatPacker().unflatten(flat, targets, layout.offsets)
            return
        for name, shape, n, off in zip(layout.names, layout.shapes, layout.numels, layout.offsets):
            self._load_one(name, flat[off:off + n].view(shape))

    def _direct_targets(self, layout) -> list[torch.Tensor] | None:
        """The destination tensors when the model holds every broadcast name as a plain
        contiguous bf16 parameter of the same shape on this HIP device (the standalone actor's
        ParamDictModel); None for models that remap names in load_weights (vLLM's fused qkv /
        gate_up, vllm1.py:89-93), which keep the per-name load."""
        params = getattr(self.model_runner.model, "params", None)
        if not isinstance(params, dict) or self.device.type != "cuda":
            return None
        out = []
        for name, shape in zip(layout.names, layout.shapes):
            p = params.get(name)
            if (p is None or p.dtype != torch.bfloat16 or tuple(p.shape) != tuple(shape) or not p.is_contiguous()
                    or p.device != self.device or p.data_ptr() % 16):
                return None
            out.append(p.detach())  # shares the version counter: the unflatten moves it
        return out

    def _load_one(self, name: str, tensor: torch.Tensor):
        loaded = self.model_runner.model.load_weights(weights=[(name, tensor)])
        if len(loaded) != 1:
            raise ValueError(f"model {name} not found in model state dict")


class ParamDictModel:
    """A minimal 'inference model': named parameters + load_weights(name -> copy)."""

    def __init__(self, module: torch.nn.Module):
        self.module = module
        self.params = dict(module.named_parameters())

    def load_weights(self, weights):
        loaded = set()
        for name, t in weights:
            p = self.params.get(name)
            if p is None:
                continue
            with torch.no_grad():
                p.copy_(t.to(p.dtype))
            loaded.add(name)
        return loaded


class StandaloneWorker(WorkerExtension):
    def __init__(self, module: torch.nn.Module, rank: int = 0, device: str | torch.device = "cpu",
                 backend: str = "nccl"):
        self.rank = rank
        self.device = torch.device(device)
        self.actor_group_backend = backend
        module.to(self.device)
        self.model_runner = types.SimpleNamespace(model=ParamDictModel(module))
        self.model_config = types.SimpleNamespace(dtype=next(module.parameters()).dtype)


def build_app(worker: StandaloneWorker):
    from fastapi import FastAPI

    app = FastAPI()
    lock = threading.Lock()

    @app.get("/health")
    def health() -> dict:
        return {"status": "ok"}

    @app.post("/receive_weight_update")
    def receive(request: dict[str, Any]) -> dict:
        with lock:  # one update at a time, like vLLM's collective_rpc
            worker.receive_weight_update(WeightUpdateRequest(**request))
        return {"status": "ok"}

    @app.get("/checksum")
    def checksum() -> dict:
        with lock:
            return {n: float(p.detach().double().sum()) for n, p in worker.model_runner.model.params.items()}

    return app


def main(argv=None):
    ap = argparse.ArgumentParser(description="stand-alone actor receiving PipelineRL weight updates")
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--actor-llm-idx", type=int, default=0)
    ap.add_argument("--weight-update-group-init-method", type=str, required=True)
    ap.add_argument("--weight-update-group-world-size", type=int, required=True)
    ap.add_argument("--disable-weight-updates", action="store_true")
    ap.add_argument("--backend", default="nccl")
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--model-config", required=True, help="HF config dir/json of the model to hold")
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    from transformers import AutoConfig, AutoModelForCausalLM

    cfg = AutoConfig.from_pretrained(args.model_config)
    module = AutoModelForCausalLM.from_config(cfg, torch_dtype=torch.bfloat16)
    worker = StandaloneWorker(module, rank=0, device=args.device, backend=args.backend)
    app = build_app(worker)
    if not args.disable_weight_updates:
        t = threading.Thread(target=worker.init_actor_update_group,
                             args=(args.actor_llm_idx, 1, args.weight_update_group_init_method,
                                   args.weight_update_group_world_size), daemon=True)
        t.start()  # the rendezvous completes when the trainer joins
    import uvicorn

    uvicorn.run(app, host=args.host, port=args.port, log_level="warning")


if __name__ == "__main__":
    main()
