"""Actor-side receive of the trainer's weight broadcast (mirror of pipelinerl/vllm1.py:53-117 and
pipelinerl/vllm0.py:51-104).

``WorkerExtension`` is a mixin for an inference worker (vLLM v1's ``worker_extension_cls``) or any
object with: ``rank``, ``device``, ``model_runner.model.load_weights(weights=[(name, t)])`` and
``model_config.dtype``.  vLLM v0 — the reference's default actor (conf/base.yaml ``use_v1: false``,
launch.py:130-131) — registers a Worker SUBCLASS instead (``parallel_config.worker_cls``,
vllm0.py:204-206): ``make_worker_class(multi_step)`` builds it over vLLM's ``Worker`` /
``MultiStepWorker`` with the same methods, and ``AsyncRLWorker`` / ``AsyncRLMultiStepWorker`` are
the two classes the reference registers by name.  Methods, arguments and errors are the reference's:

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
        self._apply_flat(flat, layout)

    def _apply_flat(self, flat: torch.Tensor, layout) -> None:
        """Load every parameter of a received flat buffer: one HIP unflatten pass straight into the
        model's storage when it resolves every name to a writable bf16 region (32 tensors per
        launch; for a fused-layout model the q / k / v and gate / up regions are row blocks of its
        qkv_proj / gate_up_proj), else the per-name load_weights path (vllm1.py:89-93)."""
        targets = self._direct_targets(layout)
        if targets is not None:
            from .weight_update import HipFlatPacker

            HipFlatPacker().unflatten(flat, targets, layout.offsets)
            return
        for name, shape, n, off in zip(layout.names, layout.shapes, layout.numels, layout.offsets):
            self._load_one(name, flat[off:off + n].view(shape))

    def _inference_model(self):
        """The model loads go to (vllm1.py:89-93: the runner's model)."""
        return self.model_runner.model

    def _direct_targets(self, layout) -> list[torch.Tensor] | None:
        """The destination region of every broadcast name, from the model's direct_target(name,
        shape) (ParamDictModel: the parameter; StackedParamsModel: a row block of a fused
        parameter), when each is a contiguous, 16-B aligned bf16 tensor on this HIP device; None
        otherwise (models without direct_target keep the per-name load)."""
        resolve = getattr(self._inference_model(), "direct_target", None)
        if resolve is None or self.device.type != "cuda":
            return None
        out = []
        for name, shape in zip(layout.names, layout.shapes):
            t = resolve(name, tuple(shape))
            if (t is None or t.dtype != torch.bfloat16 or not t.is_contiguous() or t.device != self.device
                    or t.data_ptr() % 16):
                if not getattr(self, "_warned_per_name", False):  # a slower path: say so, once
                    self._warned_per_name = True
                    why = ("no destination" if t is None else f"dtype {t.dtype}, contiguous {t.is_contiguous()}, "
                           f"device {t.device} (this worker: {self.device}), 16-B aligned {t.data_ptr() % 16 == 0}")
                    logger.warning(f"weight updates load per name (load_weights), not by one HIP unflatten: "
                                   f"{name} {tuple(shape)}: {why}")
                return None
            out.append(t)  # views share the parameter's version counter: the unflatten moves it
        return out

    def _load_one(self, name: str, tensor: torch.Tensor):
        loaded = self._inference_model().load_weights(weights=[(name, tensor)])
        if len(loaded) != 1:
            raise ValueError(f"model {name} not found in model state dict")


# ------------------------------------------------------------------------------------------
# vLLM v0 (vllm0.py:51-104): a Worker subclass registered through parallel_config.worker_cls

def is_multi_step_runner(runner) -> bool:
    """vllm0.py:90 ``isinstance(self.model_runner, MultiStepModelRunner)``; without vLLM importable
    (tests, stand-ins) a class of that name anywhere in the runner's MRO."""
    try:
        from vllm.worker.multi_step_model_runner import MultiStepModelRunner
    except ImportError:
        return any(c.__name__ == "MultiStepModelRunner" for c in type(runner).__mro__)
    return isinstance(runner, MultiStepModelRunner)


class V0WorkerMixin(WorkerExtension):
    """The receive side of vllm0.py's worker class: the v1 extension's methods (per_tensor /
    bucketed transports, the HIP unflatten into direct targets), with the model taken where the v0
    runner keeps it — a MultiStepModelRunner wraps the real runner and loads go to
    ``model_runner._base_model_runner.model`` (vllm0.py:90-95)."""

    actor_group_backend = "nccl"  # vllm0.py:75

    def _inference_model(self):
        runner = self.model_runner
        if is_multi_step_runner(runner):
            return runner._base_model_runner.model
        return runner.model


def _vllm_v0_worker_base(multi_step: bool) -> type:
    """vllm0.py:26,32,52: vLLM v0's Worker or MultiStepWorker."""
    try:
        if multi_step:
            from vllm.worker.multi_step_worker import MultiStepWorker as base
        else:
            from vllm.worker.worker import Worker as base
    except ImportError as e:
        raise ImportError("the vLLM v0 worker classes need vLLM (vllm.worker.worker / vllm.worker.multi_step_worker); "
                          "pass base_class= to make_worker_class for another engine's worker") from e
    return base


def make_worker_class(multi_step: bool, base_class: type | None = None) -> type:
    """vllm0.py:51-100: a class deriving from vLLM v0's ``MultiStepWorker`` (``multi_step``) or
    ``Worker`` — or ``base_class`` — with ``init_actor_update_group`` / ``receive_weight_update``.
    The mixin comes first in the MRO, so the base worker's own methods are untouched."""
    base = base_class if base_class is not None else _vllm_v0_worker_base(multi_step)
    name = "AsyncRLMultiStepWorker" if multi_step else "AsyncRLWorker"
    return type(name, (V0WorkerMixin, base), {"__module__": __name__, "__qualname__": name})


_V0_CLASSES: dict[str, type] = {}


def __getattr__(name: str):
    """``AsyncRLWorker`` / ``AsyncRLMultiStepWorker`` (vllm0.py:103-104), built on first access so
    this module imports without vLLM; vLLM resolves ``worker_cls`` by qualified name, which lands
    here.  One class per process, so the reference's isinstance checks (vllm0.py:127) hold."""
    if name in ("AsyncRLWorker", "AsyncRLMultiStepWorker"):
        if name not in _V0_CLASSES:
            _V0_CLASSES[name] = make_worker_class(multi_step=name == "AsyncRLMultiStepWorker")
        return _V0_CLASSES[name]
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")


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

    def direct_target(self, name: str, shape: tuple) -> torch.Tensor | None:
        p = self.params.get(name)
        return p.detach() if p is not None and tuple(p.shape) == shape else None


# vLLM's fused projections (vllm/model_executor/models/qwen2.py, vLLM 0.8.5, Qwen2Model.load_weights:
# stacked_params_mapping, applied by the reference actor's load_weights call, vllm1.py:89-93): the
# trainer's q / k / v projections are row blocks of one qkv_proj (QKVParallelLinear shard ids "q",
# "k", "v"), gate / up of one gate_up_proj (MergedColumnParallelLinear shards 0, 1), in that order;
# at tensor parallel 1 a shard's rows are contiguous.  vLLM is not importable here: the layout and the
# loader are restated from its source, and the trainer-side names are pinned by F4.
STACKED_PARAMS = (("qkv_proj", "q_proj", "q"), ("qkv_proj", "k_proj", "k"), ("qkv_proj", "v_proj", "v"),
                  ("gate_up_proj", "gate_proj", 0), ("gate_up_proj", "up_proj", 1))
_SHARD_ORDER = {"q": 0, "k": 1, "v": 2, 0: 0, 1: 1}


def fused_direct_target(params: dict[str, torch.Tensor], config):
    """direct_target(name, shape) over a model already in vLLM's fused layout (its named_parameters
    and its HF config): the trainer's q / k / v or gate / up name -> that shard's row block of the
    fused parameter (QKVParallelLinear / MergedColumnParallelLinear row offsets at tensor parallel 1),
    any other name -> the parameter of that name; None when the shape differs or the name is unknown."""
    hd = getattr(config, "head_dim", None) or config.hidden_size // config.num_attention_heads
    rows = {"q": config.num_attention_heads * hd, "k": config.num_key_value_heads * hd,
            "v": config.num_key_value_heads * hd, 0: config.intermediate_size, 1: config.intermediate_size}

    def direct_target(name: str, shape: tuple) -> torch.Tensor | None:
        for fused, part, shard in STACKED_PARAMS:
            if f".{part}." in name:
                p = params.get(name.replace(f".{part}.", f".{fused}."))
                if p is None:
                    return None
                r0 = sum(rows[s] for f, _, s in STACKED_PARAMS if f == fused and _SHARD_ORDER[s] < _SHARD_ORDER[shard])
                t = p.detach()[r0:r0 + rows[shard]]
                return t if tuple(t.shape) == shape else None
        p = params.get(name)
        return p.detach() if p is not None and tuple(p.shape) == shape else None

    return direct_target


class StackedParamsModel:
    """An inference model in vLLM's fused parameter layout, built from a trainer-layout module:
    load_weights(name -> copy into the shard's rows, returns the fused names loaded) as vLLM's
    Qwen2 model does, and direct_target(name, shape) -> the shard's row block, so the bucketed
    receive unflattens straight into qkv_proj / gate_up_proj with no per-name copy."""

    def __init__(self, module: torch.nn.Module):
        self.params: dict[str, torch.Tensor] = {}
        self.shards: dict[str, tuple[str, int, int]] = {}  # trainer name -> (fused name, first row, rows)
        groups: dict[str, list] = {}
        for name, p in module.named_parameters():
            for fused, part, shard in STACKED_PARAMS:
                if f".{part}." in name:
                    groups.setdefault(name.replace(f".{part}.", f".{fused}."), []).append((shard, name, p))
                    break
            else:
                self.params[name] = p.detach()
        for fname, members in groups.items():
            members.sort(key=lambda m: _SHARD_ORDER[m[0]])
            self.params[fname] = torch.cat([p.detach() for _, _, p in members], dim=0).contiguous()
            row = 0
            for _, name, p in members:
                self.shards[name] = (fname, row, p.shape[0])
                row += p.shape[0]

    def _region(self, name: str) -> torch.Tensor | None:
        if name in self.shards:
            fname, r0, n = self.shards[name]
            return self.params[fname][r0:r0 + n]
        return self.params.get(name)

    def load_weights(self, weights):
        loaded = set()
        for name, t in weights:
            if "rotary_emb.inv_freq" in name:
                continue
            dst = self._region(name)
            if dst is None or tuple(dst.shape) != tuple(t.shape):
                continue
            with torch.no_grad():
                dst.copy_(t.to(dst.dtype))
            loaded.add(self.shards[name][0] if name in self.shards else name)
        return loaded

    def direct_target(self, name: str, shape: tuple) -> torch.Tensor | None:
        t = self._region(name)
        return t if t is not None and tuple(t.shape) == shape else None


class StandaloneWorker(WorkerExtension):
    def __init__(self, module: torch.nn.Module, rank: int = 0, device: str | torch.device = "cpu",
                 backend: str = "nccl", layout: str = "trainer"):
        self.rank = rank
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:  # compare equal to the tensors' devices
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.actor_group_backend = backend
        module.to(self.device)
        model = StackedParamsModel(module) if layout == "vllm" else ParamDictModel(module)
        self.model_runner = types.SimpleNamespace(model=model)
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
    ap.add_argument("--layout", choices=("trainer", "vllm"), default="trainer",
                    help="parameter layout held: the trainer's names, or vLLM's fused qkv_proj / gate_up_proj")
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    from transformers import AutoConfig, AutoModelForCausalLM

    cfg = AutoConfig.from_pretrained(args.model_config)
    module = AutoModelForCausalLM.from_config(cfg, torch_dtype=torch.bfloat16)
    worker = StandaloneWorker(module, rank=0, device=args.device, backend=args.backend, layout=args.layout)
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
