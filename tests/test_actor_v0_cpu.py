"""The vLLM v0 actor binding (pipelinerl/vllm0.py:51-104, the reference's default actor:
conf/base.yaml ``use_v1: false``): ``make_worker_class`` over stand-ins of vLLM's ``Worker`` and
``MultiStepWorker`` (whose ``MultiStepModelRunner`` keeps the model at
``_base_model_runner.model``, vllm0.py:90-93).  A gloo trainer broadcasts per_tensor and bucketed
updates to one worker of each kind holding vLLM's fused qkv / gate_up layout; both end with the
trainer's exact weights.  The reference's errors (dtype AssertionError, ValueError on an unknown
name) and its group ranks are kept."""

from __future__ import annotations

import os
import sys
import types
from pathlib import Path

import pytest
import torch
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "pipelinerl-swe_amd")]


# --- stand-ins of the vLLM v0 classes the reference subclasses / checks (vllm0.py:26,32,33) ---

class ModelRunner:
    def __init__(self, model):
        self.model = model


class MultiStepModelRunner:
    """vLLM's multi-step runner wraps the real runner (no ``model`` attribute of its own)."""

    def __init__(self, base):
        self._base_model_runner = base


class Worker:
    def __init__(self, module: torch.nn.Module, rank: int = 0, device: str = "cpu"):
        from pipelinerl_amd.actor import StackedParamsModel

        self.rank = rank
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:  # as vLLM's worker: an indexed device
            self.device = torch.device("cuda", torch.cuda.current_device())
        module.to(self.device)
        self.model_config = types.SimpleNamespace(dtype=next(module.parameters()).dtype)
        self.model_runner = ModelRunner(StackedParamsModel(module))  # vLLM's fused Qwen2 layout

    def execute_model(self):  # a base-class method the mixin must leave alone
        return "executed"


class MultiStepWorker(Worker):
    def __init__(self, module: torch.nn.Module, rank: int = 0, device: str = "cpu"):
        super().__init__(module, rank, device)
        self.model_runner = MultiStepModelRunner(self.model_runner)


def _classes():
    from pipelinerl_amd.actor import make_worker_class

    return make_worker_class(False, Worker), make_worker_class(True, MultiStepWorker)


def _infos(module):
    from pipelinerl_amd.weight_update import ParameterInfo

    return [ParameterInfo(name=n, shape=list(p.shape), dtype=str(torch.bfloat16)) for n, p in module.named_parameters()]


def _trainer(port, exp, versions):
    from test_weight_update_cpu import TorchFlatPacker, make_qwen2

    from pipelinerl_amd import torch_utils
    from pipelinerl_amd.weight_update import WeightUpdateManager

    model = make_qwen2(0)
    pg = torch_utils.init_extra_process_group(group_name="actor", backend="gloo",
                                              init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=3)
    for transport, v in zip(("per_tensor", "bucketed"), versions):
        mgr = WeightUpdateManager([], model, None, pg, transport=transport, bucket_bytes=1000, overlap=True,
                                  packer=TorchFlatPacker(), write_message=lambda s, m: None)
        mgr.before_optimizer_step()
        with torch.no_grad():
            for p in model.parameters():
                p.add_(0.125 * (v + 1))
        mgr.send_weight_update(v)
        mgr.close()
        torch.save({n: p.detach().clone() for n, p in model.named_parameters()}, Path(exp) / f"trainer_v{v}.pt")


def _actor(port, exp, idx, versions):
    from test_weight_update_cpu import make_qwen2

    from pipelinerl_amd.weight_update import WeightUpdateRequest

    single, multi = _classes()
    cls = single if idx == 0 else multi
    worker = cls(make_qwen2(100 + idx), rank=0)
    worker.actor_group_backend = "gloo"  # the one-host stand-in for RCCL
    worker.init_actor_update_group(idx, 1, f"tcp://127.0.0.1:{port}", 3)
    assert worker.pg_rank == 1 + idx
    infos = _infos(make_qwen2(0))
    m = worker._inference_model()
    for transport, v in zip(("per_tensor", "bucketed"), versions):
        worker.receive_weight_update(WeightUpdateRequest(version=v, parameters_info=infos, transport=transport,
                                                         bucket_bytes=1000 if transport == "bucketed" else 0))
        torch.save({i.name: m.direct_target(i.name, tuple(i.shape)).clone() for i in infos},
                   Path(exp) / f"actor{idx}_v{v}.pt")


def _run(rank, port, exp, versions):
    os.environ["OMP_NUM_THREADS"] = "1"
    if rank == 0:
        _trainer(port, exp, versions)
    else:
        _actor(port, exp, rank - 1, versions)


def test_v0_workers_receive_both_transports_bit_exactly(tmp_path):
    from test_weight_update_cpu import free_port

    versions = [3, 7]
    mp.spawn(_run, args=(free_port(), str(tmp_path), versions), nprocs=3, join=True)
    for v in versions:
        want = torch.load(tmp_path / f"trainer_v{v}.pt")
        for idx in (0, 1):
            got = torch.load(tmp_path / f"actor{idx}_v{v}.pt")
            assert set(got) == set(want)
            for n in want:
                assert torch.equal(got[n], want[n]), (idx, v, n)


def test_v0_worker_classes_keep_the_reference_contract():
    from test_weight_update_cpu import make_qwen2

    from pipelinerl_amd.actor import V0WorkerMixin, is_multi_step_runner
    from pipelinerl_amd.weight_update import ParameterInfo, WeightUpdateRequest

    single, multi = _classes()
    assert single.__name__ == "AsyncRLWorker" and multi.__name__ == "AsyncRLMultiStepWorker"
    assert issubclass(single, Worker) and issubclass(multi, MultiStepWorker)
    assert single.__mro__[1] is V0WorkerMixin  # the receive methods come first, the base's stay
    for cls in (single, multi):
        module = make_qwen2(5)
        w = cls(module)
        assert w.execute_model() == "executed"
        runner = w.model_runner
        # where the loads go (vllm0.py:90-95): the multi-step runner's base runner's model
        assert is_multi_step_runner(runner) == (cls is multi)
        model = runner._base_model_runner.model if cls is multi else runner.model
        assert w._inference_model() is model
        # the fused layout resolves through direct_target on both runner kinds
        q = w._inference_model().direct_target("model.layers.0.self_attn.k_proj.weight", (8, 16))
        qkv = model.params["model.layers.0.self_attn.qkv_proj.weight"]
        assert q is not None and q.data_ptr() == qkv[16:24].data_ptr()
        # vllm0.py:85-87: dtype mismatch -> AssertionError, before anything is received
        bad = WeightUpdateRequest(version=1, parameters_info=[ParameterInfo(name="model.norm.weight", shape=[16],
                                                                            dtype="torch.float32")])
        with pytest.raises(AssertionError, match="mismatch dtype"):
            w.receive_weight_update(bad)
        # vllm0.py:96-97: a name the model does not load -> ValueError
        with pytest.raises(ValueError, match="not found in model state dict"):
            w._load_one("model.no_such.weight", torch.zeros(3, dtype=torch.bfloat16))
        w._load_one("model.layers.1.mlp.up_proj.weight", torch.ones(24, 16, dtype=torch.bfloat16))
        assert torch.equal(model.params["model.layers.1.mlp.gate_up_proj.weight"][24:],
                           torch.ones(24, 16, dtype=torch.bfloat16))


def test_v0_named_classes_need_vllm():
    """``worker_cls = "pipelinerl_amd.actor.AsyncRLWorker"`` resolves through the module; without
    vLLM importable the error says what is missing (vLLM is absent from this image)."""
    import importlib.util

    from pipelinerl_amd import actor

    if importlib.util.find_spec("vllm") is not None:
        assert actor.AsyncRLWorker is actor.AsyncRLWorker  # one class per process
        return
    with pytest.raises(ImportError, match="vLLM v0 worker classes need vLLM"):
        actor.AsyncRLMultiStepWorker
    with pytest.raises(AttributeError):
        actor.NoSuchWorker
