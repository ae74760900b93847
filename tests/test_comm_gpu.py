"""prl_comm (RCCL C ABI) on one MI355X: a world-1 communicator through the Python wrapper and
the weight-update sender on it.  RCCL refuses two ranks on one GPU, so the multi-rank paths
run only on the driver's multi-GPU node; the same call sequence is exercised here."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _comm():
    from pipelinerl_amd.comm import RcclComm
    from test_weight_update_cpu import free_port

    return RcclComm.create(f"tcp://127.0.0.1:{free_port()}", 0, 1, torch.device("cuda", 0))


def test_world1_collectives():
    from pipelinerl_amd.comm import CommError

    c = _comm()
    try:
        x = torch.arange(1 << 20, device="cuda", dtype=torch.float32)
        want = x.clone()
        c.broadcast(x, 0)
        c.broadcast(x, 0, bucket_bytes=1 << 16)
        for op in ("sum", "avg", "max"):
            c.all_reduce(x, op)
        y = torch.randn(4097, device="cuda").to(torch.bfloat16)
        y0 = y.clone()
        c.all_reduce(y, "sum")
        torch.cuda.synchronize()
        assert torch.equal(x, want) and torch.equal(y, y0)
        with pytest.raises(CommError):
            c.broadcast(x, 1)  # root out of range
        with pytest.raises(CommError):
            c.all_reduce(torch.zeros(3, device="cuda", dtype=torch.float16))
    finally:
        c.close()


def test_weight_update_sender_on_prl_comm():
    from pipelinerl_amd.weight_update import WeightUpdateManager

    c = _comm()
    try:
        model = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.Linear(128, 8, bias=False)).cuda()
        for transport in ("bucketed", "per_tensor"):
            mgr = WeightUpdateManager([], model, None, c, transport=transport, bucket_bytes=4096, overlap=True,
                                      write_message=lambda s, m: None)
            mgr.send_weight_update(3)
            mgr.close()
            assert mgr.completed_versions == [3]
            flat = mgr._staging
            got = torch.cat([flat[o:o + p.numel()].float() for o, p in
                             zip(_offsets(model), model.parameters())])
            want = torch.cat([p.detach().reshape(-1).to(torch.bfloat16).float() for p in model.parameters()])
            assert torch.equal(got, want)
    finally:
        c.close()


def _offsets(model):
    from pipelinerl_amd.weight_update import FlatLayout, ParameterInfo

    infos = [ParameterInfo(name=n, shape=list(p.shape), dtype=str(torch.bfloat16)) for n, p in model.named_parameters()]
    return FlatLayout.from_infos(infos).offsets
