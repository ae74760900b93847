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


def test_abort_all_tears_down_every_open_communicator():
    """bench.py's probe deadline: comm.abort_all() aborts the process's open communicators (closed
    ones are skipped) and leaves them unusable."""
    from pipelinerl_amd import comm

    a, b = _comm(), _comm()
    b.close()
    try:
        assert comm.abort_all() == 1
        assert a._h is None and comm.abort_all() == 0
        with pytest.raises(Exception):
            a.all_reduce(torch.ones(4, device="cuda"))
    finally:
        a.close()


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


def test_zero_copy_snapshot_broadcasts_the_parameters_in_place(tmp_path):
    """snapshot="zero_copy" (the default): a bf16 model's parameters are re-homed once into one
    buffer in the broadcast layout (the same Parameter objects, values bit-identical, a tied weight
    kept tied), every later update reads them in place (no re-home, no staging buffer), the next
    optimizer step is ordered after the broadcast's reads, and a checkpoint of the re-homed model
    saves and loads back exactly (safetensors refuses shared storage: host copies are saved)."""
    from transformers import AutoConfig, AutoModelForCausalLM

    from loop_helpers import tiny_model_dir
    from pipelinerl_amd.finetune.checkpoints import save_model_and_tokenizer
    from pipelinerl_amd.finetune.optim import PrlAdamW
    from pipelinerl_amd.weight_update import WeightUpdateManager

    c = _comm()
    try:
        cfg = AutoConfig.from_pretrained(tiny_model_dir(tmp_path))
        torch.manual_seed(0)
        model = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16).cuda()
        tied = model.get_input_embeddings().weight is model.get_output_embeddings().weight
        before = {n: p.detach().clone() for n, p in model.named_parameters()}
        ids = {n: id(p) for n, p in model.named_parameters()}
        mgr = WeightUpdateManager([], model, None, c, transport="bucketed", bucket_bytes=4096, overlap=True,
                                  write_message=lambda s, m: None)
        mgr.send_weight_update(1)
        mgr.wait()
        flat = mgr._flat_params
        assert flat is not None and mgr._staging is None
        offs = _offsets(model)
        for (n, p), o in zip(model.named_parameters(), offs):
            assert id(p) == ids[n] and p.data_ptr() == flat.data_ptr() + 2 * o, n
            assert torch.equal(p.detach(), before[n]), n
        assert (model.get_input_embeddings().weight is model.get_output_embeddings().weight) == tied
        # an optimizer step after the update: ordered after the broadcast, parameters stay in place
        opt = PrlAdamW(model.parameters(), lr=1e-2)
        for p in model.parameters():
            p.grad = torch.randn_like(p)
        mgr.before_optimizer_step()
        opt.step()
        mgr.send_weight_update(2)
        mgr.close()
        assert mgr._flat_params is flat and mgr.completed_versions == [1, 2]
        for (n, p), o in zip(model.named_parameters(), offs):
            assert p.data_ptr() == flat.data_ptr() + 2 * o and not torch.equal(p.detach(), before[n]), n
        # checkpoint of the re-homed model: saves, and loads back bit for bit
        out = tmp_path / "current"
        save_model_and_tokenizer(out, model, object(), safe_serialization=True)
        back = AutoModelForCausalLM.from_pretrained(out, dtype=torch.bfloat16).cuda()
        for n, p in back.named_parameters():
            assert torch.equal(p.detach(), dict(model.named_parameters())[n].detach()), n
        # snapshot="copy" keeps the parameters where they are
        m2 = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16).cuda()
        ptrs = [p.data_ptr() for p in m2.parameters()]
        mgr2 = WeightUpdateManager([], m2, None, c, transport="bucketed", bucket_bytes=4096, overlap=True,
                                   write_message=lambda s, m: None, snapshot="copy")
        mgr2.send_weight_update(1)
        mgr2.close()
        assert mgr2._flat_params is None and mgr2._staging is not None
        assert [p.data_ptr() for p in m2.parameters()] == ptrs
    finally:
        c.close()


def test_paced_read_runs_at_its_rate():
    """prl_paced_read (the emulated broadcast reads of bench.py's snapshot_overlap): 1 GiB at 153 GB/s
    over 16 workgroups takes 1 GiB / 153 GB/s within 10 % (paced, not at HBM speed), and at a rate
    above what 16 workgroups can read it simply runs unpaced."""
    import ctypes

    from pipelinerl_amd import _native

    lib = _native.load()
    buf = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(64, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream

    def run(gbps, blocks):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        assert lib.prl_paced_read(ctypes.c_void_p(buf.data_ptr()), buf.numel(), gbps, blocks,
                                  ctypes.c_void_p(sink.data_ptr()), st) == 0
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1)

    run(153.0, 16)  # warm-up
    ms = run(153.0, 16)
    want = buf.numel() / 153e9 * 1e3
    assert 0.9 * want <= ms <= 1.1 * want, (ms, want)
    assert run(1e6, 64) < 0.5 * want
