"""Trainer -> actor weight broadcast over a gloo "actor" group on CPU (world size 2 and 3).

The trainer side is WeightUpdateManager (overlapped, both transports); the actor side is the
WorkerExtension receive path.  A test-only packer (plain torch copies) stands in for the HIP
flatten kernel, which needs a device; the GPU suite covers that kernel.
"""

import json
import os
import socket
import sys
from pathlib import Path

import pytest
import torch
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


class TorchFlatPacker:
    def flatten(self, tensors, offsets, flat):
        for t, o in zip(tensors, offsets):
            flat[o:o + t.numel()].copy_(t.reshape(-1))

    def unflatten(self, flat, tensors, offsets):
        for t, o in zip(tensors, offsets):
            t.copy_(flat[o:o + t.numel()].view_as(t))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def make_model(seed):
    torch.manual_seed(seed)
    m = torch.nn.Sequential(torch.nn.Embedding(37, 16), torch.nn.Linear(16, 24), torch.nn.LayerNorm(24),
                            torch.nn.Linear(24, 37, bias=False))
    return m.to(torch.bfloat16)


def make_qwen2(seed):
    """A tiny Qwen2 (the trainer's parameter names: q/k/v_proj, gate/up_proj, GQA 2/1)."""
    from transformers import Qwen2Config, Qwen2ForCausalLM

    torch.manual_seed(seed)
    cfg = Qwen2Config(vocab_size=37, hidden_size=16, intermediate_size=24, num_hidden_layers=2,
                      num_attention_heads=2, num_key_value_heads=1, tie_word_embeddings=False)
    return Qwen2ForCausalLM(cfg).to(torch.bfloat16)


def _trainer(port, world, transport, exp, versions, use_reference_pg, qwen=False):
    sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]
    from pipelinerl_amd import torch_utils
    from pipelinerl_amd.streams import SingleStreamSpec, reset_streams_backend, set_streams_backend
    from pipelinerl_amd.weight_update import WeightUpdateManager

    reset_streams_backend()
    set_streams_backend("files")
    model = make_qwen2(0) if qwen else make_model(0)
    pg = torch_utils.init_extra_process_group(group_name="actor", backend="gloo",
                                              init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=world)
    stream = SingleStreamSpec(exp_path=Path(exp), topic="weight_update_request")
    mgr = WeightUpdateManager([], model, stream, pg, transport=transport, bucket_bytes=1000, overlap=True,
                              packer=TorchFlatPacker())
    for v in versions:
        mgr.before_optimizer_step()  # the parameters are written below: after the previous broadcast read them
        with torch.no_grad():
            for p in model.parameters():
                p.add_(0.125 * (v + 1))
        mgr.send_weight_update(v)  # returns immediately (overlapped)
    mgr.close()
    # the bf16 model is broadcast in place (snapshot="zero_copy"): its parameters live in one buffer
    flat = mgr._flat_params
    assert flat is not None and mgr._staging is None
    assert all(flat.data_ptr() <= p.data_ptr() < flat.data_ptr() + 2 * flat.numel() for p in model.parameters())
    torch.save({n: p.detach().clone() for n, p in model.named_parameters()}, Path(exp) / "trainer_params.pt")


def _actor(port, world, idx, transport, exp, nupdates, use_reference_pg, qwen=False):
    sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]
    from pipelinerl_amd.actor import StandaloneWorker
    from pipelinerl_amd.weight_update import ParameterInfo, WeightUpdateRequest

    if qwen:  # vLLM's fused layout at the actor; the request carries the trainer's names
        module = make_qwen2(100 + idx)
        names = [(n, list(p.shape)) for n, p in module.named_parameters()]
        worker = StandaloneWorker(module, rank=0, device="cpu", backend="gloo", layout="vllm")
        worker.init_actor_update_group(idx, 1, f"tcp://127.0.0.1:{port}", world)
        infos = [ParameterInfo(name=n, shape=s, dtype=str(torch.bfloat16)) for n, s in names]
        for v in range(nupdates):
            worker.receive_weight_update(WeightUpdateRequest(version=v, parameters_info=infos, transport=transport,
                                                             bucket_bytes=1000 if transport == "bucketed" else 0))
        m = worker.model_runner.model
        torch.save({"by_name": {n: m.direct_target(n, tuple(s)).clone() for n, s in names},
                    "fused": {n: p.clone() for n, p in m.params.items()}}, Path(exp) / f"actor{idx}_params.pt")
        return
    worker = StandaloneWorker(make_model(100 + idx), rank=0, device="cpu", backend="gloo")
    if use_reference_pg:  # join with the REFERENCE's group helper: pins the store-key layout
        sys.path.insert(0, "/root/reference")
        from pipelinerl.torch_utils import init_extra_process_group as ref_init

        worker.pg_rank = 1 + idx
        worker.process_group = ref_init(group_name="actor", backend="gloo", init_method=f"tcp://127.0.0.1:{port}",
                                        rank=worker.pg_rank, world_size=world)
    else:
        worker.init_actor_update_group(idx, 1, f"tcp://127.0.0.1:{port}", world)
    names = [(n, list(p.shape)) for n, p in worker.model_runner.model.params.items()]
    infos = [ParameterInfo(name=n, shape=s, dtype=str(torch.bfloat16)) for n, s in names]
    for v in range(nupdates):
        worker.receive_weight_update(WeightUpdateRequest(version=v, parameters_info=infos, transport=transport,
                                                         bucket_bytes=1000 if transport == "bucketed" else 0))
    torch.save({n: p.detach().clone() for n, p in worker.model_runner.model.params.items()},
               Path(exp) / f"actor{idx}_params.pt")
    os._exit(0)  # no gloo teardown at interpreter exit (it aborted once under a loaded pytest -n 4)


def _run(rank, port, world, transport, exp, use_reference_pg, qwen=False):
    os.environ["OMP_NUM_THREADS"] = "1"
    if rank == 0:
        _trainer(port, world, transport, exp, [3, 7], use_reference_pg, qwen)
    else:
        _actor(port, world, rank - 1, transport, exp, 2, use_reference_pg, qwen)


# world 5: C4's actor group (1 trainer + 4 actor GPUs, weight_update_group_size 5, world.py:184)
@pytest.mark.parametrize("transport,world", [("per_tensor", 2), ("bucketed", 2), ("bucketed", 3), ("per_tensor", 5),
                                             ("bucketed", 5)])
def test_broadcast_roundtrip(tmp_path, transport, world):
    port = free_port()
    mp.spawn(_run, args=(port, world, transport, str(tmp_path), False), nprocs=world, join=True)
    want = torch.load(tmp_path / "trainer_params.pt")
    for a in range(world - 1):
        got = torch.load(tmp_path / f"actor{a}_params.pt")
        assert set(got) == set(want)
        for n in want:
            assert torch.equal(got[n], want[n].to(torch.bfloat16)), n
    lines = (tmp_path / "streams" / "weight_update_request" / "0" / "0" / "0.jsonl").read_text().splitlines()
    msgs = [json.loads(x) for x in lines]
    assert [m["version"] for m in msgs if m["kind"] == "weight_update_success"] == [3, 7]


@pytest.mark.parametrize("transport", ["per_tensor", "bucketed"])
def test_broadcast_into_vllm_fused_layout(tmp_path, transport):
    """An actor holding vLLM's fused qkv_proj / gate_up_proj receives the trainer's per-projection
    names: every q / k / v and gate / up tensor lands in its row block, the rest by name, and each
    fused parameter is the concatenation of the trainer's shards in vLLM's order."""
    port = free_port()
    mp.spawn(_run, args=(port, 2, transport, str(tmp_path), False, True), nprocs=2, join=True)
    want = torch.load(tmp_path / "trainer_params.pt")
    got = torch.load(tmp_path / "actor0_params.pt")
    assert set(got["by_name"]) == set(want)
    for n in want:
        assert torch.equal(got["by_name"][n], want[n]), n
    fused = got["fused"]
    assert not any(".q_proj." in n or ".gate_proj." in n for n in fused)
    for i in range(2):
        pre = f"model.layers.{i}."
        assert torch.equal(fused[pre + "self_attn.qkv_proj.weight"],
                           torch.cat([want[pre + f"self_attn.{x}_proj.weight"] for x in "qkv"]))
        assert torch.equal(fused[pre + "self_attn.qkv_proj.bias"],
                           torch.cat([want[pre + f"self_attn.{x}_proj.bias"] for x in "qkv"]))
        assert torch.equal(fused[pre + "mlp.gate_up_proj.weight"],
                           torch.cat([want[pre + "mlp.gate_proj.weight"], want[pre + "mlp.up_proj.weight"]]))


def test_vllm_layout_load_weights_returns_the_fused_name():
    """The reference actor raises unless load_weights reports exactly one loaded parameter
    (vllm1.py:91-93); for a shard that is the fused parameter's name, as in vLLM."""
    sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]
    from pipelinerl_amd.actor import StackedParamsModel

    src = make_qwen2(1)
    m = StackedParamsModel(make_qwen2(2))
    w = dict(src.named_parameters())
    assert m.load_weights([("model.layers.0.self_attn.k_proj.weight", w["model.layers.0.self_attn.k_proj.weight"])]) \
        == {"model.layers.0.self_attn.qkv_proj.weight"}
    assert m.load_weights([("model.norm.weight", w["model.norm.weight"])]) == {"model.norm.weight"}
    assert m.load_weights([("model.layers.0.self_attn.rotary_emb.inv_freq", torch.ones(4))]) == set()
    assert m.load_weights([("no.such.param", torch.ones(4))]) == set()
    assert torch.equal(m.params["model.layers.0.self_attn.qkv_proj.weight"][16:24],
                       w["model.layers.0.self_attn.k_proj.weight"].detach())


def test_fused_direct_target_matches_the_stand_in():
    """fused_direct_target (the adapter a vLLM worker attaches to its model) over
    a fused-layout model's parameters and config resolves every trainer name to the same storage as
    StackedParamsModel's own shard map."""
    sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]
    from pipelinerl_amd.actor import StackedParamsModel, fused_direct_target

    trainer = make_qwen2(3)
    m = StackedParamsModel(make_qwen2(4))
    resolve = fused_direct_target(m.params, trainer.config)
    for n, p in trainer.named_parameters():
        a, b = resolve(n, tuple(p.shape)), m.direct_target(n, tuple(p.shape))
        assert a is not None and a.data_ptr() == b.data_ptr() and a.shape == b.shape, n
    assert resolve("model.layers.0.self_attn.q_proj.weight", (3, 3)) is None
    assert resolve("no.such.param", (1,)) is None


@pytest.mark.skipif(not Path("/root/reference/pipelinerl/torch_utils.py").exists(),
                    reason="reference checkout not present (wire-compat check runs in the build container)")
def test_actor_group_interoperates_with_reference_helper(tmp_path):
    port = free_port()
    mp.spawn(_run, args=(port, 2, "per_tensor", str(tmp_path), True), nprocs=2, join=True)
    want = torch.load(tmp_path / "trainer_params.pt")
    got = torch.load(tmp_path / "actor0_params.pt")
    for n in want:
        assert torch.equal(got[n], want[n].to(torch.bfloat16)), n


def _failing_trainer(port, exp, mode):
    """Trainer rank of the fail-fast tests: an actor HTTP server that answers 500 ('http500')
    or answers 200 but never joins the broadcast ('silent'); wait() must raise, quickly."""
    import threading
    import time
    from http.server import BaseHTTPRequestHandler, HTTPServer

    sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]
    from pipelinerl_amd import torch_utils
    from pipelinerl_amd.weight_update import WeightUpdateError, WeightUpdateManager

    class H(BaseHTTPRequestHandler):
        def do_POST(self):
            self.rfile.read(int(self.headers.get("Content-Length", 0)))
            code = 500 if mode == "http500" else 200
            self.send_response(code)
            self.end_headers()
            self.wfile.write(b'{"status": "error"}' if code == 500 else b'{"status": "ok"}')

        def log_message(self, *a):
            pass

    srv = HTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    url = f"http://127.0.0.1:{srv.server_address[1]}"
    model = make_model(0)
    pg = torch_utils.init_extra_process_group(group_name="actor", backend="gloo",
                                              init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=2)
    mgr = WeightUpdateManager([url], model, None, pg, transport="bucketed", bucket_bytes=1000, overlap=True,
                              packer=TorchFlatPacker(), write_message=lambda s, m: None, timeout_s=3.0,
                              http_timeout_s=5.0)
    before = [p.detach().clone() for p in model.parameters()]
    t0 = time.time()
    mgr.send_weight_update(1)
    err, stepped = None, False
    if mode == "silent_step":
        # the loop's next step while the broadcast still reads the parameters in place
        # (finetune_loop.py: backward, clip, wum.poll(), wum.before_optimizer_step(), optimizer.step())
        assert mgr._flat_params is not None, "a bf16 model is broadcast in place (zero-copy)"
        opt = torch.optim.AdamW(model.parameters(), lr=1e-2)
        model(torch.arange(8).view(1, 8)).float().square().mean().backward()
        try:
            mgr.poll()
            mgr.before_optimizer_step()
            opt.step()
            stepped = True
        except WeightUpdateError as e:
            err = str(e)
    else:
        try:
            mgr.wait()
        except WeightUpdateError as e:
            err = str(e)
    unchanged = all(torch.equal(a, p.detach()) for a, p in zip(before, model.parameters()))
    Path(exp, "result.json").write_text(json.dumps({"error": err, "elapsed": time.time() - t0, "stepped": stepped,
                                                    "unchanged": unchanged}))
    os._exit(0)  # the never-matched gloo broadcast stays pending: skip its destructor


def _failing_actor(port, exp):
    import time

    sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]
    from pipelinerl_amd import torch_utils

    torch_utils.init_extra_process_group(group_name="actor", backend="gloo", init_method=f"tcp://127.0.0.1:{port}",
                                         rank=1, world_size=2)
    t0 = time.time()
    while not Path(exp, "result.json").exists() and time.time() - t0 < 60:
        time.sleep(0.05)  # a dead actor: never receives
    os._exit(0)


def _run_failing(rank, port, exp, mode):
    os.environ["OMP_NUM_THREADS"] = "1"
    if rank == 0:
        _failing_trainer(port, exp, mode)
    else:
        _failing_actor(port, exp)


@pytest.mark.parametrize("mode", ["http500", "silent", "silent_step"])
def test_failed_actor_makes_the_trainer_raise(tmp_path, mode):
    """SURVEY.md §5 failure row: the reference logs an actor's HTTP error and then blocks in the
    broadcast until the process-group timeout (finetune_loop.py:155-172).  Here an HTTP 500
    raises WeightUpdateError from wait() at once; an actor that never joins the broadcast
    raises after WeightUpdateManager's timeout (3 s in this test).  ``silent_step``: the bf16
    model is broadcast in place (zero-copy, the default) and the trainer reaches its next
    optimizer step while the broadcast still reads the parameters — before_optimizer_step raises
    within the timeout (no host wait on the gloo works) and the parameters stay unwritten."""
    port = free_port()
    mp.spawn(_run_failing, args=(port, str(tmp_path), mode), nprocs=2, join=True)
    r = json.loads((tmp_path / "result.json").read_text())
    assert r["error"] is not None
    if mode == "http500":
        assert "500" in r["error"] and r["elapsed"] < 3.0
    else:
        assert ("not completed" in r["error"] or "still reading" in r["error"]) and 2.5 < r["elapsed"] < 4.5, r
    assert r["unchanged"] and not r["stepped"]


def test_f4_request_and_actor_group_layout():
    """F4 (tests/golden/make_f4.py): the request the reference trainer builds for a 0.5B-shaped
    model (finetune_loop.py:178-199, 290 entries in named_parameters order) and the actor-group
    layout of the reference's world map (world.py:133-184, vllm1.py:62).  The build's request and
    its actors' group ranks must be the same."""
    from conftest import GOLDEN
    from transformers import Qwen2Config, Qwen2ForCausalLM

    sys.path[:0] = [str(ROOT / "pipelinerl-swe_amd")]
    from pipelinerl_amd import actor as actor_mod
    from pipelinerl_amd.weight_update import FlatLayout, WeightUpdateRequest, parameters_info, unwrap_model

    f4 = json.loads((GOLDEN / "f4_weight_update.json").read_text())
    cfg = Qwen2Config(hidden_size=896, intermediate_size=4864, num_hidden_layers=24, num_attention_heads=14,
                      num_key_value_heads=2, vocab_size=151936, tie_word_embeddings=True)
    with torch.device("meta"):
        model = Qwen2ForCausalLM(cfg)
    ours = [i.model_dump() for i in parameters_info(list(unwrap_model(model).named_parameters()))]
    assert ours == f4["request"]["parameters_info"] and len(ours) == f4["num_parameters"] == 290
    # the reference's message parses into ours (the extension fields default to the compat mode)
    req = WeightUpdateRequest(**f4["request"])
    assert req.transport == "per_tensor" and req.version == 4096
    dumped = req.model_dump()
    assert {k: dumped[k] for k in ("kind", "version", "parameters_info")} == \
        {k: f4["request"][k] for k in ("kind", "version", "parameters_info")}
    layout = FlatLayout.from_infos(req.parameters_info)
    assert sum(layout.numels) == f4["numel"] and all(o % 8 == 0 for o in layout.offsets)
    # actor group ranks: every worker of every actor LLM gets the reference's pg_rank, and the
    # ranks 1..size-1 of the reference's weight_update_group_size are covered exactly once
    seen = []

    def fake_group(**kw):
        seen.append((kw["rank"], kw["world_size"]))
        return object()

    orig = actor_mod.torch_utils.init_extra_process_group
    actor_mod.torch_utils.init_extra_process_group = fake_group
    try:
        for g in f4["groups"]:
            seen.clear()
            for idx, r, pg in g["actor_pg_ranks"]:
                w = actor_mod.WorkerExtension()
                w.rank = r
                w.init_actor_update_group(idx, g["gpus_per_llm"], "tcp://127.0.0.1:1", g["weight_update_group_size"])
                assert w.pg_rank == pg
            assert sorted(x[0] for x in seen) == list(range(1, g["weight_update_group_size"]))
            assert all(x[1] == g["weight_update_group_size"] for x in seen)
    finally:
        actor_mod.torch_utils.init_extra_process_group = orig


def test_weight_snapshot_follows_flat_parameters(caplog):
    """finetune.flat_parameters=false opts out of re-homing: the snapshot defaults to the staging
    copy, and an explicit zero_copy falls back to it with a warning instead of re-homing the
    parameters after the optimizer exists."""
    from pipelinerl_amd.config import Cfg
    from pipelinerl_amd.finetune_loop import weight_snapshot_mode

    assert weight_snapshot_mode(Cfg.wrap({})) == "zero_copy"
    assert weight_snapshot_mode(Cfg.wrap({"flat_parameters": False})) == "copy"
    assert weight_snapshot_mode(Cfg.wrap({"weight_snapshot": "copy"})) == "copy"
    with caplog.at_level("WARNING"):
        assert weight_snapshot_mode(Cfg.wrap({"flat_parameters": False, "weight_snapshot": "zero_copy"})) == "copy"
    assert "flat_parameters" in caplog.text
