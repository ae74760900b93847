"""The trainer -> actor pipeline end to end, on CPU: ``run_finetuning_loop`` with
``send_weight_updates`` on (the reference's default, conf/finetune/base.yaml) and a stand-alone actor
PROCESS (``python -m pipelinerl_amd.actor``: HTTP ``/health`` and ``/receive_weight_update``, the
actor group joined at ``+me.weight_update_group_init_method`` with pg_rank 1, vllm1.py:53-117).

What the components' own tests do not cover, checked here in one run:
  * the loop's start-up order (finetune_loop.py:400-441): the actor group rendezvous, the health
    wait, the initial update at version 0 before the first micro-batch;
  * one update after every optimizer step (weight_update_interval 1) with version = samples trained
    (finetune_loop.py:795-801), each acknowledged by the actor's HTTP answer and then announced by a
    ``WeightUpdateSuccess`` on the ``weight_update_request`` topic, after that step's
    ``SamplesProcessed``;
  * the actor ends holding exactly the trainer's final weights (bf16; per-tensor checksums over
    HTTP), the bf16 trainer's parameters broadcast in place (``weight_snapshot: zero_copy``), over
    both transports.  (The staging-copy snapshot runs the HIP flatten kernel: on the GPU in
    tests/test_split_pipeline_gpu.py and tests/test_comm_gpu.py, with a torch packer in
    tests/test_weight_update_cpu.py.)
The loss is the CPU torch restatement of rl_step (tests/cpu_rl_step.py) here; tests/test_pipeline_e2e_gpu.py
runs the same pipeline with the product's rl_step and the actor on the GPU.
"""

from __future__ import annotations

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest
import torch
import torch.multiprocessing as mp

from test_finetune_loop_cpu import _setup, free_port

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "pipelinerl-swe_amd"


def _trainer(rank, exp, actor_url, group_port, transport, snapshot, device="cpu"):
    sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(PKG)]
    os.environ.update(OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        os.environ.pop(k, None)
    from cpu_rl_step import cpu_rl_step
    from loop_helpers import loop_cfg
    from pipelinerl_amd.finetune.rl import rl_step
    from pipelinerl_amd.finetune_loop import run_finetuning_loop
    from pipelinerl_amd.streams import reset_streams_backend

    reset_streams_backend()
    exp = Path(exp)
    per_step = json.loads((exp / "per_step.json").read_text())
    cfg = loop_cfg(exp, exp / "tiny_qwen2", 1, per_step, 2, dist_backend=None, send_weight_updates=True,
                   load_as_bf16=True, actor_group_backend="gloo", weight_transport=transport,
                   weight_snapshot=snapshot, weight_update_timeout_s=120.0, weight_update_http_timeout_s=120.0)
    cfg.me.weight_update_group_init_method = f"tcp://127.0.0.1:{group_port}"
    cfg.me.weight_update_group_world_size = 2
    cfg.me.llm_urls = actor_url
    captured = {}

    def step(model, batch, cur, mx, config):  # CPU: the torch restatement
        captured["model"] = model
        return cpu_rl_step(model, batch, cur, mx, config)

    m = run_finetuning_loop(cfg, step_fn=step if device == "cpu" else _Capture(rl_step, captured))
    sums = {n: float(p.detach().to(torch.bfloat16).double().sum()) for n, p in captured["model"].named_parameters()}
    (exp / "trainer.json").write_text(json.dumps({"steps": m.completed_steps, "samples": m.samples, "sums": sums}))


class _Capture:
    """rl_step itself (so the loop takes its native path: deferred statistics, loss scale), noting the model."""

    def __init__(self, fn, captured):
        self.fn, self.captured = fn, captured

    def __call__(self, model, *a, **kw):
        self.captured["model"] = model
        return self.fn(model, *a, **kw)


@pytest.mark.parametrize("transport,snapshot", [("bucketed", "zero_copy"), ("per_tensor", "zero_copy")])
def test_loop_updates_a_standalone_actor_process(tmp_path, transport, snapshot):
    run_pipeline(tmp_path, transport, snapshot, "cpu")


def run_pipeline(tmp_path, transport, snapshot, device):
    import requests

    exp = tmp_path
    per_step, _ = _setup(exp, 1)
    (exp / "per_step.json").write_text(json.dumps(per_step))
    actor_port, group_port = free_port(), free_port()
    url = f"http://127.0.0.1:{actor_port}"
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([str(PKG), os.environ.get("PYTHONPATH", "")]),
               OMP_NUM_THREADS="1")
    if device == "cpu":
        env.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    log = open(exp / "actor.log", "w")
    actor = subprocess.Popen([sys.executable, "-m", "pipelinerl_amd.actor", "--port", str(actor_port),
                              "--actor-llm-idx", "0", "--weight-update-group-init-method",
                              f"tcp://127.0.0.1:{group_port}", "--weight-update-group-world-size", "2",
                              "--backend", "gloo", "--device", device, "--model-config", str(exp / "tiny_qwen2")],
                             env=env, stdout=log, stderr=subprocess.STDOUT)
    try:
        mp.spawn(_trainer, args=(str(exp), url, group_port, transport, snapshot, device), nprocs=1, join=True)
        got = requests.get(url + "/checksum", timeout=30).json()
    finally:
        actor.terminate()
        try:
            actor.wait(timeout=20)
        except subprocess.TimeoutExpired:
            actor.kill()
        log.close()
    t = json.loads((exp / "trainer.json").read_text())
    assert t["steps"] == 2 and t["samples"] == 2 * per_step
    # the actor holds the trainer's final weights exactly
    assert set(got) == set(t["sums"]), (set(got) ^ set(t["sums"]))
    for n, s in t["sums"].items():
        assert got[n] == s, (n, got[n], s)
    # the protocol on the weight_update_request topic
    lines = (exp / "streams" / "weight_update_request" / "0" / "0" / "0.jsonl").read_text().splitlines()
    msgs = [json.loads(x) for x in lines]
    success = [m["version"] for m in msgs if m["kind"] == "weight_update_success"]
    assert success == [0, per_step, 2 * per_step], success
    processed = [m["samples_processed"] for m in msgs if m["kind"] == "samples_processed"]
    assert processed[-1] == 2 * per_step
    for v in success[1:]:  # each update is announced after the SamplesProcessed that completed its step
        i_done = next(i for i, m in enumerate(msgs) if m["kind"] == "samples_processed" and m["samples_processed"] == v)
        i_succ = next(i for i, m in enumerate(msgs) if m["kind"] == "weight_update_success" and m["version"] == v)
        assert i_done < i_succ, (v, i_done, i_succ)
    actor_log = (exp / "actor.log").read_text()
    assert actor_log.count("Weight update received") == 3, actor_log[-2000:]
    # the final checkpoint of the (re-homed) trainer loads back with the weights the actor holds
    from transformers import AutoModelForCausalLM

    back = AutoModelForCausalLM.from_pretrained(exp / "finetune" / "current", dtype=torch.bfloat16)
    for n, p in back.named_parameters():
        assert float(p.detach().double().sum()) == t["sums"][n], n
