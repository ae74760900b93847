"""Fail-fast of the zero-copy weight broadcast on device tensors (one MI355X): a gloo "actor" group
on cuda:0 parameters (the one-GPU stand-in for the RCCL group, which refuses two ranks on one GPU),
an actor that answers HTTP but never receives, and the trainer reaching its next optimizer step
while the broadcast still reads the parameters in place.  before_optimizer_step must raise
WeightUpdateError within the update's timeout, without a host wait on the gloo works, and leave the
parameters unwritten (reference behaviour it replaces: finetune_loop.py:155-172 blocks in NCCL)."""

from __future__ import annotations

import json
import os
import sys
from pathlib import Path

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _trainer(port, exp):
    import threading
    import time
    from http.server import BaseHTTPRequestHandler, HTTPServer

    sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "pipelinerl-swe_amd")]
    from pipelinerl_amd import torch_utils
    from pipelinerl_amd.finetune.optim import PrlAdamW
    from pipelinerl_amd.weight_update import WeightUpdateError, WeightUpdateManager

    class Silent(BaseHTTPRequestHandler):
        def do_POST(self):
            self.rfile.read(int(self.headers.get("Content-Length", 0)))
            self.send_response(200)
            self.end_headers()
            self.wfile.write(b'{"status": "ok"}')

        def log_message(self, *a):
            pass

    srv = HTTPServer(("127.0.0.1", 0), Silent)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Embedding(64, 256), torch.nn.Linear(256, 512), torch.nn.Linear(512, 64))
    model = model.to(device="cuda", dtype=torch.bfloat16)
    pg = torch_utils.init_extra_process_group(group_name="actor", backend="gloo",
                                              init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=2)
    mgr = WeightUpdateManager([f"http://127.0.0.1:{srv.server_address[1]}"], model, None, pg, transport="bucketed",
                              bucket_bytes=1 << 16, overlap=True, write_message=lambda s, m: None, timeout_s=3.0,
                              http_timeout_s=5.0)
    opt = PrlAdamW(model.parameters(), lr=1e-2)
    t0 = time.time()
    mgr.send_weight_update(1)
    t_send = time.time() - t0
    in_place = mgr._flat_params is not None
    before = [p.detach().clone() for p in model.parameters()]
    model(torch.arange(32, device="cuda").view(1, 32)).float().square().mean().backward()
    err, stepped = None, False
    try:
        mgr.poll()
        mgr.before_optimizer_step()
        opt.step()
        stepped = True
    except WeightUpdateError as e:
        err = str(e)
    torch.cuda.synchronize()
    unchanged = all(torch.equal(a, p.detach()) for a, p in zip(before, model.parameters()))
    Path(exp, "result.json").write_text(json.dumps(dict(error=err, elapsed=time.time() - t0, t_send=t_send,
                                                        in_place=in_place, stepped=stepped, unchanged=unchanged)))
    os._exit(0)  # the never-matched gloo broadcast stays pending: skip its destructor


def _actor(port, exp):
    import time

    sys.path[:0] = [str(ROOT), str(ROOT / "pipelinerl-swe_amd")]
    from pipelinerl_amd import torch_utils

    torch_utils.init_extra_process_group(group_name="actor", backend="gloo", init_method=f"tcp://127.0.0.1:{port}",
                                         rank=1, world_size=2)
    t0 = time.time()
    while not Path(exp, "result.json").exists() and time.time() - t0 < 60:
        time.sleep(0.05)  # joined the group, never receives
    os._exit(0)


def _run(rank, port, exp):
    os.environ["OMP_NUM_THREADS"] = "1"
    if rank == 0:
        _trainer(port, exp)
    else:
        os.environ["HIP_VISIBLE_DEVICES"] = ""  # the actor stand-in never touches the GPU
        _actor(port, exp)


def test_zero_copy_update_fails_fast_on_a_silent_actor(tmp_path):
    from test_weight_update_cpu import free_port

    mp.spawn(_run, args=(free_port(), str(tmp_path)), nprocs=2, join=True)
    r = json.loads((tmp_path / "result.json").read_text())
    assert r["in_place"], r  # a bf16 model on one device: broadcast in place (the default)
    assert r["t_send"] < 1.0, r  # the send itself never waits for the broadcast
    assert r["error"] is not None and not r["stepped"] and r["unchanged"], r
    assert 2.5 < r["elapsed"] < 4.5, r
