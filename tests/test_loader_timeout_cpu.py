"""The trainer's data loader fails instead of hanging when its stream goes idle
(finetune.data_timeout_s; the reference's loader blocks forever, finetune_loop.py:92-115)."""
import threading
import time
from queue import Queue

import torch

from pipelinerl_amd import streams
from pipelinerl_amd.finetune_loop import run_data_loader


def _spec(tmp_path):
    streams.reset_streams_backend()
    streams.set_streams_backend("files")
    return streams.SingleStreamSpec(exp_path=tmp_path, topic="training_data")


def test_idle_stream_puts_timeout_error(tmp_path):
    spec = _spec(tmp_path)
    with streams.write_to_streams(spec):  # the file exists, but no line ever arrives
        pass
    q: Queue = Queue(maxsize=1)
    t0 = time.time()
    run_data_loader(spec, q, torch.device("cpu"), stop=None, timeout=0.3)
    item = q.get(timeout=5)
    assert isinstance(item, TimeoutError) and "training_data" in str(item)
    assert time.time() - t0 < 5


def test_missing_stream_puts_timeout_error(tmp_path):
    q: Queue = Queue(maxsize=1)
    run_data_loader(_spec(tmp_path), q, torch.device("cpu"), stop=None, timeout=0.3)
    assert isinstance(q.get(timeout=5), TimeoutError)


def test_stopped_loader_puts_nothing(tmp_path):
    spec = _spec(tmp_path)
    with streams.write_to_streams(spec):
        pass
    stop = threading.Event()
    stop.set()
    q: Queue = Queue(maxsize=1)
    run_data_loader(spec, q, torch.device("cpu"), stop=stop, timeout=0.2)
    assert q.empty()
