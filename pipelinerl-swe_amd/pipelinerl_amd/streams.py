"""Inter-process streams, files backend (wire-compatible with pipelinerl/streams.py:238-346).

Layout: <exp_path>/streams/<topic>/<instance>/<partition>/0.jsonl, one JSON document per
line, appended and flushed per message.  The trainer reads its ``training_data`` partition
(one per trainer rank) and writes SamplesProcessed / WeightUpdateSuccess to the
``weight_update_request`` topic.  Pydantic models are dumped with tensors converted to
(nested) lists, which is what orjson's OPT_SERIALIZE_NUMPY produces for the reference.
The Redis backend is out of scope.
"""

from __future__ import annotations

import json
import logging
import os
import time
from pathlib import Path
from typing import Any, Iterator, Literal

import numpy as np
import torch
from pydantic import BaseModel

logger = logging.getLogger(__name__)

REREAD_DELAY = 0.1
RECHECK_DELAY = 3.0

_backend: str | None = None


def set_streams_backend(backend: str, **kwargs) -> None:
    global _backend
    if _backend is not None and _backend != backend:
        raise ValueError("Backend already set. Cannot change it.")
    if backend == "redis":
        raise NotImplementedError("the redis streams backend is not part of this build; use backend=files")
    if backend != "files":
        raise ValueError(f"Invalid backend: {backend}. Only 'redis' and 'files' are supported.")
    _backend = backend


def reset_streams_backend() -> None:  # tests
    global _backend
    _backend = None


class SingleStreamSpec(BaseModel):
    exp_path: Path
    topic: str
    instance: int = 0
    partition: int = 0

    def __str__(self):
        return f"{self.topic}/{self.instance}/{self.partition}"


class StreamRangeSpec(BaseModel):
    exp_path: Path
    topic: str
    instance: int = 0
    partition_range: tuple[int, int]


def stream_dir(exp_path: Path, topic: str, instance: int, partition: int) -> Path:
    return Path(exp_path) / "streams" / topic / str(instance) / str(partition)


def stream_file(d: Path, shard_id: int = 0) -> Path:
    return d / f"{shard_id}.jsonl"


def _jsonable(x: Any) -> Any:
    if isinstance(x, BaseModel):
        x = x.model_dump()
    if isinstance(x, dict):
        return {k: _jsonable(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_jsonable(v) for v in x]
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().tolist()
    if isinstance(x, np.ndarray):
        return x.tolist()
    if isinstance(x, (np.integer,)):
        return int(x)
    if isinstance(x, (np.floating,)):
        return float(x)
    if isinstance(x, Path):
        return str(x)
    return x


_NATIVE_ENCODE: list = [None]  # None: not tried yet; False: libprl_data unavailable in this process


def _native_encoder():
    if _NATIVE_ENCODE[0] is None:
        from . import native_data
        try:
            native_data.load()
            _NATIVE_ENCODE[0] = native_data
        except Exception as e:  # noqa: BLE001 - no library / toolchain on this host: json (same bytes)
            logger.warning(f"libprl_data unavailable ({e}); stream lines are written with json.dumps")
            _NATIVE_ENCODE[0] = False
    return _NATIVE_ENCODE[0] or None


def dumps(data: Any) -> str:
    """One stream line.  A pydantic model or dict (a PipelineBatchEncoding, a message) goes
    through libprl_data's encoder, byte-identical to json.dumps of the lists (numeric tensors /
    arrays formatted natively); anything else — or any line on a host where libprl_data neither
    loads nor builds (an actor host without g++) — through json, which writes the same bytes."""
    if isinstance(data, BaseModel):
        data = data.model_dump()
    if isinstance(data, dict) and all(isinstance(k, str) for k in data):
        enc = _native_encoder()
        if enc is not None:
            return enc.encode_document(data)
    return json.dumps(_jsonable(data), separators=(",", ":"))


class FileStreamWriter:
    def __init__(self, stream: SingleStreamSpec, mode: Literal["w", "a"] = "a"):
        self.stream = stream
        self.mode = mode

    def __enter__(self):
        d = stream_dir(self.stream.exp_path, self.stream.topic, self.stream.instance, self.stream.partition)
        os.makedirs(d, exist_ok=True)
        self._file = open(stream_file(d), self.mode)
        return self

    def __exit__(self, *exc):
        self._file.close()

    def write(self, data: Any, partition: int | None = None) -> None:
        if partition is not None:
            raise ValueError("a single-stream writer has no partitions")
        self._file.write(dumps(data))
        self._file.write("\n")
        self._file.flush()


class RoundRobinFileStreamWriter:
    def __init__(self, streams: StreamRangeSpec, mode: Literal["w", "a"] = "a"):
        a, b = streams.partition_range
        self._writers = [FileStreamWriter(SingleStreamSpec(exp_path=streams.exp_path, topic=streams.topic,
                                                           instance=streams.instance, partition=i), mode)
                         for i in range(a, b)]
        self._next = 0

    def __enter__(self):
        for w in self._writers:
            w.__enter__()
        return self

    def __exit__(self, *exc):
        for w in self._writers:
            w.__exit__(*exc)

    def write(self, data: Any, partition: int | None = None) -> None:
        if partition is not None:
            if not 0 <= partition < len(self._writers):
                raise ValueError(f"Invalid partition {partition}. Must be between 0 and {len(self._writers) - 1}")
            self._writers[partition].write(data)
        else:
            self._writers[self._next].write(data)
            self._next = (self._next + 1) % len(self._writers)


class FileStreamReader:
    """Tails a JSONL file from the beginning; blocks (polling) for new complete lines."""

    def __init__(self, stream: SingleStreamSpec, poll: float = REREAD_DELAY, timeout: float | None = None):
        self.stream = stream
        self.poll = poll
        self.timeout = timeout

    def __enter__(self):
        d = stream_dir(self.stream.exp_path, self.stream.topic, self.stream.instance, self.stream.partition)
        self._path = stream_file(d)
        t0 = time.time()
        while not self._path.exists():
            if self.timeout is not None and time.time() - t0 > self.timeout:
                raise TimeoutError(f"stream {self.stream} was not created")
            logger.warning(f"Waiting for {self.stream} to be created")
            time.sleep(min(RECHECK_DELAY, self.poll * 10))
        self._file = open(self._path, "rb")
        return self

    def __exit__(self, *exc):
        self._file.close()

    def read_lines(self) -> Iterator[bytes]:
        """Complete lines, as bytes (a line without its newline is still being written: wait
        for it).  Returns after `timeout` s without a new line."""
        pos = self._file.tell()
        idle = time.time()
        while True:
            line = self._file.readline()
            if line.endswith(b"\n"):
                pos = self._file.tell()
                idle = time.time()
                yield line
            else:
                if self.timeout is not None and time.time() - idle > self.timeout:
                    return
                self._file.seek(pos)
                time.sleep(self.poll)

    def read(self) -> Iterator[Any]:
        for line in self.read_lines():
            yield json.loads(line)


def _check_backend():
    if _backend is None:
        raise ValueError("Backend not set. Please call set_streams_backend() first.")


def read_stream(stream: SingleStreamSpec, timeout: float | None = None) -> FileStreamReader:
    _check_backend()
    if not isinstance(stream, SingleStreamSpec):
        raise ValueError(f"Invalid stream spec: {stream}")
    return FileStreamReader(stream, timeout=timeout)


def write_to_streams(streams: SingleStreamSpec | StreamRangeSpec, mode: Literal["w", "a"] = "a"):
    _check_backend()
    if isinstance(streams, SingleStreamSpec):
        return FileStreamWriter(streams, mode)
    if isinstance(streams, StreamRangeSpec):
        return RoundRobinFileStreamWriter(streams, mode)
    raise ValueError(f"Invalid stream spec: {streams}")
