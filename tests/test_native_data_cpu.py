"""libprl_data (include/prl_data.h): the training_data stream codec and the preprocessing
arithmetic in C++, against the Python path they replace.

* decode: ``native_data.decode_batch(line)`` must equal ``PipelineBatchEncoding(**json.loads(line))``
  (pipelinerl/finetune_loop.py:92-115 + types.py:48-117's numpy.asarray -> torch.as_tensor) in
  dtype, shape and every bit, including NaN / Infinity literals, ints in float fields, floats in
  int fields, exponents, whitespace, empty lists; what the native path does not take (ragged
  lists, bools, strings) goes through json and fails or succeeds exactly as Python does;
* encode: ``streams.dumps`` (native) is byte-identical to json.dumps of the lists;
* populate_rl_data's group statistics vs pandas' groupby (the reference's own aggregation,
  rl/__init__.py:408-416), collate_packed's token layout vs a direct restatement.
"""

import ctypes
import json
import re

import numpy as np
import pytest
import torch

from conftest import GOLDEN  # noqa: F401  (puts the package on sys.path)


def _fields(b):
    from pipelinerl_amd.finetune.types import PipelineBatchEncoding
    return {k: getattr(b, k) for k in PipelineBatchEncoding.model_fields}


def _assert_same(b1, b2):
    f1, f2 = _fields(b1), _fields(b2)
    for k in f1:
        v1, v2 = f1[k], f2[k]
        if isinstance(v1, torch.Tensor):
            assert isinstance(v2, torch.Tensor), k
            assert v1.dtype == v2.dtype and v1.shape == v2.shape, (k, v1.dtype, v2.dtype, v1.shape, v2.shape)
            # bit-exact, NaNs included
            if v1.dtype.is_floating_point:
                assert torch.equal(v1.view(torch.int32) if v1.dtype == torch.float32 else v1.view(torch.int64),
                                   v2.view(torch.int32) if v2.dtype == torch.float32 else v2.view(torch.int64)), k
            else:
                assert torch.equal(v1, v2), k
        else:
            assert v1 == v2, k


def _python_decode(line):
    from pipelinerl_amd.finetune.types import PipelineBatchEncoding
    return PipelineBatchEncoding(**json.loads(line))


def _packed_doc(rng, T, as_lists=True):
    f32 = lambda x: x.astype(np.float32).astype(np.float64).tolist()  # noqa: E731
    return dict(
        input_ids=[rng.integers(0, 151643, T).tolist()], attention_mask=[[1] * T],
        labels=[np.where(rng.random(T) < 0.2, -100, rng.integers(0, 151643, T)).tolist()],
        position_ids=[np.arange(T).tolist()], rewards=[f32(rng.random(T))], advantages=[f32(rng.normal(0, 1, T))],
        ref_logprobs=[f32(-rng.exponential(2, T))], old_logprobs=[(-rng.exponential(2, T)).tolist()],
        group_tokens=[[1000.0] * T], num_labels=[[float(T // 2)] * T], overflow=[[0.0] * T], model_version=7,
        sentinel=False, padding=0, is_packed=True, seq_boundaries=[0, T // 3, T], pixel_values=None,
        image_grid_thw=None)


def test_decode_packed_batch_bit_exact():
    from pipelinerl_amd import native_data
    from pipelinerl_amd.streams import dumps

    rng = np.random.default_rng(0)
    for T in (1, 7, 4096):
        line = dumps(_packed_doc(rng, T)).encode()
        for threads in (1, 4):
            _assert_same(_python_decode(line), native_data.decode_batch(line, threads=threads))


def test_decode_value_edge_cases():
    """Literal forms and conversions the reference's json + numpy path applies."""
    from pipelinerl_amd import native_data

    doc = _packed_doc(np.random.default_rng(1), 12)
    doc["rewards"] = [[0, 1, -2, 9007199254740993, 1e-05, 1E5, -0.0, 2.5e-310, 1e308, 3.4028235677973366e+38,
                       0.1, 123456789012345678]]
    doc["advantages"] = [[float("nan"), float("inf"), -float("inf")] + [0.5] * 9]
    doc["input_ids"] = [[1.7, -1.7, 2.0, 3, 4e3, -0.0, 7, 8, 9, 10, 11, 12]]  # floats in an int field: truncation
    doc["position_ids"] = [[2 ** 62, -2 ** 62] + list(range(10))]
    line = json.dumps(doc)  # Python's writer: NaN / Infinity literals, spaces after separators
    _assert_same(_python_decode(line), native_data.decode_batch(line.encode()))
    line = json.dumps(doc, indent=2)  # any whitespace
    _assert_same(_python_decode(line), native_data.decode_batch(line.encode()))


def test_decode_unpacked_and_empty_arrays():
    from pipelinerl_amd import native_data

    rng = np.random.default_rng(2)
    B, L = 3, 9
    doc = {k: (np.zeros((B, L)) if k != "labels" else np.full((B, L), -100)).tolist()
           for k in ("input_ids", "attention_mask", "labels", "rewards", "advantages", "ref_logprobs",
                     "old_logprobs", "group_tokens", "num_labels", "overflow")}
    doc["old_logprobs"] = rng.normal(size=(B, L)).tolist()
    doc.update(model_version=1, is_packed=False)
    line = json.dumps(doc, separators=(",", ":"))
    _assert_same(_python_decode(line), native_data.decode_batch(line.encode()))
    # empty lists: [] and [[]]
    doc2 = dict(doc, input_ids=[[]], attention_mask=[[]], labels=[[]], rewards=[], advantages=[[]],
                ref_logprobs=[[]], old_logprobs=[[]], group_tokens=[[]], num_labels=[[]], overflow=[[]],
                seq_boundaries=[])
    line = json.dumps(doc2)
    _assert_same(_python_decode(line), native_data.decode_batch(line.encode()))


@pytest.mark.parametrize("bad,exc", [
    ({"rewards": [[1.0, 2.0], [3.0]]}, ValueError),        # ragged: numpy refuses (inhomogeneous shape)
    ({"rewards": [["a", "b"]]}, TypeError),                # strings: torch refuses numpy str_
])
def test_decode_rejects_what_python_rejects(bad, exc):
    from pipelinerl_amd import native_data

    doc = _packed_doc(np.random.default_rng(3), 2)
    doc.update(bad)
    line = json.dumps(doc)
    with pytest.raises(exc):
        _python_decode(line)
    with pytest.raises(exc):
        native_data.decode_batch(line.encode())


def test_decode_bools_and_non_numeric_fields_follow_python():
    from pipelinerl_amd import native_data

    doc = _packed_doc(np.random.default_rng(4), 3)
    doc["attention_mask"] = [[True, False, True]]  # np.asarray(bools) -> long
    doc["sentinel"] = True
    line = json.dumps(doc)
    _assert_same(_python_decode(line), native_data.decode_batch(line.encode()))
    # a generic document: members order kept, nothing numeric requested
    d = native_data.decode_document(b'{"kind": "weight_update_request", "version": 3, "x": [1, 2]}', {})
    assert d == {"kind": "weight_update_request", "version": 3, "x": [1, 2]}


def _f32(x):
    with np.errstate(over="ignore"):
        return x.astype(np.float32)


def test_encode_byte_identical_to_json():
    from pipelinerl_amd import native_data
    from pipelinerl_amd.streams import _jsonable

    rng = np.random.default_rng(5)
    bits32 = rng.integers(0, 2 ** 32, 4096, dtype=np.uint64).astype(np.uint32).view(np.float32)
    bits64 = rng.integers(0, 2 ** 63, 4096, dtype=np.uint64).view(np.float64)
    specials = np.array([0.0, -0.0, 1e-5, 1e-4, 123.0, 1e16, 9999999999999998.0, 1e22, 5e-324, np.nan, np.inf, -np.inf,
                         0.1, 1.0 / 3, 2.0 ** 60, 1.7976931348623157e308], np.float64)
    data = {
        "f32": torch.from_numpy(bits32.reshape(64, 64)), "f64": torch.from_numpy(bits64)[None],
        "specials": specials, "f32specials": _f32(specials),
        "i64": torch.tensor([[0, -1, 2 ** 63 - 1, -2 ** 63, 151643]]), "i32": np.array([0, -2 ** 31, 2 ** 31 - 1], np.int32),
        "empty": torch.zeros(0), "empty2": torch.zeros(1, 0), "empty3": np.zeros((2, 0, 3)),
        "scalar": torch.tensor(3.5), "bf16": torch.tensor([1.5, 2.25], dtype=torch.bfloat16),
        "text": "a \"quoted\" string", "nested": {"a": [1, 2.5]}, "none": None, "flag": True,
    }
    want = json.dumps(_jsonable(data), separators=(",", ":"))
    assert native_data.encode_document(data) == want


def test_stream_roundtrip_through_the_loader(tmp_path):
    """FileStreamWriter (native encode) -> run_data_loader (native decode) on CPU == the
    PipelineBatchEncoding written; the json decode (PRL_NATIVE_DECODE=0) agrees."""
    import os
    from queue import Queue

    from pipelinerl_amd.finetune.types import PipelineBatchEncoding
    from pipelinerl_amd.finetune_loop import run_data_loader
    from pipelinerl_amd.streams import (SingleStreamSpec, reset_streams_backend, set_streams_backend,
                                        write_to_streams)

    reset_streams_backend()
    set_streams_backend("files")
    spec = SingleStreamSpec(exp_path=tmp_path, topic="training_data")
    rng = np.random.default_rng(6)
    batches = [PipelineBatchEncoding(**_packed_doc(rng, T)) for T in (5, 300)]
    with write_to_streams(spec, "w") as w:
        for b in batches:
            w.write(b)
    for native in ("1", "0"):
        os.environ["PRL_NATIVE_DECODE"] = native
        q = Queue()
        run_data_loader(spec, q, torch.device("cpu"), timeout=0.5)
        for b in batches:
            got, ntok, nseq = q.get(timeout=5)
            _assert_same(b, got)
            assert ntok == b.attention_mask.numel() and nseq == 2
        assert isinstance(q.get(timeout=5), TimeoutError)
    os.environ.pop("PRL_NATIVE_DECODE")
    reset_streams_backend()


def test_group_stats_match_pandas():
    """prl_rl_group_stats vs the reference's own aggregation (pandas groupby mean / std / mean,
    rl/__init__.py:408-416) on random rewards and lengths, groups interleaved, one singleton."""
    import pandas as pd

    from pipelinerl_amd import native_data

    rng = np.random.default_rng(7)
    n, G = 999, 40
    group = rng.integers(0, G - 1, n)
    group[17] = G - 1  # a single-rollout group: std NaN
    reward = np.where(rng.random(n) < 0.5, rng.integers(0, 2, n).astype(float), rng.normal(0.3, 2.0, n))
    length = rng.integers(1, 9000, n)
    mean, std, tok = native_data.rl_group_stats(group, G, reward, length)
    df = pd.DataFrame({"g": group, "r": reward, "n": length})
    agg = df.groupby("g").agg(m=("r", "mean"), s=("r", "std"), t=("n", "mean"))
    np.testing.assert_array_equal(mean, agg["m"].to_numpy())
    np.testing.assert_array_equal(tok, agg["t"].to_numpy())
    np.testing.assert_allclose(std, agg["s"].to_numpy(), rtol=1e-14, atol=0, equal_nan=True)
    assert np.isnan(std[G - 1])


def test_collate_arrays_layout():
    from pipelinerl_amd import native_data

    rng = np.random.default_rng(8)
    lens = np.array([5, 0, 3, 1, 7])
    ids = rng.integers(0, 100, lens.sum())
    labels = np.where(rng.random(lens.sum()) < 0.3, -100, ids)
    o_ids, o_lab, o_pos, bounds = native_data.collate_arrays(lens, ids, labels, -7)
    assert bounds.tolist() == [0, 5, 5, 8, 9, 16] and bounds.dtype == np.int32
    assert o_ids.tolist() == ids.tolist()
    want = labels.copy()
    for i in range(1, len(lens)):
        if lens[i]:
            want[bounds[i]] = -7
    assert o_lab.tolist() == want.tolist()
    assert o_pos.tolist() == [0, 1, 2, 3, 4, 0, 1, 2, 0, 0, 1, 2, 3, 4, 5, 6]
    with pytest.raises(native_data.PrlDataError):
        native_data.collate_arrays(lens, ids[:-1], labels)


def test_concat_lists_fast_path_and_fallback():
    from pipelinerl_amd import native_data
    from pipelinerl_amd.finetune.data import _concat

    seqs = [[1, 2, 3], [], [2 ** 40, -5]]
    assert native_data.concat_lists(seqs, native_data.DT_I64, 5).tolist() == [1, 2, 3, 2 ** 40, -5]
    f = native_data.concat_lists([[0.5, 1], [2 ** 60 + 1]], native_data.DT_F64, 3)
    assert f.tolist() == [0.5, 1.0, float(2 ** 60 + 1)]
    # bools / numpy scalars / overflow: not taken natively; _concat converts them like numpy
    assert native_data.concat_lists([[True, 2]], native_data.DT_I64, 2) is None
    assert native_data.concat_lists([[2 ** 70]], native_data.DT_I64, 1) is None
    assert _concat([[True, 2], np.array([3, 4])], "q", np.int64).tolist() == [1, 2, 3, 4]
    assert _concat([[0.5, np.float32(0.25)], 3.0], "d", np.float64).tolist() == [0.5, 0.25, 3.0]


def test_data_library_exports_header_symbols():
    from pipelinerl_amd import native_data

    lib = native_data.load()
    text = native_data.HEADER_PATH.read_text()
    declared = sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(prl_\w+)\s*\(", text, flags=re.M)))
    assert len(declared) == 9, declared
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.prl_data_abi_version() == native_data.ABI
    assert lib.prl_data_error_string(5001).decode() == "invalid argument"
    n = ctypes.c_int32(0)
    assert lib.prl_json_members(None, 0, None, 0, ctypes.byref(n)) == 5001
    assert lib.prl_rl_group_stats(-1, None, 0, None, None, None, None, None) == 5001
    assert lib.prl_json_array_fill(None, 1, 1) == 5001


def test_stream_writer_falls_back_to_json_without_the_library(monkeypatch):
    """A process where libprl_data neither loads nor builds (an actor host without g++) still
    writes stream lines: json.dumps, the same bytes the native encoder writes."""
    from pipelinerl_amd import native_data, streams
    from pipelinerl_amd.finetune.types import PipelineBatchEncoding

    b = PipelineBatchEncoding(input_ids=torch.tensor([[1, 2, 3]]), labels=torch.tensor([[-100, 2, 3]]),
                              attention_mask=torch.ones(1, 3, dtype=torch.long),
                              rewards=torch.tensor([[0.0, 1.0, 1.0]]), advantages=torch.tensor([[0.0, 0.5, 0.5]]),
                              ref_logprobs=torch.tensor([[0.0, -0.25, -1e-5]]),
                              old_logprobs=torch.tensor([[0.0, -0.25, -1e-5]]),
                              group_tokens=torch.ones(1, 3), num_labels=torch.full((1, 3), 2.0),
                              overflow=torch.zeros(1, 3), model_version=3)
    native = streams.dumps(b)

    def broken():
        raise native_data.PrlDataError("no g++ here")

    monkeypatch.setattr(streams, "_NATIVE_ENCODE", [None])
    monkeypatch.setattr(native_data, "load", broken)
    assert streams.dumps(b) == native
    assert streams._NATIVE_ENCODE[0] is False  # tried once per process
