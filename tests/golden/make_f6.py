"""F6 fixture: the preprocessor's sequence-packing write loop — per-trainer sample quotas,
greedy packing up to ``seq_length``, sentinel batches, round-robin over lead trainers
(pipelinerl/preprocess.py:557-613, the ``seq_packing`` branch) — run on synthetic populated
rollouts, chunk by chunk, as the reference runs it.

Run in the build container only (reads /root/reference; writes data):

    PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_f6.py

preprocess.py does not import here (litellm, tapeagents), and the loop is not a function of its
own: the ``while`` statement of the write loop is taken from the file's syntax tree and executed
in a namespace holding the loop's state, initialised as preprocess.py:430-449 does (from zero
published samples) and carried from chunk to chunk.  Its collaborators are the reference's own
``collate_packed`` / ``create_sentinel_batch``; ``write_micro_batch_slices`` records the
(lead trainer, micro-batch) it is given; ``max_model_version`` is recomputed after each chunk
is appended over the entries still queued (:542-546).  For seq_parallel > 1 each write's
slices (the reference's ``make_slices``, as ``write_micro_batch_slices`` sends them) are kept too.  After each chunk the loop is re-entered
while entries remain (the outer loop does, the trainer keeping up).
"""

from __future__ import annotations

import ast
import json
import logging
import sys
import types
from collections import deque
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REF = Path("/root/reference/pipelinerl/preprocess.py")

if "omegaconf" not in sys.modules:  # finetune/data.py names DictConfig as a type only
    _om = types.ModuleType("omegaconf")
    _om.DictConfig = dict
    sys.modules["omegaconf"] = _om

EOS = 50
FIELDS = ["input_ids", "labels", "position_ids", "attention_mask", "rewards", "advantages", "ref_logprobs",
          "old_logprobs", "group_tokens", "num_labels", "overflow"]


def write_loop_code():
    tree = ast.parse(REF.read_text())
    for node in ast.walk(tree):
        if isinstance(node, ast.While) and "processed_entries_queue" in ast.unparse(node.test) \
                and "batch_done" in ast.unparse(node.test):
            return compile(ast.Module(body=[node], type_ignores=[]), str(REF), "exec")
    raise RuntimeError("write loop not found")


def rollouts(seed: int, n_groups: int, attempts: int, max_len: int):
    from pipelinerl.finetune.rl import RLConfig, populate_rl_data, prepare_rl_fields

    rng = np.random.default_rng(seed)
    data = []
    for g in range(n_groups):
        for a in range(attempts):
            p = int(rng.integers(2, 8))
            c = int(rng.integers(1, max_len - p))
            ids = rng.integers(0, EOS, p + c).tolist()
            if rng.random() < 0.75:
                ids[-1] = EOS
            lps = np.round(rng.normal(-1.0, 0.5, c), 3).tolist()
            enc = prepare_rl_fields({"input_ids": ids, "labels": [-100] * p + ids[p:], "attention_mask": [1] * len(ids)},
                                    float(rng.integers(0, 2)), lps, lps)
            # model versions move forward, with a late straggler now and then
            enc.update(group_id=f"g{g}", rollout_index=a, step_index=0,
                       model_version=int(g // 2 - (2 if rng.random() < 0.1 else 0)))
            data.append(enc)
    return populate_rl_data(data, EOS, RLConfig(divide_advantage_by_std=False))


def run_reference(data, chunk_sizes, num_trainers, seq_parallel, per_lead, seq_length):
    from pipelinerl.finetune.data import collate_packed
    from pipelinerl.finetune.utils import create_sentinel_batch

    writes = []

    def write_micro_batch_slices(lead_trainer_id, data_writer, micro_batch, seq_parallel):
        writes.append((lead_trainer_id, micro_batch))

    num_leads = num_trainers // seq_parallel
    cfg = types.SimpleNamespace(finetune=types.SimpleNamespace(seq_packing=True, seq_length=seq_length,
                                                               seq_parallel=seq_parallel, train_batch_size=1),
                                preprocess=types.SimpleNamespace(dataset_buffer_size=0))
    ns = dict(processed_entries_queue=deque(), trainer_id=0, published_samples=0,
              samples_per_trainer={i: 0 for i in range(0, num_trainers, seq_parallel)},
              samples_per_lead_per_step=per_lead, train_batch_size=per_lead * num_leads,
              batch_boundary=per_lead * num_leads, target_samples_per_lead=per_lead, max_model_version=None,
              time_to_write=False, current_batch=[], current_length=0, cfg=cfg, num_trainers=num_trainers,
              tokenizer=types.SimpleNamespace(eos_token_id=EOS), data_writer=None, logger=logging.getLogger("f6"),
              create_sentinel_batch=create_sentinel_batch, collate_packed=collate_packed, collate=None,
              write_micro_batch_slices=write_micro_batch_slices)
    code = write_loop_code()
    pos = 0
    for size in chunk_sizes:
        for e in data[pos:pos + size]:
            ns["processed_entries_queue"].append(e)
            q = ns["processed_entries_queue"]
            ns["max_model_version"] = max(x["model_version"] for x in q) if q else 0
        pos += size
        while ns["processed_entries_queue"]:
            ns["batch_done"] = False
            exec(code, ns)
    return writes


def encode(tid, b):
    rec = {"trainer": int(tid), "sentinel": bool(b.sentinel), "model_version": int(b.model_version),
           "padding": int(b.padding), "is_packed": bool(b.is_packed),
           "seq_boundaries": [int(x) for x in b.seq_boundaries.tolist()]}
    for f in FIELDS:
        v = getattr(b, f, None)
        if v is not None:
            rec[f] = [float(x) for x in v.reshape(-1).tolist()] if v.is_floating_point() else \
                [int(x) for x in v.reshape(-1).tolist()]
    return rec


def main():
    cases = []
    for name, seed, groups, attempts, max_len, chunks, nt, sp, per_lead, seq_len in (
            ("one_trainer", 1, 6, 4, 30, [5, 7, 12], 1, 1, 6, 64),
            ("four_trainers", 2, 8, 4, 40, [3, 9, 20], 4, 1, 4, 80),
            ("seq_parallel_2", 3, 6, 4, 30, [8, 16], 4, 2, 6, 64),
            ("quota_in_one_batch", 4, 4, 8, 12, [32], 2, 1, 8, 256),
            ("late_versions", 5, 4, 4, 20, [6, 10], 2, 1, 4, 40)):
        data = rollouts(seed, groups, attempts, max_len)
        if name == "late_versions":  # the second chunk comes from an older policy: the sentinels
            for i, e in enumerate(data):  # carry the max over what is still queued, not the max seen
                e["model_version"] = 7 if i < 6 else 3
        writes = run_reference(json.loads(json.dumps(data)), chunks, nt, sp, per_lead, seq_len)
        # what write_micro_batch_slices sends each trainer of a lead's group (preprocess.py:327-338):
        # the reference's own PipelineBatchEncoding.make_slices (types.py:144-180)
        slices = [[encode(t + i, sl) for i, sl in enumerate(b.make_slices(sp))] if sp > 1 else []
                  for t, b in writes]
        cases.append({"name": name, "num_trainers": nt, "seq_parallel": sp, "samples_per_lead_per_step": per_lead,
                      "seq_length": seq_len, "chunks": chunks, "input": data,
                      "writes": [encode(t, b) for t, b in writes], "slices": slices})
        print(name, len(writes), "writes,", sum(w[1].sentinel for w in writes), "sentinels")
    (HERE / "f6_packing.json").write_text(json.dumps({"source": "pipelinerl/preprocess.py:557-613", "eos": EOS,
                                                      "cases": cases}))


if __name__ == "__main__":
    main()
