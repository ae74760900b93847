"""Generate golden vectors by running the REFERENCE rl_step in the build container.

Run (build container only; /root/reference is not on the GPU box):

    PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference's ``rl_step`` (pipelinerl/finetune/rl/__init__.py:130-377) is driven through a
stub model whose forward returns fixed logits (and value-head outputs) held as
``nn.Parameter``s, so ``loss.backward()`` yields the reference dlogits / dvalues.  The
per-token new log-probs and entropy are captured with a TorchFunctionMode at the
reference's own ``torch.gather`` / ``.sum(dim=-1)`` calls (rl/__init__.py:204, :208).

Fixtures written next to this script (data only: inputs and reference outputs):
  f1_inputs.npz   tiny packed + unpacked batches, fp32 logits (T=37, V=384)
  f1_outputs.npz  per case: dlogits, dvalues, new_logprobs, entropy
  f1_cases.json   per case: config, step, loss, stats
  f2_*.npz/json   V=151936, T=16, bf16 logits from oracle/synth.py (regenerable);
                  outputs of the bf16 reference path and of the fp32 path on the same
                  bf16-rounded logits (projections of dlogits only, to stay small)
  f3_*.json       populate_rl_data + collate_packed on synthetic rollouts
"""

from __future__ import annotations

import itertools
import json
import os
import sys
import types
from pathlib import Path

import numpy as np
import torch
from torch.overrides import TorchFunctionMode

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parents[1]))  # repo root, for oracle.synth

from oracle import synth  # noqa: E402

# omegaconf is not installed here; finetune/data.py only needs DictConfig as a type name.
if "omegaconf" not in sys.modules:
    _om = types.ModuleType("omegaconf")
    _om.DictConfig = dict
    sys.modules["omegaconf"] = _om

from pipelinerl.finetune.rl import RLConfig, rl_step, populate_rl_data  # noqa: E402
from pipelinerl.finetune.types import PipelineBatchEncoding  # noqa: E402


class _Capture(TorchFunctionMode):
    def __init__(self):
        super().__init__()
        self.gather = None
        self.negent = None

    def __torch_function__(self, func, types_, args=(), kwargs=None):
        kwargs = kwargs or {}
        out = func(*args, **kwargs)
        if func is torch.gather:
            self.gather = out.detach().clone()
        elif func is torch.Tensor.sum and kwargs.get("dim") == -1 and args[0].dim() == 3:
            self.negent = out.detach().clone()
        return out


class LogitsModel(torch.nn.Module):
    def __init__(self, logits: torch.Tensor, values: torch.Tensor | None):
        super().__init__()
        self.logits = torch.nn.Parameter(logits)
        if values is not None:
            self.value_head = torch.nn.Parameter(values)

    def forward(self, **kw):
        return types.SimpleNamespace(logits=self.logits, value=getattr(self, "value_head", None))


def run_reference(logits_np, batch_np, cfg, step, max_step, values_np=None, dtype=torch.float32):
    batch = PipelineBatchEncoding(**{k: v for k, v in batch_np.items()})
    logits = torch.tensor(logits_np, dtype=torch.float32).to(dtype)
    values = None if values_np is None else torch.tensor(values_np, dtype=torch.float32)
    model = LogitsModel(logits, values)
    cap = _Capture()
    with cap:
        loss, stats = rl_step(model, batch, step, max_step, RLConfig(**cfg))
    loss.backward()
    out = dict(loss=float(loss.item()), stats={k: float(v) for k, v in stats.items()},
               new_logprobs=cap.gather[..., 0].float().numpy() if cap.gather is not None else None,
               entropy=(-cap.negent).float().numpy() if cap.negent is not None else None,
               dlogits=model.logits.grad.float().numpy())
    if values is not None:
        out["dvalues"] = model.value_head.grad.float().numpy()
    return out


def f1_batches():
    T, V = 37, 384
    seq_lens, prompt_lens = [13, 12, 12], [4, 5, 3]
    b = synth.packed_rl_batch(11, seq_lens, prompt_lens, id_range=V, eos=7)
    rng = np.random.default_rng(1234)
    logits = (rng.standard_normal((1, T, V)) * 2.5).astype(np.float32)
    # true fp32 log-probs of the targets, for realistic old/ref
    x = logits[0, :-1].astype(np.float64)
    lse = np.log(np.exp(x - x.max(-1, keepdims=True)).sum(-1)) + x.max(-1)
    tl = x[np.arange(T - 1), b["input_ids"][0, 1:]] - lse
    lab = b["labels"][0] != -100
    old = np.zeros(T, np.float32)
    ref = np.zeros(T, np.float32)
    old[1:] = tl + rng.normal(0, 0.35, T - 1)
    ref[1:] = tl + rng.normal(0, 0.6, T - 1)
    ref[[9, 20]] += np.array([13.0, -12.0])  # trigger the KL clamp at C=10 and C=5
    old[[5, 30]] += np.array([2.0, -1.5])  # big ratios for PPO clipping
    old[~lab] = 0.0
    ref[~lab] = 0.0
    b["old_logprobs"] = old[None]
    b["ref_logprobs"] = ref[None]
    b["advantages"][0, 26:] = 0.0  # a zero-advantage sequence (PPO min() ties)
    values = (rng.standard_normal((1, T)) * 0.3 + 0.5).astype(np.float32)

    # unpacked: 2 rows of length 16 (collate pads labels with -100 and RL fields with 0)
    L = 16
    ub = {k: np.zeros((2, L), np.float32) for k in
          ["rewards", "advantages", "ref_logprobs", "old_logprobs", "group_tokens", "num_labels", "overflow"]}
    ids = synth.token_ids(5, 2 * L, V).reshape(2, L)
    labels = ids.copy()
    labels[0, :5] = -100
    labels[0, 13:] = -100  # right padding
    labels[1, :3] = -100
    ub["rewards"][0, :13] = 1.0
    ub["rewards"][1, :] = 0.0
    ub["advantages"][0, :13] = 0.5
    ub["advantages"][1, :] = -0.5
    ub["group_tokens"][:] = 14.5
    ub["num_labels"][0, :13] = 8
    ub["num_labels"][1, :] = 13
    ulog = (rng.standard_normal((2, L, V)) * 2.0).astype(np.float32)
    ux = ulog[:, :-1].astype(np.float64)
    ulse = np.log(np.exp(ux - ux.max(-1, keepdims=True)).sum(-1)) + ux.max(-1)
    utl = np.take_along_axis(ux, ids[:, 1:, None], -1)[..., 0] - ulse
    um = labels[:, 1:] != -100
    ub["old_logprobs"][:, 1:] = np.where(um, utl + rng.normal(0, 0.2, utl.shape), 0)
    ub["ref_logprobs"][:, 1:] = np.where(um, utl + rng.normal(0, 0.3, utl.shape), 0)
    ub.update(input_ids=ids, labels=labels, attention_mask=np.ones((2, L), np.int64),
              is_packed=False, model_version=0)
    uvalues = (rng.standard_normal((2, L)) * 0.3).astype(np.float32)
    return (logits, b, values), (ulog, ub, uvalues)


def f1_cases():
    cases = []
    for pol, kl, tau, ent, vh in itertools.product(["ppo", "reinforce"], [0.0, 0.1], [1.0, 0.7],
                                                  [0.0, 0.01], [False, True]):
        cases.append(dict(batch="packed", value_head=vh, step=0, max_step=10,
                          cfg=dict(policy_loss=pol, kl_coef=kl, final_kl_coef=kl, temperature=tau,
                                   entropy_bonus=ent, final_entropy_bonus=ent, batch_size=4,
                                   epsilon=0.2, value_loss_coef=0.1 if vh else 0.0)))
    grpo = dict(policy_loss="ppo", divide_advantage_by_std=False, kl_coef=0.0, final_kl_coef=0.0,
                entropy_bonus=0.0, epsilon=4, use_advantages=True, relu_log_p_weights=False,
                clamp_log_ratio_ref_new_value=5, temperature=1.0, overlong_filtering=False,
                batch_size=256, aggregate_loss="sum")  # conf/finetune/base.yaml:92-105 + grpo.yaml
    cases.append(dict(batch="packed", value_head=False, step=0, max_step=10, cfg=grpo))
    cases.append(dict(batch="packed", value_head=False, step=3, max_step=10,
                      cfg=dict(grpo, kl_coef=0.2, final_kl_coef=0.0, entropy_bonus=0.05,
                               final_entropy_bonus=0.0, group_normalization=True,
                               overlong_filtering=True, relu_log_p_weights=True)))
    cases.append(dict(batch="packed", value_head=False, step=1, max_step=4,
                      cfg=dict(policy_loss="reinforce", use_advantages=False, epsilon=0.3,
                               kl_coef=0.05, clamp_log_ratio_ref_new_value=5, batch_size=3)))
    cases.append(dict(batch="packed_nolabels", value_head=False, step=0, max_step=10,
                      cfg=dict(grpo)))
    for pol in ["ppo", "reinforce"]:
        cases.append(dict(batch="unpacked", value_head=False, step=2, max_step=10,
                          cfg=dict(policy_loss=pol, kl_coef=0.1, entropy_bonus=0.01,
                                   final_entropy_bonus=0.01, temperature=0.8, batch_size=2)))
    cases.append(dict(batch="unpacked", value_head=True, step=0, max_step=10,
                      cfg=dict(policy_loss="ppo", kl_coef=0.0, final_kl_coef=0.0, batch_size=2,
                               value_loss_coef=0.1)))
    return cases


def write_f1():
    (plog, pb, pval), (ulog, ub, uval) = f1_batches()
    nb = dict(pb)
    nb["labels"] = np.full_like(pb["labels"], -100)
    batches = {"packed": (plog, pb, pval), "packed_nolabels": (plog, nb, pval),
               "unpacked": (ulog, ub, uval)}
    arrays = {}
    for name, (lg, b, v) in batches.items():
        arrays[f"{name}__logits"] = lg
        arrays[f"{name}__values"] = v
        for k, val in b.items():
            if isinstance(val, np.ndarray):
                arrays[f"{name}__{k}"] = val
        arrays[f"{name}__is_packed"] = np.array(bool(b["is_packed"]))
    np.savez_compressed(HERE / "f1_inputs.npz", **arrays)

    outs, meta = {}, []
    for i, c in enumerate(f1_cases()):
        lg, b, v = batches[c["batch"]]
        bb = {k: (val.tolist() if isinstance(val, np.ndarray) else val) for k, val in b.items()}
        r = run_reference(lg, bb, c["cfg"], c["step"], c["max_step"], v if c["value_head"] else None)
        outs[f"case{i}__dlogits"] = r["dlogits"]
        outs[f"case{i}__new_logprobs"] = r["new_logprobs"]
        outs[f"case{i}__entropy"] = r["entropy"]
        if "dvalues" in r:
            outs[f"case{i}__dvalues"] = r["dvalues"]
        meta.append(dict(c, loss=r["loss"], stats=r["stats"]))
    np.savez_compressed(HERE / "f1_outputs.npz", **outs)
    (HERE / "f1_cases.json").write_text(json.dumps(meta, indent=1))
    print(f"F1: {len(meta)} cases")


F2_SEED, F2_T, F2_V = 2024, 16, 151936


def f2_inputs():
    b = synth.packed_rl_batch(F2_SEED, [8, 8], [3, 3], id_range=151643, eos=151643)
    ids = b["input_ids"][0]
    lg = synth.logits_rows(F2_SEED, np.arange(F2_T), F2_V, ids)
    lg = synth.to_bf16(lg)
    x = lg[:-1].astype(np.float64)
    lse = np.log(np.exp(x - x.max(-1, keepdims=True)).sum(-1)) + x.max(-1)
    tl = x[np.arange(F2_T - 1), ids[1:]] - lse
    lab = b["labels"][0] != -100
    u = synth.normal(F2_SEED + 3, np.arange(2 * F2_T, dtype=np.uint64))
    old = np.zeros(F2_T, np.float32)
    ref = np.zeros(F2_T, np.float32)
    old[1:] = tl + 0.1 * u[:F2_T - 1]
    ref[1:] = tl + 0.2 * u[F2_T:2 * F2_T - 1]
    old[~lab] = 0
    ref[~lab] = 0
    b["old_logprobs"] = old[None]
    b["ref_logprobs"] = ref[None]
    return lg[None].astype(np.float32), b


def f2_projection_vector(V: int) -> np.ndarray:
    return synth.normal(F2_SEED + 99, np.arange(V, dtype=np.uint64))


def write_f2():
    lg, b = f2_inputs()
    cfg = dict(policy_loss="ppo", kl_coef=0.05, final_kl_coef=0.05, entropy_bonus=0.01,
               final_entropy_bonus=0.01, epsilon=0.2, batch_size=2, temperature=1.0,
               clamp_log_ratio_ref_new_value=5)
    bb = {k: (val.tolist() if isinstance(val, np.ndarray) else val) for k, val in b.items()}
    proj = f2_projection_vector(F2_V)
    tgt = b["input_ids"][0, 1:]
    res = {}
    meta = {"cfg": cfg, "step": 0, "max_step": 10, "seed": F2_SEED, "T": F2_T, "V": F2_V}
    for name, dt in [("bf16", torch.bfloat16), ("fp32", torch.float32)]:
        r = run_reference(lg, bb, cfg, 0, 10, None, dtype=dt)
        d = r["dlogits"][0].astype(np.float64)
        res[f"{name}__new_logprobs"] = r["new_logprobs"]
        res[f"{name}__entropy"] = r["entropy"]
        res[f"{name}__d_target"] = d[np.arange(F2_T - 1), tgt]
        res[f"{name}__d_abssum"] = np.abs(d).sum(-1)
        res[f"{name}__d_proj"] = d @ proj
        res[f"{name}__d_cols"] = d[:, :1024].astype(np.float32)
        meta[name] = {"loss": r["loss"], "stats": r["stats"]}
    np.savez_compressed(HERE / "f2_outputs.npz", **res)
    (HERE / "f2_meta.json").write_text(json.dumps(meta, indent=1))
    print("F2 written")


def write_f3():
    """populate_rl_data (rl/__init__.py:380-501) + collate_packed (data.py:215-279)."""
    from pipelinerl.finetune.data import collate_packed
    from pipelinerl.finetune.rl import prepare_rl_fields

    rng = np.random.default_rng(77)
    eos = 50
    dataset = []
    for g in range(4):
        for a in range(8):
            steps = 2 if (g == 3 and a % 2 == 0) else 1
            reward = float(rng.integers(0, 2)) if g != 2 else 1.0  # group 2: zero variance
            for s in range(steps):
                p = int(rng.integers(3, 7))
                c = int(rng.integers(2, 9))
                ids = rng.integers(0, eos, p + c).tolist()
                if not (g == 1 and a == 0):  # one overflow rollout (no EOS)
                    ids[-1] = eos
                labels = [-100] * p + ids[p:]
                lps = rng.normal(-1.0, 0.5, c).tolist()
                enc = {"input_ids": ids, "labels": labels, "attention_mask": [1] * len(ids)}
                enc = prepare_rl_fields(enc, reward, lps, lps)
                enc.update(group_id=f"g{g}", rollout_index=a, step_index=s, model_version=g)
                dataset.append(enc)
    inputs = json.loads(json.dumps(dataset))
    res = {}
    for divide in [False, True]:
        cfg = RLConfig(divide_advantage_by_std=divide)
        out = populate_rl_data([dict(e) for e in json.loads(json.dumps(inputs))], eos, cfg)
        res[f"divide_{divide}"] = [{k: e[k] for k in ["advantages", "group_tokens", "overflow", "num_labels"]}
                                   for e in out]
    tok = types.SimpleNamespace(eos_token_id=eos)
    out = populate_rl_data([dict(e) for e in json.loads(json.dumps(inputs))], eos, RLConfig())
    packs = {}
    for sp in [1, 4]:
        pb = collate_packed(out[:5], tok, sp)
        packs[f"sp{sp}"] = {k: (v.tolist() if isinstance(v, torch.Tensor) else v)
                            for k, v in pb.model_dump().items() if v is not None}
    (HERE / "f3_rl_data.json").write_text(json.dumps({"eos": eos, "inputs": inputs, "populate": res,
                                                      "collate_packed": packs}))
    print("F3 written")


if __name__ == "__main__":
    assert os.environ.get("PYTHONDONTWRITEBYTECODE") == "1", "set PYTHONDONTWRITEBYTECODE=1"
    torch.manual_seed(0)
    meta = {"torch": torch.__version__, "numpy": np.__version__}
    import pandas
    meta["pandas"] = pandas.__version__
    (HERE / "versions.json").write_text(json.dumps(meta))
    write_f1()
    write_f2()
    write_f3()
