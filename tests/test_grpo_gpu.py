"""GPU parity of the fused GRPO loss head (HIP, through the C ABI) against the reference.

Anchors: golden vectors produced by the reference rl_step (tests/golden/make_golden.py) and the
pinned numpy oracle (oracle/grpo_oracle.py).  Tolerances (BASELINE.json north_star):
  fp32 logits: loss / stats / log-probs / entropy within 1e-4 (relative to max(1, |x|)),
               dlogits within 1e-6 + 1e-4 |d|;
  bf16 logits: vs an fp32 computation on the same bf16 values: 1e-4 on log-probs / entropy,
               dlogits (stored bf16) within 1e-2 relative + 1e-8 absolute;
               vs the reference's own bf16 path: 1e-2 relative.
"""

import json

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_f1
from gpu_helpers import LogitsModel, rel_close, to_batch
from oracle import grpo_oracle, synth

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(logits, b, cfg, step, max_step, values=None, scale=1.0):
    from pipelinerl_amd.finetune.rl import RLConfig, rl_step

    model = LogitsModel(logits, values)
    loss, stats = rl_step(model, to_batch(b), step, max_step, RLConfig(**cfg))
    (loss * scale).backward() if scale != 1.0 else loss.backward()
    torch.cuda.synchronize()
    out = dict(loss=float(loss.item()), stats=stats, dlogits=model.logits.grad.float().cpu().numpy())
    if values is not None:
        out["dvalues"] = model.value_head.grad.float().cpu().numpy()
    return out


def _rows(logits, b, cfg, step, max_step, values=None):
    from pipelinerl_amd.finetune.rl import RLConfig, linear_decay_coef
    from pipelinerl_amd.finetune.rl.fused import GrpoParams, grpo_loss, prepare_fields

    c = RLConfig(**cfg)
    p = GrpoParams(policy_loss=c.policy_loss, use_advantages=c.use_advantages,
                   relu_log_p_weights=c.relu_log_p_weights, group_normalization=c.group_normalization,
                   overlong_filtering=c.overlong_filtering, epsilon=c.epsilon,
                   kl_coef=linear_decay_coef(step, max_step, c.kl_coef, c.final_kl_coef),
                   entropy_coef=linear_decay_coef(step, max_step, c.entropy_bonus, c.final_entropy_bonus),
                   clamp_log_ratio=c.clamp_log_ratio_ref_new_value, temperature=c.temperature,
                   batch_size=c.batch_size, value_loss_coef=c.value_loss_coef if values is not None else 0.0)
    batch = to_batch(b)
    _, _, rows = grpo_loss(logits, prepare_fields(batch, logits.device), p, values)
    r = rows.cpu().numpy()
    B, L = np.asarray(b["labels"]).shape
    return r[0].reshape(B, L - 1), r[1].reshape(B, L - 1)


def _check_stats(got, want, rtol=1e-4, what=""):
    assert set(got) == set(want), (what, set(got) ^ set(want))
    for k, v in want.items():
        assert abs(got[k] - v) <= rtol * max(1.0, abs(v)), (what, k, got[k], v)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_f1_all_cases(dtype):
    batches, out, cases = load_f1()
    for i, c in enumerate(cases):
        b = batches[c["batch"]]
        lg = b["logits"] if dtype == "fp32" else synth.to_bf16(b["logits"])
        tdt = torch.float32 if dtype == "fp32" else torch.bfloat16
        logits = torch.tensor(lg, dtype=torch.float32).to(tdt).to(DEV)
        vals = torch.tensor(b["values"], device=DEV) if c["value_head"] else None
        r = _run(logits, b, c["cfg"], c["step"], c["max_step"], vals)
        if dtype == "fp32":  # straight against the reference's own outputs
            _check_stats(r["stats"], c["stats"], 1e-4, f"case{i}")
            assert abs(r["loss"] - c["loss"]) <= 1e-4 * max(1, abs(c["loss"]))
            ok, err = rel_close(r["dlogits"], out[f"case{i}__dlogits"], 1e-4, 1e-6)
            assert ok, (i, err)
            if c["value_head"]:
                ok, err = rel_close(r["dvalues"], out[f"case{i}__dvalues"], 1e-4, 1e-7)
                assert ok, (i, err)
            lp, H = _rows(logits.detach(), b, c["cfg"], c["step"], c["max_step"], vals)
            ok, err = rel_close(lp, out[f"case{i}__new_logprobs"], 1e-5, 1e-5)
            assert ok, (i, "lp", err)
            ok, err = rel_close(H, out[f"case{i}__entropy"], 1e-5, 1e-5)
            assert ok, (i, "H", err)
        else:  # bf16 logits: against the pinned oracle on the same bf16 values
            o = grpo_oracle.rl_step_oracle(lg, b, c["cfg"], c["step"], c["max_step"],
                                           values=b["values"] if c["value_head"] else None)
            _check_stats(r["stats"], o["stats"], 1e-4, f"case{i}")
            ok, err = rel_close(r["dlogits"], o["dlogits"], 1e-2, 1e-8)
            assert ok, (i, err)


def _f2():
    meta = json.loads((GOLDEN / "f2_meta.json").read_text())
    from test_oracle_golden import f2_batch
    _, lg, b = f2_batch()
    return meta, lg, b


def test_f2_full_vocab_bf16_resident_path():
    """V = 151936, bf16: the register-resident kernel (19 x 16 B per lane)."""
    meta, lg, b = _f2()
    out = np.load(GOLDEN / "f2_outputs.npz")
    logits = torch.tensor(lg, dtype=torch.float32).to(torch.bfloat16).to(DEV)
    r = _run(logits, b, meta["cfg"], meta["step"], meta["max_step"])
    ref = meta["fp32"]  # reference fp32 path on the same bf16-rounded logits
    assert abs(r["loss"] - ref["loss"]) <= 1e-4 * max(1, abs(ref["loss"]))
    _check_stats(r["stats"], ref["stats"], 1e-4, "f2 fp32")
    lp, H = _rows(logits.detach(), b, meta["cfg"], meta["step"], meta["max_step"])
    assert rel_close(lp, out["fp32__new_logprobs"], 1e-4, 1e-4)[0]
    assert rel_close(H, out["fp32__entropy"], 1e-4, 1e-4)[0]
    # the reference's own bf16 path rounds log_softmax to bf16: relative 1e-2
    assert rel_close(lp, out["bf16__new_logprobs"], 1e-2, 1e-2)[0]
    assert rel_close(H, out["bf16__entropy"], 1e-2, 1e-2)[0]
    d = r["dlogits"][0].astype(np.float64)
    T = meta["T"]
    tgt = b["input_ids"][0, 1:]
    assert rel_close(d[np.arange(T - 1), tgt], out["fp32__d_target"], 1e-2, 1e-8)[0]
    assert rel_close(d[:, :1024], out["fp32__d_cols"], 1e-2, 1e-9)[0]
    assert np.all(d[T - 1] == 0)


@pytest.mark.parametrize("V,dtype", [(1000, "bf16"), (1001, "bf16"), (1001, "fp32"), (8 * 1024 * 3 + 8, "bf16"),
                                     (152064, "bf16"), (151936, "fp32"), (152064, "fp32")])
def test_kernel_paths_vs_oracle(V, dtype):
    """Resident (bf16, V % 8 == 0), streaming vector and scalar paths, ragged last vector; fp32 logits
    (Accelerate's upcast regime: the streaming kernel) at the Qwen2.5 vocabularies."""
    T = 29
    b = synth.packed_rl_batch(3, [10, 12, 7], [3, 4, 2], id_range=V, eos=5)
    rng = np.random.default_rng(V)
    lg = rng.normal(0, 2.0, (1, T, V)).astype(np.float32)
    if dtype == "bf16":
        lg = synth.to_bf16(lg)
    b["old_logprobs"] = np.where(b["labels"] != -100, rng.normal(-7, 1, (1, T)), 0).astype(np.float32)
    b["ref_logprobs"] = np.where(b["labels"] != -100, rng.normal(-7, 1, (1, T)), 0).astype(np.float32)
    cfg = dict(policy_loss="ppo", kl_coef=0.05, entropy_bonus=0.02, final_entropy_bonus=0.02, epsilon=0.2,
               batch_size=3, temperature=0.9, clamp_log_ratio_ref_new_value=5)
    tdt = torch.float32 if dtype == "fp32" else torch.bfloat16
    logits = torch.tensor(lg).to(tdt).to(DEV)
    r = _run(logits, b, cfg, 0, 10)
    o = grpo_oracle.rl_step_oracle(lg, b, cfg, 0, 10)
    _check_stats(r["stats"], o["stats"], 1e-4, f"V={V}")
    lp, H = _rows(logits.detach(), b, cfg, 0, 10)
    assert rel_close(lp, o["new_logprobs"], 1e-5, 1e-4)[0]
    assert rel_close(H, o["entropy"], 1e-5, 1e-4)[0]
    tol = (1e-2, 1e-8) if dtype == "bf16" else (1e-4, 1e-7)
    ok, err = rel_close(r["dlogits"], o["dlogits"], *tol)
    assert ok, err


def test_upstream_gradient_scale_and_sentinel():
    batches, _, cases = load_f1()
    b = batches["packed"]
    c = cases[5]
    for scale in (0.0, 0.25, -3.0):
        logits = torch.tensor(b["logits"], device=DEV)
        r = _run(logits, b, c["cfg"], c["step"], c["max_step"], scale=scale)
        o = grpo_oracle.rl_step_oracle(b["logits"], b, c["cfg"], c["step"], c["max_step"], grad_out=scale)
        ok, err = rel_close(r["dlogits"], o["dlogits"], 1e-4, 1e-7)
        assert ok, (scale, err)
        if scale == 0.0:
            assert np.all(r["dlogits"] == 0)


def test_errors_match_reference():
    from pipelinerl_amd.finetune.rl import RLConfig, rl_step

    batches, _, _ = load_f1()
    b = batches["packed"]
    with pytest.raises(ValueError):
        rl_step(LogitsModel(torch.tensor(b["logits"], device=DEV)), to_batch(b), 0, 10,
                RLConfig(policy_loss="nope", batch_size=4))
    lg = b["logits"].copy()
    lg[0, 3, 5] = np.nan
    with pytest.raises(AssertionError):
        rl_step(LogitsModel(torch.tensor(lg, device=DEV)), to_batch(b), 0, 10, RLConfig(batch_size=4))
    bad = dict(b)
    bad["input_ids"] = b["input_ids"].copy()
    bad["input_ids"][0, 4] = 10 ** 6
    with pytest.raises(RuntimeError):
        rl_step(LogitsModel(torch.tensor(b["logits"], device=DEV)), to_batch(bad), 0, 10, RLConfig(batch_size=4))
    gn = dict(b)
    gn["group_tokens"] = np.zeros_like(b["group_tokens"])
    with pytest.raises(AssertionError):
        rl_step(LogitsModel(torch.tensor(b["logits"], device=DEV)), to_batch(gn), 0, 10,
                RLConfig(batch_size=4, group_normalization=True))
    nl = dict(b)
    nl["labels"] = np.full_like(b["labels"], -100)
    loss, stats = rl_step(LogitsModel(torch.tensor(b["logits"], device=DEV)), to_batch(nl), 0, 10,
                          RLConfig(batch_size=4))
    assert stats == {"input_size": float(b["input_ids"].size)}
    assert float(loss) == 0.0


def _c2_inputs(T: int, V: int, seq: int):
    """C2's packed micro-batch (T rows = T/seq rollouts of seq tokens, 256-token prompts) with
    per-token fields drawn so every branch of the token arithmetic is taken at full size:
    old = ATen log-prob of the target + N(0, 0.3²) (PPO clip engaged on both sides at eps 0.2),
    ref = old + N(0, 0.05²) with 1 % of the rows pushed ±6 beyond the KL clamp (C = 5), group
    advantages N(0, 1), 1 sequence in 8 overflowing (overlong filter on)."""
    g = torch.Generator(device=DEV).manual_seed(0)
    logits = torch.empty((1, T, V), device=DEV, dtype=torch.bfloat16)
    for a in range(0, T, 8192):
        logits[0, a:a + 8192] = (torch.randn((min(8192, T - a), V), generator=g, device=DEV) * 3).to(torch.bfloat16)
    nseq = T // seq
    pos = torch.arange(T, device=DEV) % seq
    ids = torch.randint(0, 151643, (1, T), generator=g, device=DEV)
    labels = torch.where(pos[None] >= 256, ids, torch.full_like(ids, -100))
    # an independent (ATen) target log-prob, only to centre old_logprobs near the policy's own
    lp = torch.zeros((1, T), device=DEV)
    for a in range(0, T - 1, 4096):
        b = min(a + 4096, T - 1)
        ls = torch.log_softmax(logits[0, a:b].float(), dim=-1)
        lp[0, a + 1:b + 1] = ls.gather(1, ids[0, a + 1:b + 1, None])[:, 0]
        del ls
    per_seq = lambda x: torch.repeat_interleave(x, seq)[None]  # noqa: E731
    old = lp + 0.3 * torch.randn((1, T), generator=g, device=DEV)
    far = (torch.rand((1, T), generator=g, device=DEV) < 0.01).float() * \
        torch.where(torch.rand((1, T), generator=g, device=DEV) < 0.5, -6.0, 6.0)
    ref = old + 0.05 * torch.randn((1, T), generator=g, device=DEV) + far
    lab = labels != -100
    f = {"input_ids": ids, "labels": labels,
         "rewards": per_seq(torch.randint(0, 2, (nseq,), generator=g, device=DEV).float()),
         "advantages": per_seq(torch.randn((nseq,), generator=g, device=DEV)),
         "ref_logprobs": torch.where(lab, ref, 0.0), "old_logprobs": torch.where(lab, old, 0.0),
         "group_tokens": torch.full((1, T), float(seq), device=DEV),
         "num_labels": torch.full((1, T), float(seq - 256), device=DEV),
         "overflow": per_seq((torch.arange(nseq, device=DEV) % 8 == 3).float())}
    return logits, {k: v.contiguous() for k, v in f.items()}, pos


C2_CFG = dict(policy_loss="ppo", epsilon=0.2, kl_coef=0.001, final_kl_coef=0.001, entropy_bonus=0.001,
              final_entropy_bonus=0.001, clamp_log_ratio_ref_new_value=5.0, batch_size=256, temperature=1.0,
              overlong_filtering=True)


def _c2_params(cfg: dict):
    from pipelinerl_amd.finetune.rl.fused import GrpoParams

    return GrpoParams(policy_loss=cfg["policy_loss"], epsilon=cfg["epsilon"], kl_coef=cfg["kl_coef"],
                      entropy_coef=cfg["entropy_bonus"], clamp_log_ratio=cfg["clamp_log_ratio_ref_new_value"],
                      batch_size=float(cfg["batch_size"]), temperature=cfg["temperature"],
                      overlong_filtering=cfg["overlong_filtering"])


def _c2_mismatches(loss: float, stats: dict, rows: np.ndarray, mask: np.ndarray, o: dict, hb: dict,
                   cfg: dict) -> list[str]:
    """Every disagreement of the kernel's loss / statistics / per-row outputs with the oracle's
    (1e-4 relative to max(1, |x|) on scalars; per row: log-prob / entropy / lse 1e-4, token loss
    and the upstream row gradients g_lp / g_h 1e-4 relative + 1e-4 of their largest magnitude).
    g_lp is a step function of the ratio at the PPO clip bounds and of ref - new at the KL clamp:
    rows within 1e-5 (relative) of a bound, where an fp32 last-bit difference in the log-prob may
    legitimately fall on the other side, are left out of the g_lp comparison (expected: ~0 rows)."""
    bad = []
    if abs(loss - o["loss"]) > 1e-4 * max(1.0, abs(o["loss"])):
        bad.append(f"loss {loss} vs {o['loss']}")
    if set(stats) != set(o["stats"]):
        bad.append(f"stat keys {set(stats) ^ set(o['stats'])}")
    for k, v in o["stats"].items():
        if k in stats and not abs(stats[k] - v) <= 1e-4 * max(1.0, abs(v)):
            bad.append(f"stat {k}: {stats[k]} vs {v}")
    for i, (name, want) in enumerate((("new_logprobs", o["new_logprobs"][0]), ("entropy", o["entropy"][0]),
                                      ("lse", o["lse"][0]))):
        ok, err = rel_close(rows[i], want, 1e-5, 1e-4)
        if not ok:
            bad.append(f"rows {name}: max err {err}")
    lp = o["new_logprobs"][0].astype(np.float64)
    ratio = np.exp(lp - hb["old_logprobs"][0, 1:])
    eps, C = cfg["epsilon"], cfg["clamp_log_ratio_ref_new_value"]
    edge = (np.abs(ratio - (1 + eps)) <= 1e-5 * (1 + eps)) | (np.abs(ratio - (1 - eps)) <= 1e-5) | \
        (np.abs(np.abs(hb["ref_logprobs"][0, 1:] - lp) - C) <= 1e-5 * C)
    for i, name, want in ((3, "token_loss", np.where(mask, o["token_loss"][0], 0.0)),
                          (4, "g_lp", np.where(edge, 0.0, o["g_lp"][0])), (5, "g_h", o["g_h"][0])):
        got = np.where(mask & ~edge if name == "g_lp" else mask, rows[i], 0.0)
        ok, err = rel_close(got, want, 1e-4, 1e-4 * float(np.abs(want).max()) + 1e-30)
        if not ok:
            bad.append(f"rows {name}: max err {err}")
    return bad


@pytest.mark.timeout(1200)
def test_c2_full_size_vs_oracle():
    """Config C2 at full size (65 536 packed rows x 151 936 vocab, bf16 logits, 19.9 GB) against the
    oracle over EVERY row (rl/__init__.py:200-366): loss and all statistics at 1e-4; every row's
    log-prob, entropy, lse, token loss and upstream gradients (g_lp, g_h); sampled rows' dlogits vs
    the oracle's own gradient (its g_lp / g_h, not the kernel's) at the bf16 bar 1e-2.  Then:
    softmax-gradient rows sum to ~0, the kernel is bitwise deterministic, and a negative control
    (the kernel run with epsilon off by 1 %) must fail the same comparison."""
    import time
    import types as _types

    from pipelinerl_amd.finetune.rl import build_stats
    from pipelinerl_amd.finetune.rl.fused import grpo_loss, prepare_fields

    T, V, seq = 65536, 151936, 2048
    logits, f, pos = _c2_inputs(T, V, seq)
    logits.requires_grad_(True)
    p = _c2_params(C2_CFG)
    fields = prepare_fields(f, logits.device)
    loss1, stats1, rows1 = grpo_loss(logits, fields, p)
    loss1.backward()
    d1 = logits.grad
    logits.grad = None
    loss2, stats2, rows2 = grpo_loss(logits, fields, p)
    loss2.backward()
    assert torch.equal(stats1, stats2) and torch.equal(rows1, rows2)
    assert torch.equal(d1, logits.grad)
    logits.grad = None
    # sum_j d_j = 0 exactly for the softmax gradient; bf16 storage rounds each d_j by 2^-9
    df = d1[0].float()
    rowsum = df.sum(-1).abs()
    absum = df.abs().sum(-1)
    assert bool(torch.all(rowsum <= 4e-3 * absum + 1e-12)), float((rowsum / (absum + 1e-30)).max())
    assert int((absum > 0).sum()) > 0
    assert torch.all(d1[0, T - 1] == 0)
    del df, rowsum, absum

    nseq = T // seq
    hb = {k: v.cpu().numpy() for k, v in f.items()} | {"position_ids": pos[None].cpu().numpy(), "is_packed": True}
    meta = _types.SimpleNamespace(is_packed=True, input_ids=f["input_ids"])
    stats = build_stats(stats1.cpu().numpy(), meta, p, p.kl_coef, p.entropy_coef, nseq, False)
    # the bf16 logits in fp32 on the host (40 GB), copied in row blocks
    lg = np.empty((1, T, V), dtype=np.float32)
    with torch.no_grad():
        for a in range(0, T, 4096):
            lg[0, a:a + 4096] = logits[0, a:a + 4096].float().cpu().numpy()
    mask = hb["labels"][0, 1:] != -100
    t0 = time.time()
    o = grpo_oracle.rl_step_oracle(lg, hb, C2_CFG, 0, 10, compute_grad=True, dtype=np.float32, threads=16,
                                   row_chunk=64, grad_rows=np.array([0]))
    t_oracle = time.time() - t0
    r1 = rows1.cpu().numpy()
    assert o["stats"]["num_output_tokens_sum"] == nseq * (seq - 256)
    bad = _c2_mismatches(float(loss1.detach()), stats, r1, mask, o, hb, C2_CFG)
    assert not bad, bad

    # the branches the token arithmetic takes at this size (so the comparison above covers them)
    ratio = np.exp(o["new_logprobs"][0] - hb["old_logprobs"][0, 1:])
    lrrn = hb["ref_logprobs"][0, 1:] - o["new_logprobs"][0]
    adv = hb["advantages"][0, 1:]
    ovf = hb["overflow"][0, 1:] > 0
    cats = {"clip_hi": mask & (ratio > 1.2) & (adv > 0), "clip_lo": mask & (ratio < 0.8) & (adv < 0),
            "clip_hi_inactive": mask & (ratio > 1.2) & (adv < 0), "kl_clamp_hi": mask & (lrrn > 5),
            "kl_clamp_lo": mask & (lrrn < -5), "overflow": mask & ovf, "plain": mask & ~ovf & (np.abs(lrrn) < 5)}
    for k, c in cats.items():
        assert c.sum() > 100, (k, int(c.sum()))
    # sampled rows: the kernel's dlogits vs the ORACLE's gradient of the same logits
    sample = np.unique(np.concatenate([[0, 1, 255, 256, 257, 4095, 30000, 65534]] +
                                      [np.nonzero(c)[0][:3] for c in cats.values()]))
    o_rows = grpo_oracle.rl_step_oracle(lg, hb, C2_CFG, 0, 10, compute_grad=True, dtype=np.float32,
                                        grad_rows=sample, rows=o)
    want = o_rows["dlogits_rows"]
    got = d1[0, torch.tensor(sample, device=DEV)].float().cpu().numpy()
    assert np.abs(want[mask[sample]]).max() > 0
    ok, err = rel_close(got, want, 1e-2, 1e-9)
    assert ok, ("sampled dlogits vs oracle", err)
    del d1

    # negative control: the kernel with epsilon off by 1 % must fail the same comparison
    cfg_bad = dict(C2_CFG, epsilon=C2_CFG["epsilon"] * 1.01)
    pb = _c2_params(cfg_bad)
    lb, sb, rb = grpo_loss(logits.detach(), fields, pb)
    stats_b = build_stats(sb.cpu().numpy(), meta, pb, pb.kl_coef, pb.entropy_coef, nseq, False)
    bad_ctl = _c2_mismatches(float(lb), stats_b, rb.cpu().numpy(), mask, o, hb, C2_CFG)
    assert bad_ctl, "epsilon x 1.01 went undetected"
    # ... and the oracle with the same perturbation agrees with that kernel run (only the token
    # arithmetic is redone: the per-row lse / entropy / log-prob of the first pass are reused)
    ob = grpo_oracle.rl_step_oracle(lg, hb, cfg_bad, 0, 10, compute_grad=True, dtype=np.float32,
                                    grad_rows=np.array([0]), rows=o)
    assert not _c2_mismatches(float(lb), stats_b, rb.cpu().numpy(), mask, ob, hb, cfg_bad)
    print(f"C2 full size: oracle {t_oracle:.1f} s over {T} x {V}; negative control caught: {bad_ctl[:3]}")


@pytest.mark.timeout(1200)
def test_c2_fp32_logits_full_size_vs_oracle():
    """C2's micro-batch in the fp32-logits regime (Accelerate mixed precision upcasts the logits,
    finetune_loop.py:381-385; 65 536 x 151 936 fp32, 39.8 GB: the streaming kernel, which re-reads
    each row for the gradient) against the oracle over every row, as the bf16 test above: loss and
    statistics at 1e-4, every row's outputs, sampled dlogits vs the oracle's gradient at the fp32
    bar (1e-4 relative).  The logits carry fp32 noise below bf16's resolution, so a kernel that
    rounded them to bf16 anywhere would fail."""
    from pipelinerl_amd.finetune.rl import build_stats
    from pipelinerl_amd.finetune.rl.fused import grpo_loss, prepare_fields

    T, V, seq = 65536, 151936, 2048
    lb, f, pos = _c2_inputs(T, V, seq)
    g = torch.Generator(device=DEV).manual_seed(1)
    logits = torch.empty((1, T, V), device=DEV, dtype=torch.float32)
    for a in range(0, T, 8192):
        b = min(a + 8192, T)
        logits[0, a:b] = lb[0, a:b].float() + 1e-3 * torch.randn((b - a, V), generator=g, device=DEV)
    del lb
    torch.cuda.empty_cache()
    logits.requires_grad_(True)
    p = _c2_params(C2_CFG)
    fields = prepare_fields(f, logits.device)
    loss1, stats1, rows1 = grpo_loss(logits, fields, p)
    loss1.backward()
    d1 = logits.grad
    logits.grad = None
    assert d1.dtype == torch.float32 and torch.all(d1[0, T - 1] == 0)
    nseq = T // seq
    hb = {k: v.cpu().numpy() for k, v in f.items()} | {"position_ids": pos[None].cpu().numpy(), "is_packed": True}
    meta = _types_ns(is_packed=True, input_ids=f["input_ids"])
    stats = build_stats(stats1.cpu().numpy(), meta, p, p.kl_coef, p.entropy_coef, nseq, False)
    lg = np.empty((1, T, V), dtype=np.float32)
    with torch.no_grad():
        for a in range(0, T, 4096):
            lg[0, a:a + 4096] = logits[0, a:a + 4096].cpu().numpy()
    mask = hb["labels"][0, 1:] != -100
    o = grpo_oracle.rl_step_oracle(lg, hb, C2_CFG, 0, 10, compute_grad=True, dtype=np.float32, threads=16,
                                   row_chunk=64, grad_rows=np.array([0]))
    bad = _c2_mismatches(float(loss1.detach()), stats, rows1.cpu().numpy(), mask, o, hb, C2_CFG)
    assert not bad, bad
    sample = np.array([0, 1, 255, 256, 257, 4095, 30000, 65534])
    o_rows = grpo_oracle.rl_step_oracle(lg, hb, C2_CFG, 0, 10, compute_grad=True, dtype=np.float32,
                                        grad_rows=sample, rows=o)
    got = d1[0, torch.tensor(sample, device=DEV)].cpu().numpy()
    want = o_rows["dlogits_rows"]
    ok, err = rel_close(got, want, 1e-4, 1e-6 * float(np.abs(want).max()))
    assert ok, ("sampled fp32 dlogits vs oracle", err)


def _types_ns(**kw):
    import types as _types

    return _types.SimpleNamespace(**kw)


def test_flatten_unflatten_and_sqnorm():
    import ctypes

    from pipelinerl_amd import _native

    lib = _native.load()
    ts = [torch.randn(n, device=DEV, dtype=dt) for n, dt in
          [(1000, torch.float32), (37, torch.bfloat16), (4096, torch.bfloat16), (8, torch.float32), (0, torch.float32)]]
    offs, o = [], 0
    for t in ts:
        offs.append(o)
        o += (t.numel() + 7) // 8 * 8
    flat = torch.zeros(o, dtype=torch.bfloat16, device=DEV)
    n = len(ts)
    P = (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])
    D = (ctypes.c_int32 * n)(*[1 if t.dtype == torch.bfloat16 else 0 for t in ts])
    N = (ctypes.c_int64 * n)(*[t.numel() for t in ts])
    Of = (ctypes.c_int64 * n)(*offs)
    st = torch.cuda.current_stream().cuda_stream
    _native.check(lib.prl_flatten_bf16(P, D, N, Of, n, flat.data_ptr(), st), "flatten")
    for t, off in zip(ts, offs):
        assert torch.equal(flat[off:off + t.numel()], t.to(torch.bfloat16))
    outs = [torch.empty_like(t) for t in ts]
    Q = (ctypes.c_void_p * n)(*[t.data_ptr() for t in outs])
    _native.check(lib.prl_unflatten_bf16(flat.data_ptr(), Q, D, N, Of, n, st), "unflatten")
    for t, u in zip(ts, outs):
        assert torch.equal(u, t.to(torch.bfloat16).to(t.dtype))
    res = torch.zeros(1, dtype=torch.float64, device=DEV)
    rp = ctypes.cast(res.data_ptr(), ctypes.POINTER(ctypes.c_double))
    assert lib.prl_grad_sqnorm(P, D, N, n, rp, None, 0, st) == 1003  # PRL_E_WORKSPACE
    ws = torch.empty(n * 256, dtype=torch.float64, device=DEV)
    _native.check(lib.prl_grad_sqnorm(P, D, N, n, rp, ws.data_ptr(), ws.numel() * 8, st), "sqnorm")
    want = sum(float((t.double() ** 2).sum()) for t in ts)
    assert abs(float(res) - want) <= 1e-9 * want
    # deterministic: the same bits on every call (fixed partials, fixed fold; no atomics)
    bits = float(res)
    for _ in range(5):
        _native.check(lib.prl_grad_sqnorm(P, D, N, n, rp, ws.data_ptr(), ws.numel() * 8, st), "sqnorm")
        assert float(res) == bits
