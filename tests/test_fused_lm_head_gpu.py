"""Label-row lm_head + loss (fused_linear.py) on the GPU.

Parity chain: the oracle's dlogits (float64 restatement of rl_step, pinned to the reference's
golden vectors) composed with the lm_head, dh = dlogits @ W and dW = dlogits^T @ h, is the
reference's autograd through ``lm_head`` (rl/__init__.py:197-208); prompt rows carry no
gradient there.  fp32 runs are held to 1e-4, bf16 runs to the bf16 bar of north_star.
"""

import numpy as np
import pytest
import torch

from gpu_helpers import rel_close, to_batch
from oracle import grpo_oracle, synth

pytestmark = pytest.mark.gpu
DEV = "cuda"
CFG = dict(policy_loss="ppo", kl_coef=0.05, final_kl_coef=0.05, entropy_bonus=0.01, final_entropy_bonus=0.01,
           epsilon=0.2, batch_size=3, clamp_log_ratio_ref_new_value=5)


def _batch(lens, prompts, V, seed):
    T = sum(lens)
    b = synth.packed_rl_batch(seed, lens, prompts, id_range=V, eos=3)
    rng = np.random.default_rng(seed)
    m = b["labels"] != -100
    b["old_logprobs"] = np.where(m, rng.normal(-6, 1, (1, T)), 0).astype(np.float32)
    b["ref_logprobs"] = np.where(m, rng.normal(-6, 1, (1, T)), 0).astype(np.float32)
    return b


def _params(cfg):
    from pipelinerl_amd.finetune.rl import RLConfig, linear_decay_coef
    from pipelinerl_amd.finetune.rl.fused import GrpoParams

    c = RLConfig(**cfg)
    return GrpoParams(policy_loss=c.policy_loss, epsilon=c.epsilon,
                      kl_coef=linear_decay_coef(0, 10, c.kl_coef, c.final_kl_coef),
                      entropy_coef=linear_decay_coef(0, 10, c.entropy_bonus, c.final_entropy_bonus),
                      clamp_log_ratio=c.clamp_log_ratio_ref_new_value, temperature=c.temperature,
                      batch_size=float(c.batch_size))


def _run_fused(h, w, b, cfg, chunk, scale=1.0):
    from pipelinerl_amd.finetune.rl.fused import prepare_fields
    from pipelinerl_amd.finetune.rl.fused_linear import linear_grpo_loss

    hp = torch.nn.Parameter(h.clone())
    wp = torch.nn.Parameter(w.clone())
    fields = prepare_fields(to_batch(b), torch.device(DEV))
    loss, stats, rows = linear_grpo_loss(hp, wp, fields, _params(cfg), chunk)
    (loss * scale).backward()
    torch.cuda.synchronize()
    return float(loss.detach()), stats.cpu().numpy(), rows, hp.grad, wp.grad


def _oracle(h, w, b, cfg):
    h64 = h.double().cpu().numpy()
    w64 = w.double().cpu().numpy()
    logits = h64 @ w64.T  # [1, T, V]
    o = grpo_oracle.rl_step_oracle(logits, b, cfg, 0, 10)
    d = o["dlogits"][0]  # [T, V]
    return o, d @ w64, d.T @ h64[0]


@pytest.mark.parametrize("chunk", [5, 4096])
def test_fp32_matches_oracle(chunk):
    V, Hd = 1000, 48
    lens, prompts = [9, 7, 12], [3, 2, 4]
    b = _batch(lens, prompts, V, seed=1)
    g = torch.Generator().manual_seed(1)
    h = (torch.randn((1, sum(lens), Hd), generator=g) * 0.5).to(DEV)
    w = (torch.randn((V, Hd), generator=g) * 0.5).to(DEV)
    loss, stats, rows, dh, dw = _run_fused(h, w, b, CFG, chunk)
    o, dh_o, dw_o = _oracle(h, w, b, CFG)
    assert abs(loss - o["loss"]) <= 1e-4 * max(1.0, abs(o["loss"]))
    from pipelinerl_amd._native import S

    nl_sum = o["stats"]["num_output_tokens_sum"]
    assert stats[S["NUM_OUT"]] == nl_sum
    ok, err = rel_close(dh.cpu().numpy()[0], dh_o, 1e-4, 1e-7)
    assert ok, err
    ok, err = rel_close(dw.cpu().numpy(), dw_o, 1e-4, 1e-7)
    assert ok, err
    # masked rows are never scored: their per-row outputs stay 0 and their dh rows are 0
    mask = (b["labels"][0, 1:] != -100)
    lp = rows[0].cpu().numpy()
    assert np.all(lp[~mask] == 0)
    ok, err = rel_close(lp[mask], o["new_logprobs"][0][mask], 1e-4, 1e-6)
    assert ok, err


@pytest.mark.parametrize("chunk", [3, 4096])
def test_bf16_resident_rows_and_upstream_scale(chunk):
    """Qwen vocab (register-resident kernel with a row map), bf16 GEMMs, upstream 0.5; several
    chunks (fp32 dW accumulator) and one chunk (dW from one bf16-output GEMM)."""
    V, Hd = 151936, 64
    lens, prompts = [6, 5], [2, 3]
    b = _batch(lens, prompts, V, seed=2)
    g = torch.Generator().manual_seed(2)
    h = (torch.randn((1, sum(lens), Hd), generator=g)).to(torch.bfloat16).to(DEV)
    w = (torch.randn((V, Hd), generator=g) * 0.3).to(torch.bfloat16).to(DEV)
    loss, stats, rows, dh, dw = _run_fused(h, w, b, CFG, chunk=chunk, scale=0.5)
    # oracle on the bf16-rounded logits the GEMM produced
    logits = (h[0].float() @ w.float().t()).to(torch.bfloat16).float().cpu().numpy()[None]
    o = grpo_oracle.rl_step_oracle(logits, b, CFG, 0, 10)
    assert abs(loss - o["loss"]) <= 2e-3 * max(1.0, abs(o["loss"]))
    d = o["dlogits"][0] * 0.5
    dh_o = d @ w.double().cpu().numpy()
    dw_o = d.T @ h[0].double().cpu().numpy()
    for got, want in ((dh.float().cpu().numpy()[0], dh_o), (dw.float().cpu().numpy(), dw_o)):
        scale = np.abs(want).max()
        assert np.abs(got - want).max() <= 2e-2 * scale


def test_zero_upstream_and_no_label_rows():
    V, Hd = 512, 32
    b = _batch([6], [5], V, seed=3)  # one label row
    h = torch.randn((1, 6, Hd), device=DEV)
    w = torch.randn((V, Hd), device=DEV)
    _, _, _, dh, dw = _run_fused(h, w, b, CFG, 16, scale=0.0)
    assert torch.count_nonzero(dh) == 0 and torch.count_nonzero(dw) == 0
    b["labels"][:] = -100
    loss, stats, rows, dh, dw = _run_fused(h, w, b, CFG, 16)
    assert loss == 0.0 and torch.count_nonzero(dh) == 0


def test_rl_step_fused_lm_head_matches_full_logits(tmp_path):
    """A tied-embedding Qwen2 (fp32): rl_step with fused_lm_head gives the same loss, stats and
    parameter gradients as the full-logits path."""
    import copy
    import types

    from loop_helpers import EOS, rollouts, tiny_model_dir
    from pipelinerl_amd.finetune.attention import register
    from pipelinerl_amd.finetune.data import collate_packed
    from pipelinerl_amd.finetune.rl import RLConfig, rl_step
    from transformers import AutoConfig, AutoModelForCausalLM

    cfg_m = AutoConfig.from_pretrained(tiny_model_dir(tmp_path))
    cfg_m.tie_word_embeddings = True
    torch.manual_seed(0)
    model = AutoModelForCausalLM.from_config(cfg_m, dtype=torch.float32, attn_implementation=register()).cuda()
    twin = copy.deepcopy(model)
    batch = collate_packed(rollouts(2, 4), types.SimpleNamespace(eos_token_id=EOS), 1).to_device("cuda")
    base = dict(policy_loss="ppo", epsilon=0.2, kl_coef=0.05, final_kl_coef=0.05, entropy_bonus=0.01,
                final_entropy_bonus=0.01, batch_size=8, clamp_log_ratio_ref_new_value=5)
    loss, stats = rl_step(model, batch, 0, 10, RLConfig(**base, fused_lm_head=True, lm_head_chunk_rows=7))
    loss.backward()
    ref_loss, ref_stats = rl_step(twin, batch, 0, 10, RLConfig(**base))
    ref_loss.backward()
    assert abs(float(loss) - float(ref_loss)) <= 1e-4 * max(1, abs(float(ref_loss)))
    for k, v in ref_stats.items():
        assert abs(stats[k] - v) <= 1e-4 * max(1.0, abs(v)), (k, stats[k], v)
    for (n, p), (_, q) in zip(model.named_parameters(), twin.named_parameters()):
        err = float((p.grad - q.grad).abs().max())
        assert err <= 1e-6 + 1e-3 * float(q.grad.abs().max()), (n, err)


def test_fp32_label_rows_at_qwen_vocab():
    """An fp32 model's label-row chunks at V = 151 936 run the part-resident fp32 kernel through
    the row map (prl_grpo_forward_rows): loss, dh and dW against the oracle composed with the
    lm_head, at the fp32 bar."""
    V, Hd = 151936, 64
    lens, prompts = [13, 17], [4, 6]
    b = _batch(lens, prompts, V, seed=5)
    g = torch.Generator().manual_seed(5)
    h = (torch.randn((1, sum(lens), Hd), generator=g) * 0.5).to(DEV)
    w = (torch.randn((V, Hd), generator=g) * 0.5).to(DEV)
    loss, stats, rows, dh, dw = _run_fused(h, w, b, CFG, 4096)
    o, dh_o, dw_o = _oracle(h, w, b, CFG)
    assert abs(loss - o["loss"]) <= 1e-4 * max(1.0, abs(o["loss"]))
    ok, err = rel_close(dh.cpu().numpy()[0], dh_o, 1e-4, 1e-5 * float(np.abs(dh_o).max()))
    assert ok, err
    ok, err = rel_close(dw.cpu().numpy(), dw_o, 1e-4, 1e-5 * float(np.abs(dw_o).max()))
    assert ok, err


class _Decoder(torch.nn.Module):
    """Decoder stub: its last hidden state is a fixed tensor (a parameter, so its gradient is read)."""

    def __init__(self, h: torch.Tensor):
        super().__init__()
        self.h = torch.nn.Parameter(h)

    def forward(self, **kw):
        import types

        return types.SimpleNamespace(last_hidden_state=self.h)


class _IdentityHeadLM(torch.nn.Module):
    """A causal LM whose lm_head is the identity [V, V]: its logits ARE the hidden states, so a
    reference batch's logits can be fed through the label-row lm_head path unchanged (fp32 GEMM
    with an identity weight is exact)."""

    def __init__(self, logits: torch.Tensor):
        super().__init__()
        import types

        V = logits.shape[-1]
        self.model = _Decoder(logits)
        self.lm_head = torch.nn.Linear(V, V, bias=False, device=logits.device)
        with torch.no_grad():
            self.lm_head.weight.copy_(torch.eye(V, device=logits.device))
        self.config = types.SimpleNamespace()

    def get_decoder(self):
        return self.model

    def get_output_embeddings(self):
        return self.lm_head

    def forward(self, logits_to_keep=0, output_hidden_states=False, **kw):
        import types

        h = self.model(**kw).last_hidden_state
        idx = slice(-logits_to_keep, None) if isinstance(logits_to_keep, int) else logits_to_keep
        return types.SimpleNamespace(logits=self.lm_head(h[:, idx, :]), hidden_states=(h,))


class _ValueHeadWrapper(torch.nn.Module):
    """value_model.py's AutoModelForCausalLMWithValueHead shape: ``pretrained_model`` + a value
    head; the values are a parameter here (the reference batch's own), their gradient read back."""

    def __init__(self, lm, values: torch.Tensor):
        super().__init__()
        self.pretrained_model = lm
        self.value_head = torch.nn.Parameter(values)

    def forward(self, **kw):
        import types

        out = self.pretrained_model(output_hidden_states=True, **kw)
        return types.SimpleNamespace(logits=out.logits, value=self.value_head)


def test_f1_value_head_cases_through_the_label_row_head():
    """The reference's default fine-tune config is actor_critic (a value head, conf/base.yaml:2):
    every F1 value-head case (generated by the reference's own rl_step, value_loss_coef 0.1) through
    rl_step's label-row lm_head path — the root forward with no logits rows, the value head on every
    row, lm_head + loss over the label rows, statistics and dvalues from the statistics pass —
    against the reference's outputs at the fp32 bar: loss, every statistic, d loss / d values, and
    d loss / d hidden (= the reference's dlogits through the identity lm_head)."""
    from conftest import load_f1
    from pipelinerl_amd.finetune import rl as rlmod
    from pipelinerl_amd.finetune.rl import RLConfig, rl_step

    batches, out, cases = load_f1()
    calls = []
    orig = rlmod.linear_grpo_loss
    rlmod.linear_grpo_loss = lambda *a, **k: (calls.append(1), orig(*a, **k))[1]
    n = 0
    try:
        for i, c in enumerate(cases):
            if not c["value_head"]:
                continue
            b = batches[c["batch"]]
            logits = torch.tensor(b["logits"], dtype=torch.float32, device=DEV)
            model = _ValueHeadWrapper(_IdentityHeadLM(logits), torch.tensor(b["values"], device=DEV))
            loss, stats = rl_step(model, to_batch(b), c["step"], c["max_step"],
                                  RLConfig(**c["cfg"], fused_lm_head=True, lm_head_chunk_rows=7))
            loss.backward()
            torch.cuda.synchronize()
            assert abs(float(loss) - c["loss"]) <= 1e-4 * max(1, abs(c["loss"])), (i, float(loss), c["loss"])
            assert set(stats) == set(c["stats"]), (i, set(stats) ^ set(c["stats"]))
            for k, v in c["stats"].items():
                assert abs(stats[k] - v) <= 1e-4 * max(1.0, abs(v)), (i, k, stats[k], v)
            ok, err = rel_close(model.value_head.grad.cpu().numpy(), out[f"case{i}__dvalues"], 1e-4, 1e-7)
            assert ok, (i, "dvalues", err)
            ok, err = rel_close(model.pretrained_model.model.h.grad.cpu().numpy(), out[f"case{i}__dlogits"], 1e-4,
                                1e-6)
            assert ok, (i, "dhidden", err)
            n += 1
    finally:
        rlmod.linear_grpo_loss = orig
    assert n == 17 and len(calls) == n  # every value-head case took the label-row path
