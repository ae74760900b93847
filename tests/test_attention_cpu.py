"""prl_varlen attention (finetune/attention.py) == SDPA with the packed block-causal mask HF
derives from position_ids; CPU exercises the per-sequence fallback."""

import types

import torch


def _models(tmp_path, device):
    from loop_helpers import tiny_model_dir
    from pipelinerl_amd.finetune.attention import register
    from transformers import AutoConfig, AutoModelForCausalLM

    d = tiny_model_dir(tmp_path)
    register()
    torch.manual_seed(0)
    a = AutoModelForCausalLM.from_config(AutoConfig.from_pretrained(d), attn_implementation="prl_varlen").to(device)
    b = AutoModelForCausalLM.from_config(AutoConfig.from_pretrained(d), attn_implementation="sdpa").to(device)
    b.load_state_dict(a.state_dict())
    return a, b


def _packed(device):
    from pipelinerl_amd.finetune.data import collate_packed
    from loop_helpers import EOS, rollouts

    return collate_packed(rollouts(2, 3), types.SimpleNamespace(eos_token_id=EOS), 1)


def check(tmp_path, device):
    """Packed forward/backward with prl_varlen == every rollout run on its own (what flash-attn
    varlen gives the reference).  Note: HF's SDPA with position_ids alone does NOT isolate
    packed sequences in this transformers version (checked below)."""
    from pipelinerl_amd.finetune.attention import packed_kwargs

    a, b = _models(tmp_path, device)
    batch = _packed(device)
    ids, pos = batch.input_ids.to(device), batch.position_ids.to(device)
    bounds = batch.seq_boundaries.tolist()
    la = a(input_ids=ids, position_ids=pos, **packed_kwargs(batch, device)).logits
    alone = torch.cat([b(input_ids=ids[:, s:e], position_ids=pos[:, s:e]).logits
                       for s, e in zip(bounds[:-1], bounds[1:])], 1)
    assert torch.allclose(la, alone, atol=2e-5, rtol=1e-4), float((la - alone).abs().max())
    la.square().mean().backward()
    alone.square().mean().backward()
    for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
        assert torch.allclose(p.grad, q.grad, atol=1e-5, rtol=1e-3), n
    # isolation: changing sequence 0 leaves sequence 1 untouched
    ids2 = ids.clone()
    ids2[0, 0] = (ids2[0, 0] + 1) % 90
    with torch.no_grad():
        la2 = a(input_ids=ids2, position_ids=pos, **packed_kwargs(batch, device)).logits
        s1 = bounds[1]
        assert torch.allclose(la2[0, s1:], la[0, s1:].detach(), atol=1e-6)
        lb = b(input_ids=ids, position_ids=pos).logits
        lb2 = b(input_ids=ids2, position_ids=pos).logits
        sdpa_isolated = torch.allclose(lb2[0, s1:], lb[0, s1:], atol=1e-6)
    return sdpa_isolated


def test_varlen_fallback_cpu(tmp_path):
    check(tmp_path, "cpu")


def test_split_plan_covers_every_block_once():
    """split_plan (host side of prl_attn_bwd_split): every (key block, kv head) is computed exactly
    once — unsplit, or as parts whose query-head ranges tile the group in order — the slots are
    0..n-1, groups point at their parts, heavy blocks of a lone sequence are split and a packing
    of many equal sequences is not (the modelled launch is no faster split)."""
    from pipelinerl_amd.finetune.attention import BLOCK, split_plan

    for bounds, heads, kv in (([0, 4096], 28, 4), ([0, 6122], 12, 2), ([0, 3000, 3400, 3500], 28, 4),
                              ([0, 8192, 16384], 28, 4), ([0, 1, 37, 300, 531, 1024, 1151], 12, 2),
                              ([0, 4096], 40, 8), ([0, 3000, 3400, 3500], 40, 8), ([0, 4096], 14, 2)):
        rep = heads // kv
        kv_rows, units, groups, slots = split_plan(bounds, heads, kv, 256)
        blocks = {(a, b, x) for a, b in zip(bounds[:-1], bounds[1:]) for x in range(a, b, BLOCK)}
        split_blocks = {(u[0], u[1], u[2]) for u in units}
        assert set(kv_rows) | split_blocks == blocks and not (set(kv_rows) & split_blocks)
        assert sorted(u[6] for u in units) == list(range(slots))
        by_slot = {u[6]: u for u in units}
        for s1, kb, g, slot0, n in groups:
            parts = [by_slot[slot0 + p] for p in range(n)]
            assert all(p[1] == s1 and p[2] == kb and p[3] == g for p in parts)
            assert [p[4] for p in parts] == [g * rep] + [p[5] for p in parts[:-1]]  # contiguous, in order
            assert parts[-1][5] == (g + 1) * rep and 2 <= n <= rep
        assert len(groups) == len({(u[0], u[1], u[2], u[3]) for u in units})
        if bounds in ([0, 4096], [0, 6122]) and heads != 40:  # 8 kv heads: enough key-block work unsplit
            assert units
        if (bounds, heads) == ([0, 3000, 3400, 3500], 40):  # a group of 5 split into parts
            assert units
        if bounds == [0, 8192, 16384]:
            assert not units


def test_split_plan_is_priced_by_the_launch_model():
    """The chosen plan's modelled makespan (list schedule of the fused launch + the partial reduce)
    is never above the unsplit launch's, and the fixed part cap of round 2 (PRL_ATTN_SPLIT_CAP=1.0)
    is still available."""
    from pipelinerl_amd.finetune import attention as A

    for lens, heads, kv in (([8511], 28, 4), ([3755, 1617, 6053], 28, 4), ([2048] * 4, 28, 4),
                            ([2048] * 32, 12, 2), ([6122], 12, 2), ([1, 700, 2200, 200], 14, 2)):
        bounds = [sum(lens[:i]) for i in range(len(lens) + 1)]
        rows = [(a, b, x) for a, b in zip(bounds[:-1], bounds[1:]) for x in range(a, b, A.BLOCK)]
        kv_rows, units, groups, slots = A.split_plan(bounds, heads, kv, 256)
        t = A._makespan(rows, kv_rows, units, slots, heads, kv, 256)
        t_one = A._makespan(rows, rows, [], 0, heads, kv, 256)
        assert t <= t_one and (not units or t < (1 - A.SPLIT_MARGIN) * t_one)
    saved = A.SPLIT_CAP_FRAC
    try:
        A.SPLIT_CAP_FRAC = 1.0
        assert not A.split_plan([0, 8511], 28, 4, 256)[1]  # below 1.2 x target: unsplit under the old rule
    finally:
        A.SPLIT_CAP_FRAC = saved
    assert A.split_plan([0, 8511], 28, 4, 256)[1]  # the model splits it (2.32 -> 2.09 ms measured)
