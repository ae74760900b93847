"""The trainer-step FLOP counter (step_flops.py) on a tiny Qwen2, against torch's own FLOP counter
over an eager forward + backward on CPU, and against a hand count."""

from __future__ import annotations

import types

import pytest
import torch


def _tiny():
    from transformers import Qwen2Config, Qwen2ForCausalLM

    cfg = Qwen2Config(vocab_size=96, hidden_size=64, intermediate_size=160, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=256,
                      tie_word_embeddings=False)
    torch.manual_seed(0)
    return cfg, Qwen2ForCausalLM(cfg).float()


def test_hand_count():
    from pipelinerl_amd.step_flops import MicroBatchShape, linear_weights_per_layer, step_flops

    cfg, _ = _tiny()
    # per layer: q 64x64, k 64x32, v 64x32, o 64x64, gate/up/down 64x160 -> 4096+2048+2048+4096+3*10240
    assert linear_weights_per_layer(cfg) == 43008
    f = step_flops(cfg, [MicroBatchShape(tokens=10, seq_lens=[6, 4], label_rows=7)])
    assert f["linear"] == 6 * 43008 * 2 * 10
    assert f["lm_head"] == 6 * 96 * 64 * 7
    # head dim 16, 4 query heads, 2 layers: 6 x 16 x 4 x 2 x (6*7 + 4*5)
    assert f["attention"] == 6 * 16 * 4 * 2 * (42 + 20)
    assert f["total"] == f["linear"] + f["lm_head"] + f["attention"]


@pytest.mark.parametrize("T", [12, 33])
def test_against_torch_flop_counter(T):
    """Eager attention multiplies the FULL score matrix (masked afterwards), and HF's lm_head forms
    logits for every row: torch's count = linear + lm_head over all T rows + 12 x d x heads x layers
    x T^2 (four forward and eight backward L x L products of one sequence).  The counter's causal
    term is that with L^2 -> L(L+1)/2 per product."""
    from torch.utils.flop_counter import FlopCounterMode

    from pipelinerl_amd.step_flops import MicroBatchShape, step_flops

    cfg, model = _tiny()
    model.config._attn_implementation = "eager"
    ids = torch.randint(0, 96, (1, T))
    with FlopCounterMode(display=False) as fc:
        out = model(input_ids=ids)
        out.logits.float().square().mean().backward()
    counted = fc.get_total_flops()
    ours = step_flops(cfg, [MicroBatchShape(tokens=T, seq_lens=[T], label_rows=T - 1)], label_row_head=False)
    d, nh, L = 16, 4, 2
    assert ours["lm_head"] == 6 * 96 * 64 * T
    full_attention = 12 * d * nh * L * T * T
    rotary = d * T  # Qwen2RotaryEmbedding's inv_freq @ positions ([d/2, 1] x [1, T]): not model FLOPs
    assert counted == ours["linear"] + ours["lm_head"] + full_attention + rotary, (counted, ours)
    assert ours["attention"] == full_attention * (T + 1) // (2 * T)


def test_shape_of_a_packed_batch():
    """Sequence lengths from seq_boundaries (a padding tail dropped), label rows = shifted labels."""
    from pipelinerl_amd.step_flops import shape_of

    labels = torch.tensor([[-100, 5, 6, -100, -100, 7, 8, 9, -100, -100]])
    b = types.SimpleNamespace(attention_mask=torch.tensor([[1] * 8 + [0, 0]]), labels=labels,
                              seq_boundaries=torch.tensor([0, 3, 8, 10]), padding=2, position_ids=None)
    s = shape_of(b)
    assert s.tokens == 8 and s.seq_lens == [3, 5] and s.label_rows == 5
    b.padding = 0
    assert shape_of(b).seq_lens == [3, 5, 2]


def test_roofline_fields():
    from pipelinerl_amd.step_flops import mfma_roofline

    f = {"linear": 6e14, "lm_head": 1e14, "attention": 3e14, "total": 1e15}
    r = mfma_roofline(f, 1.0, {"gemm_ms": 500.0, "attention_ms": 200.0, "other_ms": 100.0, "kernel_ms": 800.0,
                               "kernels": 9})
    assert r["bound"] == "mfma" and r["unit"] == "TFLOP/s" and r["achieved"] == 1000.0 and r["frac"] == 0.4
    assert r["gemm_share_of_kernel_time"] == 0.625 and r["gemm_achieved"] == 1400.0 and r["attention_achieved"] == 1500.0


def _roofline_rank(rank, port, out):
    import os
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "pipelinerl-swe_amd"), str(root / "tests")]
    os.environ["OMP_NUM_THREADS"] = "1"
    import torch.distributed as dist
    from cpu_rl_step import cpu_rl_step
    from test_split_pipeline_cpu import _tiny as tiny_bf16

    from pipelinerl_amd.trainer_probe import TrainerStep, step_roofline

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    ts = TrainerStep(tokens=64, seq=32, prompt=8, micro_batches=2, device=torch.device("cpu"), model=tiny_bf16(),
                     step_fn=cpu_rl_step, vocab=96)
    sec = ts.timed(1, 1)
    r = step_roofline(ts, sec)
    torch.save({"r": r, "sec": sec}, Path(out) / f"r{rank}.pt")
    dist.destroy_process_group()


def test_step_roofline_gloo(tmp_path):
    """TrainerStep at world 2 on CPU: the line's roofline holds the FLOPs of one rank's micro-batches
    (2 x 64 tokens: 2 sequences of 32, 24 label rows each),
    the same on both ranks, and achieved = FLOPs / step time."""
    import torch.multiprocessing as mp
    from test_weight_update_cpu import free_port

    from pipelinerl_amd.step_flops import MicroBatchShape, step_flops

    mp.spawn(_roofline_rank, args=(free_port(), str(tmp_path)), nprocs=2, join=True)
    got = [torch.load(tmp_path / f"r{i}.pt") for i in range(2)]
    r = got[0]["r"]
    assert r == got[1]["r"] or r["flops_per_step"] == got[1]["r"]["flops_per_step"]
    from test_split_pipeline_cpu import _tiny as tiny_bf16

    cfg = tiny_bf16().config
    # per micro-batch: 2 sequences of 32 with 8 prompt tokens: 2 x 24 label tokens, each the next token
    # of one logits row
    want = step_flops(cfg, [MicroBatchShape(tokens=64, seq_lens=[32, 32], label_rows=48)] * 2)
    assert r["flops_per_step"] == {k: float(want[k]) for k in ("linear", "lm_head", "attention", "total")}
    assert r["bound"] == "mfma" and abs(r["achieved"] - want["total"] / got[0]["sec"] / 1e12) < 0.06
