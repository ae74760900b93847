"""End-to-end trainer-loop throughput: ``run_finetuning_loop`` (the product path of
finetune_loop.py, reference pipelinerl/finetune_loop.py:567-719) on one GPU, fed from a
files-backend ``training_data`` stream of variable-length packed rollouts, exactly as the
preprocessor would write them (MicroBatchPacker: per-step sample quotas, sentinels).

What it adds over trainer_probe: the stream reader thread, host->device batch transfer, the
lockstep sample-count exchange, per-micro-batch stats, lr scheduler, metrics logging and the
final checkpoint write — everything the loop does around the compute.

    python tools/loop_bench.py --model 1.5b --seq-length 16384 --samples-per-step 64 --steps 4

Prints one JSON line: steady-state tokens/s from the loop's own ``throughput/*`` metrics
(step 1 excluded: it carries the kernel/library warm-up); wall clock between step logs, each
taken after a device synchronize.
"""

from __future__ import annotations

import argparse
import copy
import json
import os
import sys
import tempfile
import time
import types
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "pipelinerl-swe_amd")]

EOS = 151643  # Qwen2.5 <|endoftext|>


def make_rollouts(n: int, group: int, mean_len: int, prompt: int, vocab: int, seed: int, dist: str = "uniform"):
    """dist "uniform": length U[mean/2, 3 mean/2) with a fixed prompt; "c3": BASELINE configs[2]'s
    math rollouts, prompt U{64..512} + completion U{256..8192} (max_tokens 8192)."""
    import numpy as np

    from pipelinerl_amd.finetune.rl import RLConfig, populate_rl_data, prepare_rl_fields

    rng = np.random.default_rng(seed)
    data = []
    for i in range(n):
        if dist == "c3":
            prompt = int(rng.integers(64, 513))
            L = prompt + int(rng.integers(256, 8193))
        else:
            L = int(rng.integers(mean_len // 2, mean_len * 3 // 2))
        c = L - prompt
        ids = rng.integers(0, EOS, L).tolist()
        if rng.random() < 0.75:
            ids[-1] = EOS
        lps = (-rng.random(c) * 4).astype(np.float32).tolist()
        enc = prepare_rl_fields({"input_ids": ids, "labels": [-100] * prompt + ids[prompt:],
                                 "attention_mask": [1] * L}, float(rng.integers(0, 2)), lps, lps)
        enc.update(group_id=f"g{i // group}", rollout_index=i % group, step_index=0, model_version=0)
        data.append(enc)
    return populate_rl_data(data, EOS, RLConfig(divide_advantage_by_std=False))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="1.5b")
    ap.add_argument("--seq-length", type=int, default=16384)
    ap.add_argument("--samples-per-step", type=int, default=64)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--mean-len", type=int, default=2048)
    ap.add_argument("--prompt", type=int, default=256)
    ap.add_argument("--full-logits", action="store_true",
                    help="materialise [T, V] logits (RLConfig.fused_lm_head off; the label-row path is the default)")
    ap.add_argument("--dist", choices=["uniform", "c3"], default="uniform",
                    help="rollout lengths: uniform around --mean-len, or configs[2]'s U{64..512} + U{256..8192}")
    ap.add_argument("--eager-ops", action="store_true", help="HF element-wise chains instead of the HIP model ops")
    ap.add_argument("--grad-ckpt", action="store_true",
                    help="gradient_checkpointing: true, as the reference config sets it (conf/finetune/base.yaml:45)")
    ap.add_argument("--ckpt-policy", choices=["auto", "always"], default="auto",
                    help="gradient_checkpointing_policy (finetune/recompute.py)")
    ap.add_argument("--keep-layers", type=int, default=None,
                    help="finetune.gradient_checkpointing_keep_layers (with --grad-ckpt: the last K layers keep activations)")
    ap.add_argument("--alloc", default=None,
                    help="finetune.allocator_settings (devalloc.py; default: the product's; 'none': torch's own)")
    ap.add_argument("--workdir", default=None)
    a = ap.parse_args()

    from transformers import Qwen2Config

    from pipelinerl_amd.config import Cfg
    from pipelinerl_amd.finetune.packing import MicroBatchPacker
    from pipelinerl_amd.finetune_loop import run_finetuning_loop
    from pipelinerl_amd.streams import SingleStreamSpec, reset_streams_backend, set_streams_backend, write_to_streams
    from pipelinerl_amd.trainer_probe import QWEN

    exp = Path(a.workdir or tempfile.mkdtemp(prefix="loop_bench_"))
    model_dir = exp / "model"
    model_dir.mkdir(parents=True, exist_ok=True)
    Qwen2Config(max_position_embeddings=32768, rope_theta=1e6, rms_norm_eps=1e-6, eos_token_id=EOS,
                bos_token_id=EOS, **QWEN[a.model]).save_pretrained(model_dir)

    t0 = time.time()
    n = a.samples_per_step * a.steps
    data = make_rollouts(n, 8, a.mean_len, a.prompt, QWEN[a.model]["vocab_size"], 0, a.dist)
    reset_streams_backend()
    set_streams_backend("files")
    packer = MicroBatchPacker(1, a.seq_length, a.samples_per_step, types.SimpleNamespace(eos_token_id=EOS))
    writes = packer.feed(copy.deepcopy(data))
    with write_to_streams(SingleStreamSpec(exp_path=exp, topic="training_data", partition=0)) as w:
        for _, b in writes:
            w.write(b)
    prep_s = time.time() - t0
    reset_streams_backend()

    for k in ("RANK", "WORLD_SIZE", "MASTER_ADDR"):
        os.environ.pop(k, None)
    ft = dict(
        config_name=str(model_dir), model_class="causal-language-modeling", output_dir=str(exp / "finetune"),
        load_as_bf16=True, attn_implementation="flash_attention_2", gradient_checkpointing=a.grad_ckpt,
        gradient_checkpointing_policy=a.ckpt_policy, seq_length=a.seq_length, optim="adamw_torch",
        learning_rate=1e-6, weight_decay=0.01, lr_scheduler_type="cosine", num_warmup_steps=0,
        max_train_steps=a.steps, interrupt_train_steps=-1, gradient_accumulation_passes=a.samples_per_step,
        train_batch_size=1, seq_parallel=1, seed=42, gradient_clipping_threshold=0.3, input="training_data",
        send_weight_updates=False, weight_update_interval=1, log_each_n_steps=1, save_checkpoint_steps=10 ** 6,
        also_save_steps=[], keep_intermediate_checkpoints=False, save_final_training_state=False,
        force_restart=False, max_lag=None, dist_backend=None, data_timeout_s=600, fused_model_ops=not a.eager_ops,
        rl=dict(policy_loss="ppo", epsilon=4, kl_coef=0.0, final_kl_coef=0.0, clamp_log_ratio_ref_new_value=5,
                temperature=1.0, divide_advantage_by_std=False, aggregate_loss="sum",
                fused_lm_head=not a.full_logits))
    if a.alloc is not None:
        ft["allocator_settings"] = None if a.alloc == "none" else a.alloc
    if a.keep_layers is not None:
        ft["gradient_checkpointing_keep_layers"] = a.keep_layers
    cfg = Cfg.wrap({"output_dir": str(exp), "streams": {"backend": "files"}, "finetune": ft,
                    "me": {"weight_update_group_init_method": None, "weight_update_group_world_size": 0,
                           "llm_urls": ""}})
    import torch

    import pipelinerl_amd.finetune_loop as fl

    stamps = []
    orig_log = fl.log_metrics

    def timed_log(step, md, log_dir):  # the step's GPU work is done when its metrics are logged
        torch.cuda.synchronize()
        stamps.append(time.time())
        orig_log(step, md, log_dir)

    fl.log_metrics = timed_log
    t1 = time.time()
    m = run_finetuning_loop(cfg)
    loop_s = time.time() - t1
    ms = torch.cuda.memory_stats()
    lines = [json.loads(x) for x in (exp / "finetune" / "logs" / "metrics.jsonl").read_text().splitlines()]
    steady = lines[1:] or lines
    tok = sum(x["throughput/tokens_per_step"] for x in steady)
    # wall time between the logs of step 1 and step N: data, stats, optimizer, scheduler included
    sec = stamps[-1] - stamps[0] if len(stamps) > 1 else loop_s
    out = {"tool": "loop_bench", "model": f"Qwen2.5-{a.model} shapes (random init, bf16)",
           "seq_length": a.seq_length, "samples_per_step": a.samples_per_step, "mean_rollout_len": a.mean_len, "length_dist": a.dist,
           "fused_lm_head": not a.full_logits, "fused_model_ops": not a.eager_ops, "steps": m.completed_steps,
           "gradient_checkpointing": a.grad_ckpt, "checkpointing_policy": a.ckpt_policy, "keep_layers": a.keep_layers, "allocator_settings": ft.get("allocator_settings", "default"),
           "micro_batches_per_step": [x["throughput/micro_batches_per_step"] for x in lines],
           "tokens_per_step": [x["throughput/tokens_per_step"] for x in lines],
           "step_wall_s": [round(b - a_, 3) for a_, b in zip(stamps, stamps[1:])],
           "steady_tokens_per_s": round(tok / sec, 1),
           "compute_tokens_per_s": round(sum(x["throughput/tokens_per_sec"] for x in steady) / len(steady), 1),
           "passes_s": [round(x["throughput/sec_per_pass"] * x["throughput/micro_batches_per_step"], 3) for x in lines],
           "waiting_for_data_s": [round(b - a_, 3) for a_, b in zip([0.0] + [x["stats/time_waiting_for_data"] for x in lines],
                                                                    [x["stats/time_waiting_for_data"] for x in lines])],
           "trace_ms": {k: [x.get(k) for x in lines] for k in sorted({k for x in lines for k in x if k.startswith("trace/")})},
           "loss": [x.get("rl/loss") for x in lines], "prep_s": round(prep_s, 1), "loop_s": round(loop_s, 1),
           "allocator": {k: ms.get(k) for k in ("num_alloc_retries", "num_device_alloc", "num_device_free",
                                                  "num_ooms")} | {"peak_reserved_gb": round(ms.get("reserved_bytes.all.peak", 0) / 1e9, 2),
                                                                       "peak_allocated_gb": round(ms.get("allocated_bytes.all.peak", 0) / 1e9, 2)}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
