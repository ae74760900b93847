"""Test infrastructure for trainer-loop tests: tiny Qwen2 configs, synthetic rollouts packed
into training_data streams with the reference's quota/sentinel protocol, configs."""

from __future__ import annotations

import copy
import types
from pathlib import Path

import numpy as np

EOS = 95


def tiny_model_dir(tmp: Path, vocab: int = 96) -> Path:
    from transformers import Qwen2Config

    d = tmp / "tiny_qwen2"
    d.mkdir(parents=True, exist_ok=True)
    Qwen2Config(vocab_size=vocab, hidden_size=32, intermediate_size=64, num_hidden_layers=2, num_attention_heads=4,
                num_key_value_heads=2, max_position_embeddings=256, tie_word_embeddings=True, eos_token_id=EOS,
                bos_token_id=EOS, rms_norm_eps=1e-6).save_pretrained(d)
    return d


def rollouts(n_groups: int, attempts: int, seed: int = 0, vocab: int = 96):
    from pipelinerl_amd.finetune.rl import RLConfig, populate_rl_data, prepare_rl_fields

    rng = np.random.default_rng(seed)
    data = []
    for g in range(n_groups):
        for a in range(attempts):
            p, c = int(rng.integers(3, 9)), int(rng.integers(3, 12))
            ids = rng.integers(0, vocab - 1, p + c).tolist()
            if rng.random() < 0.75:
                ids[-1] = EOS
            labels = [-100] * p + ids[p:]
            lps = (-rng.random(c) * 4).tolist()
            enc = prepare_rl_fields({"input_ids": ids, "labels": labels, "attention_mask": [1] * len(ids)},
                                    float(rng.integers(0, 2)), lps, lps)
            enc.update(group_id=f"g{g}", rollout_index=a, step_index=0, model_version=0)
            data.append(enc)
    return populate_rl_data(data, EOS, RLConfig(divide_advantage_by_std=False))


def write_training_data(exp: Path, data, num_trainers: int, seq_length: int, per_lead: int):
    from pipelinerl_amd.finetune.packing import MicroBatchPacker
    from pipelinerl_amd.streams import SingleStreamSpec, write_to_streams

    packer = MicroBatchPacker(num_trainers, seq_length, per_lead, types.SimpleNamespace(eos_token_id=EOS))
    writes = packer.feed(copy.deepcopy(data))
    for tid in range(num_trainers):
        with write_to_streams(SingleStreamSpec(exp_path=exp, topic="training_data", partition=tid)) as w:
            for t, b in writes:
                if t == tid:
                    w.write(b)
    return writes


def loop_cfg(exp: Path, model_dir: Path, world: int, passes: int, steps: int, **finetune):
    from pipelinerl_amd.config import Cfg

    ft = dict(
        config_name=str(model_dir), model_class="causal-language-modeling", output_dir=str(exp / "finetune"),
        load_as_bf16=False, attn_implementation="flash_attention_2", gradient_checkpointing=False, optim="adamw_torch",
        learning_rate=1e-3, weight_decay=0.01, lr_scheduler_type="cosine", num_warmup_steps=0,
        max_train_steps=steps, interrupt_train_steps=-1, gradient_accumulation_passes=passes,
        train_batch_size=1, seq_parallel=1, seed=42, gradient_clipping_threshold=0.3, input="training_data",
        send_weight_updates=False, weight_update_interval=1, log_each_n_steps=1, save_checkpoint_steps=100,
        also_save_steps=[], keep_intermediate_checkpoints=False, save_final_training_state=True,
        force_restart=False, max_lag=None, dist_backend="gloo", grad_reduce="sum", data_timeout_s=60,
        rl=dict(policy_loss="ppo", epsilon=4, kl_coef=0.0, final_kl_coef=0.0, clamp_log_ratio_ref_new_value=5,
                temperature=1.0, divide_advantage_by_std=False, aggregate_loss="sum"))
    ft.update(finetune)
    return Cfg.wrap({"output_dir": str(exp), "streams": {"backend": "files"}, "finetune": ft,
                     "me": {"weight_update_group_init_method": None, "weight_update_group_world_size": 0,
                            "llm_urls": ""}})
