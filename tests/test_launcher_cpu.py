"""The reference launcher's own trainer command runs the build's entry script by path.

pipelinerl/launch.py:235-315 starts every trainer as
    python -m accelerate.commands.launch [--use_deepspeed …] --config_file conf/accelerate/<cfg>.yaml
        --rdzv_backend c10d --num_processes N pipelinerl/entrypoints/run_finetune.py
        --config-dir <exp>/conf --config-name exp_config output_dir=<exp>
        hydra.run.dir=<exp>/finetune +me.weight_update_group_init_method=tcp://… 
        +me.weight_update_group_world_size=K +me.llm_urls=…  [finetune.send_weight_updates=False]
This test runs exactly that argv (the non-DeepSpeed flavour: DeepSpeed is not installed here)
with only the script path changed, two ranks over gloo on CPU, on an exp_config composed like the
one launch.py:547 saves (the golden math + grpo config, a tiny model).  The loss step on CPU is the
torch restatement (tests/launcher_site/sitecustomize.py): the HIP loss head needs a GPU.
"""

from __future__ import annotations

import json
import os
import subprocess
import sys
from pathlib import Path

import yaml

from conftest import GOLDEN
from test_finetune_loop_cpu import _setup, free_port

ROOT = Path(__file__).resolve().parents[1]
ENTRY = ROOT / "pipelinerl-swe_amd" / "pipelinerl_amd" / "entrypoints" / "run_finetune.py"

# the keys of the reference's conf/accelerate/base_mp.yaml (the launcher's choice without
# DeepSpeed or FSDP, launch.py:276-283)
ACCELERATE_BASE_MP = dict(
    command_file=None, commands=None, compute_environment="LOCAL_MACHINE", distributed_type="MULTI_GPU",
    mixed_precision="bf16", dynamo_backend="NO", fsdp_config={}, gpu_ids=None, machine_rank=0,
    main_process_ip=None, main_process_port=None, main_training_function="main", megatron_lm_config={},
    num_processes=1, num_machines=1, rdzv_backend="c10d", same_network=True)


def test_reference_launcher_command_runs_the_entry_by_path(tmp_path):
    exp = tmp_path / "exp"
    exp.mkdir()
    world = 2
    per_step, _ = _setup(exp, world)
    raw = yaml.safe_load((GOLDEN / "exp_config_math_grpo.yaml").read_text())
    raw["model_path"] = str(exp / "tiny_qwen2")
    raw["output_dir"] = "/nonexistent"  # the launcher's output_dir= override must win
    raw["use_deepspeed"] = False
    raw["streams"] = {"backend": "files"}
    raw["finetune"].update(seq_length=28, train_batch_size=1, gradient_accumulation_passes=per_step,
                           max_train_steps=2, learning_rate=1e-3, load_as_bf16=False,
                           gradient_checkpointing=False, save_checkpoint_steps=100, log_each_n_steps=1,
                           data_timeout_s=120)
    (exp / "conf").mkdir()
    (exp / "conf" / "exp_config.yaml").write_text(yaml.safe_dump(raw))
    acc = tmp_path / "base_mp.yaml"
    acc.write_text(yaml.safe_dump(ACCELERATE_BASE_MP))
    port = free_port()
    cmd = [sys.executable, "-m", "accelerate.commands.launch", "--config_file", str(acc), "--rdzv_backend", "c10d",
           "--num_processes", str(world), str(ENTRY),
           "--config-dir", f"{exp}/conf", "--config-name", "exp_config", f"output_dir={exp}",
           f"hydra.run.dir={exp}/finetune", f"+me.weight_update_group_init_method=tcp://127.0.0.1:{free_port()}",
           "+me.weight_update_group_world_size=2", "+me.llm_urls=http://127.0.0.1:1+http://127.0.0.1:2",
           "finetune.send_weight_updates=False"]
    env = dict(os.environ, PRL_TEST_CPU_STEP="1", OMP_NUM_THREADS="1", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
               PYTHONPATH=os.pathsep.join([str(ROOT / "tests" / "launcher_site"), os.environ.get("PYTHONPATH", "")]))
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-6000:])
    fin = exp / "finetune"
    summary = json.loads((fin / "summary.json").read_text())
    assert summary["completed_steps"] == 2 and summary["samples"] == 2 * per_step
    assert (fin / "current" / "config.json").exists() and (fin / "training_state" / "training_state.pt").exists()
    lines = [json.loads(x) for x in (fin / "logs" / "metrics.jsonl").read_text().splitlines()]
    assert [ln["step"] for ln in lines] == [1, 2] and "rl/loss" in lines[-1]
    # both ranks ran (each logs to its own file)
    assert (fin / "logs" / "info_0.log").exists() and (fin / "logs" / "info_1.log").exists()


def test_reference_default_deepspeed_config_unchanged_through_torchrun(tmp_path):
    """The reference's DEFAULT exp_config — use_deepspeed true, deepspeed_config deepspeed_stage3_bf16,
    bf16 weights (conf/base.yaml:94-96) — left unchanged, launched one process per rank (torchrun:
    the launcher's accelerate --use_deepspeed needs DeepSpeed installed for accelerate itself, the
    trainer never imports it).  The trainer honours it: DeepSpeed's gradient scale, fp32 master
    weights and moments, and the ZeRO-3 layout decision logged (replicas here: a tiny model fits)."""
    exp = tmp_path / "exp"
    exp.mkdir()
    world = 2
    per_step, _ = _setup(exp, world)
    raw = yaml.safe_load((GOLDEN / "exp_config_math_grpo.yaml").read_text())
    assert raw["use_deepspeed"] is True and raw["deepspeed_config"] == "deepspeed_stage3_bf16"
    raw["model_path"] = str(exp / "tiny_qwen2")
    raw["streams"] = {"backend": "files"}
    raw["finetune"].update(seq_length=28, train_batch_size=1, gradient_accumulation_passes=per_step,
                           max_train_steps=2, learning_rate=1e-3, gradient_checkpointing=False,
                           save_checkpoint_steps=100, log_each_n_steps=1, data_timeout_s=120)
    (exp / "conf").mkdir()
    (exp / "conf" / "exp_config.yaml").write_text(yaml.safe_dump(raw))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), str(ENTRY),
           "--config-dir", f"{exp}/conf", "--config-name", "exp_config", f"output_dir={exp}",
           f"hydra.run.dir={exp}/finetune", f"+me.weight_update_group_init_method=tcp://127.0.0.1:{free_port()}",
           "+me.weight_update_group_world_size=2", "+me.llm_urls=http://127.0.0.1:1+http://127.0.0.1:2",
           "finetune.send_weight_updates=False"]
    env = dict(os.environ, PRL_TEST_CPU_STEP="1", OMP_NUM_THREADS="1", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="",
               PYTHONPATH=os.pathsep.join([str(ROOT / "tests" / "launcher_site"), os.environ.get("PYTHONPATH", "")]))
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-6000:])
    fin = exp / "finetune"
    assert json.loads((fin / "summary.json").read_text())["completed_steps"] == 2
    log = (fin / "logs" / "info_0.log").read_text()
    assert "model state layout: replicas (DeepSpeed ZeRO-3 config" in log, log[-2000:]
    assert "fp32 master weights + fp32 AdamW moments" in log
    import torch

    st = torch.load(fin / "training_state" / "training_state.pt", weights_only=True)
    s0 = st["optimizer_state"]["state"][0]
    assert s0["master"].dtype == torch.float32 and s0["exp_avg"].dtype == torch.float32
    from safetensors.torch import load_file

    assert {t.dtype for t in load_file(str(fin / "current" / "model.safetensors")).values()} == {torch.bfloat16}
