"""Trainer entrypoint (drop-in for pipelinerl/entrypoints/run_finetune.py).

The reference launcher's own command line works with only the script path changed
(launch.py:235-315 builds it; any accelerate config, ``--num_processes N``):

    python -m accelerate.commands.launch --config_file conf/accelerate/base_mp.yaml \
        --rdzv_backend c10d --num_processes N \
        pipelinerl-swe_amd/pipelinerl_amd/entrypoints/run_finetune.py \
        --config-dir exp/conf --config-name exp_config output_dir=exp hydra.run.dir=exp/finetune \
        +me.weight_update_group_init_method=tcp://HOST:9000 +me.weight_update_group_world_size=K \
        +me.llm_urls=http://a:8080+http://b:8080

It also runs as a module (``torchrun --nproc-per-node N -m pipelinerl_amd.entrypoints.run_finetune
…``).  accelerate's / DeepSpeed's ``--local_rank=N`` argument is accepted and dropped, as the
reference does (run_finetune.py:15-20); ranks come from the RANK / WORLD_SIZE / LOCAL_RANK /
MASTER_* environment the launcher sets.  Any exception kills the process (non-zero exit), so the
launcher's watchdog sees it.
"""

from __future__ import annotations

import argparse
import logging
import sys
from pathlib import Path

if __package__ in (None, ""):  # run by path (the reference launcher's form): make the package importable
    sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

from pipelinerl_amd.config import load_config  # noqa: E402
from pipelinerl_amd.finetune_loop import run_finetuning_loop  # noqa: E402


def main(argv: list[str] | None = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    argv = [a for a in argv if not a.startswith("--local_rank") and not a.startswith("--local-rank")]
    ap = argparse.ArgumentParser()
    ap.add_argument("--config-dir", required=True)
    ap.add_argument("--config-name", required=True)
    args, overrides = ap.parse_known_args(argv)
    logging.basicConfig(level=logging.INFO, format="[%(asctime)s][%(name)s][%(levelname)s] - %(message)s")
    cfg = load_config(args.config_dir, args.config_name, overrides)
    run_finetuning_loop(cfg)
    return 0


if __name__ == "__main__":
    sys.exit(main())
