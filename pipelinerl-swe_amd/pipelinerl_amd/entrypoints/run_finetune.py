"""Trainer entrypoint (drop-in for pipelinerl/entrypoints/run_finetune.py).

    torchrun --nproc-per-node N -m pipelinerl_amd.entrypoints.run_finetune \
        --config-dir exp/conf --config-name exp_config \
        +me.weight_update_group_init_method=tcp://HOST:9000 +me.weight_update_group_world_size=K \
        +me.llm_urls=http://a:8080+http://b:8080

(accelerate's / DeepSpeed's ``--local_rank=N`` argument is accepted and ignored, as in the
reference.)  Any exception kills the process (non-zero exit), so the launcher's watchdog sees it.
"""

from __future__ import annotations

import argparse
import logging
import sys

from ..config import load_config
from ..finetune_loop import run_finetuning_loop


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
