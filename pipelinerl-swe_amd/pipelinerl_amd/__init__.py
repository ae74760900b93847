"""pipelinerl_amd — MI355X-native GRPO trainer step + trainer->actor weight broadcast.

Drop-in for ServiceNow/PipelineRL-SWE's hot path: ``finetune.rl.rl_step`` (fused HIP loss
head), ``finetune_loop.run_finetuning_loop`` and the actor-side ``init_actor_update_group`` /
``receive_weight_update``.  Kernels live in ``libprl_hip.so`` (C ABI: include/prl_hip.h).
"""

__version__ = "0.1.0"
