"""A second, independent c10d group joining trainer rank 0 and every actor GPU
(contract of pipelinerl/torch_utils.py:16-65).

The group lives outside the trainer's default (DP) world: its own rendezvous
(``tcp://<master>:<world.actor_group_port>``), world size
``total_actor_llms * gpus_per_llm + 1`` (world.py:184), trainer = rank 0, actor worker w of
LLM i = ``1 + i * ngpus + w`` (vllm1.py:62).  On MI355X the "nccl" backend is RCCL over xGMI.

Wire compatibility with unmodified reference actors requires the same store key layout:
rendezvous store -> PrefixStore(group_name) -> torch's group helper (which adds
"<group_name>/<device>/").  torch exposes no public constructor for a group outside the
default world, so the (private) helper is called here exactly as torch's own
init_process_group does.
"""

from __future__ import annotations

from datetime import timedelta
from typing import Any

import torch
import torch.distributed.distributed_c10d as c10d


def collective_options(backend: str | None, high_priority: bool = True):
    """``pg_options`` for an RCCL ("nccl") group: its collectives run on high-priority HIP streams
    (ProcessGroupNCCL.Options.is_high_priority_stream).  The HIP runtime gives high-priority streams
    hardware queues of their own (tools/queue_probe.py, profiles/r06_queue_probe.json): a collective
    then never waits in the compute stream's queue behind the trainer's kernels, which run in order
    within one queue — with GPU_MAX_HW_QUEUES at its default 4 the normal-priority streams of a rank
    (compute, GradBuckets', the weight update's, the process groups' own) otherwise share four
    queues.  None for other backends (gloo runs on host threads)."""
    if not high_priority or "nccl" not in str(backend or "").lower():
        return None
    import torch.distributed as dist

    return dist.ProcessGroupNCCL.Options(is_high_priority_stream=True)


def init_extra_process_group(backend: str | None = None, init_method: str | None = None,
                             timeout: timedelta | None = None, world_size: int = -1, rank: int = -1,
                             store: Any = None, group_name: str | None = None, pg_options: Any = None,
                             device_id: torch.device | None = None):
    if store is not None and init_method is not None:
        raise ValueError("Cannot specify both init_method and store.")
    if store is not None and (world_size <= 0 or rank < 0):
        raise ValueError("world_size and rank are required with an explicit store")
    timeout = timeout or c10d.default_pg_timeout
    be = c10d.Backend(backend) if backend else c10d.Backend("undefined")
    if store is None:
        store, rank, world_size = next(c10d.rendezvous(init_method or "env://", rank, world_size, timeout=timeout))
        store.set_timeout(timeout)
        store = c10d.PrefixStore(group_name, store)
    kwargs = dict(group_name=group_name, backend_options=pg_options, timeout=timeout)
    if device_id is not None:
        kwargs["device_id"] = device_id
    pg, _ = c10d._new_process_group_helper(world_size, rank, [], be, store, **kwargs)
    c10d._world.pg_group_ranks[pg] = {i: i for i in range(world_size)}
    return pg
