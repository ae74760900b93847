"""The trainer -> actor pipeline end to end on one MI355X (tests/test_pipeline_e2e_cpu.py's checks):
``run_finetuning_loop`` on cuda:0 with the product's rl_step (HIP loss head, patched model ops) and
weight updates on, a stand-alone actor process holding its model on the same GPU (HTTP
``/receive_weight_update``, actor group over gloo: RCCL needs one GPU per rank), the trainer's
snapshot by the HIP paths — in place (zero_copy) or the prl_flatten_bf16 staging copy — and the
actor's bucketed receive by the HIP unflatten.  The final checkpoint of the trainer loads back
with the weights the actor holds."""

import pytest

from test_pipeline_e2e_cpu import run_pipeline

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("transport,snapshot", [("bucketed", "zero_copy"), ("per_tensor", "zero_copy"),
                                                ("bucketed", "copy")])
def test_loop_updates_a_standalone_actor_process_gpu(tmp_path, transport, snapshot):
    run_pipeline(tmp_path, transport, snapshot, "cuda")
