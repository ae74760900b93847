"""Build A/B experiment variants of libprl_hip.so into pipelinerl_amd/variants/ (git-ignored and
gpurun-ignored: build them on the GPU box as the first step of an A/B command, hipcc is there).
Run a variant with PRL_LIB=<path> python bench.py ...  Settled arms are retired from the source
(round 6: the phased schedule, the target fix-up, the no-entropy and folded exponent forms, the
scalar row inputs, the streaming kernels' sc1 stores, the resident row permutation, the pair
kernel's claim-order rows); profiles/README.md keeps their measurements."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "pipelinerl-swe_amd"))
from pipelinerl_amd._build import build, build_variant  # noqa: E402

VARIANTS = {  # the loss head's A/B builds (csrc/grpo_loss.hip macros); profiles/README.md cites each result
    "ld_nt_st_nt": {"PRL_LOAD_AUX": "2", "PRL_STORE_AUX": "2"},  # the round-1..2 cache policy
    "ld_def_st_nt": {"PRL_LOAD_AUX": "0", "PRL_STORE_AUX": "2"},
    "ld_def_st_def": {"PRL_LOAD_AUX": "0", "PRL_STORE_AUX": "0"},
    "st_sc1_nt": {"PRL_STORE_AUX": "18"},
    "ld_sc1_nt_st_sc1_nt": {"PRL_LOAD_AUX": "18", "PRL_STORE_AUX": "18"},
    "copy_ceiling": {"PRL_COPY_CEILING": "1"},  # same schedule, no math: the kernel's own ceiling
    "no_math": {"PRL_COPY_CEILING": "1", "PRL_NO_PASS1": "1"},  # neither pass's math (measurement only)
    "phased24": {"PRL_PHASED_MAX_NV": "24"},
    "nofence": {"PRL_STORE_FENCE": "0"},  # the round-2 store hazard (wrong results: probes only)
    "f32_u2": {"PRL_STREAM_F32_U": "2"},
    "hyb_off": {"PRL_HYB_NL": "-1"},
    "aw_u8": {"PRL_ADAMW_UNROLL": "8"},  # the fp32-master AdamW with 8 units in flight per thread (the first build)
    "aw_u2": {"PRL_ADAMW_UNROLL": "2"},
}

if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    if not sys.argv[1:]:
        build(force=True)
    for n in names:
        d = dict(VARIANTS[n])
        flags = d.pop("__flags__", "").split()
        print(build_variant(n, d, flags))
