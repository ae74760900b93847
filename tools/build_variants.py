"""Build A/B experiment variants of libprl_hip.so into pipelinerl_amd/variants/ (git-ignored,
travels to the GPU box).  Run a variant with PRL_LIB=<path> python bench.py ..."""
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
    "row_sequential": {"PRL_ROW_PERMUTE": "0"},
    "unphased": {"PRL_PHASED": "0"},
    "phased_nowait": {"PRL_PHASED": "2"},  # phased order, no wait for the stores before the next row's loads
    "phased24": {"PRL_PHASED_MAX_NV": "24"},
    "nofence": {"PRL_STORE_FENCE": "0"},  # the round-2 store hazard (wrong results: probes only)
    "f32_u2": {"PRL_STREAM_F32_U": "2"},
    "stream_store_nt": {"PRL_STREAM_STORE_SC1": "0"},
    "vec_row_inputs": {"PRL_SCALAR_ROW_INPUTS": "0"},
    "target_select": {"PRL_TARGET_FIXUP": "0"},
    "hyb_off": {"PRL_HYB_NL": "-1"},
    "pair_perm": {"PRL_PAIR_PERMUTE": "1"},  # the fp32 pair kernel's rows through perm_row (round 6 A/B)
    "fold_off": {"PRL_FOLD_EXP": "0"},  # the bf16 kernel's (x - M) c exponent forms (round 2-5)  # fp32 rows on the streaming kernel instead of the part-resident one
}

if __name__ == "__main__":
    build(force=True)
    names = sys.argv[1:] or list(VARIANTS)
    for n in names:
        d = dict(VARIANTS[n])
        flags = d.pop("__flags__", "").split()
        print(build_variant(n, d, flags))
