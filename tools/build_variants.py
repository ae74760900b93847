"""Build A/B experiment variants of libprl_hip.so into pipelinerl_amd/variants/ (git-ignored,
travels to the GPU box).  Run a variant with PRL_LIB=<path> python bench.py ..."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "pipelinerl-swe_amd"))
from pipelinerl_amd._build import build, build_variant  # noqa: E402

VARIANTS = {
    "ld_nt_st_nt": {"PRL_LOAD_AUX": "2", "PRL_STORE_AUX": "2"},  # the round-1..3 default
    "ld_def_st_nt": {"PRL_LOAD_AUX": "0", "PRL_STORE_AUX": "2"},
    "ld_nt_st_def": {"PRL_LOAD_AUX": "2", "PRL_STORE_AUX": "0"},
    "ld_def_st_def": {"PRL_LOAD_AUX": "0", "PRL_STORE_AUX": "0"},
    "copy_ceiling": {"PRL_COPY_CEILING": "1"},
    "row_sequential": {"PRL_ROW_PERMUTE": "0"},
    "swiglu_u1": {"SWIGLU_UNROLL": "1"},
    "attn_xcd_off": {"PRL_ATTN_XCD": "0"},
    "f32_u2": {"PRL_STREAM_F32_U": "2"},
    "f32_wg2": {"PRL_STREAM_F32_WG_PER_CU": "2"},
    "swiglu_u2": {"SWIGLU_UNROLL": "2"},
    "attn_fwd_1wave": {"PRL_ATTN_FWD_MINB": "1"},
    "attn_serial": {"PRL_ATTN_PIPE": "0", "PRL_ATTN_INTERLEAVE": "0"},
    "attn_exp_noload": {"PRL_ATTN_EXP_NOLOAD": "1"},
    "attn_exp_noexp": {"PRL_ATTN_EXP_NOEXP": "1"},
    "attn_exp_noload_noexp": {"PRL_ATTN_EXP_NOLOAD": "1", "PRL_ATTN_EXP_NOEXP": "1"},
    "attn_kv_regs": {"PRL_ATTN_PIPE": "0", "PRL_ATTN_KV_LDS": "0"},
    "attn_vgpr_form": {"PRL_ATTN_PIPE": "0", "PRL_ATTN_KV_LDS": "1", "__flags__": "-mllvm --amdgpu-mfma-vgpr-form=1"},
    "norm_dres_early": {"PRL_NORM_WIDE_DRES_EARLY": "1"},
    "norm_grid1536": {"PRL_NORM_GRID": "1536"},
    "norm_grid3072_early": {"PRL_NORM_GRID": "3072", "PRL_NORM_WIDE_DRES_EARLY": "1"},
    "norm_grid2048": {"PRL_NORM_GRID": "2048"},
    "norm_fwd2048": {"PRL_NORM_FWD_GRID": "2048"},
    "bf16_sw": {"PRL_HW_BF16": "0"},
    "unphased": {"PRL_PHASED": "0"},
    "phased24": {"PRL_PHASED_MAX_NV": "24"},
    "nofence": {"PRL_STORE_FENCE": "0"},
    "noslp": {"__flags__": "-fno-slp-vectorize"},
    "norm_regacc": {"PRL_NORM_BWD_LDS": "0"},
    "norm_lds768": {"PRL_NORM_LDS_GRID": "768"},
    "attn_clock": {"PRL_ATTN_CLOCK_PROBE": "1"},
    "attn_flat_stage": {"PRL_ATTN_BUF_STAGE": "0"},
    "swiglu_gridstride": {"PRL_SWIGLU_PHASED": "0"},
    "swiglu_phased_wg2": {"PRL_SWIGLU_PHASED": "1", "PRL_SWIGLU_PHASED_WG": "2"},
    "swiglu_rows_phased": {"PRL_SWIGLU_ROWS_PHASED": "1"},
    "attn_2wg": {"PRL_ATTN_PIPE": "0", "PRL_ATTN_BWD_MINB": "2", "PRL_ATTN_KV_LDS": "2", "PRL_ATTN_INTERLEAVE": "0", "PRL_ATTN_BSTAGE": "32"},
    "attn_v_lds": {"PRL_ATTN_PIPE": "0", "PRL_ATTN_KV_LDS": "2"},
    "attn_bstage32": {"PRL_ATTN_PIPE": "0", "PRL_ATTN_INTERLEAVE": "0", "PRL_ATTN_BSTAGE": "32"},
    "phased_nowait": {"PRL_PHASED": "2"},
    "attn_nopipe": {"PRL_ATTN_PIPE": "0"},
    "attn_clock_nopipe": {"PRL_ATTN_CLOCK_PROBE": "1", "PRL_ATTN_PIPE": "0"},
    "attn_pipe_sgb": {"PRL_ATTN_PIPE_SCHED": "0"},
    "attn_pipe_lead6": {"PRL_ATTN_PIPE_LEAD": "6"},
    "attn_fwd_tiles": {"PRL_ATTN_FWD_PAIR": "0"},
    "stream_store_nt": {"PRL_STREAM_STORE_SC1": "0"},
    "vec_row_inputs": {"PRL_SCALAR_ROW_INPUTS": "0"},
    "target_select": {"PRL_TARGET_FIXUP": "0"},
    "noent_form_off": {"PRL_NOENT_FORM": "0"},
    "st_sc1": {"PRL_STORE_AUX": "16"},
    "st_sc1_nt": {"PRL_STORE_AUX": "18"},
    "st_sc0_sc1": {"PRL_STORE_AUX": "17"},
    "st_sc0_sc1_nt": {"PRL_STORE_AUX": "19"},
    "ld_sc1_nt_st_sc1_nt": {"PRL_LOAD_AUX": "18", "PRL_STORE_AUX": "18"},
    "ld_sc1_st_sc1_nt": {"PRL_LOAD_AUX": "16", "PRL_STORE_AUX": "18"},
    "ld_def_st_sc1_nt": {"PRL_LOAD_AUX": "0", "PRL_STORE_AUX": "18"},
}

if __name__ == "__main__":
    build(force=True)
    names = sys.argv[1:] or list(VARIANTS)
    for n in names:
        d = dict(VARIANTS[n])
        flags = d.pop("__flags__", "").split()
        print(build_variant(n, d, flags))
