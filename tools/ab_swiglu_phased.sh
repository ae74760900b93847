# SwiGLU read/write phased kernels (PRL_SWIGLU_PHASED=1 variant: contiguous and row-strided forms)
# vs the grid-stride ones: model-op and fused-MLP tests on the variant, then tools/ew_bench.py and
# the C3 step (fused gate/up: the row-strided kernels), alternated  -> gpurun_out/ab_swiglu_phased.jsonl
set -e
mkdir -p gpurun_out
V=pipelinerl-swe_amd/pipelinerl_amd/variants
PRL_LIB=$PWD/$V/libprl_hip_swiglu_phased.so timeout -k 10 300 python -u -m pytest tests/test_model_ops_gpu.py tests/test_fused_mlp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -1
for rep in 1 2; do
  for v in main swiglu_phased; do
    if [[ $v == main ]]; then unset PRL_LIB; else export PRL_LIB=$PWD/$V/libprl_hip_$v.so; fi
    timeout -k 10 120 python -u tools/ew_bench.py | sed "s/}$/, \"variant\": \"$v\"}/" >> gpurun_out/ab_swiglu_phased.jsonl
    timeout -k 10 300 python -u tools/c3_step.py | grep '^{' | sed "s/}$/, \"variant\": \"$v\"}/" >> gpurun_out/ab_swiglu_phased.jsonl
  done
done
