# attention backward build variants (tools/build_variants.py attn_*) vs the in-tree library:
# correctness (tests/test_attn_bwd_gpu.py on each) then timings, alternated  -> gpurun_out/ab_attn_variants.jsonl
set -e
mkdir -p gpurun_out
V=pipelinerl-swe_amd/pipelinerl_amd/variants
for v in attn_2wg attn_v_lds attn_bstage32; do
  PRL_LIB=$PWD/$V/libprl_hip_$v.so timeout -k 10 200 python -u -m pytest tests/test_attn_bwd_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -1
done
for rep in 1 2; do
  for v in main attn_2wg attn_v_lds attn_bstage32; do
    if [[ $v == main ]]; then unset PRL_LIB; else export PRL_LIB=$PWD/$V/libprl_hip_$v.so; fi
    timeout -k 10 200 python -u tools/attn_bwd_bench.py lens 28 4 8192,8192 4096,4096,2048,1760 2048,2048,2048,2048,2048,1760 | sed "s/}$/, \"variant\": \"$v\"}/" >> gpurun_out/ab_attn_variants.jsonl
    timeout -k 10 200 python -u tools/attn_bwd_bench.py lens 12 2 2048,2048,2048,2048,2048,2048,2048,2048 | sed "s/}$/, \"variant\": \"$v\"}/" >> gpurun_out/ab_attn_variants.jsonl
  done
done
