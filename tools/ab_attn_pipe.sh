# attention backward: dK/dV tile pipeline (attn_pipe and its variants) vs the pair loop (in-tree
# build): correctness of the pipeline, bit identity across builds, role-split timings alternated,
# and the pair-region clocks
set -e
mkdir -p gpurun_out
V=$PWD/pipelinerl-swe_amd/pipelinerl_amd/variants
PRL_LIB=$V/libprl_hip_attn_pipe.so timeout -k 10 300 python -u -m pytest tests/test_attn_bwd_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -3
for v in main attn_pipe attn_pipe_sgb; do
  if [[ $v == main ]]; then unset PRL_LIB; else export PRL_LIB=$V/libprl_hip_$v.so; fi
  timeout -k 10 200 python -u tools/attn_bits.py | sed "s/}$/, \"arm\": \"$v\"}/" >> gpurun_out/attn_pipe_bits.jsonl
done
for rep in 1 2; do
  for v in main attn_pipe attn_pipe_sgb attn_pipe_lead6; do
    if [[ $v == main ]]; then unset PRL_LIB; else export PRL_LIB=$V/libprl_hip_$v.so; fi
    timeout -k 10 200 python -u tools/attn_role_split.py lens 28 4 8511 3755,1617,6053 8192,8192 2048,2048,2048,2048 | sed "s/}$/, \"arm\": \"$v\"}/" >> gpurun_out/ab_attn_pipe.jsonl
  done
done
unset PRL_LIB
for v in attn_clock_pipe attn_clock; do
  PRL_LIB=$V/libprl_hip_$v.so timeout -k 10 200 python -u tools/attn_clock.py lens 28 4 8511 8192,8192 | sed "s/}$/, \"arm\": \"$v\"}/" >> gpurun_out/attn_pipe_clock.jsonl
done
