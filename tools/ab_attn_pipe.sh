# attention backward: dK/dV tile pipeline (in-tree build) vs the pair loop (attn_nopipe): the attention
# GPU tests on the pipeline, bit identity across the builds, role-split timings alternated, the
# pair-region clocks, and the C3 7B step alternated   -> gpurun_out/*attn_pipe*.jsonl
set -e
mkdir -p gpurun_out
V=$PWD/pipelinerl-swe_amd/pipelinerl_amd/variants
timeout -k 10 300 python -u -m pytest tests/test_attn_bwd_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2
for v in main attn_nopipe; do
  if [[ $v == main ]]; then unset PRL_LIB; else export PRL_LIB=$V/libprl_hip_$v.so; fi
  timeout -k 10 200 python -u tools/attn_bits.py | sed "s/}$/, \"arm\": \"$v\"}/" >> gpurun_out/attn_pipe_bits.jsonl
done
for rep in 1 2; do
  for v in main attn_nopipe; do
    if [[ $v == main ]]; then unset PRL_LIB; else export PRL_LIB=$V/libprl_hip_$v.so; fi
    timeout -k 10 200 python -u tools/attn_role_split.py lens 28 4 8511 3755,1617,6053 8192,8192 2048,2048,2048,2048 | sed "s/}$/, \"arm\": \"$v\"}/" >> gpurun_out/ab_attn_pipe.jsonl
    timeout -k 10 200 python -u tools/attn_role_split.py lens 12 2 2048,2048,2048,2048,2048,2048,2048,2048 | sed "s/}$/, \"arm\": \"$v\"}/" >> gpurun_out/ab_attn_pipe.jsonl
  done
done
unset PRL_LIB
for v in attn_clock attn_clock_nopipe; do
  PRL_LIB=$V/libprl_hip_$v.so timeout -k 10 200 python -u tools/attn_clock.py lens 28 4 8511 8192,8192 | sed "s/}$/, \"arm\": \"$v\"}/" >> gpurun_out/attn_pipe_clock.jsonl
done
for rep in 1 2; do
  for v in main attn_nopipe; do
    if [[ $v == main ]]; then unset PRL_LIB; else export PRL_LIB=$V/libprl_hip_$v.so; fi
    timeout -k 10 300 python -u tools/c3_step.py | grep '^{' | sed "s/}$/, \"arm\": \"$v\"}/" >> gpurun_out/c3_attn_pipe_ab.jsonl
  done
done
