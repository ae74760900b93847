# bench's trainer_step (C2 micro-batches: 1.5B, 2 x 65 536 tokens, contiguous SwiGLU kernels):
# phased SwiGLU (default) vs grid-stride (variant), alternated   -> gpurun_out/ab_swiglu_c2.jsonl
set -e
mkdir -p gpurun_out
V=pipelinerl-swe_amd/pipelinerl_amd/variants
for rep in 1 2; do
  for v in main swiglu_gridstride; do
    if [[ $v == main ]]; then unset PRL_LIB; else export PRL_LIB=$PWD/$V/libprl_hip_$v.so; fi
    timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-c3 | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=d['trainer_step']; print(json.dumps({'variant': '$v', 'ms_per_optimizer_step': t['ms_per_optimizer_step'], 'tokens_per_s': t['tokens_per_s']}))" >> gpurun_out/ab_swiglu_c2.jsonl
  done
done
