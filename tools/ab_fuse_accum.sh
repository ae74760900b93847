# A/B of the fused weight-gradient accumulation (PRL_FUSE_GRAD_ACCUM) on the C3 7B step and the
# 1.5B C2 trainer step, interleaved, one box   -> gpurun_out/ab_fuse_accum.jsonl
set -e
mkdir -p gpurun_out
for v in 1 0 1 0; do
  PRL_FUSE_GRAD_ACCUM=$v timeout -k 10 300 python -u tools/c3_step.py | grep '^{' | sed "s/}$/, \"fuse_grad_accum\": $v, \"probe\": \"c3_dp\"}/" >> gpurun_out/ab_fuse_accum.jsonl
done
