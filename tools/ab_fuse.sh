# A/B of the decoder fusions (residual adds fused into the norms, q/k/v and gate/up input
# gradients summed in the dgrad GEMM epilogue) on the trainer micro-batch step, one box:
#   bash tools/ab_fuse.sh [1.5b|7b]  -> gpurun_out/ab_fuse.jsonl
set -e
M=${1:-1.5b}
T=65536; [[ $M == 7b ]] && T=16384
B="python -u tools/trainer_step_bench.py --mode trainer --loss fused_head --model $M --tokens $T --steps 5 --warmup 2"
for v in base new; do
  if [[ $v == base ]]; then export PRL_ADD_NORM=0 PRL_QKV_GROUP=0; else export PRL_ADD_NORM=1 PRL_QKV_GROUP=1; fi
  timeout -k 10 200 $B | sed "s/}$/, \"variant\": \"$v\"}/" | grep '^{' >> gpurun_out/ab_fuse.jsonl
done
