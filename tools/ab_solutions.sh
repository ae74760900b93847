# swept GEMM solutions on vs off (PRL_GEMM_SOLUTIONS=off: library heuristic for every backward GEMM,
# torch forward) on the trainer micro-batch step, alternated on one box:
#   bash tools/ab_solutions.sh [7b|1.5b] [tokens]  -> gpurun_out/ab_solutions.jsonl
set -e
M=${1:-7b}; T=${2:-16384}
B="python -u tools/trainer_step_bench.py --mode trainer --loss fused_head --model $M --tokens $T --steps 5 --warmup 2"
for v in off on off on; do
  if [[ $v == off ]]; then export PRL_GEMM_SOLUTIONS=off; else unset PRL_GEMM_SOLUTIONS; fi
  timeout -k 10 240 $B | sed "s/}$/, \"solutions\": \"$v\"}/" | grep '^{' >> gpurun_out/ab_solutions.jsonl
done
