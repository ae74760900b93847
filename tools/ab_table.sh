# GEMM solution table A/B on the trainer micro-batch step: the shipped table vs another table file
#   bash tools/ab_table.sh <alt.json> [model] [tokens]  -> gpurun_out/ab_table.jsonl
set -e
ALT=$1; M=${2:-1.5b}; T=${3:-16384}
B="python -u tools/trainer_step_bench.py --mode trainer --loss fused_head --model $M --tokens $T --steps 8 --warmup 2"
for v in shipped alt shipped alt; do
  if [[ $v == alt ]]; then export PRL_GEMM_SOLUTIONS=$ALT; else unset PRL_GEMM_SOLUTIONS; fi
  timeout -k 10 240 $B | sed "s/}$/, \"table\": \"$v\"}/" | grep '^{' >> gpurun_out/ab_table.jsonl
done
