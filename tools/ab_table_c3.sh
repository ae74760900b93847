# GEMM solution table A/B on the C3 7B step (tools/c3_step.py): the shipped table vs another file
#   bash tools/ab_table_c3.sh <alt.json>  -> gpurun_out/ab_table_c3.jsonl
set -e
ALT=$1
mkdir -p gpurun_out
for v in shipped alt shipped alt; do
  if [[ $v == alt ]]; then export PRL_GEMM_SOLUTIONS=$ALT; else unset PRL_GEMM_SOLUTIONS; fi
  timeout -k 10 300 python -u tools/c3_step.py | grep '^{' | sed "s/}$/, \"table\": \"$v\"}/" >> gpurun_out/ab_table_c3.jsonl
done
