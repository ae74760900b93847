# Alternate the product build with variant builds (tools/build_variants.py) of the bf16 loss head
# on one box, three rounds: bash tools/ab_variants.sh [arm ...]  (default: product copy_ceiling unphased)
set -u
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-trainer-step --no-c3 --no-fp32"
V=pipelinerl-swe_amd/pipelinerl_amd/variants
ARMS="${*:-product copy_ceiling unphased}"
for r in 1 2 3; do
  for arm in $ARMS; do
    if [ $arm = product ]; then lib=""; else lib="PRL_LIB=$V/libprl_hip_$arm.so"; fi
    line=$(env $lib timeout -k 10 120 $B 2>/dev/null | grep '^{') || exit $?
    echo "{\"round\": $r, \"arm\": \"$arm\", \"line\": $line}" >> gpurun_out/ab_variants.jsonl
    echo "$r $arm $(echo $line | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_ms"], d["roofline"]["frac"])')"
  done
done
