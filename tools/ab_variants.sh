# Alternate the product build with variant builds (tools/build_variants.py) of the bf16 loss head
# on one box, three rounds: bash tools/ab_variants.sh [arm ...]  (default: product copy_ceiling no_math).
# The variants are built here, on the box (pipelinerl_amd/variants/ is not pushed: .gpurunignore).
set -u
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-trainer-step --no-c3 --no-fp32"
V=pipelinerl-swe_amd/pipelinerl_amd/variants
ARMS="${*:-product copy_ceiling no_math}"
BUILD=$(for a in $ARMS; do [ $a = product ] || printf '%s ' $a; done)
[ -z "$BUILD" ] || timeout -k 10 600 python tools/build_variants.py $BUILD > gpurun_out/ab_variants_build.log 2>&1 || exit $?
for r in 1 2 3; do
  for arm in $ARMS; do
    if [ $arm = product ]; then lib=""; else lib="PRL_LIB=$V/libprl_hip_$arm.so"; fi
    line=$(env $lib timeout -k 10 120 $B 2>/dev/null | grep '^{') || exit $?
    echo "{\"round\": $r, \"arm\": \"$arm\", \"line\": $line}" >> gpurun_out/ab_variants.jsonl
    echo "$r $arm $(echo $line | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_ms"], d["roofline"]["frac"])')"
  done
done
