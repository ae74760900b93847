# The fp32-master AdamW step (7B parameter set) alternated with build variants of it, three rounds:
# bash tools/adamw_ab.sh [variant ...]  -> gpurun_out/adamw_ab.jsonl (variants built here, on the box)
set -u
V=pipelinerl-swe_amd/pipelinerl_amd/variants
ARMS="${*:-aw_u8 aw_u2}"
timeout -k 10 600 python tools/build_variants.py $ARMS > gpurun_out/adamw_ab_build.log 2>&1 || exit $?
for r in 1 2 3; do
  for arm in product $ARMS; do
    if [ $arm = product ]; then lib=""; else lib="PRL_LIB=$V/libprl_hip_$arm.so"; fi
    line=$(env $lib timeout -k 10 200 python tools/adamw_master_bench.py --model 7b --steps 10 2>/dev/null | grep '^{') || exit $?
    echo "{\"round\": $r, \"arm\": \"$arm\", \"line\": $line}" >> gpurun_out/adamw_ab.jsonl
  done
done
