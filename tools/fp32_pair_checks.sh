# fp32 pair-kernel checks after a change: its GPU tests, two short bench runs, the FETCH/WRITE calibration
set -u
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_grpo_edge_gpu.py tests/test_grpo_gpu.py -k "fp32 or pair or f32" > gpurun_out/pair_tests.log 2>&1 || exit $?
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-trainer-step --no-c3 --no-split-pipeline"
for r in 1 2; do
  timeout -k 10 200 $B > gpurun_out/pp_def_$r.log 2>&1 || exit $?
done
bash tools/profile_fp32_calib.sh
