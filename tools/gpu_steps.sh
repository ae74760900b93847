#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first step that faults,
# aborts, segfaults or times out (exit 124 / 134 / 137 / 139), or fails when marked "!".
# usage: tools/gpu_steps.sh "<secs>:<log name>:<command>" ...   (prefix "!" on the secs: stop on any failure)
mkdir -p gpurun_out
for spec in "$@"; do
  secs=${spec%%:*}; rest=${spec#*:}; name=${rest%%:*}; cmd=${rest#*:}
  strict=0
  if [[ $secs == !* ]]; then strict=1; secs=${secs#!}; fi
  echo "[gpu_steps] $(date +%T) $name: $cmd" >&2
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[gpu_steps] $(date +%T) $name rc=$rc" >&2
  case $rc in
    124|134|137|139) echo "[gpu_steps] stopping after $name (rc $rc)" >&2; exit $rc ;;
  esac
  if [[ $strict == 1 && $rc != 0 ]]; then exit $rc; fi
done
