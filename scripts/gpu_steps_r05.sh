#!/bin/bash
# Round-5 GPU batch: each step under its own time limit; a step that times out or crashes
# (exit >= 124) ends the batch, a failing test (exit 1) does not.
# usage: bash scripts/gpu_steps_r05.sh <tag> "<step 1>" "<step 2>" ...
TAG=$1; shift
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
i=0
for step in "$@"; do
  i=$((i + 1))
  echo "[$TAG step $i] $step" | tee -a "$OUT/steps_$TAG.log"
  bash -c "$step" > "$OUT/${TAG}_$i.log" 2>&1
  rc=$?
  echo "[$TAG step $i] rc=$rc" | tee -a "$OUT/steps_$TAG.log"
  if [ $rc -ge 124 ]; then echo "stopping: step $i rc=$rc"; exit $rc; fi
done
