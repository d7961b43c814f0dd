#!/bin/bash
# Run GPU steps in order, each under its own time limit, logging to gpurun_out/<name>.log.
# A step that fails normally (tests failing, exit 1) does not stop the sequence; a step that
# ends in a time limit (124 / 137), an abort (134) or a segmentation fault (139) does: nothing
# more touches the GPU after it.
#   scripts/gpu_steps.sh "name1|seconds|command" "name2|seconds|command" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "== $name (limit ${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  case $rc in
    124|134|137|139) echo "== stopping: $name ended with $rc"; exit $rc ;;
  esac
done
