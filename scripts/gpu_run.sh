#!/bin/bash
# Run GPU steps given as "log|limit|command" arguments, each under its own time limit; a
# fatal exit (timeout / abort / segfault, rc >= 124) ends the script so nothing else
# touches a sick GPU.  Ordinary failures (rc 1, e.g. a failing test) continue.
# usage: bash scripts/gpu_run.sh "pytest.log|600|python -m pytest ..." "b.log|300|python bench.py"
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
for spec in "$@"; do
  log=${spec%%|*}; rest=${spec#*|}; lim=${rest%%|*}; cmd=${rest#*|}
  echo "== $cmd (limit ${lim}s) -> $log"
  timeout -k 10 "$lim" bash -c "$cmd" > "$OUT/$log" 2>&1
  rc=$?
  echo "   rc=$rc"; tail -n 4 "$OUT/$log"
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc, stopping"; exit $rc; fi
done
