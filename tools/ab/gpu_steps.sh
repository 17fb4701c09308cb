#!/bin/bash
# Run GPU steps in order; each is "name|timeout_s|command".  A step that fails with an ordinary
# test/script failure (exit 1 or 2) lets the next step run; anything else (a fault, abort,
# segfault, time limit: 124/134/137/139...) stops the sequence -- no further GPU work after it.
# Usage: tools/ab/gpu_steps.sh "tests|300|python -u -m pytest ..." "bench|560|python -u bench.py ..."
mkdir -p gpurun_out
for step in "$@"; do
  name="${step%%|*}"
  rest="${step#*|}"
  t="${rest%%|*}"
  cmd="${rest#*|}"
  echo "[gpu_steps] $name (limit ${t}s): $cmd"
  timeout -k 10 "$t" bash -c "$cmd"
  rc=$?
  echo "[gpu_steps] $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 2 ]; then
    echo "[gpu_steps] stopping after $name (rc=$rc)"
    exit $rc
  fi
done
