#!/bin/bash
# Run GPU steps one after another on the box, each under its own time limit:
#   tools/gpu_steps.sh OUTDIR 'name|seconds|command' ...
# stdout/stderr of step `name` go to OUTDIR/name.out / OUTDIR/name.err.  A step that exits 0 or 1
# (a test or assertion failure) lets the next one run; anything else (a fault, an abort, a time
# limit, a signal) ends the script there with that status.  A name starting with '!' (a step that
# exercises new kernels: pytest reports a GPU fault as an ordinary failure) stops on any non-zero
# status.
OUT=$1
shift
mkdir -p "$OUT"
for step in "$@"; do
  name=${step%%|*}
  strict=0
  if [ "${name:0:1}" = "!" ]; then strict=1; name=${name:1}; fi
  rest=${step#*|}
  secs=${rest%%|*}
  cmd=${rest#*|}
  echo "[$(date +%T)] $name: $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.out" 2> "$OUT/$name.err"
  rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  echo "$rc" > "$OUT/$name.rc"
  if [ "$rc" -ne 0 ] && { [ "$rc" -ne 1 ] || [ "$strict" -eq 1 ]; }; then
    echo "stopping after $name (rc=$rc)"
    exit "$rc"
  fi
done
echo all-steps-done
