#!/bin/bash
# k_serve6 launch timing over env variants (run on the GPU box): tools/serve_sweep.sh OUT "ENV1" "ENV2" ...
OUT=$1; shift
mkdir -p "$OUT"
for v in "$@"; do
  env $v timeout -k 10 120 python tools/serve_time.py > "$OUT/t.log" 2>&1 || { echo "FAIL $v"; tail -n 5 "$OUT/t.log"; exit 1; }
  echo "$v $(tail -n 1 $OUT/t.log)"
done
