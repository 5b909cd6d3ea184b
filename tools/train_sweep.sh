#!/bin/bash
# cfg3 fused train step timing over env variants (GPU box): tools/train_sweep.sh OUT "ENV1" "ENV2" ...
OUT=$1; shift
mkdir -p "$OUT"
for v in "$@"; do
  env FUSED_ONLY=1 $v timeout -k 10 200 python tools/dp1_sweep.py 320 > "$OUT/t.log" 2>&1 || { echo "FAIL $v"; tail -n 5 "$OUT/t.log"; exit 1; }
  echo "$v $(grep '^{' $OUT/t.log | tail -n 1 | cut -c1-330)"
done
