#!/bin/bash
# Tile-block parameter sweep at C3 (one GPU): block horizon K x band W.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03${TAG:-}
mkdir -p $OUT
for k in ${KS:-4 6 8}; do
  for b in ${BANDS:-0.8 1.0 1.3}; do
    timeout -k 10 120 python -u scripts/tile_time.py --modes 1 --k $k --band $b ${ARGS:-} || exit $?
  done
done > $OUT/tile_sweep.json 2> $OUT/tile_sweep.err
rc=$?; cat $OUT/tile_sweep.json; tail -3 $OUT/tile_sweep.err; exit $rc
