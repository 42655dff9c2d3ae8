#!/bin/bash
# Round-3 GPU pass.  MODE=tile: the tile-block tests and a tile vs per-step
# timing at C3; MODE=full: every -m gpu test, smoke, the bench line and its
# rocprofv3 stats.  Every GPU step has its own time limit; a step that fails
# (other than pytest's "tests failed") ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03${TAG:-}
mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "== $*  ($(date +%T))"; }
MODE=${MODE:-tile}
if [ "$MODE" = tile ]; then
  step pytest-tile
  timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest ${TESTS:-tests/test_gpu_tile.py} -m gpu -x -v --timeout 300 \
      --timeout-method thread > $OUT/pytest_tile.log 2>&1
  rc=$?; tail -25 $OUT/pytest_tile.log; echo "pytest rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
  step tile-time
  timeout -k 10 300 python -u scripts/tile_time.py ${TIME_ARGS:-} > $OUT/tile_time.json 2> $OUT/tile_time.err
  rc=$?; cat $OUT/tile_time.json; tail -5 $OUT/tile_time.err; exit $rc
fi
if [ "$MODE" = time ]; then
  for a in "${TIME_SETS[@]:-}"; do :; done
  step tile-time
  timeout -k 10 600 python -u scripts/tile_time.py ${TIME_ARGS:-} > $OUT/tile_time.json 2> $OUT/tile_time.err
  rc=$?; cat $OUT/tile_time.json; tail -5 $OUT/tile_time.err; exit $rc
fi
if [ -z "${SKIP_TESTS:-}" ]; then
  step pytest-gpu
  timeout -k 10 ${PYTEST_TIMEOUT:-1000} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -15 $OUT/pytest_gpu.log; echo "pytest rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  step smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  rc=$?; cat $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
step bench
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; tail -3 $OUT/bench.err; [ $rc -eq 0 ] || exit $rc
if [ -z "${SKIP_PROF:-}" ]; then
  step rocprofv3
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- \
      python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/prof_bench.json 2> $OUT/prof.err
  rc=$?; cat $OUT/prof_bench.json; tail -3 $OUT/prof.err
  find $OUT/prof -name '*kernel_stats.csv' -exec head -8 {} \;
fi
