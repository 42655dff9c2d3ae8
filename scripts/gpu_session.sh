#!/bin/bash
# One GPU-box pass of this session: the driver's checks (GPU suite, smoke,
# default bench, the driver's 20-step bench) then an A/B of prebuilt library
# variants (LIBS, scripts/ablate.py).  Each step has its own time limit; the
# first failure ends the script.  SKIP_TESTS=1 skips the suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/session
mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "== $*  ($(date +%T))"; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest-gpu
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
  step smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  tail -3 $OUT/smoke.log
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  step bench
  timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
  step bench-driver-shape
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_k20.json 2> $OUT/bench_k20.err || { tail -5 $OUT/bench_k20.err; exit 1; }
  cat $OUT/bench_k20.json
fi
if [ -n "${LIBS:-}" ]; then
  step ab
  LIBS="$LIBS" SIZES="${SIZES:-256x256}" ROUNDS="${ROUNDS:-3}" timeout -k 10 600 python -u scripts/ablate.py > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
  grep "N=" $OUT/ab.txt
fi
echo "ALL DONE"
