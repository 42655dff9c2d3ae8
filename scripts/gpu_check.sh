#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/timeout (exit other than
# 0 or pytest's 1 = "tests failed") stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "== $*" ; }
step pytest-gpu
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -x ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -30 $OUT/pytest_gpu.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; cat $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
step bench
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; tail -5 $OUT/bench.err; [ $rc -eq 0 ] || exit $rc
if [ -n "${PROFILE:-1}" ]; then
  step rocprofv3
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- \
      python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/prof_bench.json 2> $OUT/prof.err
  rc=$?; cat $OUT/prof_bench.json; tail -5 $OUT/prof.err; [ $rc -eq 0 ] || exit $rc
  find $OUT/prof -name '*stats*' | head
fi
echo "ALL DONE"
