#!/bin/bash
# Helper wave in box worlds: box tests (small box worlds now take the helper
# form), C5 A/B (cooperative vs cooperative + helper), C5 pin with the helper.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03e
mkdir -p $OUT
step() { echo "== $*  ($(date +%T))"; }
step pytest-boxes
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_boxes.py > $OUT/pytest_boxes.log 2>&1 || { tail -30 $OUT/pytest_boxes.log; exit 1; }
tail -2 $OUT/pytest_boxes.log
for hm in 12288 20480; do
  step bench-c5 help_max=$hm
  RBHIP_HELP_MAX_BODIES=$hm timeout -k 10 600 python bench.py --config c5 --no-cpu-baseline > $OUT/bench_c5_help$hm.json 2> $OUT/bench_c5_help$hm.err || { tail -5 $OUT/bench_c5_help$hm.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_c5_help$hm.json')); print(d['ms_per_step']*1e3, d['roofline']['kernel'], d['roofline']['avg_launch_ms']*1e3)"
done
step c5-pin-help
RBHIP_HELP_MAX_BODIES=20480 timeout -k 10 600 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
    "tests/test_gpu_parity.py::test_config_long_run_bit_exact_vs_oracle[c5-2000-500]" > $OUT/pytest_c5.log 2>&1 || { tail -30 $OUT/pytest_c5.log; exit 1; }
tail -2 $OUT/pytest_c5.log
echo done
