#!/bin/bash
# Guarded chunks: box rollback + layout refit; C4 drift; C5 pin; frame cost;
# the C3 headline line (regression check).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03c
mkdir -p $OUT
step() { echo "== $*  ($(date +%T))"; }
step pytest
timeout -k 10 1100 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_gpu_boxes.py \
    "tests/test_gpu_parity.py::test_bucket_overflow_rolls_back_and_refits_bit_exact" \
    "tests/test_gpu_parity.py::test_config_long_run_bit_exact_vs_oracle[c5-2000-500]" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
step frame-cost
timeout -k 10 600 python scripts/frame_cost.py > $OUT/frame_cost.json 2> $OUT/frame_cost.err || { tail -5 $OUT/frame_cost.err; exit 1; }
cat $OUT/frame_cost.json
step bench-c3
timeout -k 10 600 python bench.py --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -5 $OUT/bench_c3.err; exit 1; }
cat $OUT/bench_c3.json
step bench-c5
timeout -k 10 600 python bench.py --config c5 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -5 $OUT/bench_c5.err; exit 1; }
cat $OUT/bench_c5.json
echo done
