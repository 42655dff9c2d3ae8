#!/bin/bash
# Bucket spill + partner growth: spill tests, C4 for 2,000 steps, box tests,
# drift windows, C3 headline (regression check of the wide kernel).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03f
mkdir -p $OUT
step() { echo "== $*  ($(date +%T))"; }
step pytest
timeout -k 10 1100 python -u -m pytest -x -v --timeout 900 --timeout-method thread \
    "tests/test_gpu_parity.py::test_crowded_cells_spill_bit_exact" \
    "tests/test_gpu_parity.py::test_c4_2000_steps_bit_exact" \
    "tests/test_gpu_parity.py::test_bucket_overflow_rolls_back_and_refits_bit_exact" \
    tests/test_gpu_boxes.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
step frame-cost
timeout -k 10 600 python scripts/frame_cost.py > $OUT/frame_cost.json 2> $OUT/frame_cost.err || { tail -5 $OUT/frame_cost.err; exit 1; }
cat $OUT/frame_cost.json
step bench-c3
timeout -k 10 600 python bench.py --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -5 $OUT/bench_c3.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_c3.json')); print(d['value'], d['ms_per_step']*1e3, d['roofline']['avg_launch_ms']*1e3)"
echo done
