#!/bin/bash
# Box worlds: sharded orientation exchange tests, optimistic chunks without
# the box kernel, the 2,000-step C5 pin, and the C5 bench line with the box
# kernel skipped (default) and always launched (RBHIP_BOX_OPTIMISTIC=0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03b
mkdir -p $OUT
step() { echo "== $*  ($(date +%T))"; }
step pytest-boxes
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_boxes.py \
    "tests/test_gpu_parity.py::test_shard_invariance_in_process" \
    "tests/test_gpu_shard_mp.py" > $OUT/pytest_boxes.log 2>&1 || { tail -40 $OUT/pytest_boxes.log; exit 1; }
tail -3 $OUT/pytest_boxes.log
step bench-c5
timeout -k 10 600 python bench.py --config c5 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -5 $OUT/bench_c5.err; exit 1; }
cat $OUT/bench_c5.json
step bench-c5-box-kernel-always
RBHIP_BOX_OPTIMISTIC=0 timeout -k 10 600 python bench.py --config c5 --no-cpu-baseline > $OUT/bench_c5_always.json 2> $OUT/bench_c5_always.err || { tail -5 $OUT/bench_c5_always.err; exit 1; }
cat $OUT/bench_c5_always.json
step frame-cost
timeout -k 10 600 python scripts/frame_cost.py > $OUT/frame_cost.json 2> $OUT/frame_cost.err || { tail -5 $OUT/frame_cost.err; exit 1; }
cat $OUT/frame_cost.json
step c5-pin
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread \
    "tests/test_gpu_parity.py::test_config_long_run_bit_exact_vs_oracle" > $OUT/pytest_c5.log 2>&1 || { tail -40 $OUT/pytest_c5.log; exit 1; }
tail -5 $OUT/pytest_c5.log
echo done
