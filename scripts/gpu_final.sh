#!/bin/bash
# One GPU-box pass over the final build: parity tests, smoke, C3 bench and
# its rocprofv3 stats (scripts/gpu_check.sh), the 1-GPU sweep, and the C2
# bench under rocprofv3.  Each GPU step has its own time limit; the first
# failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash scripts/gpu_check.sh || exit $?
echo "== sweep"
timeout -k 10 600 python scripts/sweep.py > gpurun_out/sweep.md 2> gpurun_out/sweep.err || exit $?
cat gpurun_out/sweep.md
echo "== c2 bench (rocprofv3)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o c2 -- \
    python bench.py --config c2 --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || exit $?
cat gpurun_out/bench_c2.json
echo "FINAL DONE"
