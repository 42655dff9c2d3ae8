#!/bin/bash
# GPU pass: all parity tests (incl. the box narrowphase), the 1-GPU sweep,
# and per-phase stamps of the step kernel at 4k / 8k / 65k bodies.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r02b
mkdir -p $OUT
export TMPDIR=/tmp
echo "== pytest $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -8 $OUT/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== sweep $(date +%T)"
timeout -k 10 400 python scripts/sweep.py > $OUT/sweep.md 2> $OUT/sweep.err
rc=$?; cat $OUT/sweep.md; tail -3 $OUT/sweep.err; [ $rc -eq 0 ] || exit $rc
echo "== stamps $(date +%T)"
STAMP_LIB=rigidbody-simulation_amd/csrc/build/libstamp.so STAMP_SIZES=64x64,128x64,256x256 timeout -k 10 300 \
    python scripts/stamps.py > $OUT/stamps.txt 2>&1
rc=$?; cat $OUT/stamps.txt; [ $rc -eq 0 ] || exit $rc
echo "ALL DONE"
