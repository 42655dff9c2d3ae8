#!/bin/bash
# A/B timing of prebuilt library variants (build/*.so) with scripts/ablate.py.
# LIBS / SIZES from the environment; PYTEST=1 first runs the GPU tests.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${PYTEST:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -5 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
LIBS="$LIBS" SIZES="${SIZES:-64x64,128x128,256x256,512x512,1024x1024}" timeout -k 10 600 python scripts/ablate.py > gpurun_out/ab.txt 2>&1
rc=$?; grep "N=" gpurun_out/ab.txt || tail gpurun_out/ab.txt; exit $rc
