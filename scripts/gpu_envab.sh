#!/bin/bash
# Diagnostic: GPU parity tests (PYTEST=1), then an A/B of runtime settings
# (ENVS, scripts/ablate.py) on the in-tree library over SIZES, then the
# sweep rows named by SWEEP (scripts/sweep.py ONLY=...).
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${PYTEST:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -5 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${ENVS:-}" ]; then
  LIBS=rigidbody-simulation_amd/rbhip/librbhip.so ENVS="$ENVS" SIZES="${SIZES:-64x64,128x64,256x256,512x512}" \
    timeout -k 10 600 python scripts/ablate.py > gpurun_out/envab.txt 2>&1
  rc=$?; grep "N=" gpurun_out/envab.txt || tail gpurun_out/envab.txt; [ $rc -eq 0 ] || exit $rc
  if [ -n "${CUBE_SIZES:-}" ]; then
    SCENE=cubes LIBS=rigidbody-simulation_amd/rbhip/librbhip.so ENVS="$ENVS" SIZES="$CUBE_SIZES" \
      timeout -k 10 600 python scripts/ablate.py > gpurun_out/envab_cubes.txt 2>&1
    rc=$?; echo "cubes:"; grep "N=" gpurun_out/envab_cubes.txt || tail gpurun_out/envab_cubes.txt; [ $rc -eq 0 ] || exit $rc
  fi
  if [ -n "${INCLINE_SIZES:-}" ]; then
    SCENE=incline LIBS=rigidbody-simulation_amd/rbhip/librbhip.so ENVS="$ENVS" SIZES="$INCLINE_SIZES" \
      timeout -k 10 600 python scripts/ablate.py > gpurun_out/envab_incline.txt 2>&1
    rc=$?; echo "incline:"; grep "N=" gpurun_out/envab_incline.txt || tail gpurun_out/envab_incline.txt; [ $rc -eq 0 ] || exit $rc
  fi
fi
if [ -n "${SWEEP:-}" ]; then
  ONLY="$SWEEP" timeout -k 10 600 python scripts/sweep.py > gpurun_out/sweep.md 2>&1
  rc=$?; cat gpurun_out/sweep.md; [ $rc -eq 0 ] || exit $rc
fi
echo ALL DONE
