#!/bin/bash
# Diagnostic: GPU parity tests, then the cooperative form with / without
# its helper wave (RBHIP_HELP_MAX_BODIES) over small scene sizes.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread ${PYTEST_K:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
LIBS="rigidbody-simulation_amd/rbhip/librbhip.so" ENVS="RBHIP_HELP_MAX_BODIES=0;RBHIP_HELP_MAX_BODIES=30000" SIZES="${SIZES:-64x64,90x91,100x100,110x110,120x120}" ROUNDS=3 timeout -k 10 400 python scripts/ablate.py > gpurun_out/ab.txt 2>&1; rc=$?; grep "N=" gpurun_out/ab.txt || tail gpurun_out/ab.txt; exit $rc
