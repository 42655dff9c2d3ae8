#!/bin/bash
# Diagnostic: the linear layout's period fitted at rb_set_state or not
# (RBHIP_FIT_PERIOD), on incline and flat sphere scenes.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for sc in incline flat; do
SCENE=$sc LIBS="build/cur.so" ENVS="RBHIP_FIT_PERIOD=1;RBHIP_FIT_PERIOD=0" SIZES="${SIZES:-256x256,128x256,512x512}" ROUNDS=2 timeout -k 10 400 python scripts/ablate.py > gpurun_out/ab_$sc.txt 2>&1 || exit $?
echo $sc; grep "N=" gpurun_out/ab_$sc.txt
done
