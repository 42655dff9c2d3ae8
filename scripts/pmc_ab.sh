#!/bin/bash
# Diagnostic: L2 hit / miss counts of the step kernel for library builds
# LIBS (";"-separated) on an NX x NY flat scene; one rocprofv3 --pmc pass per
# build, each under its own kill timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ab
mkdir -p $OUT
IFS=";" read -ra L <<< "$LIBS"
for lib in "${L[@]}"; do
  tag=$(basename $lib .so)
  LIB=$lib NX=${NX:-256} NY=${NY:-256} WARM=${WARM:-300} STEPS=10 timeout -s KILL 90 rocprofv3 --pmc ${CTRS:-TCC_HIT_sum TCC_MISS_sum} \
      --output-format csv -d $OUT/$tag -o run -- python scripts/kprobe.py > /dev/null 2> $OUT/err_$tag.log \
      || { echo "fail $tag"; tail -3 $OUT/err_$tag.log; exit 4; }
  echo "== $tag"; python scripts/pmc_summary.py $OUT/$tag step_kernel
done
