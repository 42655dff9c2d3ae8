#!/bin/bash
# Diagnostic: kernel durations of the preload probe, without (a) and with (b)
# kernel-argument preloading (scripts/preload_probe.hip; binaries in build/).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/preload
for v in a b; do
  timeout -k 10 120 build/probe_$v 2000
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/preload/$v -o run -- build/probe_$v 2000 > /dev/null 2>&1
  find gpurun_out/preload/$v -name '*kernel_stats.csv' -exec cat {} \;
done
