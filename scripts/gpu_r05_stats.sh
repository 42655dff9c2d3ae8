#!/bin/bash
# rocprofv3 --kernel-trace --stats of bench.py for the shapes named
# (tag:args) -> gpurun_out/r05stats/<tag>/ (run on the GPU box from the repo root)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r05stats
for spec in "$@"; do
  tag=${spec%%:*}; args=${spec#*:}
  echo "== stats $tag ($args)" >&2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05stats/$tag -o run -- \
    python -u bench.py $args > gpurun_out/r05stats/$tag.json
done
