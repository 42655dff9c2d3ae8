#!/bin/bash
# PMC traffic (FETCH_SIZE / WRITE_SIZE passes) of every bench shape on the
# shipped library -> profiles/pmc_traffic.json (run on the GPU box from the
# repo root; each pass under its own time limit inside collect_pmc.py)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for a in "$@"; do
  set -- $a
  echo "== pmc $a" >&2
  timeout -k 10 400 python -u profiles/collect_pmc.py $1 $2 ${3:-1} > gpurun_out/pmc_$1_$2_${3:-1}.json
done
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
