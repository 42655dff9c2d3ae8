#!/bin/bash
# Round-3 measurements: per-rank PMC traffic of the strong-scaling shards
# (c3 at P = 2, 4, 8; c4 at 8), the fp32 sweep line of configs[2], the C2
# line, and rocprofv3 kernel stats of the default bench.  Each GPU step has
# its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03m
mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "== $*  ($(date +%T))"; }
if [ -z "${SKIP_PMC:-}" ]; then
  for cp in "c3 2" "c3 4" "c3 8" "c4 8"; do
    set -- $cp
    step pmc $1 P=$2
    timeout -k 10 900 python -u profiles/collect_pmc.py $1 f64 $2 > $OUT/pmc_$1_p$2.log 2>&1 || { tail -20 $OUT/pmc_$1_p$2.log; exit 1; }
    tail -4 $OUT/pmc_$1_p$2.log
  done
  cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
fi
step bench-f32
timeout -k 10 600 python bench.py --dtype f32 > $OUT/bench_c3_f32.json 2> $OUT/bench_c3_f32.err || { tail -5 $OUT/bench_c3_f32.err; exit 1; }
step bench-c2
timeout -k 10 600 python bench.py --config c2 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -5 $OUT/bench_c2.err; exit 1; }
step rocprofv3
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- \
    python bench.py --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err || { tail -5 $OUT/prof.err; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec head -6 {} \;
echo done
