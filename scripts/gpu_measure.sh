#!/bin/bash
# One measurement pass for profiles/: the default bench line (with the CPU
# baseline), rocprofv3 kernel stats of the same command, PMC traffic of the
# step kernel, and the 1-GPU sweep.  Every GPU step has its own time limit;
# the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/measure
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 5; }
cat $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- \
    python bench.py --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 6; }
cat $OUT/prof_bench.json
timeout -k 10 900 python profiles/collect_pmc.py ${PMC_CFG:-c3} f64 > $OUT/pmc.txt 2>&1 || { tail $OUT/pmc.txt; exit 7; }
tail -12 $OUT/pmc.txt
timeout -k 10 600 python scripts/sweep.py > $OUT/sweep.md 2> $OUT/sweep.err || { tail $OUT/sweep.err; exit 8; }
cat $OUT/sweep.md
echo "ALL DONE"
