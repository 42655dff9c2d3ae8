#!/bin/bash
# Final-build measurements of round 6: PMC traffic (profiles/collect_pmc.py)
# for every shape a bench line can print, the bench lines (C3 f64 default,
# the driver's 20-step shape, C3 f32 sweep, C2, C4, C5) and rocprofv3 kernel
# stats of the default bench.  Each GPU step has its own time limit; the
# first failure ends the script.  SKIP_PMC=1 skips the counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/final6
mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "== $*  ($(date +%T))"; }
if [ "${RUN_SUITE:-0}" = 1 ]; then
  step gpu-suite
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_suite.log 2>&1
  rc=$?
  tail -2 $OUT/gpu_suite.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ "${SKIP_PMC:-0}" != 1 ]; then
  # PMC_SHAPES: "cfg dtype P" entries separated by "|"
  IFS='|' read -r -a shapes <<< "${PMC_SHAPES:-c3 f64 1|c2 f64 1|c4 f64 1|c5 f64 1|c3 f32 1|c3 f64 2|c3 f64 4|c3 f64 8|c4 f64 8}"
  for cp in "${shapes[@]}"; do
    set -- $cp
    step pmc $1 $2 P=$3
    timeout -k 10 900 python -u profiles/collect_pmc.py $1 $2 $3 > $OUT/pmc_$1_$2_p$3.log 2>&1 || { tail -20 $OUT/pmc_$1_$2_p$3.log; exit 1; }
    tail -2 $OUT/pmc_$1_$2_p$3.log
  done
  if [ "${SKIP_TILE_PMC:-0}" != 1 ]; then
    step pmc c3 f64 tile
    RBHIP_TILE=1 timeout -k 10 900 python -u profiles/collect_pmc.py c3 f64 1 _tile > $OUT/pmc_c3_f64_tile.log 2>&1 || { tail -20 $OUT/pmc_c3_f64_tile.log; exit 1; }
  fi
  cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  step bench-c3
  timeout -k 10 600 python bench.py > $OUT/bench_c3_f64.json 2> $OUT/bench_c3_f64.err || { tail -5 $OUT/bench_c3_f64.err; exit 1; }
  cat $OUT/bench_c3_f64.json | cut -c1-400
  step bench-c3-k20
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c3_k20.json 2> $OUT/bench_c3_k20.err || { tail -5 $OUT/bench_c3_k20.err; exit 1; }
  cat $OUT/bench_c3_k20.json | cut -c1-400
  for c in "--dtype f32:c3_f32" "--config c2:c2_f64" "--config c4:c4_f64" "--config c5:c5_f64"; do
    a=${c%%:*}; n=${c##*:}
    step bench $n
    timeout -k 10 600 python bench.py $a > $OUT/bench_$n.json 2> $OUT/bench_$n.err || { tail -5 $OUT/bench_$n.err; exit 1; }
    cat $OUT/bench_$n.json | cut -c1-300
  done
  step rocprofv3
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- \
      python bench.py --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err || { tail -5 $OUT/prof.err; exit 1; }
  find $OUT/prof -name '*kernel_stats.csv' -exec head -6 {} \;
  step rocprofv3-driver-shape
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_driver -o bench -- \
      python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/prof_driver_bench.json 2> $OUT/prof_driver.err || { tail -5 $OUT/prof_driver.err; exit 1; }
  find $OUT/prof_driver -name '*kernel_stats.csv' -exec head -6 {} \;
fi
echo "ALL DONE"
