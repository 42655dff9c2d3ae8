#!/bin/bash
# Round-2 GPU pass: parity tests, smoke, the default bench line (C3 strong,
# N = 1, with cpu_baseline + accuracy), rocprofv3 kernel stats of the same
# command, and 2- and 4-rank strong-scaling rehearsals (gloo group, ranks
# sharing the one GPU, p2p transport) of C3 and C4, validated bit-identical
# to one World.  Every GPU step has its own time limit; the first failure
# other than pytest's "tests failed" ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r02
mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "== $*  ($(date +%T))"; }
if [ -z "${SKIP_TESTS:-}" ]; then
  step pytest-gpu
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
      ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -15 $OUT/pytest_gpu.log; echo "pytest rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  step smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  rc=$?; cat $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
step bench
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; cat $OUT/bench.json; tail -3 $OUT/bench.err; [ $rc -eq 0 ] || exit $rc
if [ -z "${SKIP_PROF:-}" ]; then
  step rocprofv3
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- \
      python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/prof_bench.json 2> $OUT/prof.err
  rc=$?; cat $OUT/prof_bench.json; tail -3 $OUT/prof.err; [ $rc -eq 0 ] || exit $rc
fi
if [ -z "${SKIP_REHEARSE:-}" ]; then
  port=29600
  for cfg in ${REHEARSE_CFGS:-c3 c4}; do
    for n in ${REHEARSE_NS:-2 4}; do
      port=$((port + 1))
      step rehearse $cfg x$n
      RBHIP_BENCH_BACKEND=gloo RBHIP_SHARD_TRANSPORT=p2p timeout -k 10 300 python -m torch.distributed.run \
          --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n \
          --config $cfg --steps ${REHEARSE_STEPS:-100} --warmup 20 > $OUT/rehearse_${cfg}_x$n.json 2> $OUT/rehearse_${cfg}_x$n.err
      rc=$?; cat $OUT/rehearse_${cfg}_x$n.json; tail -3 $OUT/rehearse_${cfg}_x$n.err; [ $rc -eq 0 ] || exit $rc
    done
  done
fi
echo "ALL DONE"
