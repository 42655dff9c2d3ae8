#!/bin/bash
# 1-GPU sweep of the final build (scripts/sweep.py) and strong-scaling
# rehearsals of bench.py on ONE GPU (gloo group, the library's peer-to-peer
# exchange between processes sharing the device; timings are not
# measurements): C3 at 2 and 8 ranks, C4 at 8.  Each step has its own time
# limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sweep
mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "== $*  ($(date +%T))"; }
step sweep
timeout -k 10 600 python -u scripts/sweep.py > $OUT/sweep.md 2> $OUT/sweep.err || { tail -20 $OUT/sweep.err; exit 1; }
cat $OUT/sweep.md
for cp in "c3 2" "c3 8" "c4 8"; do
  set -- $cp
  step rehearse $1 x$2
  RBHIP_BENCH_BACKEND=gloo RBHIP_SHARD_TRANSPORT=p2p timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node $2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus $2 --steps 20 --warmup 5 \
      --config $1 --no-cpu-baseline > $OUT/rehearse$2_$1.json 2> $OUT/rehearse$2_$1.err || { tail -20 $OUT/rehearse$2_$1.err; exit 1; }
  cut -c1-300 $OUT/rehearse$2_$1.json
done
echo "ALL DONE"
