#!/bin/bash
# strong-scaling rehearsals of bench.py on ONE GPU (gloo group, the
# library's peer-to-peer exchange between processes sharing the device, both
# modes probed, the fused halo push among them): validates the sharded data
# path bit-for-bit against one World; timings are not measurements (the
# processes time-slice one GPU).  Then the one-rank loop costs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/rehearse6}
mkdir -p $OUT
for spec in ${SPECS:-"2 c3" "4 c3" "8 c3" "8 c4"}; do
  set -- $spec
  echo "== rehearse $1 $2 ($(date +%T))"
  RBHIP_BENCH_BACKEND=gloo RBHIP_SHARD_TRANSPORT=p2p timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node $1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus $1 --steps 20 --warmup 5 \
      --config $2 --no-cpu-baseline > $OUT/rehearse$1_$2.json 2> $OUT/rehearse$1_$2.err || { tail -20 $OUT/rehearse$1_$2.err; exit 1; }
  tail -1 $OUT/rehearse$1_$2.json
done
NX=256 NY=32 timeout -k 10 300 python -u scripts/loop_overhead.py > $OUT/loop_overhead_8k.txt 2>&1 || exit 1
CFG=c2 timeout -k 10 300 python -u scripts/loop_overhead.py > $OUT/loop_overhead_c2.txt 2>&1 || exit 1
echo done
