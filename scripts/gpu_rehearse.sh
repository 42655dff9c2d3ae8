#!/bin/bash
# Strong-scaling rehearsals of bench.py on one GPU (gloo group, the ranks
# share the card; timings are not measurements): every rank's bodies are
# validated bit-identical to one World by bench.py itself.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
port=29610
for spec in ${REHEARSE:-c3:8 c4:8 c3:2}; do
  cfg=${spec%%:*}; n=${spec#*:}; port=$((port + 1))
  echo "== rehearse $cfg x$n"
  RBHIP_BENCH_BACKEND=gloo RBHIP_SHARD_TRANSPORT=p2p timeout -k 10 300 python -m torch.distributed.run \
      --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n \
      --config $cfg --steps 100 --warmup 20 > $OUT/rehearse_${cfg}_x$n.json 2> $OUT/rehearse_${cfg}_x$n.err
  rc=$?; cat $OUT/rehearse_${cfg}_x$n.json; tail -3 $OUT/rehearse_${cfg}_x$n.err; [ $rc -eq 0 ] || exit $rc
done
echo "ALL DONE"
