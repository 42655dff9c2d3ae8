#!/bin/bash
# GPU pass for the sharded exchange: multi-process shard tests, the C3
# bench, and a 2-rank rehearsal of bench.py on one GPU (gloo group, p2p
# halo transport, validated against one World).  Stops at the first crash.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard_mp.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_shard.log 2>&1
rc=$?; tail -25 $OUT/pytest_shard.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.err
rc=$?; cat $OUT/bench_c3.json; tail -3 $OUT/bench_c3.err; [ $rc -eq 0 ] || exit $rc
RBHIP_BENCH_BACKEND=gloo RBHIP_SHARD_TRANSPORT=p2p timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 100 --warmup 20 \
    > $OUT/rehearse2.json 2> $OUT/rehearse2.err
rc=$?; cat $OUT/rehearse2.json; tail -5 $OUT/rehearse2.err; [ $rc -eq 0 ] || exit $rc
echo "ALL DONE"
