#!/bin/bash
# 8-rank strong-scaling rehearsal of bench.py on ONE GPU (gloo group, the
# library's peer-to-peer exchange between processes sharing the device):
# validates the sharded data path bit-for-bit against one World; timings are
# not measurements (8 processes time-slice one GPU).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/rehearse
mkdir -p $OUT
step() { echo "== $*  ($(date +%T))"; }
step graph-cache-test
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    "tests/test_gpu_parity.py::test_graph_cache_stays_bounded" > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for cfg in c3 c4; do
  step rehearse-8 $cfg
  RBHIP_BENCH_BACKEND=gloo RBHIP_SHARD_TRANSPORT=p2p timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --steps 20 --warmup 5 \
      --config $cfg --no-cpu-baseline > $OUT/rehearse8_$cfg.json 2> $OUT/rehearse8_$cfg.err || { tail -20 $OUT/rehearse8_$cfg.err; exit 1; }
  cat $OUT/rehearse8_$cfg.json
done
echo done
