# the fused halo push: the multi-process shard tests, then the one-rank
# loop costs at 8,192 bodies (profiles/r06/loop_overhead_8k.txt)
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard_mp.py -x -v --timeout 200 --timeout-method thread > gpurun_out/halo_tests.log 2>&1 || exit 1
NX=256 NY=32 timeout -k 10 300 python -u scripts/loop_overhead.py > gpurun_out/loop_overhead_8k.txt 2>&1 || exit 1
CFG=c2 timeout -k 10 300 python -u scripts/loop_overhead.py > gpurun_out/loop_overhead_c2.txt 2>&1 || exit 1
