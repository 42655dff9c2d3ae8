# the GPU suite, then the one-rank loop costs of the build before the fused
# halo push and of this one, interleaved (only if the suite ended normally)
OUT=gpurun_out/suite6
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_suite.log 2>&1
rc=$?
echo "suite rc=$rc" >> $OUT/gpu_suite.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for r in 1 2; do
  for lib in diag/librbhip_pre_fused.so rigidbody-simulation_amd/rbhip/librbhip.so; do
    echo "== $lib round $r" >> $OUT/loop_ab.txt
    LIB=$lib NX=256 NY=32 timeout -k 10 300 python -u scripts/loop_overhead.py 2>&1 | grep -E "graph|shard_run" >> $OUT/loop_ab.txt || exit 1
  done
done
