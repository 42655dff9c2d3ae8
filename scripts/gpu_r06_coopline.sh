# cooperative worlds on the linear layout with 4 heads per line and dense
# first slot snapshots: the suites they run, timings against the shipped
# build (diag/librbhip_shipped.so) interleaved, and one C3 rank's PMC at P = 8
OUT=gpurun_out/coopline
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_boxes.py tests/test_gpu_shard_mp.py tests/test_gpu_balls.py tests/test_gpu_shims.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $OUT/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  for lib in diag/librbhip_shipped.so rigidbody-simulation_amd/rbhip/librbhip.so; do
    timeout -k 10 200 python -u scripts/slab_time.py --lib $lib >> $OUT/times.txt 2>&1 || exit 1
    LIB=$lib NX=256 NY=32 timeout -k 10 300 python -u scripts/loop_overhead.py 2>&1 | grep -E "halo" >> $OUT/times.txt || exit 1
  done
done
timeout -k 10 500 python -u profiles/collect_pmc.py c3 f64 8 > $OUT/pmc_p8.log 2>&1 || exit 1
timeout -k 10 500 python -u profiles/collect_pmc.py c2 f64 1 > $OUT/pmc_c2.log 2>&1 || exit 1
