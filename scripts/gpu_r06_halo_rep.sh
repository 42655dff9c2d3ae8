# the multi-process shard tests, three times over (a race shows as a mismatch)
OUT=gpurun_out/halorep
mkdir -p $OUT
for r in 1 2 3; do
  timeout -k 10 600 python -u -m pytest tests/test_gpu_shard_mp.py -x -q --timeout 200 --timeout-method thread -k "two_process or halo_push or one_rank" > $OUT/run$r.log 2>&1
  rc=$?
  tail -1 $OUT/run$r.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
