# the candidate screen: parity tests first, then window timings of the build
# without it (diag/librbhip_noscreen.so) and with it, interleaved
OUT=gpurun_out/screen
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_boxes.py tests/test_gpu_tiles.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $OUT/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  for lib in diag/librbhip_noscreen.so rigidbody-simulation_amd/rbhip/librbhip.so; do
    timeout -k 10 200 python -u scripts/window_time.py --lib $lib --config c3 --warm 45 --steps 20 >> $OUT/times.txt 2>&1 || exit 1
    timeout -k 10 200 python -u scripts/window_time.py --lib $lib --config c3 --warm 450 --steps 400 --reps 1 >> $OUT/times.txt 2>&1 || exit 1
    timeout -k 10 200 python -u scripts/window_time.py --lib $lib --config c4 --warm 450 --steps 400 --reps 1 >> $OUT/times.txt 2>&1 || exit 1
    timeout -k 10 200 python -u scripts/window_time.py --lib $lib --config c2 --warm 260 --steps 200 --reps 1 >> $OUT/times.txt 2>&1 || exit 1
  done
done
