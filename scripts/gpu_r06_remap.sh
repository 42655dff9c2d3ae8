# the XCD-contiguous block order for every step form (RB_XCD_REMAP=1,
# diag/librbhip_remap.so) against the shipped build, interleaved
OUT=gpurun_out/remap
mkdir -p $OUT
for r in 1 2; do
  for lib in rigidbody-simulation_amd/rbhip/librbhip.so diag/librbhip_remap.so; do
    timeout -k 10 200 python -u scripts/window_time.py --lib $lib --config c3 --warm 25 --steps 20 >> $OUT/times.txt 2>&1 || exit 1
    timeout -k 10 200 python -u scripts/window_time.py --lib $lib --config c3 --warm 450 --steps 400 --reps 1 >> $OUT/times.txt 2>&1 || exit 1
    timeout -k 10 200 python -u scripts/window_time.py --lib $lib --config c4 --warm 450 --steps 400 --reps 1 >> $OUT/times.txt 2>&1 || exit 1
    timeout -k 10 200 python -u scripts/window_time.py --lib $lib --config c2 --warm 260 --steps 200 --reps 1 >> $OUT/times.txt 2>&1 || exit 1
  done
done
