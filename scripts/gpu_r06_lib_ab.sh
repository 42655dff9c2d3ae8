# window timings of the build before the fused halo push and this one,
# interleaved (profiles/r06/fused_ab_times.txt)
OUT=gpurun_out/libab2
mkdir -p $OUT
for r in 1 2; do
  for lib in diag/librbhip_pre_fused.so rigidbody-simulation_amd/rbhip/librbhip.so; do
    timeout -k 10 200 python -u scripts/window_time.py --lib $lib --config c3 --warm 45 --steps 20 >> $OUT/times.txt 2>&1 || exit 1
    timeout -k 10 200 python -u scripts/window_time.py --lib $lib --config c3 --warm 450 --steps 400 --reps 1 >> $OUT/times.txt 2>&1 || exit 1
    timeout -k 10 200 python -u scripts/window_time.py --lib $lib --config c2 --warm 260 --steps 200 --reps 1 >> $OUT/times.txt 2>&1 || exit 1
  done
done
LIB=rigidbody-simulation_amd/rbhip/librbhip.so NX=256 NY=32 timeout -k 10 300 python -u scripts/loop_overhead.py 2>&1 | grep -E "graph|shard_run" >> $OUT/loop_8k.txt || exit 1
