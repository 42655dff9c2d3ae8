# rb_sync polling the stream before blocking, against the shipped build:
# the bench's per-call overhead (K = 20 and 400), interleaved
OUT=gpurun_out/poll
mkdir -p $OUT
for r in 1 2 3; do
  for lib in diag/librbhip_shipped.so rigidbody-simulation_amd/rbhip/librbhip.so; do
    for k in 20 400; do
      timeout -k 10 200 python -u scripts/call_overhead.py --lib $lib --K $k >> $OUT/call_overhead.txt 2>&1 || exit 1
    done
  done
done
