# per-call overhead of short runs: graph replay against kernel-by-kernel
# launches (RBHIP_GRAPH_MIN_STEPS), K = 20 (the driver's bench shape) and 400
OUT=gpurun_out/overhead2
mkdir -p $OUT
for r in 1 2; do
  for gm in 2 64; do
    for k in 20 400; do
      RBHIP_GRAPH_MIN_STEPS=$gm timeout -k 10 200 python -u scripts/call_overhead.py --K $k >> $OUT/call_overhead.txt 2>&1 || exit 1
    done
  done
done
