set -u
OUT=gpurun_out/r03c
mkdir -p $OUT
timeout -k 10 600 python scripts/frame_cost.py > $OUT/frame_cost.json 2> $OUT/frame_cost.err || { tail -5 $OUT/frame_cost.err; exit 1; }
cat $OUT/frame_cost.json
timeout -k 10 600 python bench.py --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -5 $OUT/bench_c3.err; exit 1; }
cat $OUT/bench_c3.json
timeout -k 10 600 python bench.py --config c5 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -5 $OUT/bench_c5.err; exit 1; }
cat $OUT/bench_c5.json
