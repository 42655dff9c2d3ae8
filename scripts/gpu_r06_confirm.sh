# the round-end checks on the final tree: GPU suite, smoke, both bench shapes
OUT=gpurun_out/confirm
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_suite.log 2>&1
rc=$?
tail -1 $OUT/gpu_suite.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || exit 1
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
