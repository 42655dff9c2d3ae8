export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
LIBS="build/old.so;build/new.so" SIZES="64x64,128x128,256x256,512x512,1024x1024" timeout -k 10 300 python scripts/ablate.py > gpurun_out/ab_gen.txt 2>&1
rc=$?; cat gpurun_out/ab_gen.txt | grep "N="; exit $rc
