OUT=gpurun_out/stamps6
mkdir -p $OUT
timeout -k 10 200 python -u scripts/stamps_c4.py --lib diag/stamps.so --config c3 --warm 30 > $OUT/c3_step30.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/stamps_c4.py --lib diag/stamps.so --config c3 --warm 600 > $OUT/c3_step600.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/stamps_c4.py --lib diag/stamps.so --config c4 --warm 700 > $OUT/c4_step700.log 2>&1 || exit 1
