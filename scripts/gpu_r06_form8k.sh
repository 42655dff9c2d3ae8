# the 8,192-body slab (one C3 rank at P = 8) and C2 in each step form
OUT=gpurun_out/form8k
mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 200 python -u scripts/slab_time.py >> $OUT/times.txt 2>&1 || exit 1
  RBHIP_HELP_MAX_BODIES=0 timeout -k 10 200 python -u scripts/slab_time.py 2>&1 | sed 's/^/coop (no helper): /' >> $OUT/times.txt || exit 1
  RBHIP_COOP_MAX_BODIES=0 timeout -k 10 200 python -u scripts/slab_time.py 2>&1 | sed 's/^/wide: /' >> $OUT/times.txt || exit 1
done
