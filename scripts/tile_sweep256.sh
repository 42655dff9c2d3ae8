set -u
export RBHIP_TILE_NT=256
timeout -k 10 120 python scripts/tile_time.py --config flat:256x32 --modes 0 --warmup 850 --steps 400 || exit 1
for o in 32 64; do for b in 0.6 1.0; do for k in 4 8 12; do
  timeout -k 10 120 python scripts/tile_time.py --config flat:256x32 --modes 1 --k $k --band $b --owned $o --warmup 850 --steps 400 || exit 1
done; done; done
