set -o pipefail
timeout -k 10 200 python -u scripts/res_stamps.py --config c2 --warm 40 --k 16 || exit 1
RBHIP_RES_SKIN=0.5 RBHIP_RES_REBUILD=0 timeout -k 10 200 python -u scripts/res_stamps.py --config c3 --warm 400 --k 8 || exit 1
