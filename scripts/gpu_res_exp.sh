set -o pipefail
timeout -k 10 200 python -u scripts/res_stamps.py --config c2 --warm 40 --k 8 || exit 1
RBHIP_RES_FILL=1.0 timeout -k 10 200 python -u scripts/res_stamps.py --config c3 --warm 40 --k 8 || exit 1
RBHIP_RES_FILL=1.0 timeout -k 10 300 python -u scripts/res_check.py --configs c3 --chunks 5,20,20 --time 20 || exit 1
