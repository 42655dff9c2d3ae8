# C4's pile-up window (steps 451-850) in the wide (default) and the
# cooperative forms (profiles/r06/bench_c4_*_450.json)
set -o pipefail
timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline > gpurun_out/c4_wide_450.json 2>&1 || exit 1
RBHIP_COOP_MAX_BODIES=100000 timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline > gpurun_out/c4_coop_450.json 2>&1 || exit 1
RBHIP_COOP_MAX_BODIES=100000 RBHIP_HELP_MAX_BODIES=100000 timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline > gpurun_out/c4_coophelp_450.json 2>&1 || exit 1
