set -e
mkdir -p gpurun_out/sw
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/sw/pytest.log 2>&1
timeout -k 10 300 python -u scripts/sweep.py > gpurun_out/sw/sweep_default.md 2>&1
RBHIP_TILE=0 timeout -k 10 300 python -u scripts/sweep.py > gpurun_out/sw/sweep_hashed.md 2>&1
timeout -k 10 300 python -u scripts/tile_check.py --configs c3,flat:272:272,flat:362:362,flat:1024:1024,flat:2048:2048 --chunks 5,20,20,100,1,1,300 --time 200 > gpurun_out/sw/tile_check_ab.log 2>&1
