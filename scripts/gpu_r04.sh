#!/bin/bash
# Round-4 GPU session steps, run on the gpurun box from the repo root:
#   scripts/gpu_r04.sh STEP [STEP ...]
# Each step runs under its own time limit; a step that ends in anything but
# success or test failures (rc 0 / 1: a fault, abort, segfault, time limit)
# stops the session there.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {   # name, seconds, command...
    local name=$1 secs=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    tail -4 "gpurun_out/$name.log"
    echo "== $name rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
    return 0
}
for step in "$@"; do
    case $step in
        xbtest) run xb_tests 600 python -u -m pytest tests/test_gpu_xblock.py -x -v --timeout 300 --timeout-method thread ;;
        xbtime) run xb_time 300 python -u scripts/xb_time.py --ks 0,2,4,6,8,12,16 ;;
        xbtime8k) run xb_time_slab8k 300 python -u scripts/xb_time.py --config slab8k --ks 0,2,4,6,8,12,16 ;;
        xbtimec2) run xb_time_c2 300 python -u scripts/xb_time.py --config c2 --ks 0,2,4,6,8,12,16 ;;
        xbtimec4) run xb_time_c4 300 python -u scripts/xb_time.py --config c4 --start 260 --ks 0,4,8 ;;
        shims) run shims 300 python -u -m pytest tests/test_gpu_shims.py tests/test_gpu_threads.py -x -q --timeout 300 --timeout-method thread ;;
        xsmp) run xs_mp 600 python -u -m pytest tests/test_gpu_shard_mp.py -x -v -k "sharded_blocks or two_process_shards_match_single_world and p2p" --timeout 300 --timeout-method thread ;;
        xbl1) run xb_tests_l1 600 env RBHIP_LIB_PATH=build/xb_l1.so python -u -m pytest tests/test_gpu_xblock.py -x -q --timeout 300 --timeout-method thread &&
              run xb_time_l1 300 env RBHIP_LIB_PATH=build/xb_l1.so python -u scripts/xb_time.py --ks 0,8,16 &&
              run xb_time_l1_8k 300 env RBHIP_LIB_PATH=build/xb_l1.so python -u scripts/xb_time.py --config slab8k --ks 0,8,16 &&
              run xb_stamps_l1 300 python -u scripts/xb_stamps.py --lib build/xbstamps_l1.so --config c3 --k 8 ;;
        spab) run slotpos_ab_c3 300 env LIBS=rigidbody-simulation_amd/rbhip/librbhip.so "ENVS=RBHIP_SLOTPOS=1;RBHIP_SLOTPOS=0" SCENE=flat SIZES=256x256,128x256 WARM=20 \
              ROUNDS=3 python -u scripts/ablate.py &&
              run slotpos_ab_c4 300 env LIBS=rigidbody-simulation_amd/rbhip/librbhip.so "ENVS=RBHIP_SLOTPOS=1;RBHIP_SLOTPOS=0" SCENE=incline SIZES=256x256 WARM=500 \
              ROUNDS=2 python -u scripts/ablate.py ;;
        rareab) run rare2_tests 600 env RBHIP_LIB_PATH=build/ab_rare2.so python -u -m pytest tests/test_gpu_parity.py -x -q \
              -k "crowded or c4_2000 or past_the_head or contact_rich or c3_bench_windows" --timeout 300 --timeout-method thread &&
              run flat_tests 600 env RBHIP_LIB_PATH=build/ab_flat.so python -u -m pytest tests/test_gpu_parity.py -x -q \
              -k "crowded or c4_2000 or past_the_head or contact_rich or c3_bench_windows or xfrc or f32_bit" --timeout 300 --timeout-method thread &&
              run solve_ab_c4 300 env "LIBS=rigidbody-simulation_amd/rbhip/librbhip.so;build/ab_rare2.so;build/ab_flat.so;build/ab_both.so" SCENE=incline \
              SIZES=256x256 WARM=500 ROUNDS=3 python -u scripts/ablate.py &&
              run solve_ab_c3 300 env "LIBS=rigidbody-simulation_amd/rbhip/librbhip.so;build/ab_rare2.so;build/ab_flat.so;build/ab_both.so" SCENE=flat \
              SIZES=256x256,128x256 WARM=20 ROUNDS=3 python -u scripts/ablate.py ;;
        depthab) run depth2_tests 600 env RBHIP_LIB_PATH=build/ab_depth2.so python -u -m pytest tests/test_gpu_parity.py -x -q \
              -k "crowded or c4_2000 or past_the_head or contact_rich or c3_bench_windows or xfrc" --timeout 300 --timeout-method thread &&
              run depth_ab_c4 300 env "LIBS=rigidbody-simulation_amd/rbhip/librbhip.so;build/ab_depth2.so" SCENE=incline \
              SIZES=256x256 WARM=500 ROUNDS=3 python -u scripts/ablate.py &&
              run depth_ab_c3 300 env "LIBS=rigidbody-simulation_amd/rbhip/librbhip.so;build/ab_depth2.so" SCENE=flat \
              SIZES=256x256,128x256 WARM=20 ROUNDS=3 python -u scripts/ablate.py ;;
        blkab) run blk128_tests 600 env RBHIP_LIB_PATH=build/ab_blk128.so python -u -m pytest tests/test_gpu_parity.py -x -q \
              -k "crowded or c4_2000 or past_the_head or contact_rich or c3_bench_windows or xfrc or ragged or large_scene or shard_invariance" \
              --timeout 300 --timeout-method thread &&
              run blk_ab_c3 300 env "LIBS=rigidbody-simulation_amd/rbhip/librbhip.so;build/ab_blk128.so" SCENE=flat \
              SIZES=256x256,128x256 WARM=20 ROUNDS=3 python -u scripts/ablate.py &&
              run blk_ab_c4 300 env "LIBS=rigidbody-simulation_amd/rbhip/librbhip.so;build/ab_blk128.so" SCENE=incline \
              SIZES=256x256 WARM=500 ROUNDS=2 python -u scripts/ablate.py ;;
        atomicprobe) run atomic_probe 120 ./scripts/atomic_probe ;;
        xbstamps) run xb_stamps 300 python -u scripts/xb_stamps.py --config c3 --k 8 ;;
        xbstamps8k) run xb_stamps_8k 300 python -u scripts/xb_stamps.py --config slab8k --k 8 ;;
        stampsc4) run stamps_c4 300 python -u scripts/stamps_c4.py --warm 700 ;;
        stampsc3) run stamps_c3 300 python -u scripts/stamps_c4.py --config c3 --warm 30 ;;
        framecost) run frame_cost 300 python -u scripts/frame_cost.py --config c3 --frames 20 ;;
        framecostq) run frame_cost 300 python -u scripts/frame_cost.py --config c3 --frames 20 --skip-drift ;;
        framecost8) run frame_cost_t8 300 env RBHIP_HOST_THREADS=8 python -u scripts/frame_cost.py --config c3 --frames 20 --skip-drift ;;
        pytest) run pytest_gpu 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
        bench) run bench 300 python -u bench.py --steps 20 --warmup 5 ;;
        benchK) run bench_k400 300 python -u bench.py --steps 400 --warmup 5 ;;
        profdrv) run prof_driver 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_prof_driver_csv -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
        profk) run prof_k400 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_prof_k400_csv -o run -- python bench.py --steps 400 --warmup 5 --no-cpu-baseline ;;
        rehxs) run rehearse2_xs 600 env RBHIP_BENCH_BACKEND=gloo RBHIP_SHARD_TRANSPORT=p2p RBHIP_XB_WPG=16 RBHIP_BENCH_BLOCKS=1 \
                   python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
                   --master-port 29512 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline ;;
        pmc) run pmc_c3 600 python -u profiles/collect_pmc.py c3 f64 ;;
        c4win) run bench_c4_261 300 python -u bench.py --config c4 --warmup 60 --steps 200 --no-cpu-baseline &&
               run bench_c4_451 300 python -u bench.py --config c4 --warmup 50 --steps 400 --no-cpu-baseline &&
               run bench_c4_1801 600 python -u bench.py --config c4 --warmup 1600 --steps 200 --no-cpu-baseline ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
done
