# Attribution of one C3 rank's step-kernel traffic at P = 8
# (step_kernel_coop_help; profiles/r06/pmc_p8_attribution.txt): the early
# window (steps 51-150, spheres still in the air) and a settled one (451-550),
# then a build without the speculative bucket-slot loads (RB_QSPEC=0,
# diag/librbhip_q0.so swapped in), with the slab timings of both builds.
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc6
pmc() {   # tag counter warmup
    timeout -s KILL 180 rocprofv3 --pmc "$2" --output-format csv -d "gpurun_out/pmc6/$1_$2" -o run -- \
        python3 scripts/shard_step_run.py --config c3 --P 8 --warmup "$3" --steps 100 > /dev/null
}
timeout -k 10 200 python -u scripts/slab_time.py > gpurun_out/pmc6/slab_time.log 2>&1 || exit 1
pmc early FETCH_SIZE 50 || exit 1
pmc early WRITE_SIZE 50 || exit 1
pmc settled FETCH_SIZE 450 || exit 1
pmc settled WRITE_SIZE 450 || exit 1
cp diag/librbhip_q0.so rigidbody-simulation_amd/rbhip/librbhip.so
timeout -k 10 200 python -u scripts/slab_time.py >> gpurun_out/pmc6/slab_time.log 2>&1 || exit 1
pmc q0early FETCH_SIZE 50 || exit 1
pmc q0early WRITE_SIZE 50 || exit 1
