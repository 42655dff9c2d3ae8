set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for v in 0 1; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -DRB_ABLATE=$v -o /tmp/lib$v.so rigidbody-simulation_amd/csrc/rb_kernels.hip rigidbody-simulation_amd/csrc/rb_balls.hip rigidbody-simulation_amd/csrc/rb_p2p.hip rigidbody-simulation_amd/csrc/rb_capi.hip || exit 3
done
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM_RD"; do
  for v in 0 1; do
    i=$((i+1))
    LIB=/tmp/lib$v.so WARM=60 STEPS=10 timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmc/p${i}_v$v -o run -- python scripts/kprobe.py > /dev/null 2> gpurun_out/pmc/err_${i}_v$v.log || { echo "fail $i $v"; tail gpurun_out/pmc/err_${i}_v$v.log; exit 4; }
  done
done
echo done
