set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc2
i=0
for sz in "64 64 300" "1024 1024 60"; do
  set -- $sz
  for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY TCC_EA0_ATOMIC_sum"; do
    i=$((i+1))
    NX=$1 NY=$2 WARM=$3 STEPS=10 timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmc2/p${i}_n$1 -o run -- python scripts/kprobe.py > /dev/null 2> gpurun_out/pmc2/err_${i}.log || { echo "fail $i"; tail -5 gpurun_out/pmc2/err_${i}.log; exit 4; }
  done
done
echo done
