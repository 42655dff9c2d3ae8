# Diagnostic: L2 -> fabric request mix of the step kernel (C2 and 1M flat)
# and of the streaming calibration kernel, one counter group per pass.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmcreq
mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/calib_fetch profiles/calib_fetch.hip || exit 3
i=0
for ctrs in "TCC_EA0_RDREQ_sum TCC_BUBBLE_sum" "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "TCC_EA0_WRREQ_DRAM_sum FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/calib_$i -o run -- /tmp/calib_fetch 16777216 > /dev/null 2> $OUT/err_c$i.log || { echo "fail calib $i"; exit 4; }
  for sz in "64 64 300" "1024 1024 60"; do
    set -- $sz
    NX=$1 NY=$2 WARM=$3 STEPS=10 timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/p${i}_n$1 -o run -- python scripts/kprobe.py > /dev/null 2> $OUT/err_${i}_$1.log || { echo "fail $i $1"; tail -3 $OUT/err_${i}_$1.log; exit 4; }
  done
done
echo done
