#!/bin/bash
# PMC evidence for DESIGN §5: per step-kernel dispatch, at C2 (64x64), C3
# (256x256) and 1M (1024x1024) flat scenes after WARM steps: wave-cycle
# split (waiting / issue-stalled / issuing, VALU share), L2 hit rate, TA
# busy, HBM bytes.  One rocprofv3 --pmc pass per counter group, each under
# its own kill timeout; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_r02
mkdir -p $OUT
GROUPS_=("SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU"
         "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
         "TA_BUSY_avr TA_BUSY_max"
         "FETCH_SIZE"
         "WRITE_SIZE")
for sz in ${SIZES:-64x64 256x256 1024x1024}; do
  NX=${sz%x*}; NY=${sz#*x}
  i=0
  for ctrs in "${GROUPS_[@]}"; do
    i=$((i+1))
    NX=$NX NY=$NY WARM=${WARM:-300} STEPS=10 timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv \
        -d $OUT/$sz/g$i -o run -- python scripts/kprobe.py > /dev/null 2> $OUT/err_${sz}_$i.log \
        || { echo "fail $sz group $i"; tail -3 $OUT/err_${sz}_$i.log; exit 4; }
  done
  python scripts/pmc_summary.py $OUT/$sz step_kernel > $OUT/summary_$sz.txt
  echo "== $sz"; cat $OUT/summary_$sz.txt
done
echo "ALL DONE"
