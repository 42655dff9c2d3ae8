# Diagnostic: arbitrary rocprofv3 counter groups (PMC_GROUPS: ";"-separated,
# counters space-separated within a group) on the step kernel of a flat
# scene of NX x NY bodies, one pass per group.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmcg
mkdir -p $OUT
IFS=";" read -ra G <<< "$PMC_GROUPS"
i=0
for ctrs in "${G[@]}"; do
  i=$((i+1))
  NX=${NX:-1024} NY=${NY:-1024} WARM=${WARM:-60} STEPS=10 timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/g$i -o run -- python scripts/kprobe.py > /dev/null 2> $OUT/err_$i.log || { echo "fail $i"; tail -3 $OUT/err_$i.log; exit 4; }
done
echo done
