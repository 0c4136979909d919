#!/bin/bash
# SQ issue / wait and SQC instruction-cache counters of k_trajectory (tools/traj_only.py),
# one rocprofv3 --pmc pass each; per-dispatch means into gpurun_out/pmc_traj_<tag>.txt
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r05}
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/pmc_traj_$TAG.txt
echo "# k_trajectory (config 1, 2 chains x 200 steps): per-dispatch means" > $OUT
timeout -k 10 120 python3 $R/tools/traj_only.py >> $OUT 2>&1 || exit $?
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_IFETCH" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d /tmp/pmct$i -o run --output-format csv -- python3 $R/tools/traj_only.py > /tmp/pmct$i.log 2>&1 || { echo "pass $i failed"; tail -5 /tmp/pmct$i.log; continue; }
  f=$(find /tmp/pmct$i -name "*counter_collection.csv" | head -1)
  python3 - "$f" >> $OUT <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(list)
for r in rows:
    if "k_trajectory" in r.get("Kernel_Name", ""):
        acc[(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
per = collections.defaultdict(list)
for (d, c), v in acc.items():
    per[c].append(sum(v))
for c, v in sorted(per.items()):
    print(f"{c:28s} per-dispatch {sum(v)/len(v):.4e}  ({len(v)} dispatches)")
PY
done
cat $OUT
