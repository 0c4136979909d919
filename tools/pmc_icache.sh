#!/bin/bash
# Diagnostic: instruction-issue / I-cache PMC passes over the trajectory kernel
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_IFETCH SQ_WAIT_ANY --output-format csv -d $R/gpurun_out/pmc1 -o pmc -- python3 $R/tools/traj_only.py || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d $R/gpurun_out/pmc2 -o pmc -- python3 $R/tools/traj_only.py || exit $?
cd $R
for f in $(find gpurun_out/pmc1 gpurun_out/pmc2 -name "*counter_collection.csv"); do
  python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(float); n = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    if "k_trajectory" not in r["Kernel_Name"]: continue
    agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]].add(r["Dispatch_Id"])
for k, v in sorted(agg.items()):
    print(f"{k:24s} per-dispatch {v / len(n[k]):.4e}")
PY
done
