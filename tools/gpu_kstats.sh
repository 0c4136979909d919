#!/bin/bash
# quick kernel-time split of one bench command (rocprofv3 kernel trace, stats only; database in /tmp)
# usage: tools/gpu_kstats.sh <bench args...>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf /tmp/ocg_ks
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ocg_ks -o ks -- python3 bench.py "$@" > gpurun_out/ks.json 2> gpurun_out/ks.err || { tail -5 gpurun_out/ks.err; exit 1; }
f=$(find /tmp/ocg_ks -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:12]:
    print(f"{r['Name'][:40]:40s} calls {int(r['Calls']):7d} total {float(r['TotalDurationNs'])/1e6:9.1f} ms avg {float(r['AverageNs'])/1e3:8.1f} us {float(r['Percentage']):5.1f}%")
PY
cut -c1-300 gpurun_out/ks.json
