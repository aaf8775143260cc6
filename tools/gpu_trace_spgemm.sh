#!/bin/bash
# kernel trace of one 1M SpGEMM bench step: per-dispatch start/end to check stream overlap
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_sp -o tr --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 ${ARGS} > $O/trace_sp.log 2>&1 || { tail -20 $O/trace_sp.log; exit 1; }
cd $R
f=$(find $O/trace_sp -name "*kernel_trace.csv" | head -1)
python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows = [r for r in rows if "spgemm" in r["Kernel_Name"] or "cumsum" in r["Kernel_Name"].lower() or "scan" in r["Kernel_Name"].lower()]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
# last step only: take the second half by time
half = len(rows) // 2
for r in rows[half:half + 40]:
    nm = r["Kernel_Name"]
    i = nm.find("spgemm_")
    nm = nm[i:i + 30] if i >= 0 else nm[:30]
    print(f'{(int(r["Start_Timestamp"]) - t0) / 1e6:9.3f} {(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6:8.3f} q{r.get("Queue_Id", "?")} {nm}')
PY
