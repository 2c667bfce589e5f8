# Kernel breakdown of the DLRM bf16 model step.  Tag $1.
set -o pipefail
T=${1:-dlrmp}
mkdir -p gpurun_out/$T
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o run -- python3 tools/model_step.py ${MS_ARGS:---model dlrm --bf16} --steps 6 --warmup 3 > gpurun_out/$T/step.log 2>&1 || exit 1
f=$(find gpurun_out/$T/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows if "synth" not in r["Name"] and "insert_range" not in r["Name"])
for r in rows[:24]:
    print("%-80s %5s %9.1f us avg %8.1f" % (r["Name"][:80], r["Calls"], float(r["TotalDurationNs"]) / 1e3, float(r["AverageNs"]) / 1e3))
print("total (excl. table setup) %.1f us" % (tot / 1e3))
PY
