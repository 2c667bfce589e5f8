# Embedding training step kernel breakdown: rocprofv3 kernel stats of
# tools/train_probe.py --graph (SGD, bench shape).  Tag $1.
set -o pipefail
T=${1:-tp}
X=${2:-}   # extra train_probe flags, e.g. --bf16
mkdir -p gpurun_out/$T
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o run -- python3 tools/train_probe.py --graph --steps 8 $X > gpurun_out/$T/train.log 2>&1 || exit 1
tail -2 gpurun_out/$T/train.log
f=$(find gpurun_out/$T/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print("%-90s %6s %10.1f us avg %8.1f" % (r["Name"][:90], r["Calls"], float(r["TotalDurationNs"]) / 1e3, float(r["AverageNs"]) / 1e3))
PY
