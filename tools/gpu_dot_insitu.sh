# dot interaction kernels inside the DLRM bf16 model step, per variant
# (rocprof kernel stats).  Tag $1, variants as env assignments in $2...
set -o pipefail
T=${1:-doti}; shift
mkdir -p gpurun_out/$T
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
n=0
for V in "$@"; do
  n=$((n+1))
  env $V true
  ( export $V; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof$n -o run -- python3 tools/model_step.py --model dlrm --bf16 --steps 6 --warmup 3 > gpurun_out/$T/step$n.log 2>&1 ) || exit 1
  f=$(find gpurun_out/$T/prof$n -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$V" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if "dot" in r["Name"]:
        print(sys.argv[2], "%-70s %5s avg %8.1f" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
