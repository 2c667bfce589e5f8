# Kernel breakdown of the DLRM top tower on the hand MFMA path (rocprofv3
# stats of tools/mlp_probe.py) + the MLP tests.  Tag $1.
set -o pipefail
T=${1:-mlp}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
tail -3 gpurun_out/$T/tests.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o run -- python3 tools/mlp_probe.py --iters 10 > gpurun_out/$T/probe.log 2>&1 || exit 1
tail -2 gpurun_out/$T/probe.log
f=$(find gpurun_out/$T/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:28]:
    print("%-90s %6s %10.1f us avg %8.1f" % (r["Name"][:90], r["Calls"], float(r["TotalDurationNs"]) / 1e3, float(r["AverageNs"]) / 1e3))
PY
