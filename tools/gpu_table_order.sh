# Feature-major one-hot lookup visiting order A/B (DR_LOOKUP_TABLE_ORDER):
# lookup / rows / fused / headline tests, then the training step both ways
# and its kernel stats with table order.  Tag $1.
set -o pipefail
T=${1:-tord}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rows_grad.py tests/test_gpu_rows_sgd_fused.py tests/test_gpu_bf16.py tests/test_gpu_headline.py tests/test_gpu_configs.py -x -q --timeout 150 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; [ $rc -ne 0 ] && exit $rc
for F in 0 1 0 1; do
  DR_LOOKUP_TABLE_ORDER=$F timeout -k 10 200 python tools/train_probe.py --graph --steps 24 > gpurun_out/$T/tp.log 2>&1 || exit 1
  echo "table_order=$F $(grep '^{' gpurun_out/$T/tp.log)" | tee -a gpurun_out/$T/ab.log
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o run -- python3 tools/train_probe.py --graph --steps 8 > gpurun_out/$T/prof.log 2>&1 || exit 1
f=$(find gpurun_out/$T/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:8]:
    print("%-90s %6s %10.1f us avg %8.1f" % (r["Name"][:90], r["Calls"], float(r["TotalDurationNs"]) / 1e3, float(r["AverageNs"]) / 1e3))
PY
