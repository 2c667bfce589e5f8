# Model training steps (tools/model_step.py) of every modelzoo model at its
# BASELINE shape, then kernel stats of the DIN and WDL steps.  Tag $1.
set -o pipefail
T=${1:-models}
mkdir -p gpurun_out/$T
for m in "dlrm" "dlrm --bf16" "deepfm --dim 64 --rows 10000000" "din" "wdl" "dcn"; do
  tag=$(echo $m | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 python tools/model_step.py --model $m --steps 10 --warmup 3 > gpurun_out/$T/$tag.log 2>&1 || { tail -5 gpurun_out/$T/$tag.log; exit 1; }
  grep '^{' gpurun_out/$T/$tag.log | tail -1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in "din" "wdl"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof_$m -o run -- python3 tools/model_step.py --model $m --steps 6 --warmup 3 > gpurun_out/$T/prof_$m.log 2>&1 || exit 1
  f=$(find gpurun_out/$T/prof_$m -name "*kernel_stats.csv" | head -1)
  echo "== $m"
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:16]:
    print("%-80s %6s %9.1f us avg %8.1f  %4.1f%%" % (r["Name"][:80], r["Calls"], float(r["TotalDurationNs"]) / 1e3, float(r["AverageNs"]) / 1e3, 100 * float(r["TotalDurationNs"]) / tot))
PY
done
