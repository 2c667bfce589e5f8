# Round 6: the native engine kinds at N = 1 under rocprofv3 (kernel stats + trace).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06ab}
mkdir -p gpurun_out/$T
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o nat -- python3 -u bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --model-steps 0 --train-steps 0 --din-steps 0 --native-steps 20 > gpurun_out/$T/bench.log 2>&1 || { tail -5 gpurun_out/$T/bench.log; exit 1; }
grep "native engine" gpurun_out/$T/bench.log | cut -c1-200
python3 -c "
import csv
rows = sorted(csv.DictReader(open('gpurun_out/$T/prof/nat_kernel_stats.csv')), key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:25]:
    print('%-90s %6s %9.1f us avg' % (r['Name'][:90], r['Calls'], float(r['AverageNs']) / 1e3))
"
