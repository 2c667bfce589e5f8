# Round 6: DIN step with the rounds walk (setprio + DPP scan) vs DR_GRAD_SEG_ROUNDS=0, + kernel stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06z}
mkdir -p gpurun_out/$T
B="python -u bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --model-steps 0 --native-steps 0 --train-steps 0 --din-steps 20"
timeout -k 10 300 $B > gpurun_out/$T/bench_rounds.log 2>&1 || { tail -5 gpurun_out/$T/bench_rounds.log; exit 1; }
grep -E "din leg" gpurun_out/$T/bench_rounds.log | cut -c1-300
DR_GRAD_SEG_ROUNDS=0 timeout -k 10 300 $B > gpurun_out/$T/bench_r0.log 2>&1 || { tail -5 gpurun_out/$T/bench_r0.log; exit 1; }
grep -E "din leg" gpurun_out/$T/bench_r0.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o din -- python3 -u tools/model_step.py --model din --steps 10 > gpurun_out/$T/din_prof.log 2>&1 || exit 1
python3 -c "
import csv
rows = sorted(csv.DictReader(open('gpurun_out/$T/prof/din_kernel_stats.csv')), key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:12]:
    print('%-80s %6s %9.1f us avg' % (r['Name'][:80], r['Calls'], float(r['AverageNs']) / 1e3))
"
