# Round 6: the padding-id chain alone, per walk mode, + kernel stats of the rounds mode.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06v

timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06v/prof -o run -- python3 tools/seg_walk_probe.py --iters 10 > gpurun_out/r06v/prof.log 2>&1 &&
python3 -c "
import csv, glob
f = sorted(glob.glob('gpurun_out/r06v/prof/**/*kernel_stats.csv', recursive=True))[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:14]:
    print('%-70s %6s %10.1f us avg' % (r['Name'][:70], r['Calls'], float(r['AverageNs']) / 1e3))
"
