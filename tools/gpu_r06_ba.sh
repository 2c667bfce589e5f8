# Round 6: DIN attention backward at 4 waves / SIMD (launch bounds): DIN tests + leg + kernel time.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06ba}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_din.py -m gpu -x -q -k "fused_attention or config3 or train_step" --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -1 gpurun_out/$T/tests.log; [ $rc -ne 0 ] && exit $rc
B="python3 -u bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --model-steps 0 --train-steps 0 --native-steps 0 --din-steps 20"
timeout -k 10 300 $B > gpurun_out/$T/bench.log 2>&1 || { tail -5 gpurun_out/$T/bench.log; exit 1; }
echo "din: $(grep 'din leg' gpurun_out/$T/bench.log | grep -o '"ms_per_step": [0-9.]*\|graph_check": "[a-z]*' | tr '\n' ' ')"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o din -- $B > gpurun_out/$T/prof.log 2>&1 || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/$T/prof/din_kernel_stats.csv')):
    if 'din_mlp_bwd' in r['Name']: print(r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3, 1))
"
