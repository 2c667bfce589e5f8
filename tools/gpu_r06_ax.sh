# Round 6: two-pass DIN attention backward: DIN tests, DIN leg A/B (DR_DIN_MLP_BWD=1 one pass).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06ax}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_din.py tests/test_gpu_din_graph.py tests/test_gpu_configs.py -m gpu -x -q -k "din or dice or fcn or config3" --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -2 gpurun_out/$T/tests.log; grep -E "^FAILED|Error" gpurun_out/$T/tests.log | head -5; [ $rc -ne 0 ] && exit $rc
B="python3 -u bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --model-steps 0 --train-steps 0 --native-steps 0 --din-steps 20"
for a in 0 1; do
  DR_DIN_MLP_BWD=$a timeout -k 10 300 $B > gpurun_out/$T/bench_$a.log 2>&1 || { tail -5 gpurun_out/$T/bench_$a.log; exit 1; }
  echo "one-pass $a: $(grep 'din leg' gpurun_out/$T/bench_$a.log | grep -o '"ms_per_step": [0-9.]*\|graph_check": "[a-z]*' | tr '\n' ' ')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o din -- $B > gpurun_out/$T/prof.log 2>&1 || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/$T/prof/din_kernel_stats.csv')):
    if 'din_mlp_bwd' in r['Name']: print(r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3, 1))
"
