# Round 6: chain walk waiting every 8 positions: rows tests, isolated chain, DIN leg.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06az}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rows_grad.py tests/test_gpu_rows_deterministic.py > gpurun_out/$T/tests.log 2>&1 || { tail -20 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/prof -o run -- python3 tools/seg_walk_probe.py --terms din_pad_terms_s200.npz --modes plain --iters 5 > gpurun_out/$T/probe.log 2>&1 || { tail -5 gpurun_out/$T/probe.log; exit 1; }
python3 -c "
import csv
rows = list(csv.DictReader(open('gpurun_out/$T/prof/run_kernel_trace.csv')))
print('plain chain', [round((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3) for r in rows if 'rows_serial_plain_kernel' in r['Kernel_Name']])
"
B="python3 -u bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --model-steps 0 --train-steps 0 --native-steps 0 --din-steps 20"
timeout -k 10 300 $B > gpurun_out/$T/bench.log 2>&1 || { tail -5 gpurun_out/$T/bench.log; exit 1; }
echo "din: $(grep 'din leg' gpurun_out/$T/bench.log | grep -o '"ms_per_step": [0-9.]*\|graph_check": "[a-z]*' | tr '\n' ' ')"
