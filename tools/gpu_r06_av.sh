# Round 6: deeper short-run chunks: rows tests, DIN leg + kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06av}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rows_grad.py tests/test_gpu_rows_deterministic.py tests/test_gpu_rows_sgd_fused.py > gpurun_out/$T/tests.log 2>&1 || { tail -20 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
B="python3 -u bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --model-steps 0 --train-steps 12 --native-steps 0 --din-steps 20"
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/prof -o din -- $B > gpurun_out/$T/bench.log 2>&1 || { tail -5 gpurun_out/$T/bench.log; exit 1; }
timeout -k 10 300 $B > gpurun_out/$T/bench2.log 2>&1 || { tail -5 gpurun_out/$T/bench2.log; exit 1; }
echo "din: $(grep 'din leg' gpurun_out/$T/bench2.log | grep -o '"ms_per_step": [0-9.]*\|graph_check": "[a-z]*' | tr '\n' ' ')"
grep -o '"train_step": {"ms_per_step": [0-9.]*' gpurun_out/$T/bench2.log | head -1
python3 -c "
import csv
rows = list(csv.DictReader(open('gpurun_out/$T/prof/din_kernel_trace.csv')))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
for n in ('rows_work_kernel',):
    print(n, [round((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3, 1) for r in rows if n in r['Kernel_Name']][-12:])
"
