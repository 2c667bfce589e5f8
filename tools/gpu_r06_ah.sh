# Round 6: serial segment walk, two fp32 adds + closed form per segment: rows tests, probe
# kernel times per mode (first-step and trained terms), DIN A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06ah}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rows_grad.py > gpurun_out/$T/tests.log 2>&1 || { tail -20 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
for f in din_pad_terms.npz din_pad_terms_s200.npz; do
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/prof_$f -o run -- python3 tools/seg_walk_probe.py --terms $f --iters 5 > gpurun_out/$T/probe_$f.log 2>&1 || { tail -5 gpurun_out/$T/probe_$f.log; exit 1; }
grep "bit-equal" gpurun_out/$T/probe_$f.log
python3 -c "
import csv
rows = list(csv.DictReader(open('gpurun_out/$T/prof_$f/run_kernel_trace.csv')))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
print('$f')
for n in ('rows_serial_plain_kernel', 'rows_serial_seg_kernel'):
    print(n, [round((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3) for r in rows if n in r['Kernel_Name']])
"
done
B="python -u bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --model-steps 0 --native-steps 0 --train-steps 0 --din-steps 20"
DR_GRAD_SEG_SCAN=4096 timeout -k 10 300 $B > gpurun_out/$T/bench_seg.log 2>&1 || { tail -5 gpurun_out/$T/bench_seg.log; exit 1; }
echo "seg walk: $(grep 'din leg' gpurun_out/$T/bench_seg.log | grep -o '"ms_per_step": [0-9.]*\|graph_check": "[a-z]*' | tr '\n' ' ')"
timeout -k 10 300 $B > gpurun_out/$T/bench_plain.log 2>&1 || { tail -5 gpurun_out/$T/bench_plain.log; exit 1; }
echo "plain walk: $(grep 'din leg' gpurun_out/$T/bench_plain.log | grep -o '"ms_per_step": [0-9.]*\|graph_check": "[a-z]*' | tr '\n' ' ')"
