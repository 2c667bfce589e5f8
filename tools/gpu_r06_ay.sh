# Round 6: plain chain walker A/B with the 64-ahead walk: register-staged (1) vs LDS-DMA (2).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06ay}
mkdir -p gpurun_out/$T
for m in 2 1; do
DR_GRAD_SERIAL_PLAIN=$m timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/prof_$m -o run -- python3 tools/seg_walk_probe.py --terms din_pad_terms_s200.npz --modes plain --iters 5 > gpurun_out/$T/probe_$m.log 2>&1 || { tail -5 gpurun_out/$T/probe_$m.log; exit 1; }
python3 -c "
import csv
rows = list(csv.DictReader(open('gpurun_out/$T/prof_$m/run_kernel_trace.csv')))
print('mode $m', [(r['Kernel_Name'][:28], round((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)) for r in rows if 'rows_serial_plain' in r['Kernel_Name'] or 'rows_serial_dma' in r['Kernel_Name']][-4:])
"
done
B="python3 -u bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --model-steps 0 --train-steps 0 --native-steps 0 --din-steps 20"
for m in 2 1; do
  DR_GRAD_SERIAL_PLAIN=$m timeout -k 10 300 $B > gpurun_out/$T/bench_$m.log 2>&1 || { tail -5 gpurun_out/$T/bench_$m.log; exit 1; }
  echo "walker $m: $(grep 'din leg' gpurun_out/$T/bench_$m.log | grep -o '"ms_per_step": [0-9.]*\|graph_check": "[a-z]*' | tr '\n' ' ')"
done
