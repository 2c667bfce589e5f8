# Round 6: DIN graphs with the side-stream fork captured (DR_ROWS_SIDE_STREAM_CAPTURE=1) and
# DEBUG_HIP_FORCE_GRAPH_QUEUES: do the graph's branches run concurrently?
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06aj}
mkdir -p gpurun_out/$T
B="python3 -u bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --model-steps 0 --train-steps 0 --native-steps 0 --din-steps 20"
for q in 0 2 4; do
  if [ $q = 0 ]; then E=""; else E="DEBUG_HIP_FORCE_GRAPH_QUEUES=$q"; fi
  env DR_ROWS_SIDE_STREAM_CAPTURE=1 $E timeout -k 10 300 $B > gpurun_out/$T/bench_q$q.log 2>&1 || { tail -5 gpurun_out/$T/bench_q$q.log; exit 1; }
  echo "fork captured, queues $q: $(grep 'din leg' gpurun_out/$T/bench_q$q.log | grep -o '"ms_per_step": [0-9.]*\|graph_check": "[a-z]*' | tr '\n' ' ')"
done
DR_ROWS_SIDE_STREAM_CAPTURE=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/prof -o din -- $B > gpurun_out/$T/prof.log 2>&1 || { tail -5 gpurun_out/$T/prof.log; exit 1; }
python3 -c "
import csv, collections
rows = list(csv.DictReader(open('gpurun_out/$T/prof/din_kernel_trace.csv')))
print(collections.Counter((r['Queue_Id'], r['Stream_Id']) for r in rows).most_common(8))
"
