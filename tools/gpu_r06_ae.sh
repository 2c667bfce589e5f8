# Round 6: DIN graph replays with DEBUG_HIP_FORCE_GRAPH_QUEUES (parallel graph branches).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06ae}
mkdir -p gpurun_out/$T
B="python3 -u bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --model-steps 0 --train-steps 0 --native-steps 0 --din-steps 20"
for q in 1 2 4; do
  DEBUG_HIP_FORCE_GRAPH_QUEUES=$q timeout -k 10 300 $B > gpurun_out/$T/bench_q$q.log 2>&1 || { tail -5 gpurun_out/$T/bench_q$q.log; exit 1; }
  echo "queues $q: $(grep 'din leg' gpurun_out/$T/bench_q$q.log | grep -o '"ms_per_step": [0-9.]*\|graph_check": "[a-z]*' | tr '\n' ' ')"
done
DEBUG_HIP_FORCE_GRAPH_QUEUES=4 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/prof -o din -- $B > gpurun_out/$T/prof.log 2>&1 || { tail -5 gpurun_out/$T/prof.log; exit 1; }
echo traced
