# Round 6: DIN leg, dense Adam fused vs foreach.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06al}
mkdir -p gpurun_out/$T
B="python3 -u bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --model-steps 0 --train-steps 0 --native-steps 0 --din-steps 20"
for a in fused foreach fused; do
  DR_BENCH_DENSE_ADAM=$a timeout -k 10 300 $B > gpurun_out/$T/bench_$a.log 2>&1 || { tail -5 gpurun_out/$T/bench_$a.log; exit 1; }
  echo "adam $a: $(grep 'din leg' gpurun_out/$T/bench_$a.log | grep -o '"ms_per_step": [0-9.]*\|graph_check": "[a-z]*\|ms_per_step_eager": [0-9.]*' | tr '\n' ' ')"
done
