# Round 6: fused Dice + fused dense Adam in the DIN step: DIN tests, then the DIN leg A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06am}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_din.py tests/test_gpu_din_graph.py tests/test_gpu_graph_interleave.py tests/test_gpu_configs.py -m gpu -x -q -k "din or dice or graph or config3" --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; grep -E "^FAILED|^ERROR|Error" gpurun_out/$T/tests.log | head -10
[ $rc -ne 0 ] && exit $rc
B="python3 -u bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --model-steps 0 --train-steps 0 --native-steps 0 --din-steps 20"
for cfg in "1 fused" "0 fused" "1 foreach" "0 foreach"; do
  set -- $cfg
  DR_DIN_DICE_FUSED=$1 DR_BENCH_DENSE_ADAM=$2 timeout -k 10 300 $B > gpurun_out/$T/bench_$1_$2.log 2>&1 || { tail -5 gpurun_out/$T/bench_$1_$2.log; exit 1; }
  echo "dice fused $1 adam $2: $(grep 'din leg' gpurun_out/$T/bench_$1_$2.log | grep -o '"ms_per_step": [0-9.]*\|graph_check": "[a-z]*\|ms_per_step_eager": [0-9.]*' | tr '\n' ' ')"
done
