# Round 6: DIN with the wider Dice grid: DIN tests, DIN leg, trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06ap}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_din.py tests/test_gpu_din_graph.py tests/test_gpu_graph_interleave.py tests/test_gpu_configs.py tests/test_gpu_din_dp.py -m gpu -x -q -k "din or dice or graph or config3 or fcn" --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; grep -E "^FAILED|^ERROR|Error" gpurun_out/$T/tests.log | head -10
[ $rc -ne 0 ] && exit $rc
B="python3 -u bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --model-steps 0 --train-steps 0 --native-steps 0 --din-steps 20"
for a in 1 0; do
  DR_DIN_FUSED_FCN_INPUT=$a timeout -k 10 300 $B > gpurun_out/$T/bench_$a.log 2>&1 || { tail -5 gpurun_out/$T/bench_$a.log; exit 1; }
  echo "fused fcn input $a: $(grep 'din leg' gpurun_out/$T/bench_$a.log | grep -o '"ms_per_step": [0-9.]*\|graph_check": "[a-z]*\|ms_per_step_eager": [0-9.]*' | tr '\n' ' ')"
done
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/prof -o din -- $B > gpurun_out/$T/prof.log 2>&1 || { tail -5 gpurun_out/$T/prof.log; exit 1; }
echo traced
