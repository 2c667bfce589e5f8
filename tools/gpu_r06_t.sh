# Round 6: the wave-rounds segment walk -- rows tests (repeated terms, DIN
# padding chain, long runs), DIN tests, then the DIN step timing + kernel stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06t}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_rows_grad.py tests/test_gpu_rows_deterministic.py tests/test_gpu_din.py tests/test_gpu_din_graph.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; grep -E "^FAILED|^ERROR" gpurun_out/$T/tests.log | head -10
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --model-steps 0 --native-steps 0 --train-steps 0 --din-steps 20 > gpurun_out/$T/bench.log 2>&1 || { tail -5 gpurun_out/$T/bench.log; exit 1; }
grep -E "din leg" gpurun_out/$T/bench.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o din -- python3 -u tools/model_step.py --model din --steps 10 > gpurun_out/$T/din_prof.log 2>&1 || exit 1
echo profiled
