# Round 5, batch Z: row backwards forked onto side streams inside the
# captured DIN graphs (DR_ROWS_SIDE_STREAM_CAPTURE) -- bit-equality to eager,
# the capture-using tests, and the bench DIN leg with it on / off.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05z2}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_din_graph.py tests/test_gpu_rows_grad.py -k "graph or capture or din" -m gpu -q --timeout 500 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -2 gpurun_out/$T/tests.log; grep -E "^FAILED|^ERROR|Error" gpurun_out/$T/tests.log | head -10
[ $rc -ne 0 ] && exit $rc
DGP_MODE=eager DGP_FILE=/tmp/dgp_full.pt timeout -k 10 200 python -u tools/din_graph_probe.py --steps 12 > gpurun_out/$T/e.log 2>&1 && DGP_MODE=graph DGP_FILE=/tmp/dgp_full.pt timeout -k 10 200 python -u tools/din_graph_probe.py --steps 12 > gpurun_out/$T/g.log 2>&1; rc=$?; grep -E "==|differs" gpurun_out/$T/g.log
[ $rc -ne 0 ] && exit $rc
for e in 1 0 1; do
  DR_ROWS_SIDE_STREAM_CAPTURE=$e timeout -k 10 400 python -u bench.py --cpu-seconds 0 --steps 3 --warmup 1 --train-steps 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --model-steps 0 --native-steps 0 --din-steps 20 > gpurun_out/$T/bench$e.json 2> gpurun_out/$T/bench$e.err || exit 1
  echo "capture fork=$e: $(grep 'din leg' gpurun_out/$T/bench$e.err | grep -o '"ms_per_step": [0-9.]*, .*hipgraph": [a-z]*')"
done
