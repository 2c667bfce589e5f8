# Round 5, batch Y: the hand DIN attention weight-gradient pass
# (dr_din_mlp_wgrad, DR_DIN_WGRAD) -- DIN tests, step A/B, bench DIN leg.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05y2}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_din.py tests/test_gpu_din_graph.py tests/test_gpu_configs.py -k "din or config3" -m gpu -q --timeout 500 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -2 gpurun_out/$T/tests.log; grep -E "^FAILED|^ERROR|Error" gpurun_out/$T/tests.log | head -10
[ $rc -ne 0 ] && exit $rc
for e in hand lib hand; do
  DR_DIN_WGRAD=$e timeout -k 10 300 python -u tools/model_step.py --model din --steps 20 > gpurun_out/$T/din_$e.log 2>&1 || { tail -5 gpurun_out/$T/din_$e.log; exit 1; }
  echo "din wgrad=$e: $(tail -1 gpurun_out/$T/din_$e.log | cut -c1-120)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o din -- python3 -u tools/model_step.py --model din --steps 10 > gpurun_out/$T/din_prof.log 2>&1 || exit 1
grep -E "wgrad" $(find gpurun_out/$T/prof -name "*kernel_stats.csv") | cut -d, -f1-4
timeout -k 10 400 python -u bench.py --cpu-seconds 0 --steps 3 --warmup 1 --train-steps 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --model-steps 0 --native-steps 0 --din-steps 20 > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err; rc=$?; grep "din leg" gpurun_out/$T/bench.err | cut -c1-500
exit $rc
