# Round 5, batch G: add-chain rate probe (tools/chain_probe.hip), DIN parity
# and step after the MLP-kernel changes and the opt-in zero scan.  Tag $1.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05g}
mkdir -p gpurun_out/$T
timeout -k 10 60 tools/chain_probe > gpurun_out/$T/chain.log 2>&1 || { tail -5 gpurun_out/$T/chain.log; exit 1; }
cat gpurun_out/$T/chain.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_rows_grad.py tests/test_gpu_din.py tests/test_gpu_configs.py -k "din or long or zero or config3" -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -2 gpurun_out/$T/tests.log; grep -E "^FAILED|^ERROR" gpurun_out/$T/tests.log | head -20
[ $rc -ne 0 ] && exit $rc
for e in "X=1" "X=1"; do
  env $e timeout -k 10 300 python -u tools/model_step.py --model din --steps 20 > gpurun_out/$T/din.log 2>&1 || { tail -5 gpurun_out/$T/din.log; exit 1; }
  echo "din $e: $(tail -1 gpurun_out/$T/din.log | cut -c1-120)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/dinprof -o run -- python3 tools/model_step.py --model din --steps 10 > gpurun_out/$T/dinprof.log 2>&1 || { tail -5 gpurun_out/$T/dinprof.log; exit 1; }
echo dinprof ok
timeout -k 10 120 tools/uc_replay_probe 3 0 1 > gpurun_out/$T/uc_replay_ipc.log 2>&1 || { tail -5 gpurun_out/$T/uc_replay_ipc.log; exit 1; }
tail -2 gpurun_out/$T/uc_replay_ipc.log
