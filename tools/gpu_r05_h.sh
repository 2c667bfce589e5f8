# Round 5, batch H: DIN attention MLP with LDS-staged weights -- parity, the
# DIN step, its kernel stats.  Tag $1.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05h}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_din.py tests/test_gpu_configs.py tests/test_gpu_din_dp.py -k "din or config3" -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -2 gpurun_out/$T/tests.log; grep -E "^FAILED|^ERROR" gpurun_out/$T/tests.log | head -20
[ $rc -ne 0 ] && exit $rc
for e in "X=1" "X=1"; do
  env $e timeout -k 10 300 python -u tools/model_step.py --model din --steps 20 > gpurun_out/$T/din.log 2>&1 || { tail -5 gpurun_out/$T/din.log; exit 1; }
  echo "din $e: $(tail -1 gpurun_out/$T/din.log | cut -c1-120)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/dinprof -o run -- python3 tools/model_step.py --model din --steps 10 > gpurun_out/$T/dinprof.log 2>&1 || { tail -5 gpurun_out/$T/dinprof.log; exit 1; }
echo dinprof ok
