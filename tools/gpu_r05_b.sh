# Round 5, batch B: the DIN fixes (MLP weight-gradient padding columns,
# whole-window walks of mostly-nonzero long runs, deeper walker prefetch):
# DIN + long-run parity, DIN step A/B, the DIN step's kernel stats, then the
# default bench line.  Tag $1.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05b}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_din.py tests/test_gpu_rows_grad.py \
  tests/test_gpu_rows_deterministic.py tests/test_gpu_configs.py -m gpu -q --timeout 300 \
  --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; grep -E "^FAILED|^ERROR" gpurun_out/$T/tests.log | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for e in "X=1" "DR_GRAD_ZERO_SKIP=0" "DR_GRAD_SERIAL_MAX=8192" "DR_DIN_FUSED_ATTENTION=0"; do
  env $e timeout -k 10 300 python -u tools/model_step.py --model din --steps 10 > gpurun_out/$T/din.log 2>&1 || { tail -5 gpurun_out/$T/din.log; exit 1; }
  echo "din $e: $(tail -1 gpurun_out/$T/din.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/dinprof -o run -- python3 tools/model_step.py --model din --steps 10 > gpurun_out/$T/dinprof.log 2>&1 || { tail -5 gpurun_out/$T/dinprof.log; exit 1; }
echo dinprof ok
timeout -k 10 600 python -u bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail -5 gpurun_out/$T/bench.err; exit 1; }
tail -1 gpurun_out/$T/bench.json | cut -c1-600
