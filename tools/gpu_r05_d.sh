# Round 5, batch D: the LDS-DMA serial walker (rows_serial_dma_kernel) --
# long-run parity, DIN step A/B (DR_GRAD_SERIAL_DMA 1 / 0, pieces of 8192)
# and the DIN step's kernel stats.  Tag $1.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05d}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_rows_grad.py tests/test_gpu_rows_deterministic.py \
  tests/test_gpu_parity.py tests/test_gpu_din.py tests/test_gpu_rows_sgd_fused.py tests/test_gpu_configs.py tests/test_gpu_sharded_c.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -2 gpurun_out/$T/tests.log; grep -E "^FAILED|^ERROR" gpurun_out/$T/tests.log | head -20
[ $rc -ne 0 ] && exit $rc
for e in "X=1" "DR_GRAD_SERIAL_PLAIN=0" "DR_GRAD_SERIAL_PLAIN=2" "DR_GRAD_SERIAL_MAX=8192" "X=1"; do
  env $e timeout -k 10 300 python -u tools/model_step.py --model din --steps 10 > gpurun_out/$T/din.log 2>&1 || { tail -5 gpurun_out/$T/din.log; exit 1; }
  echo "din $e: $(tail -1 gpurun_out/$T/din.log | cut -c1-120)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/dinprof -o run -- python3 tools/model_step.py --model din --steps 10 > gpurun_out/$T/dinprof.log 2>&1 || { tail -5 gpurun_out/$T/dinprof.log; exit 1; }
echo dinprof ok
