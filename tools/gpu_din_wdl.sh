# DIN / WDL path changes: their tests, then the model steps.  Tag $1.
set -o pipefail
T=${1:-dw}
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest tests/test_gpu_rows_grad.py tests/test_gpu_rows_sgd_fused.py tests/test_gpu_din.py tests/test_gpu_wdl.py tests/test_gpu_dtypes.py tests/test_gpu_parity.py tests/test_gpu_async_decay.py -x -q --timeout 150 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; [ $rc -ne 0 ] && exit $rc
for m in "din" "wdl" "din" "wdl"; do
  timeout -k 10 300 python tools/model_step.py --model $m --steps 10 --warmup 3 > gpurun_out/$T/$m.log 2>&1 || { tail -5 gpurun_out/$T/$m.log; exit 1; }
  grep '^{' gpurun_out/$T/$m.log | tail -1
done
