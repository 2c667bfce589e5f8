# DIN step on the rows path vs the Unique path (DEEPREC_AMD_ROWS_GRAD=0), rocprof stats of each
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rows_grad.py tests/test_gpu_din.py -x -q --timeout 120 --timeout-method thread > gpurun_out/din_tests.log 2>&1
rc=$?; tail -2 gpurun_out/din_tests.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/din_rows -o run -- python3 tools/model_step.py --model din > gpurun_out/din_rows.log 2>&1 || exit 1
DEEPREC_AMD_ROWS_GRAD=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/din_uniq -o run -- python3 tools/model_step.py --model din > gpurun_out/din_uniq.log 2>&1 || exit 1
timeout -k 10 200 python3 tools/model_step.py --model din > gpurun_out/din_plain.log 2>&1 || exit 1
grep '"model"' gpurun_out/din_rows.log gpurun_out/din_uniq.log gpurun_out/din_plain.log
