set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rows_grad.py -x -v --timeout 120 --timeout-method thread > gpurun_out/rows_tests.log 2>&1
rc=$?; tail -40 gpurun_out/rows_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_rows.log 2>&1
rc=$?; tail -30 gpurun_out/gpu_tests_rows.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/train_probe.py > gpurun_out/train_rows.log 2>&1
rc=$?; cat gpurun_out/train_rows.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train_rows -o run -- python3 tools/train_probe.py > gpurun_out/train_rows_prof.log 2>&1
