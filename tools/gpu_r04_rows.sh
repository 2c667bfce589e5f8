# round 4: deterministic long-run backward -- its tests, the rows suites, the
# train step (uniform / Zipf, graph) before/after, rocprof of the Zipf step
set -o pipefail
T=${1:-x}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_rows_grad.py tests/test_gpu_ev_concurrency.py tests/test_gpu_rows_deterministic.py tests/test_gpu_rows_sgd_fused.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r04_rows_tests_$T.log 2>&1
rc=$?; tail -40 gpurun_out/r04_rows_tests_$T.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/train_probe.py --graph > gpurun_out/r04_train_$T.log 2>&1 && \
timeout -k 10 200 python -u tools/train_probe.py --graph --zipf 1.05 >> gpurun_out/r04_train_$T.log 2>&1
rc=$?; cat gpurun_out/r04_train_$T.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_prof_zipf_$T -o run -- python3 tools/train_probe.py --graph --zipf 1.05 > gpurun_out/r04_train_prof_$T.log 2>&1
exit $?
