# rows-path GPU check: its tests, the whole GPU suite, train probe (eager,
# graph), rocprof of the graph probe, bench
set -o pipefail
T=${1:-x}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rows_grad.py -x -v --timeout 120 --timeout-method thread > gpurun_out/rows_tests_$T.log 2>&1
rc=$?; tail -30 gpurun_out/rows_tests_$T.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests_$T.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/train_probe.py > gpurun_out/train_$T.log 2>&1 && \
timeout -k 10 200 python -u tools/train_probe.py --graph >> gpurun_out/train_$T.log 2>&1
rc=$?; cat gpurun_out/train_$T.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train_$T -o run -- python3 tools/train_probe.py --graph > gpurun_out/train_prof_$T.log 2>&1
rc=$?; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; tail -5 gpurun_out/bench_$T.err; cat gpurun_out/bench_$T.json; exit $rc
