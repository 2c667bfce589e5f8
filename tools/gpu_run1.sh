# usage: bash tools/gpu_run1.sh TAG  -- GPU test suite, then bench.py, then a rocprof kernel-stats pass of bench
set -o pipefail
T=${1:-x}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?
tail -25 gpurun_out/gpu_tests_$T.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?
tail -20 gpurun_out/bench_$T.err; cat gpurun_out/bench_$T.json
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$T -o run -- python3 bench.py --cpu-seconds 0 --steps 10 --warmup 3 > gpurun_out/bench_prof_$T.log 2>&1
rc=$?
tail -3 gpurun_out/bench_prof_$T.log
exit $rc
