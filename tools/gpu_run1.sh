set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_r02b.log 2>&1
rc=$?
tail -25 gpurun_out/gpu_tests_r02b.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r02b.json 2> gpurun_out/bench_r02b.err
rc=$?
tail -20 gpurun_out/bench_r02b.err; cat gpurun_out/bench_r02b.json
exit $rc
