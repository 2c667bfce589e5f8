# Round measurement: GPU test suite, full bench line, rocprofv3 kernel stats of
# a short bench, and the dominant kernel's FETCH_SIZE / WRITE_SIZE in separate
# --pmc passes (summarised on the host by tools/pmc_summary.py).  Tag $1.
set -o pipefail
T=${1:-final}
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
rc=$?; tail -2 gpurun_out/$T/bench.err; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="bench.py --no-graph --steps 2 --kernel-iters 3 --cpu-seconds 0 --train-steps 0 --no-deepfm --no-criteo --no-dcn"
# kernel stats of the headline path (steps + checks + the dominant kernel's timing loop)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/stats -o run -- python3 bench.py --cpu-seconds 0 --steps 10 --warmup 3 --train-steps 0 --no-deepfm --no-criteo --no-dcn > gpurun_out/$T/prof.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/$T/fetch -o run -- python3 $B > gpurun_out/$T/fetch.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/$T/write -o run -- python3 $B > gpurun_out/$T/write.log 2>&1 || exit 1
echo measured
