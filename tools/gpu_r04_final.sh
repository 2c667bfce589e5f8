# Round-4 measurement: GPU suite + smoke, full bench line, kernel stats of the
# headline path and the dominant kernel's FETCH_SIZE / WRITE_SIZE (own passes)
set -o pipefail
T=${1:-r04final}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/$T/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
rc=$?; tail -2 gpurun_out/$T/bench.err; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="bench.py --no-graph --steps 2 --kernel-iters 3 --cpu-seconds 0 --train-steps 0 --model-steps 0 --din-steps 0 --no-deepfm --no-criteo --no-dcn --no-hybrid"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/stats -o run -- python3 bench.py --cpu-seconds 0 --steps 10 --warmup 3 --train-steps 0 --model-steps 0 --din-steps 0 --no-deepfm --no-criteo --no-dcn --no-hybrid > gpurun_out/$T/prof.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/$T/fetch -o run -- python3 $B > gpurun_out/$T/fetch.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/$T/write -o run -- python3 $B > gpurun_out/$T/write.log 2>&1 || exit 1
echo measured
