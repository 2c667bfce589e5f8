set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train_r2 -o run -- python3 tools/train_probe.py --graph > gpurun_out/train_prof_r2.log 2>&1
rc=$?; tail -3 gpurun_out/train_prof_r2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r2.json 2> gpurun_out/bench_r2.err
rc=$?; tail -5 gpurun_out/bench_r2.err; cat gpurun_out/bench_r2.json; exit $rc
