# Round-4 data-parallel model step: its tests (multi-process on one GPU), the
# bench rehearsal, the multi-process C / IPC checks, then the N = 1 bench line
set -o pipefail
O=gpurun_out/r04dp
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dlrm_sharded.py tests/test_gpu_sharded_c.py tests/test_gpu_ipc.py tests/test_gpu_bench_rehearsal.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -12 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; tail -3 $O/bench.err; grep -E "dlrm model step|hybrid leg" $O/bench.err; exit $rc
