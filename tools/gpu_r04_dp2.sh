# data-parallel model steps: DLRM (sharded, hybrid), DCN-v2 (sharded), DIN
# (replicated) against one process; the 2-rank bench rehearsal; N = 1 bench
set -o pipefail
O=gpurun_out/r04dp2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_dlrm_sharded.py tests/test_gpu_din_dp.py tests/test_gpu_bench_rehearsal.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -14 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; grep -E "dlrm model step|din leg|train step" $O/bench.err; tail -2 $O/bench.err; exit $rc
