# data-parallel DLRM checks incl. hybrid placement
set -o pipefail
O=gpurun_out/r04dp2
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_dlrm_sharded.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -8 $O/tests.log; exit $rc
