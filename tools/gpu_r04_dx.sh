# CrossNet input-gradient kernel: DCN tests, then the crossnet roofline lines
set -o pipefail
mkdir -p gpurun_out/r04dx
timeout -k 10 300 python -u -m pytest tests/test_gpu_dcn.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04dx/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04dx/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/kernel_roofline.py --only crossnet > gpurun_out/r04dx/roofline.log 2>&1
rc=$?; grep '^{' gpurun_out/r04dx/roofline.log; exit $rc
