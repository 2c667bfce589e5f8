# Round 6: native engine kinds at N = 1 after the world-1 flush skip; sharded tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06aq}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded_capture.py tests/test_gpu_sharded_c.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -2 gpurun_out/$T/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/sharded_c_check.py > gpurun_out/$T/c_check.log 2>&1 || { tail -5 gpurun_out/$T/c_check.log; exit 1; }
grep -c '"ok": true' gpurun_out/$T/c_check.log
for i in 1 2; do
timeout -k 10 600 python3 -u bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --model-steps 0 --train-steps 0 --din-steps 0 --native-steps 40 > gpurun_out/$T/bench_$i.log 2>&1 || { tail -5 gpurun_out/$T/bench_$i.log; exit 1; }
grep "native engine" gpurun_out/$T/bench_$i.log | cut -c1-190
done
