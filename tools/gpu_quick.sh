# GPU test suite, then a short bench (no CPU baseline) -- tag $1
set -o pipefail
T=${1:-q}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; tail -5 gpurun_out/gpu_tests_$T.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --cpu-seconds 0 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; tail -3 gpurun_out/bench_$T.err; python3 -c "
import json;d=json.load(open('gpurun_out/bench_$T.json'))
print('value',d['value'],'ms',d['ms_per_step'],'roof',d['roofline']['frac'],d['roofline']['kernel_ms'],'rowgather',d['roofline_row_gather']['frac'],'train',d['train_step']['ms_per_step'],'deepfm',d['deepfm_config']['roofline']['frac'],d['deepfm_config']['train_step']['ms_per_step'])"
exit $rc
