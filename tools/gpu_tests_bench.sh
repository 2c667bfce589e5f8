# GPU: selected test files (or the whole -m gpu suite when none given), then
# a short bench line.  Usage: tools/gpu_tests_bench.sh <tag> [test files...]
set -o pipefail
T=$1; shift
mkdir -p gpurun_out/$T
if [ $# -gt 0 ]; then TESTS="$@"; else TESTS=tests; fi
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/$T/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --cpu-seconds 0 > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
rc=$?; tail -3 gpurun_out/$T/bench.err; [ $rc -ne 0 ] && exit $rc
python3 -c "
import json;d=json.load(open('gpurun_out/$T/bench.json'))
print('value',d['value'],'ms',d['ms_per_step'],'roof',d['roofline']['frac'],d['roofline']['kernel_ms'],'rowgather',d['roofline_row_gather']['frac'],'train',d['train_step']['ms_per_step'],'deepfm',d['deepfm_config']['roofline']['frac'],d['deepfm_config']['train_step']['ms_per_step'])"
