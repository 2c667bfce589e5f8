# Round 5: lookup parity tests on the line-probe / pipelined kernels, then the
# headline kernel A/B over DR_LOOKUP_KERNEL (0 slot walk, 1 line one-shot,
# 2 line pipelined), alternating.  Tag $1.
set -o pipefail
T=${1:-r05lk}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_record_major.py tests/test_gpu_parity.py tests/test_gpu_bf16.py tests/test_gpu_ev_concurrency.py tests/test_gpu_shrink.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; grep -E "FAILED|Error" gpurun_out/$T/tests.log | head -5
# a test failure (not a crash / timeout) still lets the A/B run
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
B="bench.py --cpu-seconds 0 --train-steps 0 --no-criteo --no-dcn --no-hybrid"
for v in 2 1 0 2 1 0; do
  DR_LOOKUP_KERNEL=$v timeout -k 10 300 python -u $B > gpurun_out/$T/k$v.json 2> gpurun_out/$T/k$v.err || { tail -5 gpurun_out/$T/k$v.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/$T/k$v.json').read().strip().splitlines()[-1])
print('kernel $v', 'ms', d['ms_per_step'], 'headline', d['roofline']['kernel_ms'], d['roofline']['frac'], 'gather', d['roofline_row_gather']['kernel_ms'], 'deepfm', d['deepfm_config']['roofline']['kernel_ms'], d['deepfm_config']['roofline']['frac'])"
done
