# Dominant-kernel timing only: headline bench (no legs, no train step) x2,
# then the GPU parity tests of the lookup paths.  Tag $1.
set -o pipefail
T=${1:-lk}
mkdir -p gpurun_out/$T
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-deepfm --no-criteo --no-dcn --train-steps 0 --cpu-seconds 0 > gpurun_out/$T/b$i.json 2> gpurun_out/$T/b$i.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/$T/b$i.json'));print('ms',d['ms_per_step'],'kernel',d['roofline']['kernel_ms'],'frac',d['roofline']['frac'],'gather',d['roofline_row_gather']['kernel_ms'])"
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_record_major.py tests/test_gpu_parity.py tests/test_gpu_bf16.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; exit $rc
