# Radix sort tile size A/B (DR_SORT_ROUNDS 16 / 8 / 4): the sort and the
# segment sums built on it (tools/kernel_roofline.py), the embedding
# training step (bench train_step), then the sort-dependent GPU tests with
# the default.  Tag $1.
set -o pipefail
T=${1:-sort}
mkdir -p gpurun_out/$T
for R in 16 8 4; do
  DR_SORT_ROUNDS=$R timeout -k 10 200 python -u tools/kernel_roofline.py --only sort,unsorted_segment_sum,segment_grad > gpurun_out/$T/kr_$R.log 2>&1 || exit 1
  echo "== R=$R"; grep -i "sort\|segment" gpurun_out/$T/kr_$R.log | head -8
  DR_SORT_ROUNDS=$R timeout -k 10 300 python -u bench.py --no-deepfm --no-criteo --no-dcn --cpu-seconds 0 --steps 8 --kernel-iters 4 > gpurun_out/$T/b_$R.json 2> gpurun_out/$T/b_$R.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/$T/b_$R.json'));print('R=$R train',d['train_step']['ms_per_step'])"
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_rows_grad.py tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_partitioned.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; exit $rc
