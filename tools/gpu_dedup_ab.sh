# xgmi engine at N = 1 on itself, with and without per-destination dedup, on
# uniform and Zipf(1.05) keys (bench.py legs off), then the 2-rank rehearsal
# tests.  Tag $1.
set -o pipefail
T=${1:-dd}
mkdir -p gpurun_out/$T
B="python -u bench.py --engine xgmi --no-deepfm --no-criteo --no-dcn --train-steps 0 --cpu-seconds 0 --steps 20"
for z in 0 1.05; do
  for d in "" "--dedup"; do
    n=z${z}${d}
    timeout -k 10 300 $B --zipf $z $d > gpurun_out/$T/$n.json 2> gpurun_out/$T/$n.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/$T/$n.json'));print('$n',d['ms_per_step'],d['value'],d['config']['engine'],d['config']['engine_check'])"
  done
done
timeout -k 10 500 python -u -m pytest tests/test_gpu_bench_rehearsal.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/rehearsal.log 2>&1
rc=$?; tail -3 gpurun_out/$T/rehearsal.log; exit $rc
