# bench (full, with the DeepFM leg) + dominant-kernel NB variants (measurement)
set -o pipefail
mkdir -p gpurun_out
T=${1:-x}
timeout -k 10 500 python -u bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; tail -4 gpurun_out/bench_$T.err; cat gpurun_out/bench_$T.json; [ $rc -ne 0 ] && exit $rc
for nb in 2 8 4; do
  DR_LOOKUP_NB=$nb timeout -k 10 240 python -u bench.py --cpu-seconds 0 --train-steps 0 --no-deepfm --kernel-iters 50 > gpurun_out/bench_nb$nb.json 2>/dev/null || exit $?
  python - $nb gpurun_out/bench_nb$nb.json <<'PY'
import json, sys
j = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print("NB", sys.argv[1], "value %.4g" % j["value"], "ev_lookup", j["roofline"]["kernel_ms"], j["roofline"]["frac"])
PY
done
