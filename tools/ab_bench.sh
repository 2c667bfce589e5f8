# A/B of two library builds on the bench (measurement only): prints the
# dominant-kernel and row-gather lines of each, twice, interleaved.
set -o pipefail
mkdir -p gpurun_out
AB=deeprec-1_amd/deeprec_amd/libdeeprec_amd_ab.so
for rep in 1 2; do
  for v in base ab; do
    if [ $v = ab ]; then export DEEPREC_AMD_LIB=$PWD/$AB; else unset DEEPREC_AMD_LIB; fi
    timeout -k 10 240 python -u bench.py --cpu-seconds 0 --train-steps 0 --kernel-iters 50 "$@" \
      > gpurun_out/ab_$v$rep.json 2> gpurun_out/ab_$v$rep.err || exit $?
    python - "$v" gpurun_out/ab_$v$rep.json <<'PY'
import json, sys
j = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], "value %.4g" % j["value"], "ms/step", j["ms_per_step"],
      "ev_lookup", j["roofline"]["kernel_ms"], j["roofline"]["frac"],
      "row_gather", j["roofline_row_gather"]["kernel_ms"], j["roofline_row_gather"]["frac"])
PY
  done
done
