# Lookup-kernel A/B on the headline and DeepFM legs: rows in
# flight per lane group (DR_LOOKUP_NB) and lanes per row (DR_LOOKUP_SPLIT).
set -o pipefail
O=gpurun_out/r04lk
mkdir -p $O
B="bench.py --cpu-seconds 0 --train-steps 0 --no-criteo --no-dcn --no-hybrid"
for v in "base" "DR_LOOKUP_NB=8" "DR_LOOKUP_SPLIT=2" "DR_LOOKUP_NB=2"; do
  if [ $v = base ]; then e=""; else e=$v; fi
  env $e timeout -k 10 300 python -u $B > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1])
print('$v', 'headline', d['roofline']['kernel_ms'], d['roofline']['frac'], 'deepfm', d['deepfm_config']['roofline']['kernel_ms'], d['deepfm_config']['roofline']['frac'], d['deepfm_config']['roofline']['kernel'])"
done
timeout -k 10 400 python -u bench.py --cpu-seconds 0 --train-steps 0 --no-criteo --no-dcn --no-deepfm > $O/hybrid.json 2> $O/hybrid.err || { tail -5 $O/hybrid.err; exit 1; }
grep "hybrid leg" $O/hybrid.err
