# Lookup rows-in-flight A/B, alternating (base, NB=2) x 2 on one box
set -o pipefail
O=gpurun_out/r04nb
mkdir -p $O
B="bench.py --cpu-seconds 0 --train-steps 0 --no-criteo --no-dcn --no-hybrid"
i=0
for v in base DR_LOOKUP_NB=2 base DR_LOOKUP_NB=2; do
  i=$((i+1))
  if [ $v = base ]; then e=""; else e=$v; fi
  env $e timeout -k 10 300 python -u $B > $O/$i.json 2> $O/$i.err || { tail -5 $O/$i.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$i.json').read().strip().splitlines()[-1])
print('$v', 'step', d['ms_per_step'], 'headline', d['roofline']['kernel_ms'], d['roofline']['frac'], 'gather', d['roofline_row_gather']['kernel_ms'], 'deepfm', d['deepfm_config']['roofline']['kernel_ms'], d['deepfm_config']['roofline']['frac'])"
done
