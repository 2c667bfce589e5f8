# A/B of the lookup kernel's lanes-per-row split (DR_LOOKUP_SPLIT): headline
# and DeepFM roofline fractions, alternating runs.
set -o pipefail
mkdir -p gpurun_out/split
for r in 1 2; do
  for S in 1 2; do
    DR_LOOKUP_SPLIT=$S timeout -k 10 300 python -u bench.py --cpu-seconds 0 --train-steps 0 > gpurun_out/split/b_${S}_$r.json 2> gpurun_out/split/b_${S}_$r.err || exit 1
    python3 -c "
import json;d=json.load(open('gpurun_out/split/b_${S}_$r.json'))
print('split',$S,'run',$r,'headline',d['roofline']['frac'],d['roofline']['kernel_ms'],'deepfm',d['deepfm_config']['roofline']['frac'],d['deepfm_config']['roofline']['kernel_ms'])"
  done
done
