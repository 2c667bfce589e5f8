# one box: CrossNet desync A/B, then the data-parallel model step checks + bench
set -o pipefail
bash tools/gpu_r04_desync.sh && bash tools/gpu_r04_dp.sh
