# Round 6: DLRM model-step graph timeline (kernel trace of the bench DLRM leg).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06as}
mkdir -p gpurun_out/$T
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/prof -o dlrm -- python3 -u bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --train-steps 0 --native-steps 0 --din-steps 0 --model-steps 12 > gpurun_out/$T/bench.log 2>&1 || { tail -5 gpurun_out/$T/bench.log; exit 1; }
grep "dlrm" gpurun_out/$T/bench.log | cut -c1-200
