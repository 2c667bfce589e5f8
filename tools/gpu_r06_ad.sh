# Round 6: DIN graph-replay timeline (kernel trace of the bench DIN leg).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06ad}
mkdir -p gpurun_out/$T
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/prof -o din -- python3 -u bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --model-steps 0 --train-steps 0 --native-steps 0 --din-steps 10 > gpurun_out/$T/bench.log 2>&1 || { tail -5 gpurun_out/$T/bench.log; exit 1; }
grep "din leg" gpurun_out/$T/bench.log | cut -c1-300
ls -la gpurun_out/$T/prof
