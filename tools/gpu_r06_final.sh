# Round 6 final evidence: the default bench line twice, and the DIN graph leg's kernel stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06final}
mkdir -p gpurun_out/$T
bash tools/gpu_r06_bench.sh $T || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/din -o din -- python3 -u bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --model-steps 0 --train-steps 0 --native-steps 0 --din-steps 20 > gpurun_out/$T/din.log 2>&1 || { tail -5 gpurun_out/$T/din.log; exit 1; }
echo din profiled
