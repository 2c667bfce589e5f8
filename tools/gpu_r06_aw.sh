# Round 6: native engine kinds at N = 1 with the hipGraph forward.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06aw}
mkdir -p gpurun_out/$T
for g in 1; do
DR_NATIVE_GRAPH=$g timeout -k 10 600 python3 -u bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --model-steps 0 --train-steps 0 --din-steps 0 > gpurun_out/$T/bench_$g.log 2>&1 || { tail -5 gpurun_out/$T/bench_$g.log; exit 1; }
grep "native engine" gpurun_out/$T/bench_$g.log | cut -c1-230
done
