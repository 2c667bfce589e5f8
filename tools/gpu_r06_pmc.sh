# Round-6 rocprof evidence for the bench line (each counter its own pass,
# --kernel-trace / --stats only in their own run): kernel stats of the
# headline path, FETCH_SIZE and WRITE_SIZE of the lookup kernels.
# Summaries: python tools/pmc_summary.py <stats> <fetch> <write> r06 ev_lookup_line_kernel
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06pmc}
mkdir -p $O
B="bench.py --no-graph --steps 2 --warmup 1 --kernel-iters 3 --cpu-seconds 0 --train-steps 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --din-steps 0 --model-steps 0 --native-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --cpu-seconds 0 --steps 10 --warmup 3 --no-criteo --no-dcn --no-hybrid --no-deepfm --din-steps 0 --model-steps 0 --native-steps 0 > $O/stats.log 2>&1 || { tail -5 $O/stats.log; exit 1; }
echo stats ok
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $B > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
echo fetch ok
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $B > $O/write.log 2>&1 || { tail -5 $O/write.log; exit 1; }
echo write ok
