# Round 6: PMC traffic of the DeepFM (D = 64 fp32) and DCN bf16 (D = 128 bf16)
# legs' fused lookup (tools/leg_pmc.py), each counter its own pass, plus the
# kernel trace; summarised into profiles/r06_pmc_traffic_<leg>.json.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r06q}
mkdir -p $O
for leg in deepfm dcn; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$leg/stats -o run -- python3 tools/leg_pmc.py --leg $leg > $O/$leg.stats.log 2>&1 || { tail -5 $O/$leg.stats.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$leg/fetch -o run -- python3 tools/leg_pmc.py --leg $leg --iters 6 > $O/$leg.fetch.log 2>&1 || { tail -5 $O/$leg.fetch.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$leg/write -o run -- python3 tools/leg_pmc.py --leg $leg --iters 6 > $O/$leg.write.log 2>&1 || { tail -5 $O/$leg.write.log; exit 1; }
  tail -1 $O/$leg.stats.log
  PMC_SOURCE="rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate passes, tools/leg_pmc.py --leg $leg --iters 6; median over dispatches" python3 tools/pmc_summary.py $O/$leg/stats $O/$leg/fetch $O/$leg/write r06 ev_lookup_line_kernel $leg | grep -E "bytes_per_launch|avg_ns" || exit 1
done
