# Round 6: graph + allocator churn, one graph, by piece of the DIN step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06d}
mkdir -p gpurun_out/$T
for p in fwd fwdbwd dense ev full; do
  for c in 0 1; do
    GPP_PIECE=$p GPP_CHURN=$c timeout -k 10 200 python -u tools/graph_piece_probe.py > gpurun_out/$T/${p}_$c.log 2>&1 || { tail -5 gpurun_out/$T/${p}_$c.log; exit 1; }
    grep -E "^piece|^LOSSES" gpurun_out/$T/${p}_$c.log
  done
done
