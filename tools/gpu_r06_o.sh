# Round 6: plain torch graphs under allocator churn (no deeprec_amd, then with it loaded).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06o}
mkdir -p gpurun_out/$T
for p in sum two_sums softmax; do
  TCP_PIECE=$p timeout -k 10 120 python -u tools/torch_graph_churn_probe.py 2>&1 | grep -E "^TORCH|Error" | tee -a gpurun_out/$T/probe.log
done
TCP_PIECE=softmax timeout -k 10 120 python -u tools/torch_graph_churn_probe.py --with-lib 2>&1 | grep -E "^TORCH|Error" | tee -a gpurun_out/$T/probe.log
TCP_PIECE=softmax DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 120 python -u tools/torch_graph_churn_probe.py 2>&1 | grep -E "^TORCH|Error" | sed 's/^/[nopc] /' | tee -a gpurun_out/$T/probe.log
exit 0
