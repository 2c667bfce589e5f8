# Round 6: which free block does the captured DIN forward read? NaN bisection.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06g}
mkdir -p gpurun_out/$T
GPP_BISECT=1 GPP_PIECE=attn timeout -k 10 300 python -u tools/graph_piece_probe.py > gpurun_out/$T/attn.log 2>&1 || { tail -5 gpurun_out/$T/attn.log; exit 1; }
grep -v amdgpu.ids gpurun_out/$T/attn.log | tail -30
GPP_BISECT=1 GPP_PIECE=attn GPP_POOLS=all timeout -k 10 300 python -u tools/graph_piece_probe.py > gpurun_out/$T/attn_all.log 2>&1 || { tail -5 gpurun_out/$T/attn_all.log; exit 1; }
grep -v amdgpu.ids gpurun_out/$T/attn_all.log | tail -30
