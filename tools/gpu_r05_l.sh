# Round 5, batch L: kernel statistics of the dW probe on the w4 kernel
# (slice-major order) -- splits crossnet_dw_w4_kernel from the split-K
# reduction; MFMA busy and HBM fetch of the hand kernel alone.  Tag $1.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05l}
mkdir -p gpurun_out/$T
DR_CROSSNET_DW_KERNEL=w4 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o dw -- python3 -u tools/cross_dw_probe.py > gpurun_out/$T/probe.log 2>&1 || { tail -5 gpurun_out/$T/probe.log; exit 1; }
grep -E "crossnet_dw|matmul|mm\(" gpurun_out/$T/probe.log
f=$(find gpurun_out/$T/prof -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 "$f" | head -14
DR_CROSSNET_DW_KERNEL=w4 timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/$T/mfma -o run -- python3 tools/cross_dw_probe.py --hand-only > gpurun_out/$T/mfma.log 2>&1 || { tail -5 gpurun_out/$T/mfma.log; exit 1; }
DR_CROSSNET_DW_KERNEL=w4 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/$T/fetch -o run -- python3 tools/cross_dw_probe.py --hand-only > gpurun_out/$T/fetch.log 2>&1 || { tail -5 gpurun_out/$T/fetch.log; exit 1; }
for q in mfma fetch; do f=$(find gpurun_out/$T/$q -name "*counter_collection.csv" | head -1); grep -E "crossnet_dw|Kernel_Name" "$f" | cut -c1-400 | head -12; done
