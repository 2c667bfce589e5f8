# Round-4 counter evidence, each counter group its own pass:
#  * the lookup kernels (headline ev_lookup_onehot_kernel<4,32,...> and the
#    DeepFM leg's <4,16,...>): TCC_EA0_RDREQ / TCC_EA0_WRREQ (memory-side
#    requests), TCC_HIT / TCC_MISS (L2), plus the kernel trace for durations;
#  * crossnet_8ph_kernel (tools/kernel_roofline.py --only crossnet):
#    SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, SQ_LDS_BANK_CONFLICT,
#    SQ_LDS_IDX_ACTIVE, GRBM_GUI_ACTIVE.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04pmc
mkdir -p $O
B="bench.py --no-graph --steps 2 --warmup 1 --kernel-iters 3 --cpu-seconds 0 --train-steps 0 --no-criteo --no-dcn --no-hybrid"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $B > $O/stats.log 2>&1 || { tail -5 $O/stats.log; exit 1; }
echo stats ok
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d $O/req -o run -- python3 $B > $O/req.log 2>&1 || { tail -5 $O/req.log; exit 1; }
echo req ok
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/hit -o run -- python3 $B > $O/hit.log 2>&1 || { tail -5 $O/hit.log; exit 1; }
echo hit ok
C="tools/kernel_roofline.py --only crossnet"
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $O/cross -o run -- python3 $C > $O/cross.log 2>&1 || { tail -5 $O/cross.log; exit 1; }
echo cross ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cross_stats -o run -- python3 $C > $O/cross_stats.log 2>&1 || { tail -5 $O/cross_stats.log; exit 1; }
echo cross stats ok
