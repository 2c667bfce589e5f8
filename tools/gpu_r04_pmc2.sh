# Request-size split of the lookup kernels' memory-side traffic (own passes)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04pmc2
mkdir -p $O
B="bench.py --no-graph --steps 2 --warmup 1 --kernel-iters 3 --cpu-seconds 0 --train-steps 0 --no-criteo --no-dcn --no-hybrid"
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $O/size -o run -- python3 $B > $O/size.log 2>&1 || { tail -5 $O/size.log; exit 1; }
echo size ok
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum --output-format csv -d $O/dram -o run -- python3 $B > $O/dram.log 2>&1 || { tail -5 $O/dram.log; exit 1; }
echo dram ok
