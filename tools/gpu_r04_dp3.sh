# DIN data-parallel checks, the 2-rank bench rehearsal (all legs), N = 1
# bench; then the DLRM step with and without its hipGraph, and a kernel
# profile of the DLRM bf16 model step
set -o pipefail
O=gpurun_out/r04dp3
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_din_dp.py tests/test_gpu_bench_rehearsal.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -8 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; grep -E "dlrm model step|din leg|train step" $O/bench.err; tail -2 $O/bench.err; [ $rc -ne 0 ] && exit $rc
S="bench.py --cpu-seconds 0 --no-deepfm --no-criteo --no-dcn --no-hybrid --din-steps 0 --train-steps 0 --model-steps 20"
timeout -k 10 300 python -u $S > $O/graph.json 2> $O/graph.err || { tail -5 $O/graph.err; exit 1; }
grep "dlrm model step" $O/graph.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dlrm_prof -o run -- python3 tools/model_step.py --model dlrm --bf16 --rows 2000000 > $O/dlrm_prof.log 2>&1 || { tail -5 $O/dlrm_prof.log; exit 1; }
tail -1 $O/dlrm_prof.log
