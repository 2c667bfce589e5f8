# DCN-v2 (configs[4]) step: deep MLP on the hand MFMA tower (--bf16) vs
# autocast, the DCN GPU tests, and the --bf16 step's kernel stats.  Tag $1.
set -o pipefail
T=${1:-dcn}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_dcn.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; [ $rc -ne 0 ] && exit $rc
for a in "" "--bf16" "" "--bf16"; do
  timeout -k 10 300 python -u tools/model_step.py --model dcn $a >> gpurun_out/$T/steps.log 2>>gpurun_out/$T/steps.err || exit 1
done
cat gpurun_out/$T/steps.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/stats -o run -- python3 tools/model_step.py --model dcn --bf16 --steps 5 > gpurun_out/$T/prof.log 2>&1 || exit 1
echo done
