# gemm_tn with its reductions in one launch: MLP tests, then the DLRM bf16
# model step (model_step.py) and the bench DLRM leg
set -o pipefail
O=gpurun_out/r04tn
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_modelzoo.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/model_step.py --model dlrm --bf16 > $O/dlrm.log 2>&1 || { tail -3 $O/dlrm.log; exit 1; }
tail -1 $O/dlrm.log
timeout -k 10 300 python -u bench.py --cpu-seconds 0 --no-deepfm --no-criteo --no-dcn --no-hybrid --din-steps 0 --train-steps 0 --model-steps 20 > $O/b.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
grep "dlrm model step" $O/b.err
