# Round 5, batch A: the parity tests touched this round (lookup kernels,
# exact long runs, fused DIN attention, RCCL world-1, sharded C long runs),
# then the headline kernel A/B over DR_LOOKUP_KERNEL (2 pipelined, 1 line
# one-shot, 0 slot walk), then DIN / train-step timings.  Tag $1.
set -o pipefail
T=${1:-r05a}
mkdir -p gpurun_out/$T
timeout -k 10 1000 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_record_major.py \
  tests/test_gpu_parity.py tests/test_gpu_rows_grad.py tests/test_gpu_rows_deterministic.py \
  tests/test_gpu_din.py tests/test_gpu_rccl_comm.py tests/test_gpu_sharded_c.py tests/test_gpu_bf16.py \
  tests/test_gpu_configs.py tests/test_gpu_dcn.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$T/tests.log; grep -E "^FAILED|^ERROR" gpurun_out/$T/tests.log | head -20
# a test failure (rc 1) still lets the timings run; a crash / timeout stops here
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
B="bench.py --cpu-seconds 0 --train-steps 0 --no-criteo --no-dcn --no-hybrid --no-deepfm --din-steps 0 --model-steps 0 --native-steps 0"
for v in 2 1 0 2 1 0; do
  DR_LOOKUP_KERNEL=$v timeout -k 10 300 python -u $B > gpurun_out/$T/k$v.json 2> gpurun_out/$T/k$v.err || { tail -5 gpurun_out/$T/k$v.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/$T/k$v.json').read().strip().splitlines()[-1])
print('kernel $v', 'ms', d['ms_per_step'], 'headline', d['roofline']['kernel_ms'], d['roofline']['frac'], 'gather', d['roofline_row_gather']['kernel_ms'])"
done
for v in 1 0 1 0; do
  DR_DIN_FUSED_ATTENTION=$v timeout -k 10 300 python -u tools/model_step.py --model din --steps 10 > gpurun_out/$T/din$v.log 2>&1 || { tail -5 gpurun_out/$T/din$v.log; exit 1; }
  echo "din fused=$v: $(tail -1 gpurun_out/$T/din$v.log)"
done
DR_GRAD_SERIAL_MAX=8192 timeout -k 10 300 python -u tools/model_step.py --model din --steps 10 > gpurun_out/$T/din_pieces.log 2>&1 || { tail -5 gpurun_out/$T/din_pieces.log; exit 1; }
echo "din pieces of 8192 (A/B): $(tail -1 gpurun_out/$T/din_pieces.log)"
timeout -k 10 200 python -u tools/cross_dw_probe.py > gpurun_out/$T/cross_dw.log 2>&1 || { tail -5 gpurun_out/$T/cross_dw.log; exit 1; }
cat gpurun_out/$T/cross_dw.log
timeout -k 10 120 tools/uc_replay_probe 3 0 > gpurun_out/$T/uc_replay.log 2>&1 || { tail -5 gpurun_out/$T/uc_replay.log; exit 1; }
tail -2 gpurun_out/$T/uc_replay.log
timeout -k 10 120 tools/uc_replay_probe 3 1 > gpurun_out/$T/uc_replay_control.log 2>&1 || { tail -5 gpurun_out/$T/uc_replay_control.log; exit 1; }
tail -1 gpurun_out/$T/uc_replay_control.log
