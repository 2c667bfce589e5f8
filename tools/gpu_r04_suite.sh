# Round-4 full GPU suite + smoke, then the DCN-v2 bf16 model step with the
# hand dx kernel and with the library addmm (A/B, same box)
set -o pipefail
T=${1:-r04suite}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1
rc=$?; tail -8 gpurun_out/$T/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/$T/smoke.log; [ $rc -ne 0 ] && exit $rc
for v in hand lib hand lib; do
  if [ $v = lib ]; then export DR_CROSSNET_DX_LIB=1; else unset DR_CROSSNET_DX_LIB; fi
  timeout -k 10 200 python -u tools/model_step.py --model dcn --bf16 > gpurun_out/$T/dcn_$v.log 2>&1 || { tail -5 gpurun_out/$T/dcn_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/$T/dcn_$v.log)"
done
