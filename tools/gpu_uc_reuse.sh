# Uncached-reuse hazard (DESIGN §7 "Coherence of peer-written buffers"): the
# peer-write tests then test_xgmi_serve_grows_small_tables, with freed
# uncached IPC blocks handed back to hipFree after a device sync
# (DR_IPC_RELEASE=2), then at once (=1, the round-2 behaviour that corrupted
# EV rows).  A data mismatch is a test failure, not a fault: both variants run
# unless one faults / aborts / times out.
set -o pipefail
T=${1:-ucr}
mkdir -p gpurun_out/$T
for v in ${VARIANTS:-2 1}; do
  DR_IPC_RELEASE=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -k "xgmi" -q --timeout 200 --timeout-method thread > gpurun_out/$T/release$v.log 2>&1
  rc=$?
  echo "DR_IPC_RELEASE=$v rc=$rc"; tail -4 gpurun_out/$T/release$v.log
  case $rc in 0|1) ;; *) exit $rc ;; esac
done
