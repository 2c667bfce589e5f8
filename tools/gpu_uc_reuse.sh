# Uncached-reuse hazard (DESIGN §7 "Coherence of peer-written buffers"): the
# peer-write tests then test_xgmi_serve_grows_small_tables, run against the
# DIAGNOSTIC build of the library (make -C deeprec-1_amd ab AB_FLAGS=-DDR_UC_DIAG
# -> libdeeprec_amd_ab.so), where DR_IPC_RELEASE=1 hands freed uncached IPC
# blocks back to hipFree (the round-2 behaviour that corrupted EV rows).  The
# diagnostic build poisons every new pool / default row with 0xFF (kernel
# fill) and checks each default row written by hipMemcpy H2D and each grown
# pool's head, read back both by D2H copy and by a kernel, logging whether
# the buffer sits on a freed uncached range ([uc-diag] lines on stderr).
set -o pipefail
T=${1:-ucr}
mkdir -p gpurun_out/$T
export DEEPREC_AMD_LIB=$PWD/deeprec-1_amd/deeprec_amd/libdeeprec_amd_ab.so
for v in ${VARIANTS:-1}; do
  DR_IPC_RELEASE=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -k "xgmi" -q -s --timeout 200 --timeout-method thread > gpurun_out/$T/release$v.log 2>&1
  rc=$?
  echo "DR_IPC_RELEASE=$v rc=$rc"; grep -c "uc-diag" gpurun_out/$T/release$v.log; tail -4 gpurun_out/$T/release$v.log
  case $rc in 0|1) ;; *) exit $rc ;; esac
done
