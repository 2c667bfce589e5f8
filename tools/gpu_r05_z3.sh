# Round 5: the DIN backward without the zeroed tail + the P-bounded weight-
# gradient pass -- DIN GPU tests,
# the DIN graph test, the bench (DIN leg), its kernel stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05z4}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_din.py tests/test_gpu_din_graph.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -2 gpurun_out/$T/tests.log; grep -E "^FAILED|^ERROR" gpurun_out/$T/tests.log | head -10
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/$T/bench.log 2>&1 || { tail -5 gpurun_out/$T/bench.log; exit 1; }
tail -1 gpurun_out/$T/bench.log > gpurun_out/$T/bench.json
python3 -c "import json;d=json.load(open('gpurun_out/$T/bench.json'));print('value',d['value'],'ms',d['ms_per_step']);print({k:v for k,v in d.items() if 'din' in k.lower()})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o din -- python3 -u tools/model_step.py --model din --steps 10 > gpurun_out/$T/din_prof.log 2>&1 || exit 1
echo profiled
