# Round 5: the hand DIN weight-gradient pass as the default -- DIN GPU tests,
# the DIN graph test, the bench (DIN leg), its kernel stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r05z2}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_din.py tests/test_gpu_din_graph.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -2 gpurun_out/$T/tests.log; grep -E "^FAILED|^ERROR" gpurun_out/$T/tests.log | head -10
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/$T/bench.log 2>&1 || { tail -5 gpurun_out/$T/bench.log; exit 1; }
tail -1 gpurun_out/$T/bench.log > gpurun_out/$T/bench.json
python3 -c "import json;d=json.load(open('gpurun_out/$T/bench.json'));print('value',d['value'],'ms',d['ms_per_step']);print({k:v for k,v in d.items() if 'din' in k.lower()})"
