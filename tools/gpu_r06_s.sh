# Round 6: the default bench (graph checks, native engine kinds, cpu_baseline).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${1:-r06s}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u bench.py > gpurun_out/$T/bench.log 2>&1 || { tail -5 gpurun_out/$T/bench.log; exit 1; }
tail -1 gpurun_out/$T/bench.log > gpurun_out/$T/bench.json
grep -E "native engine|din leg|dlrm model step|train step" gpurun_out/$T/bench.log | cut -c1-400
python3 -c "import json;d=json.load(open('gpurun_out/$T/bench.json'));print('value',d['value'],'ms',d['ms_per_step'],'frac',d['roofline']['frac']);print(json.dumps(d.get('cpu_baseline'))[:700])"
