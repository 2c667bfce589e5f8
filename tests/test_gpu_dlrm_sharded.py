"""The data-parallel DLRM step with row-sharded embeddings
(modelzoo.DLRM(engine=...) + train_step_sharded: sharded lookup, local loss /
world, dense gradients all-reduced, embedding gradient rows to their owners,
SGD + KV SGD) across PROCESSES on one GPU, against one process training the
same DLRM with the full tables on the whole global batch
(tools/dlrm_sharded_check.py): loss, dense weights and every owned EV row
within fp32 tolerance (1e-5 relative) after each of three steps.  Engines:
the RCCL all-to-all form (staged through gloo on one GPU) and the xGMI
peer-write form (real HIP IPC mappings between the processes); and hybrid
placement (two features replicated on every rank, their gradient slices
gathered by sharded.sync_replicated_grads, every replica equal to the
reference table); and DCN-v2 (configs[4]) with sharded tables, at bf16
tolerance."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world,engine,hybrid,model", [
    (2, "a2a", False, "dlrm"), (3, "a2a", False, "dlrm"), (2, "xgmi", False, "dlrm"),
    (2, "a2a", True, "dlrm"), (3, "xgmi", True, "dlrm"), (2, "xgmi", False, "dcn")])
def test_dlrm_sharded_step_matches_one_process(world, engine, hybrid, model):
    env = dict(os.environ)
    env["MASTER_ADDR"] = "127.0.0.1"
    cmd = [sys.executable, os.path.join(ROOT, "tools", "dlrm_sharded_check.py"),
           "--world", str(world), "--engine", engine, "--model", model] + (
               ["--hybrid"] if hybrid else [])
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=170)
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-4000:]
    assert sorted(x["rank"] for x in lines) == list(range(world))
    assert all(x["ok"] for x in lines), lines
