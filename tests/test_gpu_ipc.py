"""The peer-write engine across PROCESSES through real HIP IPC mappings
(tools/xgmi_ipc_check.py): 2 and 3 ranks, each its own process on cuda:0,
inboxes / outputs / gradient buffers in uncached memory (dr_ipc_alloc)
exported with dr_ipc_export and mapped with dr_ipc_import.  Three forward
steps bit-exact against the CPU oracle and each backward's pulled gradient
rows exact.  The checker runs as a child process started with subprocess
(its ranks are spawned before any of them touches the GPU); the RCCL / xGMI
transport between distinct GPUs is the driver's multi-GPU run."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world", [2, 3])
def test_xgmi_ipc_multiprocess(world):
    env = dict(os.environ)
    env["MASTER_ADDR"] = "127.0.0.1"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "xgmi_ipc_check.py"),
                        "--world", str(world)], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=110)
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert sorted(x["rank"] for x in lines) == list(range(world))
    assert all(x["ipc_peer_write_ok"] and x["ipc_grad_pull_ok"] for x in lines)
