"""The N > 1 bench path, rehearsed on one GPU (VERDICT r02 "next" #6): two
bench.py ranks started by torch.distributed.run, both on cuda:0, the
row-sharded tables split by owner = key % 2, the all-to-alls staged through
host memory over gloo (DR_BENCH_GLOO_STAGED=1; a 1-GPU box cannot host two
RCCL ranks).  bench.py's own engine check must pass on every rank: the
peer-write (xGMI IPC) engine's output equals the all-to-all engine's bit for
bit on steps 0-3 before timing, and on the last timed step plus two more
after it -- each output consumed by the next step's reads, as in a model
step -- and the sampled headline rows equal the synthetic tables' rows.
The rehearsal also runs the N > 1 training step (sharded forward + backward
to the owners + owner SGD), the data-parallel DLRM model step (dense
gradients all-reduced) and the hybrid-placement Criteo-TB leg (large
vocabularies capped for time).  Never a reported number: the timing of
staged steps means nothing."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("engine", ["xgmi", "xgmi-dedup", "a2a"])
def test_bench_two_rank_rehearsal(engine):
    env = dict(os.environ)
    env.update(DR_BENCH_GLOO_STAGED="1", MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1",
           "--master-port", {"xgmi": "29531", "xgmi-dedup": "29533", "a2a": "29532"}[engine],
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "6", "--warmup", "2",
           "--rows", "200000", "--batch", "8192", "--tables", "8", "--cpu-seconds", "0",
           "--check-rows", "4096", "--engine", engine.split("-")[0], "--train-steps", "3",
           "--hybrid-cap", "1000000", "--model-steps", "3", "--din-steps", "3",
           "--din-batch", "1024", "--native-steps", "4"]
    if engine == "xgmi-dedup":
        cmd += ["--dedup", "--zipf", "1.05"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=170)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    line = lines[0]
    assert line["n_gpus"] == 2
    assert line["correctness"]["bitexact"] and line["correctness"]["checked_rows"] == 4096
    cfg = line["config"]
    if engine.startswith("xgmi"):
        assert cfg["engine"] == "xgmi peer-write" + (" + dedup" if "dedup" in engine else ""), cfg
        assert cfg["engine_check"].count("True") == 2 and "False" not in cfg["engine_check"], cfg
    else:
        assert cfg["engine"] == "RCCL all-to-all", cfg
    # the N > 1 training step (sharded forward + backward + owner SGD) ran
    assert line["train_step"]["engine"] == cfg["engine"] and line["train_step"]["steps"] == 3
    # the data-parallel DLRM model step with the sharded lookup
    dl = line["dlrm_train_step"]
    assert dl["global_batch"] == 2 * 8192 and dl["steps"] == 3 and dl["engine"] == cfg["engine"]
    # the data-parallel DIN leg (replicated EVs)
    assert line["din_config"]["n_gpus"] == 2 and line["din_config"]["global_batch"] == 2048
    # the hybrid-placement leg: replicated small features + sharded large
    # ones, sampled rows bit-exact and (xgmi) equal to the all-to-all engine
    hy = line["criteo_tb_hybrid"]
    assert hy["bitexact"] and hy["n_gpus"] == 2 and hy["checked_rows"] > 0, hy
