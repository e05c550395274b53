"""Bucketed data-parallel training step on the GPU box: 2 ranks on one MI355X
over gloo (tests/ddp_worker.py), compared bit for bit with a 1-process step."""
import os
import subprocess
import sys
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_ddp_bucketed_step_matches_single_process():
    out = os.path.join(tempfile.mkdtemp(), "ddp.txt")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", "29631", os.path.join(REPO, "tests", "ddp_worker.py"), out]
    r = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    same, diff, nb = open(out).read().split()
    assert int(nb) > 3, "expected several buckets"
    assert same == "1", f"DDP step differs from the single-process step (max |diff| {diff})"
