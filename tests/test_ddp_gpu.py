"""Bucketed data-parallel training step on the GPU box: 2 and 3 ranks on one MI355X
over gloo (tests/ddp_worker.py), each on its own batch, against the 1-process
update from the averaged gradients -- eager and graph-segmented replay (3 ranks:
the non-power-of-two world size averages the gradient in a pass of its own)."""
import os
import subprocess
import sys
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_ddp_bucketed_step_matches_mean_gradient_update(world):
    out = os.path.join(tempfile.mkdtemp(), "ddp")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(29631 + world),
           os.path.join(REPO, "tests", "ddp_worker.py"), out]
    r = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    for rank in range(world):
        f = open(f"{out}.{rank}").read().split()
        same, diff, graph_same, run_eager, run_graph, agree, nb, nsegs, distinct = f
        assert int(distinct) == 1, "the two ranks' batches must give different gradients"
        assert int(nb) > 3 and int(nsegs) > 1, "expected several buckets and graph segments"
        assert same == "1", f"rank {rank}: DDP step != AdamW on the mean gradient (max |diff| {diff})"
        assert graph_same == "1", f"rank {rank}: graph-segmented DDP step != eager DDP step"
        assert run_eager == "1" and run_graph == "1", f"rank {rank}: local BN running stats differ"
        assert agree == "1", "ranks hold different parameters"
