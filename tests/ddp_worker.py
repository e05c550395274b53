"""Worker of tests/test_ddp_gpu.py (launched by torch.distributed.run, 2 or 3 ranks on
ONE GPU over gloo: RCCL needs a GPU per rank; 3 ranks exercise the non-power-of-two
average pass).  argv: OUT [B [BUCKET_MB]] -- B = 4 with 2 MB buckets (many buckets and
segments on a small model step), or BASELINE configs[4]'s per-rank workload: B = 32 with
the trainer's default 25 MB buckets (what bench.py --gpus N builds).  Each rank trains one step on its
OWN batch (seed 77 + rank) through the bucketed all-reduce path
(RGBDGeometricTrainer with a process group), eagerly and replayed from the
segmented graphs.  Rank 0 also builds the expected update in one process: the
gradients of the two batches from two 1-process trainers, averaged, fed to the
same clip-norm + AdamW step.  With two ranks the all-reduce sum is exact
(a + b == b + a), so the parameters must agree bit for bit; each rank's BatchNorm
running statistics must equal a 1-process step on its own batch (local BN)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    out = sys.argv[1]
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from bench import synth_batch
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    from pose6d.train import RGBDGeometricTrainer
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    bucket = float(sys.argv[3]) if len(sys.argv) > 3 else 2.0
    batches = [synth_batch(B, dev, seed=77 + r) for r in range(world)]

    def trainer(pg, bucket_mb=bucket):
        torch.manual_seed(0)
        model = PoseNetRGBDGeometric(pretrained=False).to(dev)
        for m in model.modules():
            if isinstance(m, torch.nn.Dropout):
                m.eval()
        return RGBDGeometricTrainer(model, B, dtype=torch.bfloat16, process_group=pg, bucket_mb=bucket_mb)

    def buffers(tr):
        return torch.cat([v.float().flatten() for k, v in tr.model.state_dict().items() if "running" in k])

    # eager bucketed step (small buckets: many all-reduces overlap backward)
    tr = trainer(dist.group.WORLD)
    tr.step_eager(batches[rank])
    torch.cuda.synchronize()
    flat_eager, n_buckets, run_eager = tr.arena.flat.clone(), len(tr.bucket_ends), buffers(tr)
    # graph-segmented bucketed step: capture() runs 2 eager warm-up steps; re-seed the
    # parameters/moments/buffers afterwards so the replayed step starts from the same state
    trg = trainer(dist.group.WORLD)
    snap = trg.snapshot()
    trg.capture(batches[rank])
    trg.restore(snap)
    trg.step()
    torch.cuda.synchronize()
    flat_graph, run_graph, n_segs = trg.arena.flat.clone(), buffers(trg), len(trg.graphs) - 1

    # every rank holds the same parameters
    mine = flat_eager.cpu()
    others = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(others, mine)
    ranks_agree = all(torch.equal(o, mine) for o in others)

    # 1-process reference: own-batch step (BN running stats) + mean-gradient update
    ref = trainer(None)
    ref.step_eager(batches[rank])
    torch.cuda.synchronize()
    run_ref = buffers(ref)
    grads = []
    for r in range(world):
        t = trainer(None)
        t.step_eager(batches[r])
        torch.cuda.synchronize()
        grads.append(t.arena.grad.clone())
    t = trainer(None)
    with torch.no_grad():
        total = grads[0].clone()
        for g in grads[1:]:
            total += g
        t.arena.grad.copy_(total)
        t.arena.grad.mul_(1.0 / world)
    t._optimizer()
    torch.cuda.synchronize()
    flat_ref = t.arena.flat
    # two ranks: the all-reduce sum is exact, so bit for bit; more ranks: gloo's summation
    # order may differ from this left-to-right sum by an ulp, then ~1e-4 relative after AdamW
    if world == 2:
        same = torch.equal(flat_eager, flat_ref)
    else:
        same = bool(((flat_eager - flat_ref).abs() <= 1e-7 + 1e-4 * flat_ref.abs()).all())
    res = [int(same), float((flat_eager - flat_ref).abs().max()),
           int(torch.equal(flat_graph, flat_eager)), int(torch.equal(run_eager, run_ref)),
           int(torch.equal(run_graph, run_ref)), int(ranks_agree), n_buckets, n_segs,
           int(not torch.equal(grads[0], grads[1]))]
    with open(f"{out}.{rank}", "w") as f:
        f.write(" ".join(str(x) for x in res) + "\n")
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
