"""Worker of tests/test_ddp_gpu.py (launched by torch.distributed.run, 2 ranks on
ONE GPU over gloo: RCCL needs a GPU per rank).  Both ranks train one step on the
same batch through the bucketed all-reduce path (RGBDGeometricTrainer with a
process group); the averaged gradient then equals each rank's own, so the
updated parameters must equal a single-process step bit for bit."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    out = sys.argv[1]
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from bench import synth_batch
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    from pose6d.train import RGBDGeometricTrainer
    B = 4
    data = synth_batch(B, dev, seed=77)

    def run(pg, bucket_mb):
        torch.manual_seed(0)
        model = PoseNetRGBDGeometric(pretrained=False).to(dev)
        for m in model.modules():
            if isinstance(m, torch.nn.Dropout):
                m.eval()
        tr = RGBDGeometricTrainer(model, B, dtype=torch.bfloat16, process_group=pg, bucket_mb=bucket_mb)
        tr.step_eager(data)
        torch.cuda.synchronize()
        return tr.arena.flat.clone(), tr

    flat_ddp, tr = run(dist.group.WORLD, 2.0)    # small buckets: many all-reduces overlap backward
    n_buckets = len(tr.bucket_ends)
    if rank == 0:
        flat_one, _ = run(None, 2.0)
        same = bool(torch.equal(flat_ddp, flat_one))
        diff = float((flat_ddp - flat_one).abs().max())
        with open(out, "w") as f:
            f.write(f"{int(same)} {diff} {n_buckets}\n")
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
