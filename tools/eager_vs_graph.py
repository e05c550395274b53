"""Host issue time of the eager training step vs the GPU time, and the graph-replayed
step: whether the eager (DDP) backward can keep the GPU fed.
usage: python tools/eager_vs_graph.py"""
import sys, time, torch
sys.path[:0] = [".", "6d-pose-estimation_amd"]
from bench import synth_batch
from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
from pose6d.train import RGBDGeometricTrainer
torch.manual_seed(0)
dev = torch.device("cuda")
m = PoseNetRGBDGeometric(pretrained=False).to(dev)
tr = RGBDGeometricTrainer(m, 32, dtype=torch.bfloat16)
data = synth_batch(32, dev, seed=0)
for _ in range(3): tr.step_eager(data)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20): tr.step_eager(data)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"eager: host issue {(t1-t0)/20*1e3:.2f} ms/step, wall {(t2-t0)/20*1e3:.2f} ms/step")
tr.capture(data)
for _ in range(3): tr.step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20): tr.step()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"graph: wall {(t2-t0)/20*1e3:.2f} ms/step")
