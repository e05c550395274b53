"""ORACLE — test infrastructure only.

CPU restatements of the reference hot path (SFR-Vision/6d-pose-estimation) used
as the checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
Nothing in the product (6d-pose-estimation_amd/) imports, links or calls this
package; the product fails loudly without its HIP library instead.

  oracle/add_core.c   ADD / ADD-S arithmetic with torch-CPU rounding (C, gcc)
  oracle/add_loss.py  ADDLoss.eval_metrics / forward / loader restatement
  oracle/pose_loss.py PoseLoss restatement (torch-CPU fp32, autograd for grads)
  oracle/resnet.py    ResNet50 trunk + the four PoseNet heads (torch-CPU fp32)

Pinning: add_loss/pose_loss are checked against tests/golden/*.npz, which
tools/gen_goldens.py produced by running the reference's own pose_loss.py and
add_loss.py.  resnet.py restates torchvision==0.24.1's ResNet50 (third-party,
absent from the image) and the reference's head code; it is pinned by structure
(state_dict names/shapes/param counts measured in SURVEY.md §8a) and by the
reference-pinned loss/metric code downstream of it -- model forward values are
"parity unpinned" by the reference.
"""
