"""Score the four pose models on a LineMOD split with the device path: the
main() of scripts/visualization/compare_all_models.py:110-190, plus the
per-object filter of SURVEY.md §8f #3 (`--objects 06` = cat).

    python tools/compare_models.py --data-root .../Linemod_preprocessed/data \
        --model-dir .../Linemod_preprocessed/models --weights RGBD-Geometric=best_pose_model.pth [--objects 06]

Checkpoints are the reference's torch.save dicts ({'model_state_dict': ...});
they are opened with torch.load(weights_only=True) (the reference uses
weights_only=False), so a file holding anything beyond tensors and plain
containers is refused rather than unpickled.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

import torch  # noqa: E402

MODELS = {   # name -> (module, class, is_rgbd, needs_geometry); compare_all_models.py:40-51,146-165
    "RGB": ("models.pose_net_rgb", "PoseNetRGB", False, False),
    "RGB-Geometric": ("models.pose_net_rgb_geometric", "PoseNetRGBGeometric", False, True),
    "RGBD": ("models.pose_net_rgbd", "PoseNetRGBD", True, False),
    "RGBD-Geometric": ("models.pose_net_rgbd_geometric", "PoseNetRGBDGeometric", True, True),
}


def load_model(name, path, device):
    """compare_all_models.py:32-60 (prints and returns None on a missing file or error)."""
    import importlib
    if not os.path.exists(path):
        print(f"  {name}: Weights not found")
        return None
    try:
        mod, cls, _, _ = MODELS[name]
        model = getattr(importlib.import_module(mod), cls)(pretrained=False)
        ckpt = torch.load(path, map_location="cpu", weights_only=True)
        model.load_state_dict(ckpt["model_state_dict"])
        model = model.to(device).eval()
        print(f"  {name}: Loaded")
        return model
    except Exception as e:  # the reference reports and carries on
        print(f"  {name}: Error - {e}")
        return None


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--data-root", required=True)
    ap.add_argument("--model-dir", required=True)
    ap.add_argument("--weights", action="append", default=[], metavar="NAME=PATH",
                    help="model name (RGB, RGB-Geometric, RGBD, RGBD-Geometric) = checkpoint path")
    ap.add_argument("--mode", default="val")
    ap.add_argument("--batch-size", type=int, default=16)
    ap.add_argument("--objects", nargs="*", default=None, help="object folders to keep (06 = cat)")
    a = ap.parse_args(argv)
    from models.add_loss import ADDLoss
    from pose6d.linemod import LineMODSet, evaluate_model
    device = "cuda"
    print(f"\nModel Comparison on {device}\n")
    criterion = ADDLoss(a.model_dir, device)
    sets = {rgbd: LineMODSet(a.data_root, a.mode, rgbd=rgbd, augment_bbox=False, objects=a.objects)
            for rgbd in (False, True)}
    print(f"  {len(sets[False])} {a.mode} samples\n")
    weights = dict(w.split("=", 1) for w in a.weights)
    results = {}
    for name, (_, _, is_rgbd, geo) in MODELS.items():
        if name not in weights:
            continue
        model = load_model(name, weights[name], device)
        if model is not None:
            results[name] = evaluate_model(model, name, sets[is_rgbd].batches(a.batch_size, device), criterion,
                                           is_rgbd=is_rgbd, needs_geometry=geo)
    print("\nResults:\n" + "-" * 60)
    print(f"{'Model':<20} {'ADD (mm)':<12} {'ADD-S (mm)':<12} {'ADD-0.1d (%)':<12}")
    print("-" * 60)
    for name, m in results.items():
        print(f"{name:<20} {m['ADD (mm)']:<12.2f} {m['ADD-S (mm)']:<12.2f} {m['ADD-0.1d (%)']:<12.1f}")
    print("-" * 60)
    return results


if __name__ == "__main__":
    main()
