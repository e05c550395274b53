"""Per-conv roofline estimates of the ResNet50 trunk at batch B (bf16): MFMA time
at the dense bf16 peak vs HBM time of one read of the input + weights and one
write of the output.  python tools/conv_roof.py [B]"""
import sys


def resnet50_convs():
    convs = [("stem", 224, 3, 64, 7, 2, 112)]
    H, cin = 56, 64
    for li, (w, nb, s) in enumerate([(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]):
        for b in range(nb):
            st = s if b == 0 else 1
            Ho = H // st
            if b == 0:   # the trunk's forward order: downsample first (pose6d/trunk.py)
                convs.append((f"l{li + 1}.{b}.ds", H, cin, 4 * w, 1, st, Ho))
            convs.append((f"l{li + 1}.{b}.c1", H, cin, w, 1, 1, H))
            convs.append((f"l{li + 1}.{b}.c2", H, w, w, 3, st, Ho))
            convs.append((f"l{li + 1}.{b}.c3", Ho, w, 4 * w, 1, 1, Ho))
            cin, H = 4 * w, Ho
    return convs


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    tf = tm_all = th_all = 0.0
    for n, H, ci, co, k, s, Ho in resnet50_convs():
        M, K = B * Ho * Ho, k * k * ci
        f = 2 * M * co * K
        by = (B * H * H * ci + M * co + co * K) * 2
        tm, th = f / 2.5e15 * 1e6, by / 6.3e12 * 1e6
        tf += f
        tm_all += tm
        th_all += max(tm, th)
        print(f"{n:10s} M={M:7d} N={co:5d} K={K:5d} GF={f / 1e9:6.2f} MB={by / 1e6:6.1f} "
              f"t_mfma={tm:5.1f}us t_hbm={th:5.1f}us wg64={(M + 63) // 64 * ((co + 63) // 64)}")
    print(f"total fwd GFLOP {tf / 1e9:.1f}  sum t_mfma {tm_all:.0f} us  sum max(t_mfma, t_hbm) {th_all:.0f} us")


if __name__ == "__main__":
    main()
