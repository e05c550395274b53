"""Condense a tools/conv_bench.py log: per shape and pass, the auto pick and the best variant."""
import re
import sys

for line in open(sys.argv[1]):
    if "|" not in line:
        print(line.strip()[:200])
        continue
    head, rest = line.split("|", 1)
    out = {}
    for tag, us, tf in re.findall(r"(\w+?):\s*([\d.]+)us/\s*(\d+)T", rest):
        out.setdefault(tag[0], []).append((float(us), tag[1:], int(tf)))
    s = head.strip()
    for p in ("f", "d", "w"):
        if p in out:
            auto = [x for x in out[p] if x[1] in ("fautosauto", "bauto", "fauto")]
            best = min(out[p])
            s += f"  {p}: auto {auto[0][0] if auto else float('nan'):6.1f} best {best[0]:6.1f} ({best[1]}, {best[2]}T)"
    print(s)
