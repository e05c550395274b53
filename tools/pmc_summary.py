"""Join rocprofv3 --pmc passes into per-kernel-symbol HBM traffic per launch.

    python tools/pmc_summary.py OUT.json fetch_dir write_dir [mfma_dir]

Each *_dir holds one `rocprofv3 --pmc ... --output-format csv` pass
(*_counter_collection.csv).  Corrections per MI355X_MICROARCH.md § HBM:
FETCH_SIZE (KiB) reports half of the bytes of wide coalesced streaming reads on
gfx950 -> doubled; WRITE_SIZE (KiB) is exact for 16-B streaming stores.
Only dispatches between the step_profile.py markers (pinhole_z_fwd launches) are
counted, so the numbers are per launch inside the training step.
"""
import collections
import glob
import json
import os
import re
import subprocess
import sys


def _itanium_template(name):
    """_ZN12_GLOBAL__N_1<len><ident>I<args>E... -> ident<args> (the forms our kernels
    use: Li<n>E integers, DF16b = __bf16, f = float); GNU c++filt on this image
    does not know DF16b."""
    m = re.match(r"_ZN12_GLOBAL__N_1(\d+)", name)
    if not m:
        return None
    n = int(m.group(1))
    rest = name[m.end():]
    ident, rest = rest[:n], rest[n:]
    if not rest.startswith("I"):
        return ident
    args, rest = [], rest[1:]
    while rest and not rest.startswith("E"):
        t = re.match(r"Li(-?\d+)E", rest)
        b = re.match(r"Lb([01])E", rest)
        if t:
            args.append(t.group(1)); rest = rest[t.end():]
        elif b:
            args.append("true" if b.group(1) == "1" else "false"); rest = rest[b.end():]
        elif rest.startswith("DF16b"):
            args.append("__bf16"); rest = rest[5:]
        elif rest.startswith("f"):
            args.append("float"); rest = rest[1:]
        else:
            return None
    return f"{ident}<{', '.join(args)}>"


def demangle(name):
    if name.startswith("_Z"):
        t = _itanium_template(name)
        if t:
            return t
        name = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*$", "", name).strip()
    name = re.sub(r"^void ", "", name)
    return name


def load(d, counter):
    """{dispatch_id: (symbol, value)} of one pass, restricted to the marker window."""
    import csv
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    rows = collections.OrderedDict()
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            did = int(r["Dispatch_Id"])
            sym, v = rows.get(did, (r["Kernel_Name"], 0.0))
            rows[did] = (sym, v + float(r["Counter_Value"]))
    ids = sorted(rows)
    marks = [i for i in ids if "pinhole_z_fwd" in rows[i][0]]
    if len(marks) >= 2:
        ids = [i for i in ids if marks[0] < i < marks[-1]]
    return {i: (demangle(rows[i][0]), rows[i][1]) for i in ids}


def main():
    out, fdir, wdir = sys.argv[1:4]
    mdir = sys.argv[4] if len(sys.argv) > 4 else None
    fetch, write = load(fdir, "FETCH_SIZE"), load(wdir, "WRITE_SIZE")
    agg = collections.OrderedDict()
    for src, key in ((fetch, "fetch_kib"), (write, "write_kib")):
        for _, (sym, v) in src.items():
            a = agg.setdefault(sym, {"launches_fetch": 0, "launches_write": 0, "fetch_kib": 0.0, "write_kib": 0.0})
            a[key] += v
            a["launches_" + key.split("_")[0]] += 1
    if mdir:
        mf = load(mdir, "SQ_VALU_MFMA_BUSY_CYCLES")
        for _, (sym, v) in mf.items():
            a = agg.setdefault(sym, {})
            a["mfma_busy_cycles"] = a.get("mfma_busy_cycles", 0.0) + v
            a["launches_mfma"] = a.get("launches_mfma", 0) + 1
    res = {}
    for sym, a in agg.items():
        nf, nw = a.get("launches_fetch", 0), a.get("launches_write", 0)
        r = {"launches": max(nf, nw)}
        if nf and nw:
            fb = 2.0 * a["fetch_kib"] * 1024 / nf      # gfx950 FETCH_SIZE correction (x2)
            wb = a["write_kib"] * 1024 / nw
            r.update({"fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb, "hbm_bytes_per_launch": fb + wb})
        if a.get("launches_mfma"):
            r["mfma_busy_cycles_per_launch"] = a["mfma_busy_cycles"] / a["launches_mfma"]
        res[sym] = r
    json.dump({"source": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE | SQ_VALU_MFMA_BUSY_CYCLES, separate passes, "
                         "eager training steps between markers (tools/step_profile.py --eager)",
               "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); KiB -> bytes",
               "kernels": res}, open(out, "w"), indent=1)
    for sym, r in sorted(res.items(), key=lambda kv: -kv[1].get("hbm_bytes_per_launch", 0))[:20]:
        print(f"{r.get('hbm_bytes_per_launch', 0) / 1e6:9.2f} MB/launch  x{r['launches']:4d}  {sym[:90]}")


if __name__ == "__main__":
    main()
