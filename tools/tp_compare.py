"""Per-op backward time of two tools/tapeprof.py --csv runs (side stream off, medians): which ops a change moved.

    python tools/tp_compare.py before.csv after.csv
"""
import collections
import csv
import sys


def load(f):
    ops, meta = collections.defaultdict(list), {}
    for r in csv.DictReader(open(f)):
        if not r["label"]:
            continue
        k, ph = r["label"].split(":")
        meta[int(k)] = (r["kind"], r["ks"], r["stride"], r["M_out"], r["cin"], r["cout"])
        if ph != "fwd":
            ops[int(k)].append((r["entry"].replace("seg_", "").replace("_bf16io", ""), float(r["us"])))
    return ops, meta


def main(a_path, b_path):
    a, meta = load(a_path)
    b, _ = load(b_path)
    tot = 0.0
    for k in sorted(a):
        sa, sb = sum(x[1] for x in a[k]), sum(x[1] for x in b.get(k, []))
        tot += sb - sa
        m = meta[k]
        print(f"{k:3d} {m[0]:6s} k{m[1]}s{m[2]} M={m[3]:>8s} {m[4]:>5s}->{m[5]:<5s} before {sa:7.1f} after {sb:7.1f} "
              f"d {sb - sa:+7.1f} | " + " ".join(f"{n}:{u:.0f}" for n, u in b.get(k, [])))
    print(f"backward kernel time delta (both streams, side stream off): {tot:+.1f} us")


if __name__ == "__main__":
    main(*sys.argv[1:3])
