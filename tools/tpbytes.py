"""Per-launch HBM rates from a tools/tapeprof.py --csv dump: for the memory-bound entry points
(BatchNorm passes, depthwise, 1x1 convs) the algorithmic bytes of the launch / its median time.

    python tools/tpbytes.py gpurun_out/<tag>/tp_bf16io.csv [--elem 2] [--entry seg_bn_backward]
"""
import argparse
import collections
import csv


def traffic(entry, kind, ks, m_out, m_in, cin, cout, s):
    """Algorithmic bytes of one launch (elements x storage size)."""
    if entry.startswith("seg_bn_backward"):
        return 5 * m_out * cout * s           # partial: dA, y; apply: dA, y -> dY
    if entry.startswith("seg_bn_apply"):
        return 2 * m_out * cout * s
    if entry.startswith("seg_bn_stats"):
        return m_out * cout * s
    if entry.startswith("seg_dw_fwd") or entry.startswith("seg_dw_dgrad"):
        return (m_in + m_out) * cout * s
    if entry.startswith("seg_conv_igemm") and ks == 1:
        return (m_in * cin + m_out * cout) * s
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--elem", type=int, default=2)
    ap.add_argument("--entry", default="")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    tot = collections.defaultdict(lambda: [0.0, 0.0, 0])
    out = []
    for r in rows:
        if a.entry and not r["entry"].startswith(a.entry):
            continue
        try:
            ks, m_out, m_in, cin, cout = (int(r[k]) for k in ("ks", "M_out", "M_in", "cin", "cout"))
        except ValueError:
            continue
        us = float(r["us"])
        b = traffic(r["entry"], r["kind"], ks, m_out, m_in, cin, cout, a.elem)
        if not b:
            continue
        t = tot[r["entry"]]
        t[0] += us
        t[1] += b
        t[2] += 1
        out.append((us, b / us / 1e3, r["label"], r["entry"], f"{r['kind']} k{ks} M={m_out} {cin}->{cout}"))
    for us, gbs, label, entry, desc in sorted(out, reverse=True):
        print(f"{us:8.1f} us {gbs:7.0f} GB/s  {label:9s} {entry:28s} {desc}")
    print()
    for e, (us, b, n) in sorted(tot.items(), key=lambda kv: -kv[1][0]):
        print(f"{e:32s} {n:3d} launches {us / 1e3:7.3f} ms  {b / 1e9:6.2f} GB  {b / us / 1e3:7.0f} GB/s")


if __name__ == "__main__":
    main()
