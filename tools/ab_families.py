"""Compare per-family kernel time of two rocprofv3 --stats runs (A/B of two builds).

    python tools/ab_families.py gpurun_out/abp_old_f32 gpurun_out/abp_new_f32
"""
import csv
import re
import sys


def families(d):
    out, tot = {}, 0.0
    for r in csv.DictReader(open(f"{d}/run_kernel_stats.csv")):
        n = r["Name"]
        m = re.search(r"(\w+_kernel\w*?)(?:<|\(|I|E|$)", n)
        key = m.group(1) if m else n[:40]
        if "chan_partial" in n:
            k = re.search(r"chan_partial_kernel(?:<|ILi)(\d)", n)
            key = f"chan_partial<{k.group(1)}>" if k else key
        t = float(r["TotalDurationNs"])
        out[key] = out.get(key, 0.0) + t
        tot += t
    return out, tot


a, ta = families(sys.argv[1])
b, tb = families(sys.argv[2])
print(f"total {ta / 1e6:.2f} -> {tb / 1e6:.2f} ms")
for k in sorted(set(a) | set(b), key=lambda k: -abs(b.get(k, 0) - a.get(k, 0)))[:12]:
    print(f"{k:40s} {a.get(k, 0) / 1e6:8.3f} -> {b.get(k, 0) / 1e6:8.3f} ms")
