"""Per-HIP-queue busy time of one training step from a rocprofv3 --kernel-trace of
bench.py (the span between the last two pack_batch launches), by kernel family.

    python tools/queues.py gpurun_out/<dir>/run_kernel_trace.csv
"""
import collections
import csv
import re
import sys


def family(n):
    n = n.replace("(anonymous namespace)::", "")
    mm = re.search(r"(igemm_conv_kernel)ILi\d+ELi\d+ELi\d+ELi\d+ELi(\d)E.*DF16b", n)
    if mm:  # rocprofv3 leaves the __bf16 instantiations mangled
        return f"{mm.group(1)}{mm.group(2)}_bf16"
    m = re.match(r"(?:void )?([A-Za-z_0-9]+)(<[^(]*>)?", n)
    base = m.group(1)
    if base in ("igemm_conv_kernel", "wgrad_kernel"):
        base += "3" if ", 3," in (m.group(2) or "") or ", 3>" in (m.group(2) or "") else "1"
    return base


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "pack_batch" in r["Kernel_Name"]]
    a, b = idx[-2], idx[-1]
    step = rows[a:b]
    t0, t1 = int(step[0]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    print(f"step span {(t1 - t0) / 1e3:.0f} us, {len(step)} kernels")
    byq = collections.defaultdict(collections.Counter)
    for r in step:
        byq[r["Queue_Id"]][family(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for q, c in byq.items():
        print(f"queue {q}: busy {sum(c.values()):.0f} us")
        for k, v in c.most_common(18):
            print(f"  {v:8.0f}  {k}")
    ce = [r for r in step if "ce_up_loss" in r["Kernel_Name"]]
    if ce:
        print(f"forward (to the CE loss) {(int(ce[0]['Start_Timestamp']) - t0) / 1e3:.0f} us")
    # idle gaps of the busiest queue (the data-gradient chain): where the step waits
    q = max(byq, key=lambda k: sum(byq[k].values()))
    main = [r for r in step if r["Queue_Id"] == q]
    gaps, tail = [], 0.0
    for p, n in zip(main, main[1:]):
        g = (int(n["Start_Timestamp"]) - int(p["End_Timestamp"])) / 1e3
        if g > 20:
            gaps.append((g, family(p["Kernel_Name"]), family(n["Kernel_Name"]),
                         (int(p["End_Timestamp"]) - t0) / 1e3))
    tail = (t1 - int(main[-1]["End_Timestamp"])) / 1e3
    print(f"queue {q} idle: {sum(g[0] for g in gaps):.0f} us in {len(gaps)} gaps > 20 us, "
          f"{tail:.0f} us after its last kernel")
    for g, a_, b_, at in sorted(gaps, reverse=True)[:12]:
        print(f"  {g:7.0f} us at {at:7.0f} us: {a_} -> {b_}")


if __name__ == "__main__":
    main()
