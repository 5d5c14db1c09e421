"""Side-stream contention table: every main-queue kernel of one training step, its duration
with the weight-gradient side stream on (overlapped) and off (alone), and the side-queue kernels that ran beside
the worst-inflated ones.

    python tools/contention.py <trace overlapped.csv> <trace alone.csv> [--top 40] [--md out.md]

Both inputs are rocprofv3 --kernel-trace CSVs of `bench.py` runs of the same workload (SEG_OVERLAP=1 / 0).  A step
is the span between the last two seg_pack_batch launches (the first launch of every step).  The main queue is the
busiest one; the tape issues the same main-queue launches in the same order with the side stream on or off (off:
the side stream's launches interleave on the one queue), so the overlapped run's main-queue sequence is matched in
order inside the alone run's.
"""
import argparse
import collections
import csv
import re


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    m = re.search(r"_ZN12_GLOBAL__N_1\d+(\w+?)I", n)
    if m:  # rocprofv3 leaves __bf16 instantiations mangled
        return m.group(1) + "<bf16>"
    m = re.match(r"(?:void )?([A-Za-z_0-9]+)(<[^(]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:60]


def step_kernels(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "pack_batch" in r["Kernel_Name"]]
    a, b = idx[-2], idx[-1]
    step = rows[a:b]
    busy = collections.Counter()
    for r in step:
        busy[r["Queue_Id"]] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    main_q = max(busy, key=busy.get)
    t0 = int(step[0]["Start_Timestamp"])
    ks = [(short(r["Kernel_Name"]), (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3,
           r["Queue_Id"] == main_q) for r in step]
    span = (int(rows[b]["Start_Timestamp"]) - t0) / 1e3
    return ks, span


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("overlapped")
    ap.add_argument("alone")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    ko, span_o = step_kernels(a.overlapped)
    ka, span_a = step_kernels(a.alone)
    mo = [k for k in ko if k[3]]
    side = [k for k in ko if not k[3]]
    # with the side stream off its launches run on the main queue, interleaved in program order: the overlapped
    # main-queue sequence is a subsequence of the alone trace (greedy match by name)
    ma, j = [], 0
    for k in ka:
        if j < len(mo) and k[0] == mo[j][0]:
            ma.append(k)
            j += 1
    if len(ma) != len(mo):
        raise SystemExit(f"main-queue launches not found in the alone trace ({len(ma)} of {len(mo)} matched)")
    rows = []
    for i, (o, al) in enumerate(zip(mo, ma)):
        d_o, d_a = o[2] - o[1], al[2] - al[1]
        beside = collections.Counter()
        for s in side:
            ov = min(o[2], s[2]) - max(o[1], s[1])
            if ov > 0:
                beside[s[0]] += ov
        rows.append((d_o - d_a, i, o[0], d_a, d_o, o[1], beside))
    bo = sum(k[2] - k[1] for k in mo)
    ba = sum(k[2] - k[1] for k in ma)  # the same launches without the side stream
    sb = sum(k[2] - k[1] for k in side)
    out = [f"# Side-stream contention: one training step, main queue with the side stream on vs off", "",
           f"* step span: {span_o:.0f} us overlapped, {span_a:.0f} us with the side stream off",
           f"* main-queue busy: {bo:.0f} us overlapped vs {ba:.0f} us alone (+{bo - ba:.0f} us, {len(mo)} kernels); "
           f"side queue busy {sb:.0f} us ({len(side)} kernels)", ""]
    fam = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for infl, i, name, d_a, d_o, st, _ in rows:
        f = fam[name]
        f[0] += 1
        f[1] += d_a
        f[2] += d_o
    out += ["## By main-queue kernel", "", "| kernel | launches | alone us | overlapped us | inflation us |",
            "|---|---|---|---|---|"]
    for name, (n, da, do) in sorted(fam.items(), key=lambda kv: -(kv[1][2] - kv[1][1]))[:25]:
        out.append(f"| `{name[:70]}` | {n} | {da:.0f} | {do:.0f} | {do - da:+.0f} |")
    out += ["", f"## The {a.top} most-inflated main-queue launches and the side-queue kernels beside them", "",
            "| # | at us | kernel | alone us | overlapped us | side kernels overlapping (us of overlap) |",
            "|---|---|---|---|---|---|"]
    for infl, i, name, d_a, d_o, st, beside in sorted(rows, key=lambda r: -r[0])[:a.top]:
        bs = ", ".join(f"{k[:40]} {v:.0f}" for k, v in beside.most_common(3))
        out.append(f"| {i} | {st:.0f} | `{name[:60]}` | {d_a:.1f} | {d_o:.1f} | {bs} |")
    text = "\n".join(out) + "\n"
    if a.md:
        with open(a.md, "w") as fh:
            fh.write(text)
    print(text)


if __name__ == "__main__":
    main()
