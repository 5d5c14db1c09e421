"""One inference frame's kernel sequence from a rocprofv3 --kernel-trace of
`bench.py --workload infer` (the launches after one frame's argmax through the next frame's).

    python tools/trace_frame.py gpurun_out/<dir>/run_kernel_trace.csv > profiles/<name>.md
"""
import csv
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    # a frame = the launches after one argmax (its last kernel) up to and including the next
    idx = [i for i, r in enumerate(rows) if "argmax" in r["Kernel_Name"]]
    a, b = idx[-3] + 1, idx[-2] + 1
    t0 = int(rows[a]["Start_Timestamp"])
    tot = 0
    print("| start us | dur us | grid (work-items) | kernel |\n|---|---|---|---|")
    for r in rows[a:b]:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        tot += d
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        print(f"| {(int(r['Start_Timestamp']) - t0) / 1e3:.1f} | {d / 1e3:.1f} | {r['Grid_Size_X']}x{r['Grid_Size_Y']} "
              f"| `{name}` |")
    print(f"\n{b - a} kernels, sum of kernel durations {tot / 1e3:.1f} us, span under the profiler "
          f"{(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
