"""Per-kernel SQ / TCC counter table from rocprofv3 --pmc passes (VERDICT r5 item 2:
what binds the bf16 dense 3x3 kernels).

    python tools/sq_report.py <out.md> <pass_dir> [<pass_dir> ...]

Each pass dir holds one rocprofv3 `--pmc ... --kernel-trace` run (run_counter_collection.csv).
Counters are summed per kernel symbol over every dispatch of the run.  Units (MI355X_MICROARCH.md
"rocprofv3 PMC slots" / cycle constants): SQ_WAVE_CYCLES, SQ_WAIT_*, SQ_ACTIVE_INST_* count
quad-cycles summed over waves, and WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~= WAVE_CYCLES;
SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed over SIMDs; GRBM_GUI_ACTIVE is summed over the 8 XCDs.
"""
import csv
import os
import re
import sys
from collections import defaultdict

FAMILY = re.compile(r"igemm2_kernel|halo3x3_kernel|igemm_conv_kernel|wgrad_kernel|wgrad2_kernel|wino_")


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*$", "", n) if not n.startswith("_Z") else n
    return n[:110]


def load(dirs):
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for d in dirs:
        path = None
        for root, _, files in os.walk(d):
            for f in files:
                if f.endswith("counter_collection.csv"):
                    path = os.path.join(root, f)
        if path is None:
            print(f"sq_report: no counter_collection.csv under {d}", file=sys.stderr)
            continue
        for r in csv.DictReader(open(path)):
            k = short(r["Kernel_Name"])
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(k, d)].add(r["Dispatch_Id"])
    calls = defaultdict(int)
    for (k, d), s in disp.items():
        calls[k] = max(calls[k], len(s))
    return tot, calls


def ratio(a, b):
    return a / b if b else float("nan")


def main(out, *dirs):
    tot, calls = load(dirs)
    rows = []
    for k, c in tot.items():
        if not FAMILY.search(k):
            continue
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        gui = c.get("GRBM_GUI_ACTIVE", 0.0)
        rows.append((c.get("SQ_WAVE_CYCLES", 0.0), k, {
            "calls": calls[k],
            "wait_any": ratio(c.get("SQ_WAIT_ANY", 0), wc),
            "wait_inst_any": ratio(c.get("SQ_WAIT_INST_ANY", 0), wc),
            "active_inst_any": ratio(c.get("SQ_ACTIVE_INST_ANY", 0), wc),
            "wait_inst_lds": ratio(c.get("SQ_WAIT_INST_LDS", 0), wc),
            "active_lds": ratio(c.get("SQ_ACTIVE_INST_LDS", 0), wc),
            "active_vmem": ratio(c.get("SQ_ACTIVE_INST_VMEM", 0), wc),
            "active_valu": ratio(c.get("SQ_ACTIVE_INST_VALU", 0), wc),
            "lds_conflict": ratio(c.get("SQ_LDS_BANK_CONFLICT", 0), c.get("SQ_LDS_IDX_ACTIVE", 0)),
            "mfma_busy": ratio(c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0), gui / 8 * 1024) if gui else float("nan"),
            "l2_hit": ratio(c.get("TCC_HIT_sum", 0), c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0)),
            "waves": c.get("SQ_WAVES", 0.0),
        }))
    rows.sort(key=lambda r: -r[0])
    cols = ["calls", "wait_any", "wait_inst_any", "active_inst_any", "wait_inst_lds", "active_lds", "active_vmem",
            "active_valu", "lds_conflict", "mfma_busy", "l2_hit"]
    lines = [f"# SQ / TCC counters per kernel ({', '.join(dirs)})", "",
             "wait_any / wait_inst_any / active_inst_any / wait_inst_lds / active_* = share of SQ_WAVE_CYCLES; "
             "lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE; mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / "
             "(GRBM_GUI_ACTIVE / 8 x 1024 SIMDs); l2_hit = TCC_HIT / (HIT + MISS).", "",
             "| kernel | " + " | ".join(cols) + " |", "|---" * (len(cols) + 1) + "|"]
    for _, k, d in rows:
        cells = [str(d["calls"])] + [f"{d[c]:.3f}" for c in cols[1:]]
        lines.append(f"| `{k}` | " + " | ".join(cells) + " |")
    with open(out, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(*sys.argv[1:])
