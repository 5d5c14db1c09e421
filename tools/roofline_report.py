"""Summarise a rocprofv3 kernel-trace/stats run and its PMC passes for the
dominant kernel family, and write it under profiles/.

    python tools/roofline_report.py <prof_dir> <pmc_dir> <steps_profiled> <out_prefix> [MobileNetV2UNet|UNet]

prof_dir: `rocprofv3 --kernel-trace --stats` output of bench.py (run_kernel_stats.csv)
pmc_dir:  FETCH_SIZE/ and WRITE_SIZE/ passes (run_counter_collection.csv), each
          its own rocprofv3 run with --pmc + --kernel-trace only.
HBM bytes per dispatch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: on gfx950
FETCH_SIZE reports exactly half of the bytes of wide (16 B/lane) coalesced reads
(MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact for 16-B stores.  The
256 MiB Infinity Cache can absorb re-reads, so these are evidence, not the metric.
"""
import csv
import json
import re
import statistics
import sys
from collections import defaultdict

FAMILIES = {  # "conv3" = the dense 3x3 conv forward + data gradient (bench.py's roofline kernel family)
    # (rocprofv3 leaves the __bf16 / _Float16 instantiations mangled: ILi..E forms)
    # igemm2_kernel<BM, BN, WM, WN, KS, XF> (csrc/igemm2.hip:91; six template parameters since 53539df --
    # round 4's three-parameter pattern matched none of them)
    "conv3": re.compile(r"igemm_conv_kernel<\d+, \d+, \d+, \d+, 3, \d+|igemm_conv_kernelILi\d+ELi\d+ELi\d+ELi\d+ELi3E"
                        r"|wino_gemm_kernel|wino_out_kernel|wino_fused_kernel|halo3x3_kernel"
                        r"|igemm2_kernel<\d+, \d+, \d+, \d+, 3[,>]|igemm2_kernelILi\d+ELi\d+ELi\d+ELi\d+ELi3E"),
    "igemm1": re.compile(r"igemm_conv_kernel<\d+, \d+, \d+, \d+, 1, \d+|igemm_conv_kernelILi\d+ELi\d+ELi\d+ELi\d+ELi1E"
                         r"|igemm2_kernel<\d+, \d+, \d+, \d+, 1[,>]|igemm2_kernelILi\d+ELi\d+ELi\d+ELi\d+ELi1E"),
    # BatchNorm backward (csrc/bn.hip): the dA/y reduction, its finalizes and the dY apply pass
    "bn_bwd": re.compile(r"chan_partial_kernel<1,|chan_partial_kernelILi1E|bn_bwd_finalize_kernel"
                         r"|bn_bwd_finalize_tiles_kernel|bn_bwd_apply_rt_kernel|bn_bwd_apply_kernel"),
    "wgrad3": re.compile(r"wgrad_kernel<\d+, \d+, \d+, \d+, 3[,>]|wgrad_kernelILi\d+ELi\d+ELi\d+ELi\d+ELi3E"
                         r"|wino_wgrad"),
    "wgrad1": re.compile(r"wgrad_kernel<\d+, \d+, \d+, \d+, 1[,>]|wgrad_kernelILi\d+ELi\d+ELi\d+ELi\d+ELi1E"),
}
# conv ops per step of the profiled model: MobileNetV2UNet 17 (8 decoder convs fwd + 8 dgrad + the stem fwd),
# UNet 27 (14 convs fwd + 13 dgrad); a two-launch Winograd op is two kernels (wino_gemm + wino_out), every other op
# (the fused Winograd kernel included) one
OPS_PER_STEP = {"MobileNetV2UNet": 17, "UNet": 27}


def family(name):
    for k, rx in FAMILIES.items():
        if rx.search(name):
            return k
    return None


def main(prof_dir, pmc_dir, steps, out_prefix, model="MobileNetV2UNet"):
    steps = int(steps)
    ops = OPS_PER_STEP[model]
    stats = list(csv.DictReader(open(f"{prof_dir}/run_kernel_stats.csv")))
    total = sum(float(r["TotalDurationNs"]) for r in stats)
    fam = defaultdict(lambda: {"calls": 0, "ns": 0.0, "symbols": []})
    for r in stats:
        f = family(r["Name"])
        if f:
            fam[f]["calls"] += int(r["Calls"])
            fam[f]["ns"] += float(r["TotalDurationNs"])
            fam[f]["symbols"].append((r["Name"].replace("(anonymous namespace)::", ""), int(r["Calls"]),
                                      float(r["AverageNs"]) / 1e3))
    traffic = defaultdict(list)
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = list(csv.DictReader(open(f"{pmc_dir}/{c}/run_counter_collection.csv")))
        per = defaultdict(float)
        names = {}
        for r in rows:
            per[r["Dispatch_Id"]] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for d, v in per.items():
            f = family(names[d])
            if f:
                traffic[(f, c)].append(v)
    # MFMA activity (optional pass): per family, MFMA-busy cycles summed over the SIMDs and
    # GRBM_GUI_ACTIVE summed over the 8 XCDs.  busy_frac = MFMA_BUSY / (GUI_ACTIVE / 8 * 1024 SIMDs):
    # the share of SIMD-cycles inside the family's dispatches in which a matrix instruction was busy.
    mfma = defaultdict(lambda: [0.0, 0.0])
    import os
    mpath = f"{pmc_dir}/MFMA/run_counter_collection.csv"
    if os.path.exists(mpath):
        for r in csv.DictReader(open(mpath)):
            f = family(r["Kernel_Name"])
            if f:
                k = 0 if r["Counter_Name"].startswith("SQ_VALU_MFMA_BUSY") else 1
                mfma[f][k] += float(r["Counter_Value"])
    import subprocess
    try:
        commit = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], capture_output=True, text=True,
                                cwd=os.path.dirname(os.path.abspath(__file__))).stdout.strip() or None
    except OSError:
        commit = None
    # stamp: the profile these counters came from and the commit of the tree that ran
    # (bench.py reports both beside `traffic`, which it does not measure itself)
    commit = os.environ.get("SEG_COMMIT", commit)
    out = {"profile": os.path.basename(out_prefix), "commit": commit, "profiled_steps": steps,
           "kernel_ms_per_step": total / 1e6 / steps, "families": {}}
    lines = [f"# rocprofv3 summary ({out_prefix})", "",
             f"Kernel time per step (all kernels): {total / 1e6 / steps:.2f} ms over {steps} profiled steps.", "",
             "| family | calls/step | ms/step | share | avg launch us | HBM bytes/launch (2*FETCH+WRITE)*1KiB "
             "| MFMA-busy share of SIMD-cycles |",
             "|---|---|---|---|---|---|---|"]
    for f, d in sorted(fam.items(), key=lambda kv: -kv[1]["ns"]):
        fetch = traffic.get((f, "FETCH_SIZE"), [])
        write = traffic.get((f, "WRITE_SIZE"), [])
        hbm = (2 * statistics.mean(fetch) + statistics.mean(write)) * 1024 if fetch and write else None
        avg_us = d["ns"] / d["calls"] / 1e3
        out["families"][f] = {"calls_per_step": d["calls"] / steps, "ms_per_step": d["ns"] / 1e6 / steps,
                              "avg_launch_us": avg_us, "hbm_bytes_per_launch": hbm,
                              "symbols": d["symbols"]}
        if mfma[f][1] > 0:
            out["families"][f]["mfma_busy_cycles"] = mfma[f][0]
            out["families"][f]["grbm_gui_active"] = mfma[f][1]
            out["families"][f]["mfma_busy_frac"] = mfma[f][0] / (mfma[f][1] / 8 * 1024)
        if f == "conv3" and fetch and write:
            # per conv op (a Winograd op is two kernels): family bytes per step / ops per step
            per_step = (2 * sum(fetch) + sum(write)) * 1024 / (len(fetch) / (d["calls"] / steps))
            out["families"][f]["ops_per_step"] = ops
            out["families"][f]["hbm_bytes_per_op"] = per_step / ops
        if f == "bn_bwd" and fetch and write:
            out["families"][f]["hbm_bytes_per_step"] = (2 * sum(fetch) + sum(write)) * 1024 / (
                len(fetch) / (d["calls"] / steps))
        lines.append(f"| {f} | {d['calls'] / steps:.0f} | {d['ns'] / 1e6 / steps:.2f} | {d['ns'] / total:.1%} | "
                     f"{avg_us:.1f} | {hbm / 1e6 if hbm else float('nan'):.1f} MB | "
                     f"{out['families'][f].get('mfma_busy_frac', float('nan')):.3f} |")
    # self-check: every conv3 op of the step must be in the family -- one kernel per op plus
    # the second kernel (wino_out_kernel) of each Winograd op
    wino_out = sum(int(r["Calls"]) for r in stats if "wino_out_kernel" in r["Name"]) / steps
    want = ops + wino_out
    got = fam["conv3"]["calls"] / steps if "conv3" in fam else 0
    if abs(got - want) > 1e-6:
        raise SystemExit(f"roofline_report: conv3 family has {got:g} launches per step, the {model} step has {want:g} "
                         f"({ops} ops + {wino_out:g} Winograd output transforms): a kernel name escaped the pattern")
    out["families"]["conv3"]["expected_calls_per_step"] = want
    lines += ["", f"conv3 self-check: {got:g} launches per step = {ops} ops + {wino_out:g} Winograd output transforms.",
              "", "Top kernels:", "", "| kernel | calls | avg us | total ms |", "|---|---|---|---|"]
    for r in sorted(stats, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
        lines.append(f"| `{r['Name'].replace('(anonymous namespace)::', '')[:90]}` | {r['Calls']} | "
                     f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['TotalDurationNs']) / 1e6:.2f} |")
    with open(out_prefix + ".md", "w") as fh:
        fh.write("\n".join(lines) + "\n")
    with open(out_prefix + ".json", "w") as fh:
        json.dump(out, fh, indent=1)
    print("\n".join(lines[:12]))


if __name__ == "__main__":
    main(*sys.argv[1:])
