"""Per-step kernel time by family from a rocprofv3 --stats run of bench.py.

    python tools/kstats.py gpurun_out/<dir>/run_kernel_stats.csv [steps]
"""
import collections
import csv
import re
import sys


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    cat, cnt = collections.Counter(), collections.Counter()
    for r in csv.DictReader(open(path)):
        n = r["Name"]
        m = re.search(r"(\w+_kernel|\w+copyBuffer|\w+)(<[^(]*>)?\(", n)
        k = m.group(1) if m else n[:40]
        if k in ("igemm_conv_kernel", "wgrad_kernel"):
            k += re.search(r"<([^>]*)>", n).group(1).split(",")[4].strip()
        cat[k] += int(r["TotalDurationNs"]) / steps / 1e6
        cnt[k] += int(r["Calls"]) / steps
    print("total kernel ms/step %.2f launches/step %.0f" % (sum(cat.values()), sum(cnt.values())))
    for k, v in cat.most_common():
        print("%-32s %6.3f ms %5.0f launches" % (k, v, cnt[k]))


if __name__ == "__main__":
    main()
