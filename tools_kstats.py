import csv, sys
d = sys.argv[1]; steps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print("kernel ms per step %.2f" % (tot / 1e6 / steps))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    n = r['Name'].replace('(anonymous namespace)::', '')[:80]
    print("%7.2f ms/step %5.1f%% calls/step %5.0f avg %8.1f us  %s" % (float(r['TotalDurationNs']) / 1e6 / steps,
          float(r['Percentage']), int(r['Calls']) / steps, float(r['AverageNs']) / 1e3, n))
