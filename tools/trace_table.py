"""dev: per-kernel, per-grid mean durations from a rocprofv3 kernel trace."""
import collections, csv, re, sys
agg = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(k_\w+)(<[^>]*>)?", r["Kernel_Name"])
    if not m:
        continue
    agg[(m.group(1) + (m.group(2) or ""), r["Grid_Size_X"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = 0.0
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print("%-60s grid=%-8s n=%-4d mean=%8.2f us" % (k[0][:60], k[1], len(v), sum(v) / len(v)))
