"""dev: per-kernel mean of every counter collected by tools/prof_counters.sh."""
import csv, re, sys, os, collections
d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for sub in sorted(os.listdir(d)):
    f = os.path.join(d, sub, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)(<[^>]*>)?", r["Kernel_Name"])
        if not m or "hic::" not in r["Kernel_Name"]:
            continue
        key = m.group(1) + (m.group(2) or "") + " g=" + r["Grid_Size"] + " v=" + r["VGPR_Count"]
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    print(k)
    for c, v in sorted(cs.items()):
        print("   %-22s %16.1f" % (c, sum(v) / len(v)))
