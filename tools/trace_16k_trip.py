"""dev: per-kernel time of one 16K round trip from a kernel trace of the default bench
command (the 16k_roundtrip extra's timed indexed trips: from its 2nd to its 6th
encode launch).  usage: python3 tools/trace_16k_trip.py run_kernel_trace.csv"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
enc = [i for i, r in enumerate(rows) if "k_encode420" in r["Kernel_Name"] and int(r["Grid_Size_X"]) == 2097152]
start, end = enc[1], enc[5]
agg = collections.OrderedDict()
for r in rows[start:end]:
    m = re.search(r"(k_\w+)(<[^>(]*>)?", r["Kernel_Name"])
    n = (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"][:40]
    n += " grid=%s" % r["Grid_Size_X"]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    agg.setdefault(n, [0.0, 0])
    agg[n][0] += d
    agg[n][1] += 1
wall = (int(rows[end - 1]["End_Timestamp"]) - int(rows[start]["Start_Timestamp"])) / 1e3
print("16K round trip, 4 trips: wall %.1f us per trip, kernels %.1f us per trip" % (wall / 4, sum(v[0] for v in agg.values()) / 4))
for k, v in agg.items():
    print("  %-64s %7.1f us per trip (%d launches)" % (k, v[0] / 4, v[1]))
