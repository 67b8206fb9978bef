"""Average rocprofv3 --pmc counter values per dispatch of kernels matching a name
substring (dev tool).  usage: pmc_kernel.py <run_counter_collection.csv> <substr>"""
import collections
import csv
import sys

acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print("%-22s %16.1f  (n=%d)" % (k, sum(v) / len(v), len(v)))
