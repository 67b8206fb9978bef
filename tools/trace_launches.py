"""dev: launches of the kernels whose name contains a substring, in dispatch order,
from a rocprofv3 --kernel-trace CSV: per (kernel, grid) group the count and every
duration, with the gap since the previous launch of any kernel.
usage: python3 tools/trace_launches.py run_kernel_trace.csv SUBSTR [SUBSTR ...]"""
import csv
import sys


def main():
    path, subs = sys.argv[1], sys.argv[2:] or ["k_dct"]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    prev_end = None
    groups = {}
    order = []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"]
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        prev_end = e if prev_end is None else max(prev_end, e)
        if not any(x in name for x in subs):
            continue
        grid = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
        key = (name[:70], grid)
        if key not in groups:
            groups[key] = []
            order.append(key)
        groups[key].append(((e - s) / 1e3, gap))
    for key in order:
        d = groups[key]
        us = sorted(x for x, _ in d)
        print("%s grid %s: %d launches, median %.2f us, min %.2f, max %.2f" % (key[0], key[1], len(d), us[len(us) // 2],
                                                                          us[0], us[-1]))
        print("   in order (us, gap before):", " ".join("%.1f/%.1f" % x for x in d))


if __name__ == "__main__":
    main()
