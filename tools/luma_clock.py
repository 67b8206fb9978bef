"""dev: the shader clock per dispatch of north_star's pass, from a rocprofv3 run that
collected GRBM_GUI_ACTIVE / SQ_BUSY_CYCLES beside its kernel trace (tools/profile.sh
luma): per k_dct_planes dispatch its duration, GRBM_GUI_ACTIVE / duration (the GPU's
clock while busy) and SQ_BUSY_CYCLES / duration, and the duration per plane
normalised to the median clock.
usage: python3 tools/luma_clock.py <rocprofv3 -d dir> [planes_per_launch=16]"""
import csv
import statistics
import sys


def main():
    d = sys.argv[1]
    planes = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    trace = {int(r["Dispatch_Id"]): r for r in csv.DictReader(open(d + "/run_kernel_trace.csv"))}
    ctr = {}
    for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
        if "k_dct_planes" not in r["Kernel_Name"]:
            continue
        ctr.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    rows = []
    for did in sorted(ctr):
        t = trace.get(did)
        if t is None:
            continue
        ns = int(t["End_Timestamp"]) - int(t["Start_Timestamp"])
        c = ctr[did]
        rows.append((did, ns, c.get("GRBM_GUI_ACTIVE", 0) / 8 / ns * 1e3, c.get("SQ_BUSY_CYCLES", 0) / ns * 1e3))
    med = statistics.median(r[2] for r in rows)
    print("dispatch  us  us/plane  clock MHz (GRBM_GUI_ACTIVE/8/us)  SQ_BUSY_CYCLES/us  us/plane at the median clock")
    for did, ns, f, sq in rows:
        print("%6d %8.2f %7.3f %10.1f %12.1f %9.3f" % (did, ns / 1e3, ns / 1e3 / planes, f, sq,
                                                      ns / 1e3 / planes * f / med))
    print("median clock (GRBM_GUI_ACTIVE / 8 per us): %.1f MHz over %d dispatches" % (med, len(rows)))


if __name__ == "__main__":
    main()
