"""Split a rocprofv3 kernel trace of `bench.py` into its phases and average one
kernel's dispatch durations per phase, so the trace can be compared with the
bench line's HIP-event numbers (dev tool).

bench.py at N=1 launches the roofline kernel W (warmup) + K (timed) times, then
24 more single-stream encodes for the isolated roofline measurement (8 untimed,
16 with every 4th timestamped), then the extras.  usage:

  python tools/trace_phases.py run_kernel_trace.csv KERNEL_SUBSTRING W K [out.json]
"""
import csv
import json
import sys


def main():
    path, key, W, K = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    rows = [r for r in csv.DictReader(open(path)) if key in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    phases = {"warmup": us[:W], "timed": us[W:W + K], "isolated_all24": us[W + K:W + K + 24],
              "isolated_timestamped": us[W + K + 8:W + K + 24][::4], "after": us[W + K + 24:]}
    out = {"trace": path, "kernel_substring": key, "dispatches": len(us), "warmup": W, "steps": K,
           "kernel_name": rows[0]["Kernel_Name"] if rows else None}
    for name, v in phases.items():
        out[name] = {"n": len(v), "avg_us": round(sum(v) / len(v), 3) if v else None,
                     "min_us": round(min(v), 3) if v else None, "max_us": round(max(v), 3) if v else None}
    out["all"] = {"n": len(us), "avg_us": round(sum(us) / len(us), 3) if us else None}
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 5:
        open(sys.argv[5], "w").write(s + "\n")


if __name__ == "__main__":
    main()
