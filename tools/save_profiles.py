"""dev: copy a tools/prof_round.sh run into profiles/ (tracked): kernel stats of the
bench command, the bench JSON line, PMC rows of our kernels, the DCT traffic json.
usage: python tools/save_profiles.py gpurun_out/prof_<tag> profiles/<round> <suffix>"""
import csv
import json
import os
import subprocess
import sys

src, dst, suf = sys.argv[1], sys.argv[2], sys.argv[3]
os.makedirs(dst, exist_ok=True)
rows = list(csv.DictReader(open(os.path.join(src, "bench", "run_kernel_stats.csv"))))
with open(os.path.join(dst, "bench_kernel_stats_%s.csv" % suf), "w", newline="") as f:
    w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
    w.writeheader()
    for r in rows:
        w.writerow(r)
lines = [l for l in open(os.path.join(src, "bench.json.log")) if l.startswith("{")]
open(os.path.join(dst, "bench_%s.json.log" % suf), "w").write(lines[-1])
plain = os.path.join(src, "bench_plain.json.log")
if os.path.exists(plain):
    pl = [l for l in open(plain) if l.startswith("{")]
    open(os.path.join(dst, "bench_full_%s.json.log" % suf), "w").write(pl[-1])
for sub in ("pmc_FETCH_SIZE", "pmc_WRITE_SIZE", "cal_FETCH_SIZE", "cal_WRITE_SIZE"):
    p = os.path.join(src, sub, "run_counter_collection.csv")
    keep = [r for r in csv.DictReader(open(p)) if "hic::" in r["Kernel_Name"] or "k_pattern" in r["Kernel_Name"]]
    with open(os.path.join(dst, "%s_%s.csv" % (sub, suf)), "w", newline="") as f:
        fields = ["Dispatch_Id", "Grid_Size", "Kernel_Name", "VGPR_Count", "Counter_Name", "Counter_Value",
                  "Start_Timestamp", "End_Timestamp"]
        w = csv.DictWriter(f, fieldnames=fields)
        w.writeheader()
        for r in keep:
            w.writerow({k: r[k] for k in fields})
out = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "pmc_summary.py"), src,
                      os.path.join("profiles", "pmc_dct.json")], capture_output=True, text=True)
print(out.stdout[-400:], out.stderr[-400:])
print(json.loads(lines[-1])["roofline"])
