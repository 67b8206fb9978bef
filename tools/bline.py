"""dev: summarise bench JSON lines from logs: python tools/bline.py log..."""
import json
import sys

for f in sys.argv[1:]:
    for line in open(f):
        if line.startswith('{"metric"'):
            d = json.loads(line)
            r = d["roofline"]
            print("%-28s value %10.1f  ms/step %.4f  roof %7.2f us  frac %.4f  overlapped %s" % (
                f.split("/")[-1], d["value"], d["ms_per_step"], r["avg_launch_us"], r["frac"],
                r.get("avg_launch_us_overlapped")))
