"""Instruction census of one kernel in a hipcc -S listing, split at sched_barrier
markers (dev tool).  usage: asm_census.py file.s name_substring"""
import collections
import re
import sys

src = open(sys.argv[1]).read()
key = sys.argv[2]
labels = [m for m in re.finditer(r"^(\S+):\s*;\s*@", src, re.M) if key in m.group(1)]
lab = labels[0]
body = src[lab.end():src.index(".Lfunc_end", lab.end())]
regions, cur = [], collections.Counter()
for line in body.split("\n"):
    t = line.strip()
    if "sched_barrier" in t:
        regions.append(cur)
        cur = collections.Counter()
        continue
    if not t or t.startswith((".", ";")) or t.endswith(":"):
        continue
    op = t.split()[0]
    cls = ("valu64" if op.startswith("v_") and "f64" in op else
           "valu" if op.startswith("v_") else
           "salu" if op.startswith("s_") and not op.startswith(("s_waitcnt", "s_load", "s_buffer", "s_cbranch", "s_branch")) else
           "lds" if op.startswith("ds_") else "vmem" if op.startswith(("global_", "buffer_", "flat_")) else "other")
    cur[cls] += 1
    cur["op:" + op] += 1
regions.append(cur)
print(lab.group(1), "regions", len(regions))
tot = collections.Counter()
for i, r in enumerate(regions):
    tot.update(r)
    print("%3d valu %5d (f64 %4d) salu %4d lds %3d vmem %3d" % (i, r["valu"] + r["valu64"], r["valu64"], r["salu"], r["lds"], r["vmem"]))
print("total valu %d (f64 %d) salu %d lds %d vmem %d" % (tot["valu"] + tot["valu64"], tot["valu64"], tot["salu"], tot["lds"], tot["vmem"]))
if len(sys.argv) > 3:
    lo, hi = map(int, sys.argv[3].split(":"))
    c = collections.Counter()
    for r in regions[lo:hi]:
        c.update({k[3:]: v for k, v in r.items() if k.startswith("op:")})
    for k, v in c.most_common(40):
        print("%6d %s" % (v, k))
