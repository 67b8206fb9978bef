"""dev: summarise a tools/prof_r2.sh run into one JSON (per encode kernel: calls,
average duration from the kernel trace, HBM bytes from FETCH_SIZE / WRITE_SIZE
corrected by the calibration kernel of the same access pattern, SQ wave-cycle
breakdown).  usage: python tools/prof_r2_summary.py gpurun_out/prof_<tag> out.json"""
import collections
import csv
import json
import os
import re
import sys

# encode kernel -> calibration kernel with its load pattern (tools/micro/cal_patterns.hip)
PATTERN = {"k_encode420": "k_cal_rgb24", "k_dct_planes": "k_cal_blk8", "k_rgb_ycrcb420_walk": "k_cal_q12",
           "k_rle_emit16b": "k_cal_d16", "k_rle_scan16b": "k_cal_d16"}
CAL_BYTES = {}  # filled from cal_patterns.log: name -> (read, write)


def short(name):
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name[:40]


def pattern_of(k):
    for p, cal in PATTERN.items():
        if k.startswith(p):
            return cal
    return "k_cal_d16"


def per_kernel(path, counter):
    out = collections.defaultdict(list)
    with open(os.path.join(path, "run_counter_collection.csv")) as fh:
        for row in csv.DictReader(fh):
            if row["Counter_Name"] == counter:
                out[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return out


def mean(v):
    v = v[2:] if len(v) > 4 else v  # drop the first (warm-up) dispatches
    return sum(v) / len(v)


def main():
    d, dst = sys.argv[1], sys.argv[2]
    for line in open(os.path.join(d, "cal_patterns.log")):
        m = re.match(r"(k_cal_\w+): ([\d.]+) us/launch, read (\d+) B, write (\d+) B", line)
        if m:
            CAL_BYTES[m.group(1)] = (int(m.group(3)), int(m.group(4)), float(m.group(2)))
    cal_f = per_kernel(os.path.join(d, "cal_FETCH_SIZE"), "FETCH_SIZE")
    cal_w = per_kernel(os.path.join(d, "cal_WRITE_SIZE"), "WRITE_SIZE")
    factors = {}
    for k, (rb, wb, us) in CAL_BYTES.items():
        factors[k] = {"fetch_counter_per_byte": mean(cal_f[k]) * 1024 / rb,
                      "write_counter_per_byte": mean(cal_w[k]) * 1024 / wb, "us": us,
                      "achieved_gbs": (rb + wb) / us / 1e3}
    stats = {}
    with open(os.path.join(d, "trace", "run_kernel_stats.csv")) as fh:
        for row in csv.DictReader(fh):
            stats[short(row["Name"])] = {"calls": int(row["Calls"]), "avg_us": float(row["AverageNs"]) / 1e3}
    f = per_kernel(os.path.join(d, "pmc_FETCH_SIZE"), "FETCH_SIZE")
    w = per_kernel(os.path.join(d, "pmc_WRITE_SIZE"), "WRITE_SIZE")
    sq = {c: per_kernel(os.path.join(d, "pmc_sq"), c) for c in
          ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU",
           "SQ_INSTS_SALU", "SQ_INSTS_LDS")}
    res = {"source": d, "calibration": factors, "kernels": {}}
    for k in sorted(stats):
        if not k.startswith("k_"):
            continue
        e = dict(stats[k])
        if k in f:
            cal = factors.get(pattern_of(k))
            fb, wb = mean(f[k]) * 1024, mean(w[k]) * 1024
            e.update({"fetch_counter_bytes": round(fb), "write_counter_bytes": round(wb),
                      "calibrated_with": pattern_of(k)})
            if cal:
                e["read_bytes"] = round(fb / cal["fetch_counter_per_byte"])
                e["write_bytes"] = round(wb / cal["write_counter_per_byte"])
                e["hbm_bytes"] = e["read_bytes"] + e["write_bytes"]
                e["hbm_gbs"] = round(e["hbm_bytes"] / e["avg_us"] / 1e3, 1)
        if k in sq["SQ_WAVE_CYCLES"]:
            wc = mean(sq["SQ_WAVE_CYCLES"][k])
            e["sq"] = {"wait_any": round(mean(sq["SQ_WAIT_ANY"][k]) / wc, 3),
                       "wait_inst_any": round(mean(sq["SQ_WAIT_INST_ANY"][k]) / wc, 3),
                       "active_valu": round(mean(sq["SQ_ACTIVE_INST_VALU"][k]) / wc, 3),
                       "insts_valu": round(mean(sq["SQ_INSTS_VALU"][k])),
                       "insts_salu": round(mean(sq["SQ_INSTS_SALU"][k])),
                       "insts_lds": round(mean(sq["SQ_INSTS_LDS"][k]))}
        res["kernels"][k] = e
    txt = json.dumps(res, indent=1)
    print(txt)
    with open(dst, "w") as fh:
        fh.write(txt + "\n")


if __name__ == "__main__":
    main()
