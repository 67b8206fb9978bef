"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (dev tool).

usage: python tools/pmc_summary.py gpurun_out/prof_<tag> [profiles/pmc_dct.json]

Reads <dir>/pmc_{FETCH,WRITE}_SIZE (the 8K 3-plane DCT driver, tools/prof_dct.py)
and <dir>/cal_{FETCH,WRITE}_SIZE (tools/micro/cal_traffic.hip: the DCT's access
pattern with known bytes).  It then writes the per-launch HBM traffic of the
DCT kernel (Y + Cr + Cb in one launch).  Units: FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950,
FETCH_SIZE reports half the bytes of wide streaming reads
(MI355X_MICROARCH.md, HBM section).  Our read pattern is 8 B per lane, so the
read factor is calibrated on cal_traffic rather than assumed.
"""
import csv
import json
import os
import re
import sys

H, W = 4320, 7680


def per_kernel(path, counter):
    """{kernel short name: [values per dispatch]} (value in bytes)."""
    f = os.path.join(path, "run_counter_collection.csv")
    out = {}
    with open(f) as fh:
        for row in csv.DictReader(fh):
            if row["Counter_Name"] != counter:
                continue
            name = row["Kernel_Name"]
            m = re.search(r"(k_\w+)(<[^>]*>)?", name)
            key = (m.group(1) + (m.group(2) or "")) if m else name[:40]
            key += " grid=%s" % row["Grid_Size"]
            out.setdefault(key, []).append(float(row["Counter_Value"]) * 1024.0)
    return out


def mean(v):
    return sum(v) / len(v)


def main():
    d = sys.argv[1]
    dst = sys.argv[2] if len(sys.argv) > 2 else None
    cpx = H * W  # calibration kernel: one 8K plane
    px = H * W + 2 * (H // 2) * (W // 2)  # the DCT launch: Y + Cr + Cb
    res = {"source": d, "planes": [[H, W], [H // 2, W // 2], [H // 2, W // 2]], "algorithmic_read_bytes": px,
           "algorithmic_write_bytes": 2 * px}
    cal_f = per_kernel(os.path.join(d, "cal_FETCH_SIZE"), "FETCH_SIZE")
    cal_w = per_kernel(os.path.join(d, "cal_WRITE_SIZE"), "WRITE_SIZE")
    kf = [k for k in cal_f if k.startswith("k_pattern")][0]
    kw = [k for k in cal_w if k.startswith("k_pattern")][0]
    rf = mean(cal_f[kf][4:]) / cpx          # counter bytes per known read byte
    rw = mean(cal_w[kw][4:]) / (2 * cpx)    # counter bytes per known written byte
    res["calibration"] = {"kernel": "tools/micro/cal_traffic.hip k_pattern", "fetch_counter_per_byte": round(rf, 4),
                          "write_counter_per_byte": round(rw, 4)}
    f = per_kernel(os.path.join(d, "pmc_FETCH_SIZE"), "FETCH_SIZE")
    w = per_kernel(os.path.join(d, "pmc_WRITE_SIZE"), "WRITE_SIZE")
    res["kernels"] = {}
    for k in sorted(f):
        if not k.startswith("k_"):
            continue
        fb = mean(f[k][2:] if len(f[k]) > 2 else f[k])
        wb = mean(w[k][2:] if len(w.get(k, [])) > 2 else w.get(k, [0.0]))
        res["kernels"][k] = {"fetch_counter_bytes": round(fb), "write_counter_bytes": round(wb),
                             "read_bytes_calibrated": round(fb / rf), "write_bytes_calibrated": round(wb / rw)}
    dk = [k for k in res["kernels"] if k.startswith("k_dct_planes<-1, 2, 15")]
    if dk:
        r = res["kernels"][dk[0]]
        res["dct_kernel"] = dk[0]
        res["hbm_bytes_per_launch"] = r["read_bytes_calibrated"] + r["write_bytes_calibrated"]
    txt = json.dumps(res, indent=1)
    print(txt)
    if dst:
        with open(dst, "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main()
