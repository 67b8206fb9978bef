"""Where the MFMA plane kernel's time goes (dev tool; run with
HICCUP_HIP_LIB=hiccup_amd/lib/libhiccup_hip_dev.so): 8K luma with parts of the
kernel switched off by the dev knob (results invalid), against the full kernel
and the float64 AAN kernel."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import bench  # noqa: E402
from hiccup_amd import _lib  # noqa: E402

BITS = {0: "full", 1: "no transform", 2: "no stores/records", 4: "no (4,4) tie path", 8: "no pixel loads",
        16: "no records", 1 | 4: "no transform, no tie", 2 | 8: "no memory", 1 | 2 | 4 | 8: "nothing"}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    var = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    for r in range(reps):
        with _lib.knobs(dct_path=1):
            print(json.dumps({"rep": r, "arm": "aan", "8k_luma_us": bench.extra_8k_plane_dct(luma_only=True)[
                "median_launch_us"]}), flush=True)
        for bits, name in BITS.items():
            with _lib.knobs(dct_path=5, dct_mfma=var, dev=bits):
                print(json.dumps({"rep": r, "arm": name, "dev": bits, "8k_luma_us": bench.extra_8k_plane_dct(
                    luma_only=True)["median_launch_us"]}), flush=True)


if __name__ == "__main__":
    main()
