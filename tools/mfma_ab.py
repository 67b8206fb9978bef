"""A/B of the forward plane paths on one GPU (dev tool, not product): the
integer-MFMA kernel (dct_path 5) against the float64 AAN kernel (1) on the
bench's plane measurements, alternating paths so box drift hits both."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import bench  # noqa: E402
from hiccup_amd import _lib  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    nplanes = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    out = []
    for r in range(reps):
        for path in (_lib.DCT_PATH_MFMA, _lib.DCT_PATH_F64):
            with _lib.knobs(dct_path=path):
                row = {"rep": r, "path": path,
                       "8k_luma_us": bench.extra_8k_plane_dct(luma_only=True)["median_launch_us"],
                       "8k_planes_us": bench.extra_8k_plane_dct()["median_launch_us"],
                       "4k_luma_us": bench.extra_4k_luma()["avg_launch_us"]}
                b = bench.extra_8k_luma_batched(nplanes)
                row["8k_luma_batched_us_per_plane"] = b["us_per_plane"]
                row["batched_frac"] = b["frac"]
            print(json.dumps(row), flush=True)
            out.append(row)


if __name__ == "__main__":
    main()
