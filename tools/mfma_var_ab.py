"""A/B of the MFMA plane kernel's variants (knob dct_mfma: bit 0 prefetch, bit 1
2 waves per SIMD) against the float64 AAN path, alternating (dev tool)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import bench  # noqa: E402
from hiccup_amd import _lib  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    arms = [(1, 0)] + [(5, int(v)) for v in os.environ.get("ARMS", "0,1,2,3,4,5,6,7,8,9").split(",")]
    for r in range(reps):
        for path, var in arms:
            with _lib.knobs(dct_path=path, dct_mfma=var):
                row = {"rep": r, "path": path, "var": var,
                       "8k_luma_us": bench.extra_8k_plane_dct(luma_only=True)["median_launch_us"],
                       "4k_luma_us": bench.extra_4k_luma()["avg_launch_us"],
                       "8k_luma_x8_us_per_plane": bench.extra_8k_luma_batched(8)["us_per_plane"]}
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
