"""A/B of the forward plane DCT paths on the bench's own workloads (dev tool):
8K luma pass, 8K Y+Cr+Cb planes, 4K luma (BASELINE configs[1]), each under the
packed-float32 path (dct_path 4, default) and the float64 AAN path (1)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from hiccup_amd import _lib  # noqa: E402


def main():
    paths = [int(a) for a in sys.argv[1:]] or [4, 1]
    extra = {}
    for a in os.environ.get("AB_KNOBS", "").split(","):
        if "=" in a:
            k, v = a.split("=")
            extra[k] = int(v)
    for rep in range(2):
        for p in paths:
            with _lib.knobs(dct_path=p, **extra):
                r = {"path": p, "rep": rep,
                     "luma_us": bench.extra_8k_plane_dct(luma_only=True)["median_launch_us"],
                     "planes_us": bench.extra_8k_plane_dct()["median_launch_us"],
                     "luma4k_us": bench.extra_4k_luma()["avg_launch_us"]}
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
