"""dev: time k_dct_planes on the 8K planes and the 8K luma plane (bench.py's
extras) under knob settings.  usage:
  HICCUP_HIP_LIB=... python tools/dct_ab.py "label:knob=v,..." ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from hiccup_amd import _lib  # noqa: E402


def main():
    lib = os.path.basename(os.environ.get("HICCUP_HIP_LIB", "default"))
    for spec in sys.argv[1:] or ["default:"]:
        label, _, kv = spec.partition(":")
        kw = {k: int(v) for k, v in (p.split("=") for p in kv.split(",") if p)}
        with _lib.knobs(**kw):
            a = bench.extra_8k_plane_dct()
            b = bench.extra_8k_plane_dct(luma_only=True)
            c = bench.extra_4k_luma()
            d = bench.extra_8k_luma_batched()
        print("%-28s %-24s planes %7.2f us (%.3f)  luma %7.2f us (%.3f)  4k %7.2f us (%.3f)  luma x8 %7.2f us/plane "
              "(%.3f)" % (lib, label, a["median_launch_us"], a["frac"], b["median_launch_us"], b["frac"],
                          c["avg_launch_us"], c["frac"], d["us_per_plane"], d["frac"]), flush=True)


if __name__ == "__main__":
    main()
