"""dev: time the forward plane kernels (bench.py's extras) under knob settings,
alternating the specs `rounds` times.  usage:
  python tools/dct_ab.py [-r ROUNDS] "label:knob=v,..." ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from hiccup_amd import _lib  # noqa: E402


def one(label, kw):
    with _lib.knobs(**kw):
        a = bench.extra_8k_plane_dct()
        b = bench.extra_8k_plane_dct(luma_only=True)
        c = bench.extra_4k_luma()
        d = bench.extra_8k_luma_batched()
    print("%-24s planes %6.2f us (%.3f)  luma %6.2f (%.3f)  4k %6.2f (%.3f)  luma x16 free %6.2f us/plane (%.3f) "
          "rec %6.2f (%.3f)  single free %6.2f (%.3f)"
          % (label, a["median_launch_us"], a["frac"], b["median_launch_us"], b["frac"], c["median_launch_us"],
             c["frac"], d["us_per_plane"], d["frac"], d["with_rle_records"]["us_per_plane"],
             d["with_rle_records"]["frac"], d["single_launch"]["median_launch_us"], d["single_launch"]["frac"]),
          flush=True)


def main():
    args = sys.argv[1:]
    rounds = 1
    if args[:1] == ["-r"]:
        rounds, args = int(args[1]), args[2:]
    specs = []
    for spec in args or ["default:"]:
        label, _, kv = spec.partition(":")
        specs.append((label, {k: int(v) for k, v in (p.split("=") for p in kv.split(",") if p)}))
    for _ in range(rounds):
        for label, kw in specs:
            one(label, kw)


if __name__ == "__main__":
    main()
