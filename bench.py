#!/usr/bin/env python3
"""bench.py -- hiccup encode throughput on MI355X (BASELINE.json metric).

N = 1 (default; BASELINE configs[2], the 8K encode the metric is quoted on): a
7680 x 4320 RGB uint8 image, already resident in HBM, through the full encode
front end = compression.jpeg_compression + the zig-zag / DC / RLE half of
codec.jpeg_encode:
  RGB -> YCrCb + 4:2:0 pyrDown, 8x8 DCT + quantize + zig-zag (3 planes,
  bit-exact vs float64), DC DPCM + AC RLE symbols of every 64-block (Y) / 32-block
  (Cr, Cb) record: ONE kernel (hic_encode420_slots_u8, the slot layout: no int16
  coefficients in HBM); the zero runs carried across records, each record's first
  symbol and the record index: ONE scan launch (hic_rle_slots_close).
One "step" encodes one such image; its stream is complete on the device (the
contiguous form is one more launch, hic_rle_slots_compact, for callers that want it).
--no-slots: the round-5 chain (the fused kernel writes coefficients + records, then
a scan and an emit kernel).

--gpus N > 1 (BASELINE configs[3]): one process per GPU over RCCL.  `python
bench.py --gpus N` starts the N ranks itself (torch.multiprocessing, before any
GPU call in the parent); under torch.distributed.run it joins the given ranks.
  --mode strong (default): ONE 8K image split N ways by block rows; each rank
                 transforms its shard (colour with halo, DCT + quantize + zig-zag +
                 RLE tile records) and ships its blocks in the lossless wire format
                 (hic_wire_pack_i16: per-slot widths proven per table, 637 / 597 bits
                 per block; 61.1 MB per 8K image with the records)
                 to the image's gathering rank, which unpacks them and runs the
                 scan + emit of the whole image: each timed image ends as ONE
                 encoded stream (codec.jpeg_encode's DC / RLE symbols) on one rank.
                 Image j of each group of N consecutive images lands on rank j, and
                 the group's N gathers go out as ONE grouped batch
                 (sharding.gather_streams_group) on a process group of their own:
                 every xGMI link carries data in both directions, where N gathers
                 into rank 0 would queue on its 7 ingress links.
                 --gather-kind blocks: round 2's exchange instead (each rank codes
                 its slice of the stream after a summary all-gather; the int16
                 blocks + DC are gathered, the symbol slices stay distributed).
  --mode weak:   an (N*H) x W image, one H-row shard per rank (no gather).
--workload 4k: 4096 x 4096 RGB instead of 7680 x 4320 (north_star's 4K point).
value = pixels encoded by all ranks / max-over-ranks wall time of the K steps.
"""
import argparse
import json
import pickle
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

H8K, W8K = 4320, 7680
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
XGMI_LINK_GBS = 153.0  # per xGMI link of an MI355X (7 per GPU), the figure given with this build
ROT_BYTES = 1.2e9          # rotate >= 1.2 GB of inputs: defeats the 256 MiB Infinity Cache
REGION_REPEATS = 7         # extra timed regions for the ms_per_step spread (p10 / p50 / p90)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mode", choices=("weak", "strong"), default="strong")
    ap.add_argument("--workload", choices=("8k", "4k"), default="8k")
    ap.add_argument("--gather-kind", choices=("stream", "blocks"), default="stream",
                    help="strong mode: 'stream' = wire-format blocks to the gathering rank, which codes the whole "
                         "stream (default); 'blocks' = per-shard stream slices + int16 block gather (round 2)")
    ap.add_argument("--no-gather", action="store_true",
                    help="strong mode: leave the coefficient blocks distributed (no RCCL gather)")
    ap.add_argument("--transport", choices=("torch", "c-abi"), default="torch",
                    help="strong mode's gather: torch.distributed P2P batch (default) or the C-ABI's own RCCL "
                         "communicator (hic_gather_*, sharding.RcclGather; nccl backend only)")
    ap.add_argument("--master-port", type=int, default=29541, help="self-launched N > 1 runs only")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                    help="nccl (= RCCL) for the real multi-GPU run; gloo only to rehearse it")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank on cuda:0 (use with --dist-backend gloo)")
    ap.add_argument("--streams", type=int, default=None,
                    help="HIP streams the consecutive images alternate over (each image's chain stays on one); "
                         "default 4 on one GPU (0.1020-0.1028 vs 0.1025-0.1037 ms/step for 2 in 3 alternating "
                         "pairs, profiles/r03/s2/streams/), 2 with N > 1 ranks")
    ap.add_argument("--unfused", action="store_true",
                    help="A/B: colour and DCT as two kernels (the planes round-trip HBM) instead of hic_encode420_u8")
    ap.add_argument("--no-slots", action="store_true",
                    help="A/B: the coefficient chain (fused kernel writes int16 coefficients, scan + emit kernels) "
                         "instead of the slot layout (the fused kernel writes the symbols, one closing scan)")
    ap.add_argument("--knob", action="append", default=[], metavar="NAME=VALUE",
                    help="A/B: set a library knob (hiccup_amd._lib.KNOBS; every knob is bit-exact)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget-s", type=float, default=25.0)
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the BASELINE configs[1] / configs[4] side measurements (at N > 1: configs[4], "
                         "the sharded 16K round trip)")
    return ap.parse_args()


def _cpu_encode_band(rgb):
    """hiccup's CPU encode path (restated in C: oracle/hiccup_oracle.c) on one band of
    rows: colour + 4:2:0 pyrDown, DCT + quantize, zig-zag, DC DPCM, AC RLE."""
    import oracle.oracle_c as orcc
    y, cr, cb = orcc.rgb_to_ycrcb(rgb)
    for p, t in ((y, 0), (orcc.pyr_down(cr), 1), (orcc.pyr_down(cb), 1)):
        zz = orcc.zigzag_blocks(orcc.dct_channel(p, t), 8)
        orcc.dpcm(zz[:, 0].copy())
        orcc.rle_encode(zz[:, 1:].reshape(-1), 15)


def cpu_baseline(budget_s):
    """The C restatement of hiccup's CPU path (oracle/; bit-identical to the GPU
    path) on bounded samples of the same 8K workload, timed on this host: 1 thread
    over 1088-row bands, then as many threads as the box grants this process (its
    CPU affinity, capped by OMP_NUM_THREADS when that is set: 16 on the GPU box),
    one 1088-row band per thread.  Each band is encoded as its own stream (colour +
    pyrDown, DCT + quantize, zig-zag, DC DPCM, AC RLE); the cross-band stitch that
    would join the bands into one image stream (the carried zero run and the DC
    difference at each band edge, a few words per band) is NOT timed."""
    from concurrent.futures import ThreadPoolExecutor
    rows = 1088  # 1/4 of the 8K frame (multiple of 16)
    rng = np.random.default_rng(3)
    band = rng.integers(0, 256, (rows, W8K, 3), dtype=np.uint8)
    host = host_description()
    # 1 thread: bands until ~budget/3
    done, t_single = 0, 0.0
    while t_single < budget_s / 3:
        t0 = time.perf_counter()
        _cpu_encode_band(band)
        t_single += time.perf_counter() - t0
        done += rows * W8K
    single = done / t_single / 1e6
    # all usable cores (capped by OMP_NUM_THREADS, the box's CPU share): one band per
    # thread (ctypes releases the GIL in the C calls)
    nt = max(1, host["usable_cpus"] or 1)
    cap_src = "CPU affinity (%d usable CPUs)" % nt
    if os.environ.get("OMP_NUM_THREADS", "").isdigit() and int(os.environ["OMP_NUM_THREADS"]) < nt:
        nt = int(os.environ["OMP_NUM_THREADS"])
        cap_src = "OMP_NUM_THREADS=%d (below the %d usable CPUs: the box's CPU share for this job)" % (
            nt, host["usable_cpus"] or 0)
    host["threads_used"] = nt
    host["thread_cap_source"] = cap_src
    bands = [rng.integers(0, 256, (rows, W8K, 3), dtype=np.uint8) for _ in range(min(nt, 64))]
    # rounds of one band per thread until ~budget/3 of wall time
    rounds, t_all = 0, 0.0
    with ThreadPoolExecutor(nt) as ex:
        while t_all < budget_s / 3:
            t0 = time.perf_counter()
            list(ex.map(_cpu_encode_band, [bands[i % len(bands)] for i in range(nt)]))
            t_all += time.perf_counter() - t0
            rounds += 1
    multi = rounds * nt * rows * W8K / t_all / 1e6
    return {"value": round(multi, 3), "unit": "Mpixels/s", "cores": nt, "kind": "port",
            "sample": "%d rounds of %d threads x one %d x %d RGB band of the 8K workload each (%.1f s): per band "
                      "colour + pyrDown, DCT + quantize, zig-zag, DC DPCM and AC RLE as the band's own stream, "
                      "oracle/hiccup_oracle.c (C restatement of hiccup's CPU path, bit-identical to the GPU path); "
                      "the cross-band stitch into one image stream (carried zero run + DC at each band edge) is not "
                      "timed; threads: %s" % (rounds, nt, rows, W8K, t_all, cap_src),
            "single_thread": {"value": round(single, 3), "cores": 1,
                              "sample": "%d bands of %d x %d RGB, %.1f s" % (done // (rows * W8K), rows, W8K,
                                                                             t_single)},
            "host": host,
            "reference_measured_in_build_container": "hiccup's own numpy path ~0.7 Mpix/s (8K 4:2:0 DCT+quantize, "
                                                     "BASELINE.md); its RLE is quadratic (infeasible at 8K)"}


def plane_kernel(tmf):
    """The forward plane kernel the library runs for ZIGZAG_I16 planes (dct_path knob)."""
    from hiccup_amd import _lib
    return ("k_dct_planes<T,ZIGZAG_I16,%d> (float64 AAN; T = the planes' table when they share one, -1 = per "
            "plane at run time)" % tmf)


def spread(ts_us):
    """min / median / max / p10 / p90 of per-launch times (us)."""
    ts = np.asarray(ts_us, dtype=np.float64)
    return {"min": round(float(ts.min()), 2), "p10": round(float(np.percentile(ts, 10)), 2),
            "median": round(float(np.median(ts)), 2), "p90": round(float(np.percentile(ts, 90)), 2),
            "max": round(float(ts.max()), 2), "n": int(ts.size)}


def extra_4k_luma(steps=24, warmup=8, floor_us=None):
    """BASELINE configs[1]: 4096 x 4096 random luminance, DCT + quantize + zig-zag on
    one GPU (hic_dct_quant_u8_timed: the launch's own begin / end timestamps), with
    >= 1.2 GB of rotating planes so every launch reads HBM, not the Infinity Cache.
    The median over `steps` launches after `warmup` untimed ones (round 4 reported a
    mean of 20 after 3, which one slow launch moved by 47 %), with the spread."""
    from hiccup_amd import _lib, device
    n = 4096
    rot = int(np.ceil(ROT_BYTES / (n * n * 3)))
    g = torch.Generator(device="cuda")
    g.manual_seed(2)
    planes = [torch.randint(0, 256, (n, n), dtype=torch.uint8, device="cuda", generator=g) for _ in range(rot)]
    outs = [device.empty((n * n // 64, 64), torch.int16) for _ in range(rot)]
    evs = [device.KernelEvents() for _ in range(steps)]

    def launch(i, ev=None):
        p, o = planes[i % rot], outs[i % rot]
        _lib.call("hic_dct_quant_u8_timed", device.ptr(p), n, n, n, _lib.TABLE_LUMINANCE, _lib.LAYOUT_ZIGZAG_I16,
                  device.ptr(o), None, ev.start if ev else None, ev.stop if ev else None)

    for i in range(warmup):
        launch(i)
    torch.cuda.synchronize()
    for i in range(steps):
        launch(warmup + i, evs[i])
    torch.cuda.synchronize()
    ts = [e.elapsed_ms() * 1e3 for e in evs]
    us = float(np.median(ts))
    gbs = n * n * 3 / (us * 1e-6) / 1e9
    del planes, outs
    torch.cuda.empty_cache()
    return {"workload": "4096x4096 uint8 luminance -> quantized int16 zig-zag blocks (BASELINE configs[1])",
            "kernel": plane_kernel(-1), "median_launch_us": round(us, 2), "launch_us": spread(ts),
            "mpix_s": round(n * n / us, 1), "achieved_gbs": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
            "algorithmic_bytes": n * n * 3, "timed_launches": steps, "warmup_launches": warmup,
            "memory_floor_us_measured": floor_us,
            "frac_of_measured_floor": round(floor_us / us, 4) if floor_us else None}


def extra_rgb_encode(H=4096, W=4096, steps=40, n_streams=2, fused=None):
    """A full RGB encode on one GPU (fused colour + DCT/quantize/zig-zag, DC DPCM +
    AC RLE; fused=False: the two-kernel chain), consecutive images alternating over
    `n_streams` streams, >= 1.2 GB of rotating inputs, wall time of `steps` images
    between two synchronisations."""
    from hiccup_amd import pipeline
    nin = int(np.ceil(ROT_BYTES / (H * W * 3)))
    g = torch.Generator(device="cuda")
    g.manual_seed(6)
    xs = [torch.randint(0, 256, (H, W, 3), dtype=torch.uint8, device="cuda", generator=g) for _ in range(nin)]
    encs = [pipeline.Encoder(H, W, fused=fused) for _ in range(4)]
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(n_streams - 1)]
    torch.cuda.synchronize()

    def run(i0, k):
        for i in range(i0, i0 + k):
            with torch.cuda.stream(streams[i % len(streams)]):
                encs[i % 4].encode(xs[i % nin])

    run(0, 8)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(8, steps)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    for e in encs:
        for ci, c in enumerate(e.counts.cpu().tolist()):
            pipeline.check_count(int(c), pipeline.CHANNELS[ci])
    used = encs[0].fused
    del xs, encs
    torch.cuda.empty_cache()
    return {"fused": used, "ms_per_image": round(dt * 1e3, 4), "mpix_s": round(H * W / dt / 1e6, 1),
            "timed_images": steps, "streams": n_streams}


def extra_4k_rgb_encode(steps=40, n_streams=4):
    """north_star's 4K point on one GPU: 4096 x 4096 random RGB, the headline's chain
    on the headline's 4 streams (a 4K launch is 2048 waves, two thirds of the chip's
    wave slots: images overlap to fill it)."""
    out = {"workload": "4096x4096 RGB -> YCrCb 4:2:0 full encode (the headline's chain at north_star's 4K point), "
                       "1 GPU, %d streams" % n_streams}
    out.update(extra_rgb_encode(4096, 4096, steps, n_streams))
    return out


def extra_ragged_rgb_encode(H, W, steps=40, n_streams=2):
    """H x W with W % 512 != 0 (the fused kernel's ragged last strip) full encode:
    the default (fused, one RLE record per strip segment, the scan / emit walking row
    segments) against the two-kernel chain on the same inputs."""
    out = {"workload": "%dx%d RGB -> YCrCb 4:2:0 full encode, 1 GPU, %d streams (fused: ragged last strip, one RLE "
                       "record per strip segment; chain: colour kernel + plane DCT)" % (W, H, n_streams)}
    out["fused"] = extra_rgb_encode(H, W, steps, n_streams, fused=True)
    out["two_kernel_chain"] = extra_rgb_encode(H, W, steps, n_streams, fused=False)
    return out


def extra_8k_plane_dct(steps=24, luma_only=False, floor_us=None):
    """The north_star's DCT+quantize pass on its own: k_dct_planes over the 8K Y +
    Cr + Cb planes (4320 x 7680 + 2 x 2160 x 3840 uint8 -> int16 zig-zag blocks +
    RLE tile records, one launch, the two-kernel chain's second kernel), or over the
    8K luminance plane alone (luma_only: SURVEY.md section 8(d)'s measurement point
    for north_star's >= 0.70 target, 99.5 MB, <= 17.8 us), rotating >= 1.2 GB of
    planes, timed by the launch's own events.  Algorithmic bytes 3 B per plane
    pixel (1 read + 2 written); read_only_frac counts the 1 B read alone."""
    from hiccup_amd import _lib, device
    shapes = [(H8K, W8K, 0)] if luma_only else [(H8K, W8K, 0), (H8K // 2, W8K // 2, 1), (H8K // 2, W8K // 2, 1)]
    n = len(shapes)
    px = sum(h * w for h, w, _ in shapes)
    rot = int(np.ceil(ROT_BYTES / (px * 3)))
    g = torch.Generator(device="cuda")
    g.manual_seed(4)
    sets = []
    for _ in range(rot):
        planes, outs, wss = [], [], []
        jobs = (_lib.DctPlaneJob * n)()
        for i, (h, w, t) in enumerate(shapes):
            nblk = (h // 8) * (w // 8)
            planes.append(torch.randint(0, 256, (h, w), dtype=torch.uint8, device="cuda", generator=g))
            outs.append(device.empty((nblk, 64), torch.int16))
            wss.append(device.workspace(_lib.load().hic_rle_workspace_bytes(nblk, 64)))
            jobs[i] = _lib.DctPlaneJob(planes[i].data_ptr(), h, w, w, t, outs[i].data_ptr(), wss[i].data_ptr())
        sets.append((planes, outs, wss, jobs))
    evs = [device.KernelEvents() for _ in range(steps)]
    for i in range(4):
        _lib.call("hic_dct_quant_rle_u8_batch", n, sets[i % rot][3], 15, device.stream_ptr(), None, None)
    for i, e in enumerate(evs):
        _lib.call("hic_dct_quant_rle_u8_batch", n, sets[(4 + i) % rot][3], 15, device.stream_ptr(), e.start, e.stop)
    torch.cuda.synchronize()
    us = float(np.median([e.elapsed_ms() for e in evs])) * 1e3
    gbs = px * 3 / (us * 1e-6) / 1e9
    del sets
    torch.cuda.empty_cache()
    out = {"workload": ("8K luminance plane (4320 x 7680 uint8) -> quantized int16 zig-zag blocks + RLE tile "
                        "records: SURVEY.md 8(d)'s measurement point for north_star's >= 0.70 target "
                        "(<= 17.8 us for 99.5 MB)" if luma_only else
                        "8K Y + Cr + Cb planes -> quantized int16 zig-zag blocks + RLE tile records (k_dct_planes, "
                        "the DCT+quantize pass without the colour stage)"),
           "kernel": plane_kernel(15), "median_launch_us": round(us, 2),
           "achieved_gbs": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4), "algorithmic_bytes": px * 3,
           "read_only_frac": round(px / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4), "timed_launches": steps}
    if luma_only and floor_us:
        # the pass's own byte pattern without the DCT, measured in this run
        # (measure_floors: hic_probe_plane on the same plane size)
        out["memory_floor_us_measured"] = floor_us
        out["frac_of_measured_floor"] = round(floor_us / us, 4)
    return out


def _luma_sets(nplanes, records, seed=12):
    """Rotating sets (>= 1.2 GB in all) of `nplanes` 8K luminance planes with their
    outputs and a hic_dct_plane_job array each (records: RLE workspaces, else NULL =
    the records-free pass)."""
    from hiccup_amd import _lib, device
    h, w = H8K, W8K
    px = h * w
    rot = max(2, int(np.ceil(ROT_BYTES / (nplanes * 3 * px))))
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    nblk = px // 64
    sets = []
    for _ in range(rot):
        planes = [torch.randint(0, 256, (h, w), dtype=torch.uint8, device="cuda", generator=g) for _ in range(nplanes)]
        outs = [device.empty((nblk, 64), torch.int16) for _ in range(nplanes)]
        wss = [device.workspace(_lib.load().hic_rle_workspace_bytes(nblk, 64)) if records else None
               for _ in range(nplanes)]
        jobs = (_lib.DctPlaneJob * nplanes)()
        for i in range(nplanes):
            jobs[i] = _lib.DctPlaneJob(planes[i].data_ptr(), h, w, w, 0, outs[i].data_ptr(),
                                       wss[i].data_ptr() if records else None)
        sets.append((planes, outs, wss, jobs))
    return sets


def _time_batches(sets, nplanes, steps, warmup):
    from hiccup_amd import _lib, device
    rot = len(sets)
    evs = [device.KernelEvents() for _ in range(steps)]
    for i in range(warmup):
        _lib.call("hic_dct_quant_rle_u8_batch", nplanes, sets[i % rot][3], 15, device.stream_ptr(), None, None)
    for i, e in enumerate(evs):
        _lib.call("hic_dct_quant_rle_u8_batch", nplanes, sets[(warmup + i) % rot][3], 15, device.stream_ptr(),
                  e.start, e.stop)
    torch.cuda.synchronize()
    return [e.elapsed_ms() * 1e3 for e in evs]


def extra_8k_luma_batched(nplanes=16, steps=16, warmup=8, floor_us_per_plane=None):
    """north_star's DCT+quantize pass measured the way the product runs planes back to
    back: ONE hic_dct_quant_rle_u8_batch launch over `nplanes` 8K luminance planes of
    consecutive images (each 4320 x 7680 uint8 -> quantized int16 zig-zag blocks),
    >= 1.2 GB rotating, timed by the launch's own events; the figure is the median
    launch time / nplanes (the per-launch ramp and tail amortised over the batch).
    Two variants: records-free (DCT + quantize + zig-zag: north_star's pass and
    what transform.dct_channel / configs[1] run; the headline of this entry) and with
    the RLE tile records fused into the epilogue (what the two-kernel chain runs);
    plus the records-free pass as one launch per plane."""
    h, w = H8K, W8K
    px = h * w
    out = {"workload": "%d x 8K luminance planes (4320 x 7680 uint8, consecutive images) per launch -> quantized "
                       "int16 zig-zag blocks: north_star's DCT+quantize pass back to back (SURVEY.md 8(d): >= 0.70 "
                       "= <= 17.8 us per plane)" % nplanes,
           "kernel": plane_kernel(-1), "planes_per_launch": nplanes, "algorithmic_bytes_per_plane": 3 * px}
    for records in (False, True):
        sets = _luma_sets(nplanes, records)
        ts = _time_batches(sets, nplanes, steps, warmup)
        del sets
        torch.cuda.empty_cache()
        us = float(np.median(ts)) / nplanes
        gbs = 3 * px / (us * 1e-6) / 1e9
        v = {"us_per_plane": round(us, 2), "launch_us": spread(ts), "achieved_gbs": round(gbs, 1),
             "frac": round(gbs / HBM_PEAK_GBS, 4), "timed_launches": steps, "warmup_launches": warmup}
        if records:
            v["kernel"] = plane_kernel(15)
            out["with_rle_records"] = v
        else:
            out.update(v)
            if floor_us_per_plane:
                out["memory_floor_us_per_plane"] = floor_us_per_plane
                out["frac_of_measured_floor"] = round(floor_us_per_plane / us, 4)
    sets = _luma_sets(1, False, seed=13)
    ts = _time_batches(sets, 1, 24, 8)
    del sets
    torch.cuda.empty_cache()
    us = float(np.median(ts))
    gbs = 3 * px / (us * 1e-6) / 1e9
    out["single_launch"] = {"median_launch_us": round(us, 2), "launch_us": spread(ts), "achieved_gbs": round(gbs, 1),
                            "frac": round(gbs / HBM_PEAK_GBS, 4)}
    return out


def slot_symbols(enc):
    """Symbols a slot-layout encode wrote into its slots (the n_r of every record:
    the stream's symbols less the virtual fillers and the EOB)."""
    return int(sum(int(enc.sidx[k].view(-1, 4)[:, 0].sum().item()) for k in enc.sidx))


def measure_floors(steps=20, slots=False):
    """In-run memory floors (hic_probe_copy / hic_probe_plane, memory-only probes in
    the product library), each timed by the launches' own HIP events over >= 1.2 GB
    of rotating buffers:
      device_copy_gbs: a streaming device copy (read + write bytes / time);
      luma_pattern:    the forward plane pass's own byte pattern without the DCT
                       (8x8 block loads, LDS stage, 1 KiB nontemporal stores, 1 B
                       read + 2 B written per pixel), on 1x / 2x / 4x the 8K luma
                       plane per launch -- whether the pass's floor is the access
                       pattern or the per-launch ramp and tail."""
    from hiccup_amd import _lib, device
    out = {}
    nbytes = 256 << 20
    nbuf = int(np.ceil(ROT_BYTES / (2 * nbytes)))
    bufs = [(device.empty((nbytes,), torch.uint8), device.empty((nbytes,), torch.uint8)) for _ in range(nbuf)]
    for a, _ in bufs:
        a.fill_(7)
    evs = [device.KernelEvents() for _ in range(steps)]

    def timed(launch):
        for i in range(steps + 3):
            ev = evs[i - 3] if i >= 3 else None
            launch(i, ev.start if ev else None, ev.stop if ev else None)
        torch.cuda.synchronize()
        return float(np.median([e.elapsed_ms() for e in evs])) * 1e3

    # the best of three grid sizes (the probes claim a floor, so they get the best
    # configuration this run finds)
    per = {}
    for wpc in (8, 16, 32):
        per[wpc] = timed(lambda i, e0, e1: _lib.call("hic_probe_copy", device.ptr(bufs[i % nbuf][0]),
                                                     device.ptr(bufs[i % nbuf][1]), nbytes, wpc,
                                                     device.stream_ptr(), e0, e1))
    best = min(per, key=per.get)
    us = per[best]
    out["device_copy_gbs"] = round(2 * nbytes / (us * 1e-6) / 1e9, 1)
    out["device_copy"] = {"bytes_per_launch": nbytes, "median_launch_us": round(us, 2), "waves_per_cu": best,
                          "frac_of_8tbs": round(2 * nbytes / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                          "us_by_waves_per_cu": {k: round(v, 2) for k, v in per.items()}}
    del bufs
    torch.cuda.empty_cache()
    pat = {}
    for mult in (1, 2, 4, "4k"):
        h, w = (4096, 4096) if mult == "4k" else (H8K * mult, W8K)
        px = h * w
        rot = max(2, int(np.ceil(ROT_BYTES / (3 * px))))
        g = torch.Generator(device="cuda")
        g.manual_seed(9)
        planes = [torch.randint(0, 256, (h, w), dtype=torch.uint8, device="cuda", generator=g) for _ in range(rot)]
        outs = [device.empty((px // 64, 64), torch.int16) for _ in range(rot)]
        per = {}
        for wpc in (12, 16):
            per[wpc] = timed(lambda i, e0, e1: _lib.call("hic_probe_plane", device.ptr(planes[i % rot]), h, w,
                                                         device.ptr(outs[i % rot]), wpc, device.stream_ptr(), e0, e1))
        best = min(per, key=per.get)
        us = per[best]
        pat["4k_luma" if mult == "4k" else "%dx" % mult] = {"plane_hw": [h, w], "bytes_per_launch": 3 * px, "median_launch_us": round(us, 2),
                             "waves_per_cu": best, "us_by_waves_per_cu": {k: round(v, 2) for k, v in per.items()},
                             "gbs": round(3 * px / (us * 1e-6) / 1e9, 1),
                             "frac_of_8tbs": round(3 * px / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}
        del planes, outs
        torch.cuda.empty_cache()
    out["luma_pattern"] = pat
    # the fused encoder's own byte pattern (hic_probe_encode420: the same grid, unit
    # order and 19 row loads per unit, stage and 1 KiB stores, no arithmetic) on the
    # 8K RGB image: k_encode420's in-run memory floor
    h, w = H8K, W8K
    px = h * w
    if slots:
        # the slot layout's pattern (hic_probe_encode420_slots): each rotating image
        # encoded once for real, then its records' symbol counts replayed
        from hiccup_amd import pipeline
        rot = max(2, int(np.ceil(ROT_BYTES / (7 * px))))
        g = torch.Generator(device="cuda")
        g.manual_seed(10)
        imgs = [torch.randint(0, 256, (h, w, 3), dtype=torch.uint8, device="cuda", generator=g) for _ in range(rot)]
        encs = [pipeline.Encoder(h, w) for _ in range(rot)]
        for e, x in zip(encs, imgs):
            e.encode(x)
        torch.cuda.synchronize()
        nbytes = 3 * px + 3 * slot_symbols(encs[0]) + 4 * sum(e.shape[0] for e in encs[0].coef.values())
        jobs = [e._slot_jobs() for e in encs]
        us = timed(lambda i, e0, e1: _lib.call("hic_probe_encode420_slots", device.ptr(imgs[i % rot]), h, w,
                                               jobs[i % rot], device.stream_ptr(), e0, e1))
        out["encode420_pattern"] = {"image_hw": [h, w], "kernel": "hic_probe_encode420_slots", "bytes_per_launch": nbytes,
                                    "median_launch_us": round(us, 2), "gbs": round(nbytes / (us * 1e-6) / 1e9, 1),
                                    "frac_of_8tbs": round(nbytes / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}
        del imgs, encs, jobs
        torch.cuda.empty_cache()
        return out
    rot = max(2, int(np.ceil(ROT_BYTES / (6 * px))))
    g = torch.Generator(device="cuda")
    g.manual_seed(10)
    imgs = [torch.randint(0, 256, (h, w, 3), dtype=torch.uint8, device="cuda", generator=g) for _ in range(rot)]
    co = [(device.empty((px // 64, 64), torch.int16), device.empty((px // 256, 64), torch.int16),
           device.empty((px // 256, 64), torch.int16)) for _ in range(rot)]
    rec_y = device.empty(((h // 8) * (w // 512) * 3,), torch.int64)
    rec_c = device.empty(((h // 16) * (w // 512) * 3,), torch.int64)
    us = timed(lambda i, e0, e1: _lib.call("hic_probe_encode420", device.ptr(imgs[i % rot]), h, w,
                                           *[device.ptr(t) for t in co[i % rot]], device.ptr(rec_y),
                                           device.ptr(rec_c), device.stream_ptr(), e0, e1))
    out["encode420_pattern"] = {"image_hw": [h, w], "bytes_per_launch": 6 * px, "median_launch_us": round(us, 2),
                                "gbs": round(6 * px / (us * 1e-6) / 1e9, 1),
                                "frac_of_8tbs": round(6 * px / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)}
    del imgs, co, rec_y, rec_c
    torch.cuda.empty_cache()
    return out


def extra_16k_roundtrip(steps=4):
    """BASELINE configs[4] on one GPU: 16384 x 16384 random RGB, full encode (colour,
    DCT/quantize/zig-zag, DPCM/RLE) then full decode (RLE expand, DC integrate,
    izigzag, dequantize/IDCT, pyrUp, YCrCb -> RGB).  The symbol counts cross to the
    host between the halves (the decoder sizes its workspace from them).  PSNR is
    of the reconstruction against the input; its bit-exactness against the CPU
    restatement is tests/test_gpu_codec.py::test_16k_roundtrip_vs_oracle."""
    from hiccup_amd import pipeline
    n = 16384
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    xs = [torch.randint(0, 256, (n, n, 3), dtype=torch.uint8, device="cuda", generator=g) for _ in range(2)]
    enc, dec = pipeline.Encoder(n, n, index=True), pipeline.Decoder(n, n)
    slots = enc.slots

    def trip(i, indexed):
        enc.encode(xs[i % 2])
        if indexed:  # encoder-side tile index, counts stay on the device: no host sync
            return dec.decode(enc.sym_len, enc.sym_val, enc.counts, enc.dc, index=enc.index)
        enc.compact()  # slot layout: the contiguous stream a bare-stream decoder reads
        counts = enc.counts.cpu().tolist()
        return dec.decode(enc.sym_len, enc.sym_val, counts, enc.dc)

    res = {}
    for indexed in (True, False):
        trip(0, indexed)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            out = trip(1 + i, indexed)
        torch.cuda.synchronize()
        res[indexed] = (time.perf_counter() - t0) / steps
        dec.check_status()
    dt = res[True]
    x = xs[steps % 2]
    mse = float(((out.float() - x.float()) ** 2).mean())
    del out
    # the same trips pipelined: consecutive trips alternate over two streams, each
    # with its own encoder / decoder, so one trip's decode overlaps the next one's
    # encode (per-trip time = throughput; ms_per_roundtrip above is the latency)
    enc2, dec2 = pipeline.Encoder(n, n, index=True), pipeline.Decoder(n, n)
    pairs = [(enc, dec), (enc2, dec2)]
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]

    def trip2(i):
        e, d = pairs[i % 2]
        with torch.cuda.stream(streams[i % 2]):
            e.encode(xs[i % 2], streams[i % 2])
            return d.decode(e.sym_len, e.sym_val, e.counts, e.dc, stream=streams[i % 2], index=e.index)

    trip2(0)
    trip2(1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(2 * steps):
        trip2(i)
    torch.cuda.synchronize()
    dt2 = (time.perf_counter() - t0) / (2 * steps)
    dec.check_status()
    dec2.check_status()
    out_a = dec2.rgb.clone()  # trip 2 * steps + 1: xs[1], against a one-stream trip of it
    ref = trip(1, True)
    torch.cuda.synchronize()
    same = bool(torch.equal(ref, out_a))
    del xs, enc, dec, enc2, dec2, pairs, ref, out_a
    torch.cuda.empty_cache()
    return {"workload": "16384x16384 RGB encode + decode round trip, 1 GPU (BASELINE configs[4] at N=1); %s"
                        % ("slot-layout encode (hic_encode420_slots_u8 + hic_rle_slots_close), decode from the "
                           "slots through the record index (Cr + Cb decode + IDCT in one launch, Y decode + IDCT + "
                           "pyrUp + colour in one), no host sync between the halves" if slots else
                           "decode from the encoder-side tile index, RLE decode + IDCT fused per plane "
                           "(hic_rle_decode_idct_u8_indexed), no host sync between the halves"),
            "ms_per_roundtrip": round(dt * 1e3, 3), "mpix_s": round(n * n / dt / 1e6, 1),
            "ms_per_roundtrip_unindexed_decode": round(res[False] * 1e3, 3),
            "unindexed_decode_is": "the contiguous stream (hic_rle_slots_compact in the trip), counts through the host, "
                                   "the bare-stream decode chain",
            "ms_per_roundtrip_2streams": round(dt2 * 1e3, 3), "two_stream_output_equal": same,
            "psnr_db_vs_input": round(10 * np.log10(255.0 ** 2 / mse), 3), "timed_roundtrips": steps}


def extra_8k_encode_from_host(steps=8):
    """The headline encode with its input starting in pinned host memory (the
    reference API hands over numpy arrays): each image's RGB crosses PCIe
    (non-blocking H2D copy) and is encoded on the same stream, two streams
    alternating so one image's copy overlaps the other's encode.  PCIe-inclusive
    rate; never the headline value."""
    from hiccup_amd import pipeline
    g = torch.Generator()
    g.manual_seed(4)
    hosts = [torch.randint(0, 256, (H8K, W8K, 3), dtype=torch.uint8, generator=g).pin_memory() for _ in range(2)]
    devs = [torch.empty((H8K, W8K, 3), dtype=torch.uint8, device="cuda") for _ in range(2)]
    encs = [pipeline.Encoder(H8K, W8K) for _ in range(2)]
    streams = [torch.cuda.Stream() for _ in range(2)]

    def run(i0, k):
        for i in range(i0, i0 + k):
            j = i % 2
            with torch.cuda.stream(streams[j]):
                devs[j].copy_(hosts[j], non_blocking=True)
                encs[j].encode(devs[j])

    run(0, 2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(2, steps)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    # the copy alone
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for i in range(steps):
        devs[i % 2].copy_(hosts[i % 2], non_blocking=True)
    torch.cuda.synchronize()
    dc = (time.perf_counter() - t1) / steps
    del hosts, devs, encs
    torch.cuda.empty_cache()
    nbytes = H8K * W8K * 3
    return {"workload": "7680x4320 RGB encode with the input in pinned host memory (H2D copy + encode, 2 streams)",
            "ms_per_image": round(dt * 1e3, 3), "mpix_s": round(H8K * W8K / dt / 1e6, 1),
            "h2d_ms_per_image": round(dc * 1e3, 3), "h2d_gbs": round(nbytes / dc / 1e9, 1), "timed_images": steps}


def extra_8k_jpeg_decode(steps=3):
    """codec.jpeg_decode of a real 8K .hic, end to end from its bytes: container
    parse, the nine trees from the tables (host), the nine Huffman streams decoded
    on the GPU (hic_huffman_decode), RLE decode + DC integration + izigzag on the
    GPU, the float64 planes copied back (the reference's CompressedImage).  The
    .hic comes from the GPU encoder on a random 8K RGB image."""
    from hiccup_amd import codec, device, hicimage, pipeline, settings
    debug, settings.DEBUG = settings.DEBUG, False  # the reference's progress prints would break the JSON line
    try:
        return _extra_8k_jpeg_decode(steps, codec, device, hicimage, pipeline)
    finally:
        settings.DEBUG = debug


def _extra_8k_jpeg_decode(steps, codec, device, hicimage, pipeline):
    g = torch.Generator(device="cuda")
    g.manual_seed(9)
    x = torch.randint(0, 256, (H8K, W8K, 3), dtype=torch.uint8, device="cuda", generator=g)
    enc = pipeline.Encoder(H8K, W8K)
    enc.encode(x)
    blob = pickle.dumps(enc.hic_image().byte_stream())  # the .hic file's bytes (HicImage.write_file)
    symbols = int(sum(enc.counts.cpu().tolist()) * 2 + sum(enc.dc[k].numel() for k in pipeline.CHANNELS))
    enc.materialize()  # slot layout: the blocks, for the DC check below
    want = device.to_host(enc.coef["lum"][:, 0])
    del x
    t_parse, t_dec = [], []
    for _ in range(steps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        img = hicimage.HicImage.from_bytes(hicimage._loads(blob))  # HicImage.from_file minus the read
        t1 = time.perf_counter()
        out = codec.jpeg_decode(img)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        t_parse.append(t1 - t0)
        t_dec.append(t2 - t1)
    lum = out.as_dict["lum"]
    # the decoded DC coefficients equal the encoder's (full parity: tests/test_gpu_codec.py)
    ok = bool(np.array_equal(lum[::8, ::8].reshape(-1), want.astype(np.float64)))
    ms = lambda v: round(float(np.median(v[1:])) * 1e3, 1)  # noqa: E731
    return {"workload": "codec.jpeg_decode of an 8K (7680x4320) .hic from bytes (GPU Huffman + RLE decode)",
            "hic_bytes": len(blob), "symbols": symbols, "ms_parse": ms(t_parse), "ms_jpeg_decode": ms(t_dec),
            "msym_s": round(symbols / float(np.median(t_dec[1:])) / 1e6, 1), "dc_matches_encoder": ok,
            "timed_decodes": steps}


def pinned_rates(nbytes=256 << 20, reps=4):
    """Pinned host <-> device copy rates of this box (GB/s), torch copies of one
    256 MiB buffer."""
    h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    out = {}
    for name, f in (("h2d_gbs", lambda: d.copy_(h, non_blocking=True)),
                    ("d2h_gbs", lambda: h.copy_(d, non_blocking=True))):
        f()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            f()
        torch.cuda.synchronize()
        out[name] = round(reps * nbytes / (time.perf_counter() - t) / 1e9, 1)
    return out


def extra_8k_reference_api(steps=3):
    """The drop-in surface at 8K from host arrays, as a user of the reference calls
    it: compression.jpeg_compression (RGB -> quantized planes), codec.jpeg_encode
    (-> HicImage), codec.jpeg_decode (HicImage -> planes) and
    compression.jpeg_decompression (-> RGB); wall time per call, median of `steps`
    after one untimed call, host copies included (PCIe-inclusive, never the headline)."""
    from hiccup_amd import codec, compression, settings
    debug, settings.DEBUG = settings.DEBUG, False
    try:
        rgb = np.random.default_rng(1).integers(0, 256, (H8K, W8K, 3), dtype=np.uint8)

        def med(f):
            ts, r = [], None
            for _ in range(steps + 1):
                t = time.perf_counter()
                r = f()
                ts.append(time.perf_counter() - t)
            return r, round(float(np.median(ts[1:])) * 1e3, 1)

        ci, t_comp = med(lambda: compression.jpeg_compression(rgb))
        hic, t_enc = med(lambda: codec.jpeg_encode(ci))
        ci2, t_dec = med(lambda: codec.jpeg_decode(hic))
        rec, t_decomp = med(lambda: compression.jpeg_decompression(ci2))
        same = all(np.array_equal(a, b) for a, b in zip(ci.as_dict.values(), ci2.as_dict.values()))
        # each call's PCIe floor: the bytes it must move at this box's pinned rates
        rates = pinned_rates()
        px = H8K * W8K
        bits = sum(int(p.packed_bits()[0].size) for p in hic.payloads[9:18])
        moved = {"jpeg_compression": (3 * px, 4 * px * 3 // 2), "jpeg_encode": (4 * px * 3 // 2, bits),
                 "jpeg_decode": (bits, 8 * px * 3 // 2), "jpeg_decompression": (8 * px * 3 // 2, 3 * px)}
        walls = {"jpeg_compression": t_comp, "jpeg_encode": t_enc, "jpeg_decode": t_dec,
                 "jpeg_decompression": t_decomp}
        floors = {}
        for k, (up, down) in moved.items():
            f = up / rates["h2d_gbs"] / 1e6 + down / rates["d2h_gbs"] / 1e6
            floors[k] = {"bytes_up": up, "bytes_down": down, "floor_ms": round(f, 2),
                         "ratio": round(walls[k] / f, 2)}
        return {"workload": "8K RGB through the reference API from host arrays (jpeg_compression, jpeg_encode, "
                            "jpeg_decode, jpeg_decompression), host copies included",
                "ms_jpeg_compression": t_comp, "ms_jpeg_encode": t_enc, "ms_jpeg_decode": t_dec,
                "ms_jpeg_decompression": t_decomp, "pcie": dict(rates, **floors),
                "pcie_note": "floor = the call's host<->device bytes (uint8 RGB, int32 planes for jpeg_compression's "
                             "result / jpeg_encode's input, the coded bits, float64 planes for jpeg_decode's result / "
                             "jpeg_decompression's input) at the pinned H2D / D2H rates measured here; ratio = "
                             "wall / floor",
                "planes_equal_after_entropy_round_trip": same,
                "rgb_out_shape": list(rec.shape), "timed_calls": steps}
    finally:
        settings.DEBUG = debug


def measure_link(rank, world, group=None, nbytes=256 << 20, reps=5, device="cuda"):
    """The xGMI rate of one link, measured in this run: every rank sends `nbytes` to
    rank + 1 and receives as much from rank - 1 (a ring: each rank's traffic crosses
    one link per direction, and every rank of the group takes part in each P2P batch,
    as RCCL's batched P2P expects), one batch per repetition on the default stream,
    the slowest rank's time, median of `reps` after one warmup.  Returns GB/s per
    link and direction."""
    buf_s = torch.empty(nbytes, dtype=torch.uint8, device=device)
    buf_r = torch.empty(nbytes, dtype=torch.uint8, device=device)
    nxt, prv = (rank + 1) % world, (rank - 1) % world
    times = []
    for i in range(reps + 1):
        dist.barrier(group=group)
        if device == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        ops = [dist.P2POp(dist.isend, buf_s, nxt, group=group), dist.P2POp(dist.irecv, buf_r, prv, group=group)]
        for req in dist.batch_isend_irecv(ops):
            req.wait()
        if device == "cuda":
            torch.cuda.synchronize()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        if i:
            times.append(float(t.item()))
    del buf_s, buf_r
    return round(nbytes / float(np.median(times)) / 1e9, 1)


def extra_16k_roundtrip_sharded(rank, world, backend, steps=4):
    """BASELINE configs[4] at N ranks: a 16384 x 16384 random RGB image tile-sharded
    by block rows.  Each rank encodes its shard (ShardEncoder: colour with halo, DCT,
    its slice of the single DC / RLE stream after the summary all-gather) and then
    decodes its own slice (ShardDecoder: carried-zero skip, DC chain from the stitch
    record, one chroma halo row per neighbour over the process group for pyrUp,
    YCrCb -> RGB of its rows).  Each rank's symbol counts cross to its host between
    the halves.  PSNR of the whole reconstruction vs the input (squared errors
    summed over ranks); its bit-exactness vs the single-GPU decode is
    tests/test_dist_gpu.py / test_gpu_codec.py::test_shards_stitch_to_single_stream."""
    from hiccup_amd import sharding
    n = 16384
    se = sharding.ShardEncoder(n, n, rank=rank, world=world)
    sd = sharding.ShardDecoder(n, n, rank=rank, world=world)
    a, b = se.span
    g = torch.Generator(device="cuda")
    g.manual_seed(5 + rank)
    xs = [torch.randint(0, 256, (b - a, n, 3), dtype=torch.uint8, device="cuda", generator=g) for _ in range(2)]

    def trip(i):
        se.encode(xs[i % 2])
        counts = se.enc.counts.cpu().tolist()
        return sd.decode(se.enc.sym_len, se.enc.sym_val, counts, se.enc.dc, se.stitch)

    trip(0)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        out = trip(1 + i)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    sd.check_status()
    x = xs[steps % 2]
    o0, o1 = sd.out_rows
    sq = float(((out.float() - x[o0 - a:o1 - a].float()) ** 2).sum())
    dev = "cuda" if backend == "nccl" else "cpu"
    t = torch.tensor([dt, sq], dtype=torch.float64, device=dev)
    tmax = t.clone()
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    dt, mse = float(tmax[0].item()), float(t[1].item()) / (n * n * 3)
    del xs, se, sd
    torch.cuda.empty_cache()
    return {"workload": "16384x16384 RGB encode + decode round trip, tile-sharded over %d ranks "
                        "(BASELINE configs[4]; sharded encode + sharded decode with pyrUp halo exchange)" % world,
            "ms_per_roundtrip": round(dt * 1e3, 3), "mpix_s": round(n * n / dt / 1e6, 1),
            "psnr_db_vs_input": round(10 * np.log10(255.0 ** 2 / mse), 3), "timed_roundtrips": steps}


def load_pmc_traffic(fused, slots=False):
    """HBM bytes per launch of the roofline kernel from the committed rocprofv3 PMC
    summary (profiles/pmc_encode_slots.json for the slot-layout kernel,
    pmc_encode.json for the fused encoder writing coefficients, pmc_dct.json for the
    two-kernel chain's DCT: FETCH_SIZE / WRITE_SIZE calibrated on kernels of known
    traffic with the same access pattern, MI355X_MICROARCH.md HBM section)."""
    p = os.path.join(HERE, "profiles", "pmc_encode_slots.json" if slots else
                     "pmc_encode.json" if fused else "pmc_dct.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f)


def host_description():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count()
    return {"cpu_model": model, "os_cpu_count": os.cpu_count(), "usable_cpus": usable}


def _spawn_worker(local, args_list, world, port):
    """torch.multiprocessing entry: one rank of a self-launched N-GPU run."""
    os.environ.update(RANK=str(local), LOCAL_RANK=str(local), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.argv = [sys.argv[0]] + list(args_list)
    main()


def launch_ranks(args):
    """`bench.py --gpus N` without torch.distributed.run: start the N ranks here.
    The parent makes no GPU call (device counting does not initialise HIP)."""
    import torch.multiprocessing as mp
    n = torch.cuda.device_count()
    if n < args.gpus and not args.same_device:
        raise SystemExit("--gpus %d: only %d visible GPUs (use --same-device --dist-backend gloo to rehearse)"
                         % (args.gpus, n))
    ctx = mp.start_processes(_spawn_worker, args=(sys.argv[1:], args.gpus, args.master_port), nprocs=args.gpus,
                             join=False, start_method="spawn")
    while not ctx.join():
        pass


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1 and args.gpus > 1:
        launch_ranks(args)
        return
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.same_device:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    from hiccup_amd import _lib, device, pipeline, sharding
    device.require_gpu()
    for kv in args.knob:
        name, _, val = kv.partition("=")
        _lib.set_knob(name, int(val))

    H0, W0 = (H8K, W8K) if args.workload == "8k" else (4096, 4096)
    strong = world > 1 and args.mode == "strong"
    gather = strong and not args.no_gather
    # strong mode with the gather: image j of each group of `world` consecutive
    # images is gathered to rank j, the group's gathers in ONE grouped RCCL batch on
    # a process group of their own (its own RCCL stream, so the next group's
    # encodes -- and their 96-byte summary all-gathers -- run beside it); 2 x world
    # encoders, so a group's buffers are reused only after the group before it
    n_enc = max(4, 2 * world) if gather else 4
    xgroup = dist.new_group(list(range(world))) if gather else None
    if xgroup is not None:
        dist.barrier(group=xgroup)  # its communicator is set up before any timing
    rgather = None
    if gather and args.transport == "c-abi":
        if args.dist_backend != "nccl":
            raise SystemExit("--transport c-abi needs --dist-backend nccl (one GPU per rank)")
        rgather = sharding.RcclGather()
    if world > 1:
        H = H0 * world if not strong else H0
        make = lambda j: sharding.ShardEncoder(H, W0, rank=rank, world=world,  # noqa: E731
                                               gather_to=j % world if gather else None,
                                               gather_kind=args.gather_kind if gather else "blocks",
                                               fused=False if args.unfused else None)
    else:
        H = H0
        make = lambda j: pipeline.Encoder(H0, W0, fused=False if args.unfused else None,  # noqa: E731
                                          slots=False if (args.no_slots or args.unfused) else None)
    encs = [make(j) for j in range(n_enc)]  # rotate outputs too (~1.2 GB per 4)
    span = encs[0].span if world > 1 else (0, H)
    in_rows = span[1] - span[0]
    nin = max(2, int(np.ceil(ROT_BYTES / (in_rows * W0 * 3))))
    g = torch.Generator(device="cuda")
    g.manual_seed(3 + rank)
    inputs = [torch.randint(0, 256, (in_rows, W0, 3), dtype=torch.uint8, device="cuda", generator=g)
              for _ in range(nin)]
    enc0 = encs[0].enc if world > 1 else encs[0]
    dct_px = sum(h * w for h, w in enc0.shapes.values())  # Y + Cr + Cb: one DCT launch
    px_per_step_rank = enc0.pixels
    fused = enc0.fused

    timed_events = []
    event_pool = [device.KernelEvents() for _ in range((args.steps + 3) // 4)]
    gather_ev = []  # (start, stop) torch events around each timed step's gather

    # consecutive images alternate over the streams (4 rotating encoders: an
    # encoder's buffers are reused only by later work on its own stream when
    # len(streams) divides 4)
    if args.streams is None:
        args.streams = 4 if world == 1 else 2
    assert 4 % args.streams == 0, "--streams must be 1, 2 or 4"
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(args.streams - 1)]
    torch.cuda.synchronize()  # inputs / buffers were made on the current stream

    exch_done = [None] * len(encs)  # event: the gather of the encoder's last image completed
    pending = []  # (encoder index, input, DCT events) of the group being collected
    n_groups = [0]

    def flush(record=False):
        """The pending images (a group of up to N): their sharded encodes with the
        exchange steps batched (sharding.encode_group), then their gathers as one
        grouped batch (image j of the group to rank j), on the group's stream
        (groups alternate over the streams)."""
        if not pending:
            return
        st = streams[n_groups[0] % len(streams)]
        n_groups[0] += 1
        for j, _, _ in pending:
            if exch_done[j] is not None:
                st.wait_event(exch_done[j])  # the encoder's previous image has left
        with torch.cuda.stream(st):
            group_encs = [encs[j] for j, _, _ in pending]
            sharding.encode_group(group_encs, [x for _, x, _ in pending], st, [ev for _, _, ev in pending])
            if record:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
            if args.gather_kind == "stream":
                sharding.gather_streams_group(group_encs, group=xgroup, rccl=rgather, stream=st)
            elif rgather is not None:
                rgather.gather_encoders(group_encs, st)
            else:
                sharding.gather_coefficients_group(group_encs, group=xgroup)
            done = torch.cuda.Event()
            done.record()
            if record:
                b.record()
                gather_ev.append((a, b, len(pending)))
        for j, _, _ in pending:
            exch_done[j] = done
        pending.clear()

    def step(i, record=False):
        e = encs[i % len(encs)]
        x = inputs[i % nin]
        ev = None
        # HIP events carrying the DCT kernel's own begin/end timestamps, on every 4th
        # timed step (a timestamped dispatch costs the stream a few us)
        if record and (i - args.warmup) % 4 == 0:
            ev = event_pool[len(timed_events)]
            timed_events.append(ev)
        if gather:
            pending.append((i % len(encs), x, ev))
            if len(pending) == world:
                flush(record)
            return
        with torch.cuda.stream(streams[i % len(streams)]):
            e.encode(x, dct_events=ev)

    for i in range(args.warmup):
        step(i)
    if gather:
        flush()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i, record=True)
    if gather:
        flush(True)  # a last, partial group: every timed image is gathered
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0

    def max_over_ranks(v):
        if world == 1:
            return v
        t = torch.tensor([v], dtype=torch.float64, device="cuda" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    elapsed = max_over_ranks(elapsed)
    # the same K-step region (same brackets) repeated: `value` is the median region
    # (a ~2 ms region moves with box clocks and queue timing), the first
    # region is reported beside it
    region_ms = [elapsed / args.steps * 1e3]
    for rep in range(REGION_REPEATS):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        base = args.warmup + args.steps * (rep + 1)
        for i in range(args.steps):
            step(base + i)
        if gather:
            flush()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        region_ms.append(max_over_ranks(time.perf_counter() - t1) / args.steps * 1e3)
    # every step's symbol counts are valid (a failed step would report a negative count);
    # in stream-gather mode the streams live on the gathering ranks
    stream_gather = gather and args.gather_kind == "stream"

    # N > 1 stream gather: one more group of N copies of one full image (every rank
    # makes the same image, encodes its row shard); each gathering rank's received
    # whole-image streams must equal a single-GPU Encoder's of that image, bit for bit
    verify = None
    if stream_gather and world > 1:
        gv = torch.Generator(device="cuda")
        gv.manual_seed(99)
        full = torch.randint(0, 256, (H, W0, 3), dtype=torch.uint8, device="cuda", generator=gv)
        xs = full[span[0]:span[1]].contiguous()
        torch.cuda.synchronize()
        for j in range(world):
            pending.append((j, xs, None))
        flush()
        torch.cuda.synchronize()
        ref = pipeline.Encoder(H, W0)
        ref.encode(full)
        ref.materialize()  # slot layout: the contiguous stream and the blocks compared below
        torch.cuda.synchronize()
        got = encs[rank].whole
        same = True
        for ci, k in enumerate(pipeline.CHANNELS):
            c = int(got.counts[ci].item())
            same = same and c == int(ref.counts[ci].item()) and c > 0
            same = same and torch.equal(got.sym_len[k][:c], ref.sym_len[k][:c])
            same = same and torch.equal(got.sym_val[k][:c], ref.sym_val[k][:c])
            same = same and torch.equal(got.dc[k], ref.dc[k]) and torch.equal(got.coef[k], ref.coef[k])
        t = torch.tensor([1 if same else 0], dtype=torch.int64,
                         device="cuda" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        verify = {"received_stream_bit_exact_vs_single_gpu": bool(t.item()),
                  "checked": "every rank's gathered image (coefficients, DC differences, both symbol arrays, "
                             "counts) vs pipeline.Encoder on the whole image, one extra group after the timing"}
        del full, xs, ref

    def counts_of(e):
        if world == 1:
            return e.counts
        if stream_gather:
            return e.whole.counts if e.whole is not None else None
        return e.enc.counts

    for e in encs:
        counts = counts_of(e)
        if counts is None:
            continue
        for ci, c in enumerate(counts.cpu().tolist()):
            pipeline.check_count(int(c), pipeline.CHANNELS[ci])
            assert c > 0, "empty symbol stream"
    mine = [e for e in encs if counts_of(e) is not None]
    symbols = [int(c) for c in counts_of(mine[0]).cpu().tolist()] if mine else None
    wire_flags = [int(e.wire_flag.item()) for e in encs if stream_gather]
    assert not any(wire_flags), "a coefficient outside its wire width"
    # per image: each grouped batch's span / the images it carried
    gather_us = (float(sum(a.elapsed_time(b) for a, b, _ in gather_ev) / sum(n for _, _, n in gather_ev)) * 1e3
                 if gather_ev else None)

    # the gather's own bound: xGMI links, not HBM.  Per group of N images each rank
    # receives (N - 1) / N of one image's blocks + DC stream over its N - 1 links to
    # the other ranks (one link per peer); a group's batch therefore needs at least
    # (image bytes / N) / link rate.  XGMI_LINK_GBS is the figure this build was
    # given (7 links x ~153 GB/s per MI355X), not a measurement.
    gather_link = None
    if gather_ev and world > 1:
        img_bytes = (encs[0].wire_bytes if stream_gather else
                     sum(encs[0].ranges[k][-1][1] * (64 * 2 + 4) for k in pipeline.CHANNELS))
        span_us = float(np.mean([a.elapsed_time(b) for a, b, n in gather_ev if n == world] or
                                [a.elapsed_time(b) for a, b, _ in gather_ev])) * 1e3
        per_link = img_bytes / world / (span_us * 1e-6) / 1e9
        gather_link = {"image_bytes": img_bytes, "bytes_per_link_per_group": img_bytes // world,
                       "group_span_us": round(span_us, 2), "per_link_GBps_achieved": round(per_link, 1),
                       "per_link_GBps_assumed_peak": XGMI_LINK_GBS,
                       "link_bound_us_per_image": round(img_bytes / world / (XGMI_LINK_GBS * 1e3) / world, 2)}

    # ---- roofline kernel: the DCT+quantize+zig-zag pass (one launch for the three
    # planes).  hic_dct_quant_rle_u8_batch hands the two HIP events to
    # hipExtLaunchKernelGGL: they hold that dispatch's begin / end timestamps.
    dct_us = float(np.mean([ev.elapsed_ms() for ev in timed_events])) * 1e3
    roof_note = "timed region (every 4th step)"
    dct_us_overlapped = None
    if len(streams) > 1 or gather:
        # with images overlapped on several streams (or a gather in the step) the DCT
        # shares the chip with other kernels, so its launch duration is no longer its
        # own: the roofline kernel is timed apart, on the same encoders and inputs,
        # one stream, right after the timed region
        dct_us_overlapped = dct_us
        # as in the timed region: back-to-back steps, the DCT timestamped on every
        # 4th (8 untimed steps first: the launches right after the overlapped region
        # run 5-15 % slow in the kernel trace, profiles/r01/bench_s2_kernel_trace_v9)
        iso = [device.KernelEvents() for _ in range(16)]
        for j in range(24):
            ev = iso[j - 8] if j >= 8 else None
            encs[j % len(encs)].encode(inputs[j % nin], dct_events=ev)
        torch.cuda.synchronize()
        dct_us = float(np.median([ev.elapsed_ms() for ev in iso])) * 1e3
        timed_events = iso
        roof_note = ("median of 16 single-stream encodes (each timestamped, after 8 untimed) right after the timed "
                     "region; the timed region overlaps images on %d stream(s)%s"
                     % (len(streams), " and grouped gathers" if gather else ""))
    # algorithmic bytes of the timed launch: the two-kernel chain's DCT reads 1 B and
    # writes 2 B per plane pixel; the fused kernel reads the RGB (3 B per image
    # pixel) and writes the same coefficients -- or, in the slot layout, the symbols
    # it emits (1 B length + 2 B value each) and the DC differences (4 B per block)
    slots = world == 1 and enc0.slots
    nsym_slots = slot_symbols(enc0) if slots else None
    if slots:
        roof_bytes = px_per_step_rank * 3 + 3 * nsym_slots + 4 * (dct_px // 64)
    else:
        roof_bytes = dct_px * 2 + (px_per_step_rank * 3 if fused else dct_px)
    achieved = roof_bytes / (dct_us * 1e-6) / 1e9

    # context for the gathered strong-scaling line: the same steps with the stream
    # left distributed (no gather), timed the same way -- the sharded encode itself
    # scales; the gathers are bound by the xGMI links
    no_gather = None
    if gather and not stream_gather:
        dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for g0 in range(0, args.steps, world):  # the same groups, encode_group only
            idx = list(range(g0, min(g0 + world, args.steps)))
            sharding.encode_group([encs[i % len(encs)] for i in idx], [inputs[i % nin] for i in idx],
                                  streams[((g0 // world) % 2) % len(streams)])
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t = torch.tensor([time.perf_counter() - t1], dtype=torch.float64,
                         device="cuda" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ng = float(t.item())
        no_gather = {"value": round(px_per_step_rank * world * args.steps / ng / 1e6, 2),
                     "ms_per_step": round(ng / args.steps * 1e3, 4),
                     "note": "same sharded encode and steps with the stream left distributed on the ranks "
                             "(no gather); not the headline value"}
    per_rank_rows = in_rows if world == 1 else encs[0].rows[1] - encs[0].rows[0]
    # read off the encoders now: the N > 1 extras below free them first
    gather_bytes = ((encs[0].wire_bytes if stream_gather else
                     sum(encs[0].ranges[k][-1][1] * (64 * 2 + 4) for k in pipeline.CHANNELS))
                    if gather else None)
    extra_sharded = None
    link_gbs = None
    if world > 1 and args.dist_backend == "nccl" and not args.same_device:
        # the per-link rate the gather model uses, measured here (not assumed)
        link_gbs = measure_link(rank, world)
    if world > 1 and not args.no_extras:
        # free the 8K run's buffers first (every rank holds ~1.2 GB of inputs)
        del encs, inputs, enc0
        torch.cuda.empty_cache()
        extra_sharded = extra_16k_roundtrip_sharded(rank, world, args.dist_backend)

    if rank == 0:
        total_px = px_per_step_rank * world * args.steps
        # value: the median of the 8 timed regions (each K steps between barriers and
        # synchronisations); the first region's rate beside it
        med_ms = float(np.median(region_ms))
        value = total_px / (med_ms * args.steps * 1e-3) / 1e6
        value_first = total_px / elapsed / 1e6
        pmc = load_pmc_traffic(fused, slots)
        cfg_idx = 2 if world == 1 else 3
        wl = ("%dx%d RGB -> YCrCb 4:2:0 full encode: colour+pyrDown, 8x8 DCT+quantize+zig-zag (3 planes), "
              "DC DPCM + AC RLE (3 planes)" % (W0, H0))
        if world > 1:
            wl += ("; %s: %s, block-row tile shards over %d ranks%s"
                   % ("BASELINE configs[3]" if (strong and args.workload == "8k") else "multi-GPU",
                      "one image split N ways" if strong else "one %d-row shard per rank" % H0, world,
                      (", each image's blocks gathered to one rank in the per-slot-width wire format with their RLE "
                       "tile records, where the whole image's DC / RLE stream is coded (image j of each group of "
                       "%d to rank j, the group's gathers in one grouped RCCL batch)" % world) if stream_gather else
                      (", each image's coefficient blocks + DC stream gathered to one rank (image j of each "
                       "group of %d to rank j, the group's gathers in one grouped RCCL batch)" % world)
                      if gather else ""))
        else:
            wl = ("BASELINE configs[2]: " if args.workload == "8k" else "") + wl
        out = {
            "metric": "Mpixels/s encode (DCT+quantize+zig-zag) at 8K; % HBM roofline, 1/2/4/8 GPU",
            "value": round(value, 2),
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(med_ms, 4),
            "value_first_region": round(value_first, 2),
            "ms_per_step_first_region": round(elapsed / args.steps * 1e3, 4),
            "value_is": "median over the %d timed regions of K steps" % len(region_ms),
            "ms_per_step_p10": round(float(np.percentile(region_ms, 10)), 4),
            "ms_per_step_p50": round(float(np.percentile(region_ms, 50)), 4),
            "ms_per_step_p90": round(float(np.percentile(region_ms, 90)), 4),
            "ms_per_step_regions": [round(v, 4) for v in region_ms],
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (uniform random uint8 RGB, resident in HBM)",
            "config": {
                "workload": wl,
                "image_hw": [H, W0],
                "per_rank_rows": per_rank_rows,
                "mode": "single" if world == 1 else args.mode,
                "streams": args.streams,
                "gather": "image j of each group of %d to rank j, one grouped RCCL batch per group (%s)"
                          % (world, "torch.distributed P2P" if rgather is None else "C-ABI hic_gather_bytes")
                          if gather else None,
                "gather_kind": args.gather_kind if gather else None,
                "gather_bytes_per_image": gather_bytes,
                "gather_us_per_image": None if gather_us is None else round(gather_us, 2),
                "gather_link": gather_link,
                "xgmi_link_gbs_measured": link_gbs,
                "without_gather": no_gather,
                "symbols_per_image_rank0": symbols,
                "gather_verify": verify,
                "stream_ends_on": "the gathering rank (whole-image scan + emit)" if stream_gather else
                ("every rank holds its slice" if world > 1 else "this GPU"),
                "dist_backend": None if world == 1 else args.dist_backend + (" (same device)" if args.same_device
                                                                              else ""),
                "parallelism": "dp%d tile-shard" % world,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": ("k_encode420<15,slots> (RGB -> YCrCb + 4:2:0 pyrDown + AAN DCT + quantize + zig-zag + the "
                           "AC symbols and DC differences of every RLE record, slot layout, in one launch; algorithmic "
                           "bytes = 3 B RGB read per pixel + 3 B per symbol written (%d symbols, the last image's) + "
                           "4 B per block's DC difference)" % nsym_slots if slots else
                           "k_encode420<15> (RGB -> YCrCb + 4:2:0 pyrDown + AAN DCT + quantize + zig-zag + RLE "
                           "tile records of the rank's image/shard in one launch; algorithmic bytes = 3 B RGB read + "
                           "2 B int16 written per Y / Cr / Cb coefficient)" if fused else
                           plane_kernel(15) + " (Y + Cr + Cb of the rank's image/shard in one launch: "
                           "DCT + quantize + zig-zag + RLE tile records, per-plane table; 1 B read + 2 B "
                           "written per plane pixel)"),
                "timed_launches": len(timed_events),
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": pmc.get("hbm_bytes_per_launch") if (pmc and world == 1 and args.workload == "8k")
                else None,
                "algorithmic_bytes": roof_bytes,
                "avg_launch_us": round(dct_us, 2),
                "timed_over": roof_note,
                "avg_launch_us_overlapped": None if dct_us_overlapped is None else round(dct_us_overlapped, 2),
            },
        }
        if world == 1:
            floors = measure_floors(slots=slots)
            out["memory_floors"] = floors
            out["roofline"]["device_copy_gbs"] = floors["device_copy_gbs"]
            out["roofline"]["frac_of_device_copy"] = round(achieved / floors["device_copy_gbs"], 4)
            if fused and args.workload == "8k":
                # the kernel's own byte pattern without its arithmetic, measured in this run
                fl = floors["encode420_pattern"]["median_launch_us"]
                out["roofline"]["memory_floor_us"] = fl
                out["roofline"]["frac_of_memory_floor"] = round(fl / dct_us, 4)
                out["roofline"]["memory_floor_source"] = ("memory_floors.encode420_pattern (%s, this run)" %
                                                          ("hic_probe_encode420_slots" if slots else
                                                           "hic_probe_encode420"))
            # the headline normalised by this box's own streaming copy rate (box-to-box
            # HBM / clock spread divides out): Mpix/s per GB/s of measured device copy
            out["value_per_copy_gbs"] = round(value / floors["device_copy_gbs"], 5)
        if not args.no_extras and world == 1:
            out["extra_configs"] = {"4k_rgb_encode": extra_4k_rgb_encode(),
                                    "3840x2160_rgb_encode": extra_ragged_rgb_encode(2160, 3840),
                                    # 1080 rows are not a multiple of 16 (the fused kernel's unit): 1088
                                    "1920x1088_rgb_encode": extra_ragged_rgb_encode(1088, 1920),
                                    "4k_luma_dct": extra_4k_luma(
                                        floor_us=floors["luma_pattern"]["4k_luma"]["median_launch_us"]),
                                    "8k_plane_dct": extra_8k_plane_dct(),
                                    "8k_luma_dct": extra_8k_plane_dct(
                                        luma_only=True, floor_us=floors["luma_pattern"]["1x"]["median_launch_us"]),
                                    "8k_luma_dct_back_to_back": extra_8k_luma_batched(
                                        floor_us_per_plane=round(floors["luma_pattern"]["4x"]["median_launch_us"] / 4,
                                                                 2)),
                                    "8k_jpeg_decode": extra_8k_jpeg_decode(),
                                    "8k_encode_from_host": extra_8k_encode_from_host(),
                                    "16k_roundtrip": extra_16k_roundtrip(),
                                    "8k_reference_api": extra_8k_reference_api()}
        if extra_sharded is not None:
            out["extra_configs"] = {"16k_roundtrip": extra_sharded}
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(args.cpu_budget_s)
        elif not args.no_cpu_baseline:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if rgather is not None:
        torch.cuda.synchronize()
        rgather.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
