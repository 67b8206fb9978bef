/*
 * hiccup_hip.h -- C-ABI of libhiccup_hip.so, the MI355X (gfx950) implementation
 * of hiccup's 8x8 block DCT -> quantize -> zig-zag -> DC-DPCM / AC-RLE encode
 * path and its inverse.
 *
 * The reference (nhomble/hiccup) is pure Python and has no FFI: its drop-in
 * boundary is the Python function surface listed below.  Each entry point here
 * is what that surface binds (through ctypes, see hiccup_amd/_lib.py and
 * INTEGRATION.md); the comment on each cites the reference function it
 * replaces (/root/reference/<file>:<line>).
 *
 * Conventions (all entry points):
 *   - plain pointers and sizes; no Python / torch types cross the ABI;
 *   - every array pointer is a DEVICE pointer (hipMalloc / torch CUDA tensor)
 *     unless the parameter name starts with h_;
 *   - caller-allocated outputs; the library never allocates on the hot path;
 *   - `stream` is a hipStream_t passed as void* (NULL = legacy default stream);
 *     calls are asynchronous on that stream and may be captured in a hipGraph;
 *   - return value: HIC_OK (0) or a negative HIC_ERR_*; hic_last_error() gives
 *     the message of the last failure on the calling thread.  Nothing throws.
 */
#ifndef HICCUP_HIP_H
#define HICCUP_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HIC_ABI_VERSION 4

#define HIC_OK 0
#define HIC_ERR_ARG (-1)      /* bad shape / pointer / enum: the reference asserts or raises */
#define HIC_ERR_HIP (-2)      /* HIP runtime failure (launch, memcpy) */
#define HIC_ERR_CAPACITY (-3) /* caller's output buffer too small */
#define HIC_COUNT_SCAN_TIMEOUT INT64_MIN /* *d_count of an RLE encode whose scan hand-off timed out */
#define HIC_COUNT_WIRE_OVERFLOW (INT64_MIN + 1) /* a gathered stream whose wire segment carried a sender's
                                                   out-of-width flag (hic_wire_pack_i16): the stream is invalid */

/* model.QTables (model.py:25-27) -> quantization.table (quantization.py:14-37) */
#define HIC_TABLE_LUMINANCE 0
#define HIC_TABLE_CHROMINANCE 1

/* Coefficient layouts in HBM.
 * RASTER_I32: the reference's "coefficient image" (transform.dct_channel output,
 *             transform.py:182-193): int32 H x W, block (i,j) coef (u,v) at [8i+u][8j+v].
 * RASTER_I16: same, int16 (lossless: |q| <= 3277).
 * ZIGZAG_I16: block-major stream: for every 8x8 block in raster block order
 *             (padded blocks included), 64 int16 in transposed zig-zag order
 *             (transform.zigzag, transform.py:106-135); coefficients whose
 *             position falls outside H x W are 0 (jpeg_encode re-splits the
 *             cropped coefficient image with zero padding, codec.py:287-294). */
#define HIC_LAYOUT_RASTER_I32 0
#define HIC_LAYOUT_RASTER_I16 1
#define HIC_LAYOUT_ZIGZAG_I16 2

int hic_abi_version(void);
/* Copies the last error message of this thread into buf (NUL-terminated). */
int hic_last_error(char *h_buf, size_t n);
/* Number of visible HIP devices. */
int hic_device_count(int *h_n);

/* Code-path selection for A/B tests (not part of the reference's surface).
 * Every selectable path is bit-exact: a knob never changes results, only which
 * kernel variant computes them.  The library reads no environment variables.
 * Values are process-wide; -1 restores the default. */
#define HIC_KNOB_DCT_PATH 0         /* forward DCT of aligned planes: 1 / 2 float64 AAN (the default; 2's LDS-DMA prefetch form, measured within noise in round 6, was removed), 0 exact replica; 3 / 4 (packed float32, two lanes per block: removed in round 5) are refused */
#define HIC_KNOB_DCT_WAVES_PER_CU 1 /* forward DCT persistent grid (waves per CU; 0 = one wave per set) */
#define HIC_KNOB_COLOR_TILED 2      /* 1: LDS-tiled colour kernels instead of the wave-walk ones */
#define HIC_KNOB_COLOR_SEG 3        /* wave-walk colour: chroma rows per segment (8 default, 16) */
#define HIC_KNOB_COLOR_NT 4         /* 1: nontemporal plane stores in the colour kernel */
#define HIC_KNOB_RLE_NT 5           /* 0: plain (not nontemporal) symbol stores in the RLE emit */
#define HIC_KNOB_RLD_NT 6           /* 1: nontemporal block stores in the RLE decode */
#define HIC_KNOB_RLD_GENERIC 7      /* 1: the generic (any block size) RLE decode */
#define HIC_KNOB_DEV 8              /* dev builds only (-DHIC_DEV): timing bits that skip work; refused otherwise */
/* knobs 9-12 were retired in rounds 4-5 (encode waves / nontemporal stores / integer-MFMA
 * transforms: measured slower, removed); hic_set_knob refuses any value but -1 for them
 * (-1, the default, is a no-op: resetting every knob 0 .. HIC_KNOB_COUNT - 1 works) */
#define HIC_KNOB_ENCODE_ORDER 13     /* hic_encode420_u8 unit order: 0 row-major; + 2: workgroups remapped XCD-major (neighbouring units on one XCD's L2); + 4: odd unit rows run their colour rows bottom-up (the halo rows two unit rows share fetched at the same time); default 6; odd values refused */
/* 14, 15: retired in round 5 with the packed-float32 transforms (refused, -1 a no-op) */
#define HIC_KNOB_COUNT 16
int hic_set_knob(int knob, int value);
int hic_get_knob(int knob, int *h_value);
/* Synchronises `stream`; returns HIC_ERR_HIP if an earlier async launch failed. */
int hic_stream_sync(void *stream);

/* ---- measurement probes (bench.py; no reference counterpart: SURVEY.md 8(d) asks
 *      for the box's device-copy bandwidth beside the roofline).  Memory-only, no
 *      arithmetic; ev_start / ev_stop (hipEvent_t or NULL) receive the launch's own
 *      begin / end timestamps.
 *  hic_probe_copy: dst[0, bytes) = src[0, bytes) (16-byte aligned, bytes % 16 == 0),
 *    16 B per lane loads, nontemporal stores: the streaming copy rate.
 *  hic_probe_plane: the forward plane pass's byte pattern without the DCT: a uint8
 *    H x W plane (pitch W, multiples of 8) read as 8x8 blocks (one per lane), 128 B
 *    per block written to out (nblk x 64 int16) through the LDS stage and 1 KiB
 *    nontemporal stores of k_dct_planes, persistent grid: the pass's memory floor.
 *  waves_per_cu: persistent grid size (0 = default: 16 for the copy, 12 for the plane).
 *  hic_probe_encode420: hic_encode420_u8's byte pattern without its arithmetic, on a
 *    whole H x W RGB image (W % 512 == 0, H % 16 == 0): the same grid, unit order
 *    (knob encode_order) and 19 row loads per 16-row unit, the LDS stage and 1 KiB
 *    nontemporal stores of the Y / Cr / Cb blocks (coef_*: the encoder's outputs'
 *    sizes) and one 24 B record per tile (rec_y: H/8 * W/512 records, rec_c: H/16 *
 *    W/512): the fused kernel's memory floor. */
int hic_probe_copy(const void *src, void *dst, int64_t bytes, int waves_per_cu, void *stream, void *ev_start,
                   void *ev_stop);
int hic_probe_plane(const uint8_t *plane, int64_t H, int64_t W, int16_t *out, int waves_per_cu, void *stream,
                    void *ev_start, void *ev_stop);
int hic_probe_encode420(const uint8_t *rgb, int64_t H, int64_t W, int16_t *coef_y, int16_t *coef_cr, int16_t *coef_cb,
                        int64_t *rec_y, int64_t *rec_c, void *stream, void *ev_start, void *ev_stop);

/* ---- forward transform: replaces transform.dct_channel (transform.py:182-193) =
 *      offset -128 (:186), split_matrix/pad (:33-42), dct2 (:67-84, scipy pocketfft
 *      DCT-II bit-exact), jpeg_quantize (quantization.py:47-52,80-81:
 *      round-half-even(b / T)), merge_blocks/crop (:45-64).
 *  plane: uint8 H x W with row pitch `stride` bytes.  out: per `layout`. */
int hic_dct_quant_u8(const uint8_t *plane, int64_t H, int64_t W, int64_t stride, int table_id,
                     int layout, void *out, void *stream);
/* Same, and the kernel's own begin / end timestamps are recorded into two
 * events from hic_event_create (hipExtLaunchKernelGGL): the measurement
 * bench.py reports as the kernel's launch duration.  Null events = untimed. */
int hic_dct_quant_u8_timed(const uint8_t *plane, int64_t H, int64_t W, int64_t stride, int table_id,
                           int layout, void *out, void *stream, void *ev_start, void *ev_stop);
/* Forward transform to HIC_LAYOUT_ZIGZAG_I16 with the RLE tile pass of
 * hic_rle_encode_i16 (its first kernel) fused into the epilogue: the per-tile
 * records land in `rle_workspace` (hic_rle_workspace_bytes(nblk, 64) bytes).
 * Follow with hic_rle_encode_i16_tiles (and, for a row shard, first
 * hic_rle_shard_summary_tiles).  Events as in hic_dct_quant_u8_timed (nullable). */
int hic_dct_quant_rle_u8(const uint8_t *plane, int64_t H, int64_t W, int64_t stride, int table_id, int max_len,
                         int16_t *out, void *rle_workspace, void *stream, void *ev_start, void *ev_stop);
/* hic_dct_quant_rle_u8 for up to 16 planes (the Y, Cr, Cb of one image, or the
 * planes of consecutive images): ONE launch, a persistent grid over all their
 * 64-block sets (each plane's table read at run time).  Each job names its plane,
 * table, ZIGZAG_I16 output and RLE workspace; rle_workspace NULL for every job
 * (round 5) = the records-free pass (DCT + quantize + zig-zag only, no tile
 * records).  Events (nullable) time that launch.  Ragged planes (H or W not a
 * multiple of 8) take separate launches. */
typedef struct {
  const uint8_t *plane;
  int64_t H, W, stride;
  int table_id;
  int16_t *out;
  void *rle_workspace;
} hic_dct_plane_job;
int hic_dct_quant_rle_u8_batch(int n, const hic_dct_plane_job *jobs, int max_len, void *stream, void *ev_start,
                               void *ev_stop);
/* ---- fused 4:2:0 encode front end: replaces compression.jpeg_compression's
 *      cvtColor(RGB2YCrCb) + pyrDown(Cr), pyrDown(Cb) + dct_channel x3
 *      (compression.py:16-39, transform.py:151-157,182-193) and the zig-zag of
 *      codec.jpeg_encode (codec.py:286-301), in ONE kernel: the planes never reach
 *      HBM.  Output identical to hic_rgb_to_ycrcb420_rows + hic_dct_quant_rle_u8_batch.
 *  rgb_rows: image rows [in_row0, in_row0 + in_rows) of an H x W x 3 uint8 image
 *  (8-byte aligned), covering output rows [out_row0, out_row0 + out_rows) plus the
 *  pyrDown halo (2 rows above, 1 below, clamped to the image).  W % 16 == 0,
 *  H % 16 == 0, out_row0 / out_rows multiples of 16.
 *  coef_*: ZIGZAG_I16 blocks of the output rows' Y ((out_rows/8) x (W/8) blocks) and
 *  Cr / Cb ((out_rows/16) x (W/16)).  ws_* (all or none): RLE workspaces that
 *  receive the tile records for hic_rle_encode_i16_tiles_batch -- Y one per
 *  64-block tile (records_per_tile 1); Cr / Cb one per 32-block half tile
 *  (records_per_tile 2) when W % 512 == 0, else one per 64-block tile
 *  (records_per_tile 1: a tile pass after the launch); max_len as there.
 *  ev_start / ev_stop (optional): events carrying the fused launch's own begin /
 *  end timestamps. */
int hic_encode420_u8(const uint8_t *rgb_rows, int64_t in_row0, int64_t in_rows, int64_t H, int64_t W,
                     int64_t out_row0, int64_t out_rows, int16_t *coef_y, int16_t *coef_cr, int16_t *coef_cb,
                     void *ws_y, void *ws_cr, void *ws_cb, int max_len, void *stream, void *ev_start,
                     void *ev_stop);
/* hic_encode420_u8 with one RLE record per strip segment for any W % 16 == 0 (round
 * 4): each block row is cut into 512-pixel strips (64 Y / 32 chroma blocks per
 * record), the last strip's record covering what remains -- no tile pass after the
 * launch.  Identical to hic_encode420_u8 when W % 512 == 0.  Consume the records with
 * hic_rle_encode_i16_rows_batch (row_blocks W/8 for Y, W/16 for Cr / Cb,
 * records_per_tile 1 / 2).  ws_bytes_y / ws_bytes_c: the sizes of ws_y and of each of
 * ws_cr / ws_cb; at least hic_rle_rows_workspace_bytes(nblk, row_blocks,
 * records_per_tile) of the plane (a narrow image has more records than 64-block
 * tiles), else HIC_ERR_ARG and nothing is launched (round 5). */
int hic_encode420_seg_u8(const uint8_t *rgb_rows, int64_t in_row0, int64_t in_rows, int64_t H, int64_t W,
                         int64_t out_row0, int64_t out_rows, int16_t *coef_y, int16_t *coef_cr, int16_t *coef_cb,
                         void *ws_y, void *ws_cr, void *ws_cb, int64_t ws_bytes_y, int64_t ws_bytes_c, int max_len,
                         void *stream, void *ev_start, void *ev_stop);
/* hic_encode420_batch_u8: n <= 8 hic_encode420_u8 calls in ONE launch (the row
 * shards of a multi-GPU group, one per image: a shard alone fills a sixth of the chip
 * at N = 8).  Each job as hic_encode420_u8's arguments; with workspaces, W % 512 == 0
 * (the records come from the kernel).  Every job is checked before the launch; the
 * events (nullable) time the whole launch. */
typedef struct {
  const uint8_t *rgb_rows;
  int64_t in_row0, in_rows, H, W, out_row0, out_rows;
  int16_t *coef_y, *coef_cr, *coef_cb;
  void *ws_y, *ws_cr, *ws_cb;
} hic_encode420_job;
int hic_encode420_batch_u8(int n, const hic_encode420_job *jobs, int max_len, void *stream, void *ev_start,
                           void *ev_stop);
/* ---- slot-layout encode (round 6): hic_encode420_u8 + hic_rle_encode_i16_tiles_batch
 *      (compression.jpeg_compression's transform + codec.jpeg_encode's DC DPCM and AC
 *      RLE, compression.py:16-39, codec.py:47-99,286-301) with the symbols written by
 *      the fused kernel itself: the int16 coefficients never reach HBM and no emit
 *      kernel re-reads them.
 *  Slot layout of a channel: its blocks form records of 64 (Y, records_per_tile 1)
 *  or 32 (Cr / Cb, records_per_tile 2) consecutive blocks; record r owns symbols
 *  [r * cap, r * cap + n_r) of slot_len / slot_val (cap = 63 x its blocks, so the
 *  slot arrays hold nblk * 63 entries).  The channel's symbol stream -- exactly
 *  what hic_rle_encode_i16 writes -- is, over the records in order, nfill_r fillers
 *  (max_len - 1, 0) followed by the slot's n_r symbols, then the EOB (0, 0) when
 *  the stream ends in a zero.  max_len must be 15 (4-bit lengths in the kernel's
 *  stage).  Whole images only, W % 512 == 0, H % 16 == 0.
 *  hic_encode420_slots_u8: jobs[0..2] = Y, Cr, Cb (nblk (H/8)(W/8) and
 *    (H/16)(W/16), records_per_tile 1 and 2): the slots, dc_diff (each record's first
 *    block still holding its raw DC) and the records in `workspace`.  Events as in
 *    hic_encode420_u8 (nullable).
 *  hic_rle_slots_close: the records' scan: writes each record's first symbol length,
 *    subtracts the previous record's last DC from its first block's dc_diff, fills
 *    d_index (4 int32 per record: n_r, P_r = the record-relative AC position after
 *    which its first symbol's zeros start (<= 0: the run is carried in), pdc_r = the
 *    DC of the block before the record, nfill_r), *d_count (the stream's symbols,
 *    fillers and EOB included; HIC_COUNT_SCAN_TIMEOUT if a hand-off timed out) and
 *    the EOB into sym_len / sym_val.
 *  hic_rle_slots_compact: the contiguous stream into sym_len / sym_val (sym_cap >=
 *    the count; after hic_rle_slots_close).
 *  Decoders: hic_rle_decode_i16_slots / hic_rle_decode_idct_u8_slots[_pair] /
 *    hic_rle_decode_idct_rgb_slots are their *_indexed counterparts reading the slots
 *    through d_index (records_per_tile as the job's; *d_status = nblk * 63, or -1
 *    when *d_nsym < 1). */
typedef struct {
  int64_t nblk;             /* blocks of the channel */
  int64_t records_per_tile; /* 1: a record per 64 blocks; 2: per 32 blocks */
  uint8_t *slot_len;        /* nblk * 63 bytes, 16-byte aligned */
  int16_t *slot_val;        /* nblk * 63 int16, 16-byte aligned */
  int32_t *dc_diff;         /* nblk */
  int32_t *d_index;         /* 4 int32 per record (hic_rle_slots_close) */
  void *workspace;          /* hic_rle_slots_workspace_bytes(nblk, records_per_tile) bytes,
                               zero-filled before its first use */
  int64_t workspace_bytes;
  int64_t *d_count;         /* device int64: the stream's symbol count */
  uint8_t *sym_len;         /* the contiguous stream: its EOB (close) and the rest (compact) */
  int16_t *sym_val;
  int64_t sym_cap;
} hic_slot_job;
size_t hic_rle_slots_workspace_bytes(int64_t nblk, int records_per_tile);
int hic_encode420_slots_u8(const uint8_t *rgb, int64_t H, int64_t W, const hic_slot_job *jobs, int max_len,
                           void *stream, void *ev_start, void *ev_stop);
int hic_rle_slots_close(int n, const hic_slot_job *jobs, int max_len, void *stream);
int hic_rle_slots_compact(int n, const hic_slot_job *jobs, int max_len, void *stream);
int hic_rle_decode_i16_slots(const uint8_t *slot_len, const int16_t *slot_val, const int64_t *d_nsym,
                             const int32_t *dc_diff, int64_t nblk, int records_per_tile, const int32_t *d_index,
                             int16_t *blocks, int64_t *d_status, void *stream);
int hic_rle_decode_idct_u8_slots(const uint8_t *slot_len, const int16_t *slot_val, const int64_t *d_nsym,
                                 const int32_t *dc_diff, const int32_t *d_index, int records_per_tile, int64_t H,
                                 int64_t W, int table_id, uint8_t *out, int64_t out_stride, int64_t *d_status,
                                 void *stream);
int hic_rle_decode_idct_u8_slots_pair(const uint8_t *const *h_slot_len, const int16_t *const *h_slot_val,
                                      const int64_t *const *h_d_nsym, const int32_t *const *h_dc_diff,
                                      const int32_t *const *h_d_index, int records_per_tile, int64_t H, int64_t W,
                                      int table_id, uint8_t *const *h_out, int64_t out_stride,
                                      int64_t *const *h_d_status, void *stream);
int hic_rle_decode_idct_rgb_slots(const uint8_t *slot_len, const int16_t *slot_val, const int64_t *d_nsym,
                                  const int32_t *dc_diff, const int32_t *d_index, int records_per_tile, int64_t H,
                                  int64_t W, const uint8_t *cr, const uint8_t *cb, uint8_t *rgb, int64_t rgb_stride,
                                  int64_t *d_status, void *stream);
/* hic_probe_encode420_slots: the slot-layout kernel's byte pattern, memory only (a
 * probe as hic_probe_encode420, bench.py's in-run floor): the same grid, unit order
 * and row loads, and per record the n_r symbols its jobs' d_index holds from an
 * earlier hic_encode420_slots_u8 + hic_rle_slots_close into the same buffers (16 +
 * 32 B nontemporal stores per 16 symbols), the DC differences, the record and its
 * last DC, with garbage values. */
int hic_probe_encode420_slots(const uint8_t *rgb, int64_t H, int64_t W, const hic_slot_job *jobs, void *stream,
                              void *ev_start, void *ev_stop);
/* Timing events (hipEvent_t handles) for the *_timed entry points. */
int hic_event_create(void **h_event);
int hic_event_destroy(void *event);
/* Records an event on a stream (hipEventRecord). */
int hic_event_record(void *event, void *stream);
/* Milliseconds between two completed events (synchronises on `stop`). */
int hic_event_elapsed_ms(void *start, void *stop, float *h_ms);

/* ---- inverse transform: replaces transform.inv_dct_channel (transform.py:169-179) =
 *      split (:174), invert_jpeg_quantize q*T (quantization.py:55-57), idct2
 *      (:87-103, pocketfft DCT-III bit-exact, /256), merge/crop, +128,
 *      astype(uint8) (truncate toward zero, wrap mod 256).
 *  coef: per `layout` (H x W coefficient image, or the zig-zag block stream of it).
 *  out : uint8 H x W with row pitch out_stride. */
int hic_dequant_idct_u8(const void *coef, int layout, int64_t H, int64_t W, int table_id,
                        uint8_t *out, int64_t out_stride, void *stream);

/* ---- block-level helpers on batches of 8x8 blocks (float64 bit-exact):
 *  hic_dct2_f64  = transform.dct2  (transform.py:67-84)  in[nblk][8][8] -> out
 *  hic_idct2_f64 = transform.idct2 (transform.py:87-103, includes /256)
 *  hic_quantize_f64   = quantization.jpeg_quantize (quantization.py:47-52,80-81) -> int32
 *  hic_dequantize_i32 = quantization.invert_jpeg_quantize (quantization.py:55-57) -> int64 */
int hic_dct2_f64(const double *in, int64_t nblk, double *out, void *stream);
int hic_idct2_f64(const double *in, int64_t nblk, double *out, void *stream);
int hic_quantize_f64(const double *in, int64_t nblk, int table_id, int32_t *out, void *stream);
int hic_dequantize_i32(const int32_t *in, int64_t nblk, int table_id, int64_t *out, void *stream);

/* ---- colour + chroma resampling (compression.py:21,56; transform.py:151-166).
 *      OpenCV 8U semantics restated (parity UNPINNED: cv2 absent).
 *  hic_rgb_to_ycrcb420: rgb H x W x 3 (pitch W*3) -> y H x W, cr/cb (H/2) x (W/2)
 *      = cvtColor(RGB2YCrCb) then pyrDown(dstsize=(W/2,H/2)) on Cr and Cb. */
int hic_rgb_to_ycrcb420(const uint8_t *rgb, int64_t H, int64_t W, uint8_t *y, uint8_t *cr,
                        uint8_t *cb, void *stream);
/* Row-shard form for tile-sharded encode: rgb_rows holds image rows
 * [in_row0, in_row0 + in_rows) of an H x W image (the shard plus the 2-row pyrDown
 * halo on each side, clipped at the image border); writes Y rows
 * [out_row0, out_row0 + out_rows) and chroma rows [out_row0/2, out_row0/2 + ceil..)
 * to y / cr / cb (relative to the shard).  out_row0 must be even; reflect-101 is
 * applied only at the true image border, so shard outputs equal the whole-image rows. */
int hic_rgb_to_ycrcb420_rows(const uint8_t *rgb_rows, int64_t in_row0, int64_t in_rows, int64_t H,
                             int64_t W, int64_t out_row0, int64_t out_rows, uint8_t *y, uint8_t *cr,
                             uint8_t *cb, void *stream);
/* cv2.cvtColor(RGB2YCrCb), full resolution, no resampling. */
int hic_rgb_to_ycrcb(const uint8_t *rgb, int64_t H, int64_t W, uint8_t *y, uint8_t *cr,
                     uint8_t *cb, void *stream);
/* transform.down_sample = cv2.pyrDown(src, dstsize=(DW, DH)) */
int hic_pyr_down_u8(const uint8_t *src, int64_t H, int64_t W, uint8_t *dst, int64_t DH,
                    int64_t DW, void *stream);
/* transform.up_sample = cv2.pyrUp(src, dstsize=(DW, DH)) */
int hic_pyr_up_u8(const uint8_t *src, int64_t H, int64_t W, uint8_t *dst, int64_t DH,
                  int64_t DW, void *stream);
/* compression.jpeg_decompression tail (compression.py:47-56): pyrUp cr/cb (h x w) to
 * 2h x 2w, crop y (row pitch y_stride) to that (transform.force_merge,
 * transform.py:269-277), cvtColor(YCrCb2RGB) -> rgb (2h) x (2w) x 3. */
int hic_ycrcb420_to_rgb(const uint8_t *y, int64_t y_stride, const uint8_t *cr, const uint8_t *cb,
                        int64_t h, int64_t w, uint8_t *rgb, void *stream);
/* Row-range form of hic_ycrcb420_to_rgb for a tile shard's decode
 * (compression.jpeg_decompression on rows of the image, compression.py:42-56):
 * chroma rows [s0, s1) of the h x w chroma planes -> RGB rows [2 s0, 2 s1).
 * y and rgb point at output row 2 s0; cr / cb hold c_rows chroma rows starting at
 * image chroma row c_row0, which must cover the pyrUp halo [max(0, s0 - 1),
 * min(h, s1 + 1)). */
int hic_ycrcb420_to_rgb_rows(const uint8_t *y, int64_t y_stride, const uint8_t *cr, const uint8_t *cb,
                             int64_t c_row0, int64_t c_rows, int64_t h, int64_t w, int64_t s0,
                             int64_t s1, uint8_t *rgb, void *stream);

/* ---- generic block split + zig-zag for any block size N (codec.jpeg_encode with
 *      settings.JPEG_BLOCK_SIZE != 8, codec.py:287-294; transform.zigzag):
 *      raster int32 H x W -> out[nblk][N*N] int32, zero padding.  And its inverse
 *      (izigzag + merge_blocks + crop, codec.py:415-425). */
int hic_zigzag_blocks_i32(const int32_t *raster, int64_t H, int64_t W, int N, int32_t *out,
                          void *stream);
/* hic_zigzag_blocks_i32 for N = 8 into int16 blocks (codec.jpeg_encode's fast path,
 * then hic_rle_encode_i16): *d_wide (device int32) = 1 if any value of the raster is
 * outside int16 -- those blocks are then not exact and the caller re-runs the plane
 * through the int32 calls -- else 0. */
int hic_zigzag8_blocks_i16(const int32_t *raster, int64_t H, int64_t W, int16_t *out, int32_t *d_wide, void *stream);
int hic_izigzag_blocks_i32(const int32_t *blocks, int64_t H, int64_t W, int N, int32_t *raster,
                           void *stream);

/* ---- entropy front end: DC DPCM (codec.differential_coding, codec.py:47-52) and
 *      global AC run-length coding (codec.run_length_coding, codec.py:55-99) over
 *      the AC stream of `nblk` blocks of `block_len` coefficients (AC = slots
 *      1..block_len-1 of every block, blocks in order).
 *  Symbols are written SoA: sym_len[i] zeros followed by sym_val[i]; a trailing
 *  zero run becomes the single EOB (0,0); runs >= max_len are split into
 *  (max_len-1, 0) fillers (max_len 0 = no split, reference max_len=None).
 *  *d_count (device int64) receives the symbol count, HIC_COUNT_SCAN_TIMEOUT if a
 *  cross-workgroup scan hand-off timed out (never expected), or -(needed) if sym_cap was
 *  too small (nothing past sym_cap is written).
 *  Sharded use (tile-sharded image, one stream across ranks): d_stitch (device,
 *  int64[4] = {carry_zeros, emit_eob, has_prev_dc, prev_dc}) or NULL for a whole
 *  stream {0, 1, 0, 0}.  hic_rle_shard_summary fills d_summary (device int64[4]
 *  = {trailing_zeros, has_nonzero, first_dc, last_dc}) for the exchange step. */
/* The workspace must be zero-filled before its first use (it carries tagged
 * hand-off records between the scan's workgroups); it may be reused after. */
size_t hic_rle_workspace_bytes(int64_t nblk, int block_len);
int hic_rle_shard_summary_i16(const int16_t *blocks, int64_t nblk, int block_len,
                              void *workspace, int64_t *d_summary, void *stream);
int hic_rle_encode_i16(const int16_t *blocks, int64_t nblk, int block_len, int max_len,
                       const int64_t *d_stitch, int32_t *dc_diff, uint8_t *sym_len,
                       int16_t *sym_val, int64_t sym_cap, int64_t *d_count, void *workspace,
                       void *stream);
/* hic_rle_encode_i16 for int16 zig-zag blocks of 64 whose tile records are already
 * in `workspace` (hic_dct_quant_rle_u8): runs only the scan and emit kernels. */
int hic_rle_encode_i16_tiles(const int16_t *blocks, int64_t nblk, int max_len, const int64_t *d_stitch,
                             int32_t *dc_diff, uint8_t *sym_len, int16_t *sym_val, int64_t sym_cap,
                             int64_t *d_count, void *workspace, void *stream);
/* The tile records hic_rle_encode_i16_tiles reads (one per 64-block tile, into
 * `workspace`) of int16 zig-zag blocks of 64 (16-byte aligned) that a transform
 * did not record: codec.run_length_coding's per-tile state (codec.py:55-99). */
int hic_rle_tile_records_i16(const int16_t *blocks, int64_t nblk, int max_len, void *workspace, void *stream);
/* hic_rle_encode_i16_tiles for up to 4 streams (e.g. the Y, Cr, Cb planes of one
 * image) in two launches in total; all with the same max_len. */
typedef struct {
  const int16_t *blocks;
  int64_t nblk;
  const int64_t *d_stitch;
  int32_t *dc_diff;
  uint8_t *sym_len;
  int16_t *sym_val;
  int64_t sym_cap;
  int64_t *d_count;
  void *workspace;
  int64_t records_per_tile; /* 0 or 1: one tile record per 64 blocks (hic_dct_quant_rle_u8);
                               2: one per 32 blocks (hic_encode420_u8's chroma planes) */
  int64_t workspace_bytes;  /* size of `workspace` (round 5): checked against the job's
                               records when > 0; required by hic_rle_encode_i16_rows_batch */
  int64_t *d_index;         /* optional (round 5), hic_rle_encode_i16_tiles_batch only, no
                               d_stitch: the emit also writes the job's tile index, exactly
                               what hic_rle_tile_index_i16 writes ((nblk+63)/64 x 3 int64),
                               with no launch of its own; NULL: none */
} hic_rle_job16;
int hic_rle_encode_i16_tiles_batch(int n, const hic_rle_job16 *jobs, int max_len, void *stream);
/* The same over records per row segment (round 4; hic_encode420_seg_u8's records):
 * job k's blocks are rows of h_row_blocks[k] blocks (dividing nblk), each row cut into
 * tiles of 64 blocks from its start (the last one shorter) with records_per_tile
 * records per full tile (1: per tile; 2: per 32 blocks, the last one shorter).  With
 * h_row_blocks[k] % 64 == 0 identical to hic_rle_encode_i16_tiles_batch. */
int hic_rle_encode_i16_rows_batch(int n, const hic_rle_job16 *jobs, const int64_t *h_row_blocks, int max_len,
                                  void *stream);
/* Workspace bytes of a row-segment job (hic_encode420_seg_u8 /
 * hic_rle_encode_i16_rows_batch): nblk blocks in rows of row_blocks, records_per_tile
 * as the job's; never less than hic_rle_workspace_bytes(nblk, 64). */
size_t hic_rle_rows_workspace_bytes(int64_t nblk, int64_t row_blocks, int records_per_tile);
/* hic_rle_shard_summary_i16 from the tile records of hic_dct_quant_rle_u8. */
int hic_rle_shard_summary_tiles(const int16_t *blocks, int64_t nblk, void *workspace, int64_t *d_summary,
                                void *stream);
/* The same for records_per_tile 1 or 2 (hic_encode420_u8's chroma records). */
int hic_rle_shard_summary_records(const int16_t *blocks, int64_t nblk, int records_per_tile,
                                  void *workspace, int64_t *d_summary, void *stream);
int hic_rle_shard_summary_i32(const int32_t *blocks, int64_t nblk, int block_len,
                              void *workspace, int64_t *d_summary, void *stream);
int hic_rle_encode_i32(const int32_t *blocks, int64_t nblk, int block_len, int max_len,
                       const int64_t *d_stitch, int32_t *dc_diff, int32_t *sym_len,
                       int32_t *sym_val, int64_t sym_cap, int64_t *d_count, void *workspace,
                       void *stream);
/* codec.run_length_coding (codec.py:55-99) on an arbitrary 1-D int32 array of n
 * elements (n = 0 gives the single EOB).  Same symbol / count conventions. */
int hic_rle_stream_encode_i32(const int32_t *arr, int64_t n, int max_len, int32_t *sym_len,
                              int32_t *sym_val, int64_t sym_cap, int64_t *d_count, void *workspace,
                              void *stream);
/* Computes this rank's d_stitch from all ranks' summaries (device int64, rank r's
 * 4 values at d_all_summaries[r * rank_stride], e.g. after an all-gather): carry = trailing zeros of the preceding ranks back to
 * the last one holding a nonzero; EOB only on the last rank; prev_dc = last DC of
 * rank-1. */
int hic_rle_stitch(const int64_t *d_all_summaries, int world, int rank, int rank_stride,
                   int64_t *d_stitch, void *stream);

/* ---- entropy front end, inverse: codec.decode_run_length (codec.py:102-113) +
 *      utils.group_tuples (:412) + utils.invert_differences (utils.py:66-73) +
 *      [dc, *ac] reassembly (codec.py:415-421) -> zig-zag blocks (nblk x block_len).
 *  *d_status (device int64) receives the decoded AC length (EOB zero-fill
 *  included); the reference asserts unless it equals nblk*(block_len-1). */
size_t hic_rld_workspace_bytes(int64_t nsym, int64_t nblk);
int hic_rle_decode_i16(const uint8_t *sym_len, const int16_t *sym_val, int64_t nsym,
                       const int32_t *dc_diff, int64_t nblk, int block_len, int16_t *blocks,
                       int64_t *d_status, void *workspace, void *stream);
/* Encoder-side tile index (no reference counterpart: it lets a device-to-device
 * decoder skip the symbol-tile pass, the scans and the DC chain that find block
 * boundaries in a bare stream).  hic_rle_tile_index_i16: after
 * hic_rle_encode_i16_tiles[_batch] (its workspace holds the scan's offsets), per
 * 64-block tile t: d_index[3t] = offset of the tile's first symbol, [3t + 1] = the
 * stream's last nonzero AC position before the tile (-1: none), [3t + 2] = DC of
 * block 64t - 1 (0 for t = 0).  records_per_tile as the encode job's.
 * hic_rle_decode_i16_indexed: hic_rle_decode_i16's result (codec.py:102-113,
 * 397-421 for one channel, 64-slot int16 blocks) from such an index: one wave per
 * 64-block tile; *d_status as hic_rle_decode_i16's (-1 when *d_nsym < 1).
 * Whole streams only (no stitch).  d_nsym: the symbol count on the device (the
 * encoder's d_count, EOB included): no host round trip between encode and decode. */
int hic_rle_tile_index_i16(const int16_t *blocks, int64_t nblk, int records_per_tile, const void *workspace,
                           int64_t *d_index, void *stream);
int hic_rle_decode_i16_indexed(const uint8_t *sym_len, const int16_t *sym_val, const int64_t *d_nsym,
                               const int32_t *dc_diff, int64_t nblk, const int64_t *d_index, int16_t *blocks,
                               int64_t *d_status, void *stream);
/* hic_rle_decode_i16_indexed + hic_dequant_idct_u8 in ONE kernel: each wave
 * assembles its 64-block tile in LDS and every lane inverts its block from there
 * into the uint8 H x W plane `out` (row pitch out_stride): no zig-zag blocks in
 * HBM.  The blocks are the plane's ((H+7)/8) x ((W+7)/8); table_id as
 * hic_dequant_idct_u8; *d_status as hic_rle_decode_i16_indexed. */
int hic_rle_decode_idct_u8_indexed(const uint8_t *sym_len, const int16_t *sym_val, const int64_t *d_nsym,
                                   const int32_t *dc_diff, const int64_t *d_index, int64_t H, int64_t W,
                                   int table_id, uint8_t *out, int64_t out_stride, int64_t *d_status,
                                   void *stream);
/* Two planes of the same shape and table (Cr and Cb of one image) through
 * hic_rle_decode_idct_u8_indexed in ONE launch, so the two share one tail.  Every
 * h_ argument is a host array of 2 device pointers (plane 0, plane 1); the rest as
 * hic_rle_decode_idct_u8_indexed, for both planes. */
int hic_rle_decode_idct_u8_indexed_pair(const uint8_t *const *h_sym_len, const int16_t *const *h_sym_val,
                                        const int64_t *const *h_d_nsym, const int32_t *const *h_dc_diff,
                                        const int64_t *const *h_d_index, int64_t H, int64_t W, int table_id,
                                        uint8_t *const *h_out, int64_t out_stride, int64_t *const *h_d_status,
                                        void *stream);
/* The luminance plane's hic_rle_decode_idct_u8_indexed fused with
 * hic_ycrcb420_to_rgb (compression.jpeg_decompression, compression.py:48-56: the
 * Y channel's decode + inv_dct_channel, pyrUp(Cr), pyrUp(Cb), cvtColor YCrCb2RGB):
 * each lane turns its 8x8 block of Y straight into 8x8 RGB pixels, reading the
 * already decoded H/2 x W/2 chroma planes cr / cb (row pitch W/2, 4-byte aligned);
 * the Y plane never reaches HBM.  H, W multiples of 8; rgb: H x W x 3, row pitch
 * rgb_stride (>= 3W, multiple of 8, 8-byte aligned).  The bytes equal
 * hic_rle_decode_idct_u8_indexed (table 0) followed by hic_ycrcb420_to_rgb;
 * *d_status as hic_rle_decode_i16_indexed. */
int hic_rle_decode_idct_rgb_indexed(const uint8_t *sym_len, const int16_t *sym_val, const int64_t *d_nsym,
                                    const int32_t *dc_diff, const int64_t *d_index, int64_t H, int64_t W,
                                    const uint8_t *cr, const uint8_t *cb, uint8_t *rgb, int64_t rgb_stride,
                                    int64_t *d_status, void *stream);
/* One tile shard's slice of the channel stream (the sharded decode of
 * codec.jpeg_decode, codec.py:397-425): d_stitch is the shard's device record from
 * hic_rle_stitch {carry zeros, closes the stream, has previous DC, previous DC}.
 * The slice's first symbol continues a zero run that started `carry` positions
 * before the shard's first block; the DC chain starts at the previous DC; a shard
 * that does not close the stream ends in zeros.  *d_status = nblk * 63 for a
 * consistent slice.  Hot-path form only (64-slot int16 blocks, 16-byte aligned). */
int hic_rle_decode_i16_shard(const uint8_t *sym_len, const int16_t *sym_val, int64_t nsym,
                             const int32_t *dc_diff, int64_t nblk, const int64_t *d_stitch,
                             int16_t *blocks, int64_t *d_status, void *workspace, void *stream);
int hic_rle_decode_i32(const int32_t *sym_len, const int32_t *sym_val, int64_t nsym,
                       const int32_t *dc_diff, int64_t nblk, int block_len, int32_t *blocks,
                       int64_t *d_status, void *workspace, void *stream);
/* codec.decode_run_length on a bare symbol list: out (room for out_cap int32,
 * out_cap a multiple of 64 and >= max(length, sum(len+1))) receives the decoded
 * list; *d_status its length (EOB zero-fill to `length` included).
 * workspace >= hic_rld_workspace_bytes(nsym, out_cap / 64). */
int hic_rle_stream_decode_i32(const int32_t *sym_len, const int32_t *sym_val, int64_t nsym,
                              int64_t length, int32_t *out, int64_t out_cap, int64_t *d_status,
                              void *workspace, void *stream);

/* ---- Huffman back end, device half (codec.jpeg_encode's trees and bit strings,
 *      codec.py:304-334; huffman.py:11-58,131-142; iohelper.py:35-56).  The trees
 *      (a heap over the distinct keys) are built on the host.
 *  keys: int8 (key_bytes 1, unsigned), int16 (2) or int32 (4) device streams.
 *  hic_key_range: d_minmax (device int32[2]) = {min, max} of the n keys.
 *  hic_key_histogram: for key k in [key_min, key_min + nbins): d_counts[k - key_min]
 *    (uint32) = its count and d_first[...] = the index of its first appearance
 *    (0xFFFFFFFF if absent) -- utils.group_by's order, which the tree's ties follow.
 *  hic_huffman_pack: symbol i gets code d_code_bits[k] (right-aligned, <= 64 bits)
 *    of length d_code_len[k]; out (zeroed here) receives the concatenated codes
 *    MSB-first (the bit string of encode_data, as iohelper packs it after its
 *    pad-length byte); *d_nbits = the total bits.  out_bytes (multiple of 4) must
 *    hold ceil(total / 32) words (sum of count x length); words past it are not
 *    written.  workspace >= hic_huffman_pack_workspace_bytes(n). */
int hic_key_range(const void *keys, int key_bytes, int64_t n, int32_t *d_minmax, void *stream);
int hic_key_histogram(const void *keys, int key_bytes, int64_t n, int32_t key_min, int32_t nbins,
                      uint32_t *d_counts, uint32_t *d_first, void *stream);
size_t hic_huffman_pack_workspace_bytes(int64_t n);
int hic_huffman_pack(const void *keys, int key_bytes, int64_t n, int32_t key_min, int32_t nbins,
                     const uint64_t *d_code_bits, const uint8_t *d_code_len, uint8_t *out,
                     int64_t out_bytes, int64_t *d_nbits, void *workspace, void *stream);
/* hic_huffman_decode: HuffmanTree.decode_data (huffman.py:149-178) of the nbits-bit
 *    MSB-first stream at d_bits (4-byte aligned, ceil(nbits / 32) * 4 readable bytes; the payload bytes after
 *    iohelper's pad-length byte, iohelper.py:35-56) -- codec.jpeg_decode's nine
 *    huffman_data_decode calls (codec.py:372-388).  The tree is a host array:
 *    h_child[2n] / h_child[2n + 1] = node n's '1' (left) / '0' (right) child, >= 0
 *    an internal node, -1 none, <= -2 the leaf -2 - c; node 0 is the root.  Symbol
 *    k gets d_out[k] = h_values[leaf] (h_values null: the leaf index).  Trailing
 *    bits that finish no code are dropped, as the reference's reduce does.
 *    *h_count = symbols decoded.  Synchronises the stream.  HIC_ERR_ARG when a code
 *    walks into a missing child (the reference's AttributeError; *h_count = the
 *    symbols before it), HIC_ERR_CAPACITY when *h_count > out_cap (nbits is always
 *    enough).  workspace >= hic_huffman_decode_workspace_bytes(nbits, nnodes, nleaves). */
size_t hic_huffman_decode_workspace_bytes(int64_t nbits, int32_t nnodes, int32_t nleaves);
int hic_huffman_decode(const uint8_t *d_bits, int64_t nbits, const int32_t *h_child, int32_t nnodes,
                       const int32_t *h_values, int32_t nleaves, int32_t *d_out, int64_t out_cap,
                       int64_t *h_count, void *workspace, void *stream);
/* hic_huffman_decode_batch: n hic_huffman_decode calls (codec.jpeg_decode's nine
 *    streams) on one stream with their host round trips shared: every job is
 *    checked before anything is queued (HIC_ERR_ARG, nothing run), then the streams
 *    go through each phase together.  Per job: count = symbols decoded, status =
 *    HIC_OK / HIC_ERR_ARG (missing child) / HIC_ERR_CAPACITY as hic_huffman_decode
 *    returns them; the call returns the first job's non-OK status (its message in
 *    hic_last_error) or HIC_OK.  Each job needs its own workspace. */
typedef struct {
  const uint8_t *d_bits;
  int64_t nbits;
  const int32_t *h_child;
  int32_t nnodes;
  const int32_t *h_values;
  int32_t nleaves;
  int32_t *d_out;
  int64_t out_cap;
  void *workspace;
  int64_t count;  /* out */
  int32_t status; /* out */
} hic_huffman_decode_job;
int hic_huffman_decode_batch(int n, hic_huffman_decode_job *jobs, void *stream);

/* ---- Huffman trees, host side (native, no device work; hufftree.hip).
 *  hic_huffman_build: HuffmanTree._construct (huffman.py:60-79) over n >= 1 leaves
 *    whose frequencies h_counts[] are in first-appearance order (utils.group_by):
 *    heapq's heap compared on frequency only, the first node popped the left child,
 *    left = '1'.  Leaf i's code: h_len[i] bits, right-aligned in h_code[i] (MSB =
 *    the edge at the root).  One leaf: code "1".  HIC_ERR_ARG if a code would pass
 *    64 bits (needs > 2^44 symbols).  h_text (may be null; >= 65 n bytes): the
 *    codes as text, each followed by one space.
 *  hic_huffman_from_codes: construct_from_coding (huffman.py:30-58) + the
 *    breadth-first layout hic_huffman_decode takes, for a table of n >= 2 codes
 *    that is a complete prefix code: code i is h_chars[h_off[i] .. h_off[i + 1])
 *    ('0' / '1'; a repeated code keeps its last entry, as the reference's dict
 *    does).  h_child (>= 2n int32) receives the tree, *h_nodes its internal node
 *    count, h_leaf_seg (>= n int32) the table entry of each leaf in the tree's leaf
 *    order, *h_minlen the shortest code.  Any other table: HIC_ERR_ARG ("irregular
 *    table ..."), nothing written; the caller then builds the reference's own tree. */
int hic_huffman_build(const int64_t *h_counts, int64_t n, uint8_t *h_len, uint64_t *h_code, char *h_text);
int hic_huffman_from_codes(const char *h_chars, const int64_t *h_off, int64_t n, int32_t *h_child,
                           int32_t *h_leaf_seg, int64_t *h_nodes, int32_t *h_minlen);

/* ---- the gather's wire format (no reference counterpart: the bytes that carry a
 *      shard's quantized zig-zag blocks -- codec.jpeg_encode's input after
 *      dct_channel, codec.py:286-301 -- to the gathering rank, losslessly).  Zig-zag
 *      slot z of a block takes a fixed number of bits (two's complement) proven
 *      sufficient for the plane's table by tools/check/wire_widths.py (hiccup's
 *      unnormalised DCT bound 4 * 128 * S_u * S_v over the table entry): 637 bits
 *      per luminance block, 597 per chrominance block; a 64-block tile is
 *      2 * bits 32-bit little-endian words, stored at a stride rounded up to 16 B.
 *  hic_wire_bytes: the wire size of nblk blocks of table table_id (whole tiles).
 *  hic_wire_pack_i16: blocks (nblk x 64 int16, 16-byte aligned) -> wire; *d_flag
 *    (device int, caller-zeroed) becomes 1 if a value does not fit its slot's
 *    width (then the wire is not lossless: send the raw blocks).
 *  hic_wire_unpack_i16: wire -> blocks (the inverse; nblk and table as packed).
 *  hic_rle_records_rebase: nrec RLE tile records (3 int64: first / last nonzero
 *    stream position or -1, symbol count) copied to d_dst with pos_shift added to
 *    the positions: a shard's records placed in the whole image's record array
 *    (pos_shift = the shard's first block x 63; its records must start on a
 *    record boundary of the whole image). */
size_t hic_wire_bytes(int64_t nblk, int table_id);
int hic_wire_pack_i16(const int16_t *blocks, int64_t nblk, int table_id, uint8_t *wire, int *d_flag, void *stream);
int hic_wire_unpack_i16(const uint8_t *wire, int64_t nblk, int table_id, int16_t *blocks, void *stream);
/* The batched forms (a multi-GPU group's segments: 3 channels x up to 7 peers in 3
 * launches).  Each job: its blocks and wire segment (nblk 0: records only), its
 * table, the out-of-width flag (pack: cleared, then raised), its RLE records
 * (rec_src / nrec, nullable) copied to rec_dst rebased by pos_shift (as
 * hic_rle_records_rebase), and d_count (hic_wire_flags_apply).  n <= 32; every job
 * checked before the first launch.
 *  hic_wire_pack_batch: hic_wire_pack_i16 + hic_rle_records_rebase of every job.
 *  hic_wire_unpack_batch: hic_wire_unpack_i16 + hic_rle_records_rebase of every job.
 *  hic_wire_flags_apply: *d_count = HIC_COUNT_WIRE_OVERFLOW for each job whose
 *    *d_flag (a received sender flag) is set -- after the stream's scan. */
typedef struct {
  int16_t *blocks;
  uint8_t *wire;
  int64_t nblk;
  int32_t table_id;
  int32_t *d_flag;
  const int64_t *rec_src;
  int64_t nrec, pos_shift;
  int64_t *rec_dst;
  int64_t *d_count;
} hic_wire_job;
int hic_wire_pack_batch(int n, const hic_wire_job *jobs, void *stream);
int hic_wire_unpack_batch(int n, const hic_wire_job *jobs, void *stream);
int hic_wire_flags_apply(int n, const hic_wire_job *jobs, void *stream);
int hic_rle_records_rebase(const int64_t *d_src, int64_t nrec, int64_t pos_shift, int64_t *d_dst, void *stream);

/* ---- Multi-GPU gather over RCCL (SURVEY.md section 8(b) hic_gather_*; the
 *      whole-image buffers it reassembles are what codec.jpeg_encode consumes,
 *      codec.py:275-334, after compression.jpeg_compression, compression.py:16-39,
 *      which the tile-sharded encode splits over the ranks).  One rank per GPU;
 *      RCCL is opened at run time (librccl.so.1), the other entry points do not
 *      need it.
 *  hic_gather_unique_id: one rank makes the communicator id (HIC_GATHER_ID_BYTES
 *    host bytes) and hands it to the others by any host channel.
 *  hic_gather_comm_init: collective over the `world` ranks, after the caller has
 *    selected its GPU (hipSetDevice); *h_comm is an opaque handle.
 *  hic_gather_bytes: a variable-size gather: every rank's d_send (send_bytes)
 *    lands at d_recv + h_recv_offsets[rank] on `root` (h_recv_bytes[rank] bytes;
 *    root-only arguments, NULL elsewhere).  The root's own slice is copied unless
 *    d_send already is that address.  One RCCL group of sends / receives on
 *    `stream`; no host synchronisation.
 *  hic_gather_group_begin / _end: gathers posted between them (e.g. image j of a
 *    group of N to root j) go out as ONE RCCL group. */
#define HIC_GATHER_ID_BYTES 128
int hic_gather_unique_id(uint8_t *h_id);
int hic_gather_comm_init(void **h_comm, const uint8_t *h_id, int world, int rank);
int hic_gather_comm_info(void *comm, int *h_world, int *h_rank);
int hic_gather_comm_destroy(void *comm);
int hic_gather_group_begin(void);
int hic_gather_group_end(void);
int hic_gather_bytes(void *comm, const void *d_send, int64_t send_bytes, void *d_recv,
                     const int64_t *h_recv_offsets, const int64_t *h_recv_bytes, int root, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* HICCUP_HIP_H */
