// hic_common.h -- shared plumbing for the libhiccup_hip.so C-ABI: error state,
// launch checks, wave-level helpers.  gfx950 only (wave64).
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/hiccup_hip.h"

namespace hic {

// Per-thread last-error text (hic_last_error).
void set_error(const char *fmt, ...);
// Current value of an A/B knob (hic_set_knob; the default when unset).
int knob(int k);

inline int arg_error(const char *what) {
  set_error("invalid argument: %s", what);
  return HIC_ERR_ARG;
}
template <typename... A>
inline int arg_error(const char *fmt, A... args) {
  char buf[200];
  snprintf(buf, sizeof buf, fmt, args...);
  set_error("invalid argument: %s", buf);
  return HIC_ERR_ARG;
}

inline int check_launch(const char *kernel) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s launch failed: %s", kernel, hipGetErrorString(e));
    return HIC_ERR_HIP;
  }
  return HIC_OK;
}

inline int hip_status(hipError_t e, const char *what) {
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return HIC_ERR_HIP;
  }
  return HIC_OK;
}

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int kWave = 64;

// Round n up to a multiple of a.
__host__ __device__ inline int64_t round_up(int64_t n, int64_t a) { return (n + a - 1) / a * a; }
__host__ __device__ inline int64_t ceil_div(int64_t n, int64_t a) { return (n + a - 1) / a; }

// Compute units of the current device (cached).
inline int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
      n = prop.multiProcessorCount;
    if (n <= 0) n = 256;
  }
  return n;
}

// A launch's hand-off epoch in [1, 2^30 - 1], unique per call (until it wraps):
// tags of the RLE scan's and the one-pass encode's granules, shared so that one
// workspace used by both never sees a stale granule match.
uint32_t next_epoch();

// Cross-file launchers (rle.hip): the hot-path RLE tile pass on int16 zig-zag
// blocks of 64, for callers whose transform did not fuse it.
int rle_tile16_launch(const int16_t *blocks, int64_t nblk, int max_len, int64_t *tiles, hipStream_t s);
// Slot layout (slots.h, rle.hip): the int64 word of a slot job's workspace where
// its records' last DCs (int32 per record) start, after the scan's records,
// offsets and hand-off granules; and the job's record count.
int64_t slot_rdc_word(int64_t nrec);
inline int64_t slot_nrec(int64_t nblk, int64_t records_per_tile) {
  return (nblk * records_per_tile + 63) / 64;
}

}  // namespace hic
