// common.hip -- error state and small runtime entry points of the C-ABI.
#include <string.h>

#include "hic_common.h"

namespace hic {
static thread_local char g_last_error[512] = "";

void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof g_last_error, fmt, ap);
  va_end(ap);
}
}  // namespace hic

extern "C" int hic_abi_version(void) { return HIC_ABI_VERSION; }

extern "C" int hic_last_error(char *h_buf, size_t n) {
  if (!h_buf || n == 0) return HIC_ERR_ARG;
  strncpy(h_buf, hic::g_last_error, n - 1);
  h_buf[n - 1] = '\0';
  return HIC_OK;
}

extern "C" int hic_device_count(int *h_n) {
  if (!h_n) return hic::arg_error("null pointer");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) n = 0;
  *h_n = n;
  return HIC_OK;
}

extern "C" int hic_stream_sync(void *stream) {
  return hic::hip_status(hipStreamSynchronize(hic::as_stream(stream)), "hipStreamSynchronize");
}

extern "C" int hic_event_create(void **h_event) {
  if (!h_event) return hic::arg_error("null pointer");
  hipEvent_t e = nullptr;
  const int rc = hic::hip_status(hipEventCreate(&e), "hipEventCreate");
  *h_event = rc == HIC_OK ? (void *)e : nullptr;
  return rc;
}

extern "C" int hic_event_destroy(void *event) {
  if (!event) return hic::arg_error("null event");
  return hic::hip_status(hipEventDestroy((hipEvent_t)event), "hipEventDestroy");
}

extern "C" int hic_event_elapsed_ms(void *start, void *stop, float *h_ms) {
  if (!start || !stop || !h_ms) return hic::arg_error("null pointer");
  int rc = hic::hip_status(hipEventSynchronize((hipEvent_t)stop), "hipEventSynchronize");
  if (rc != HIC_OK) return rc;
  return hic::hip_status(hipEventElapsedTime(h_ms, (hipEvent_t)start, (hipEvent_t)stop), "hipEventElapsedTime");
}
