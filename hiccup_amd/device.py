"""Device plumbing: PyTorch-ROCm provides HBM allocations and the HIP stream;
the compute is entirely in libhiccup_hip.so.  No CPU fallback: without a HIP
device every entry point raises ``HipUnavailable``."""
import contextlib
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import HipUnavailable

_checked = False


def require_gpu():
    global _checked
    if not _checked:
        _lib.load()
        if not torch.cuda.is_available():
            raise HipUnavailable("no HIP device visible: hiccup_amd runs only on MI355X (gfx950); "
                                 "there is no CPU fallback")
        _checked = True


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def on_stream(stream=None):
    """Context that makes `stream` torch's current stream (a no-op for None): the
    allocations made inside belong to it, and host reads (.cpu()) wait for the
    kernels launched on it."""
    return torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()


def ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def to_device(a):
    require_gpu()
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")


def empty(shape, dtype):
    require_gpu()
    return torch.empty(shape, dtype=dtype, device="cuda")


def zeros(shape, dtype):
    require_gpu()
    return torch.zeros(shape, dtype=dtype, device="cuda")


def workspace(nbytes):
    """Zero-filled int64 scratch (the RLE scan's hand-off granules expect zeros
    before their first use; see hic_rle_workspace_bytes)."""
    return zeros((max(int(nbytes), 8) + 7) // 8, torch.int64)


def sync(stream=None):
    _lib.call("hic_stream_sync", stream_ptr(stream))


def to_host(t):
    sync()
    return t.cpu().numpy()


_staging = None  # pinned host staging for to_host_f64 (grown on demand, reused)
_cast_pool = None
_staging_lock = None


def to_host_f64(t):
    """A device int32 tensor as a new float64 numpy array (the reference's planes are
    float64): one DMA into a reused pinned buffer, then the cast split over host
    threads.  A pageable copy runs at ~4 GB/s here and the single-threaded cast after
    it doubled the time (8K luma: 48 ms, tools/prof_d2h.py)."""
    global _staging, _cast_pool, _staging_lock
    import threading
    from concurrent.futures import ThreadPoolExecutor
    assert t.dtype == torch.int32 and t.is_cuda
    n = t.numel()
    sync()
    if _staging_lock is None:
        _staging_lock = threading.Lock()
    out = np.empty(n, np.float64)
    with _staging_lock:  # one staging buffer: callers on several threads take turns
        if _staging is None or _staging.numel() < n:
            _staging = torch.empty(max(n, 1), dtype=torch.int32, pin_memory=True)
        _staging[:n].copy_(t.reshape(-1))
        src = _staging[:n].numpy()
        if _cast_pool is None:
            _cast_pool = ThreadPoolExecutor(8)
        k = 8 if n >= (1 << 20) else 1
        bounds = [(i * n // k, (i + 1) * n // k) for i in range(k)]
        list(_cast_pool.map(lambda ab: np.copyto(out[ab[0]:ab[1]], src[ab[0]:ab[1]]), bounds))
    return out.reshape(tuple(t.shape))


class KernelEvents:
    """A pair of HIP events that a *_timed entry point fills with one kernel's
    own begin / end timestamps (hipExtLaunchKernelGGL)."""

    def __init__(self):
        require_gpu()
        self._lib = _lib.load()
        a, b = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.call("hic_event_create", ctypes.byref(a))
        _lib.call("hic_event_create", ctypes.byref(b))
        self.start, self.stop = a, b

    def elapsed_ms(self):
        ms = ctypes.c_float()
        _lib.call("hic_event_elapsed_ms", self.start, self.stop, ctypes.byref(ms))
        return float(ms.value)

    def __del__(self):
        for e in (getattr(self, "start", None), getattr(self, "stop", None)):
            if e is not None and e.value:
                self._lib.hic_event_destroy(e)
