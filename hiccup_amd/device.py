"""Device plumbing: PyTorch-ROCm provides HBM allocations and the HIP stream;
the compute is entirely in libhiccup_hip.so.  No CPU fallback: without a HIP
device every entry point raises ``HipUnavailable``."""
import contextlib
import ctypes
import threading

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
    """A host array as a new device tensor.  Large arrays (>= 4 MiB) go through the
    pinned staging buffer in chunks of at most _PIN_MAX bytes (threaded host copy,
    then one DMA each): a pageable copy runs at ~4 GB/s on the MI355X boxes
    (tools/prof_d2h.py)."""
    require_gpu()
    a = np.ascontiguousarray(a)
    if a.nbytes < _PIN_MIN or a.dtype.hasobject:
        return torch.from_numpy(a).to("cuda")
    out = torch.empty(tuple(a.shape), dtype=torch.from_numpy(a[:0].reshape(-1)).dtype, device="cuda")
    ob, ab = out.reshape(-1).view(torch.uint8), a.reshape(-1).view(np.uint8)
    with _staging_lock:
        for o, n in _chunks(a.nbytes):
            st = _stage(n)
            _par_copy(st.numpy(), ab[o:o + n])
            ob[o:o + n].copy_(st)  # synchronous: the buffer is reused by the next chunk
    return out


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
    """A device tensor as a new numpy array (through the pinned buffer when large)."""
    sync()
    nbytes = t.numel() * t.element_size()
    if nbytes < _PIN_MIN or not t.is_cuda:
        return t.cpu().numpy()
    t = t.contiguous()
    out = np.empty(tuple(t.shape), torch.empty(0, dtype=t.dtype).numpy().dtype)
    tb, ob = t.reshape(-1).view(torch.uint8), out.reshape(-1).view(np.uint8)
    with _staging_lock:
        for o, n in _chunks(nbytes):
            st = _stage(n)
            st.copy_(tb[o:o + n])
            _par_copy(ob[o:o + n], st.numpy())
    return out


def to_host_f64(t):
    """A device int32 tensor as a new float64 numpy array (the reference's planes are
    float64): DMA into the pinned buffer, then the cast split over host threads.
    A pageable copy runs at ~4 GB/s here and the single-threaded cast after it
    doubled the time (8K luma: 48 vs 17 ms, tools/prof_d2h.py)."""
    assert t.dtype == torch.int32 and t.is_cuda
    sync()
    t = t.contiguous()
    n = t.numel()
    out = np.empty(n, np.float64)
    ti = t.reshape(-1)
    with _staging_lock:
        for o, nb in _chunks(4 * n):
            st = _stage(nb)
            st.view(torch.int32).copy_(ti[o // 4:(o + nb) // 4])
            _par_copy(out[o // 4:(o + nb) // 4], st.numpy().view(np.int32))
    return out.reshape(tuple(t.shape))


def to_device_i32(a, nonint_msg, range_msg):
    """A host array of integer values as a new int32 device tensor, refusing
    non-integer (ValueError(nonint_msg)) or out-of-int32 (ValueError(range_msg))
    values as the host checks did.  Large float arrays (the reference's float64
    planes) are checked and cast on the GPU after one pinned copy: np.mod, min / max
    and two casts of an 8K float64 plane took ~0.2 s on the host."""
    a = np.asarray(a)
    if a.dtype == np.int32:  # already in range
        return to_device(a)
    if a.dtype.kind != "f" or a.nbytes < _PIN_MIN:
        if a.size and a.dtype.kind not in "iub" and not np.all(np.mod(a, 1) == 0):
            raise ValueError(nonint_msg)
        b = a.astype(np.int64)
        if b.size and (b.min() < -(1 << 31) or b.max() >= (1 << 31)):
            raise ValueError(range_msg)
        return to_device(b.astype(np.int32))
    t = to_device(a)
    if not bool((torch.remainder(t, 1) == 0).all()):
        raise ValueError(nonint_msg)
    if bool(((t < -(1 << 31)) | (t >= (1 << 31))).any()):
        raise ValueError(range_msg)
    return t.to(torch.int32)


# one pinned host staging buffer (grown on demand up to _PIN_MAX bytes, reused;
# callers on several threads take turns under _staging_lock; larger copies go in
# _PIN_MAX chunks, so the buffer never holds more than that) and a small thread
# pool for the host side of the copies
_PIN_MIN = 4 << 20
_PIN_MAX = 256 << 20
_staging = None
_staging_lock = threading.Lock()
_pool = None


def _chunks(nbytes):
    """(offset, length) pieces of a copy of nbytes, each <= _PIN_MAX (a multiple of 8)."""
    return [(o, min(_PIN_MAX, nbytes - o)) for o in range(0, nbytes, _PIN_MAX)]


def _stage(nbytes):
    """The first nbytes (<= _PIN_MAX) of the pinned uint8 buffer (call with
    _staging_lock held)."""
    global _staging
    assert nbytes <= _PIN_MAX
    if _staging is None or _staging.numel() < nbytes:
        _staging = None
        _staging = torch.empty(min(_PIN_MAX, max(2 * int(nbytes), _PIN_MIN)), dtype=torch.uint8, pin_memory=True)
    return _staging[:nbytes]


def _par_copy(dst, src):
    """dst[...] = src (same shape; a cast if the dtypes differ) in 8 row ranges on
    host threads (numpy releases the GIL while it copies)."""
    global _pool
    if _pool is None:
        from concurrent.futures import ThreadPoolExecutor
        _pool = ThreadPoolExecutor(8)
    d, s_ = dst.reshape(-1), src.reshape(-1)
    n = d.size
    k = 8 if n >= (1 << 20) else 1
    bounds = [(i * n // k, (i + 1) * n // k) for i in range(k)]
    list(_pool.map(lambda ab: np.copyto(d[ab[0]:ab[1]], s_[ab[0]:ab[1]], casting="unsafe"), bounds))


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
