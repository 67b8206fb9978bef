"""Device plumbing: PyTorch-ROCm provides HBM allocations and the HIP stream;
the compute is entirely in libhiccup_hip.so.  No CPU fallback: without a HIP
device every entry point raises ``HipUnavailable``."""
import contextlib
import ctypes
import os
import sys
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


def to_device(a, wait=True):
    """A host array as a new device tensor.  Large arrays (>= 4 MiB) go through two
    pinned staging buffers in chunks of _CHUNK bytes: the threaded host copy of one
    chunk overlaps the DMA of the one before it (a pageable copy runs at ~4 GB/s on
    the MI355X boxes).  wait=False (an array in a pinned pool buffer only): return
    with its DMA still queued -- the caller keeps `a` unchanged until it next
    synchronises the current stream."""
    require_gpu()
    a = np.ascontiguousarray(a)
    if a.nbytes < _PIN_MIN or a.dtype.hasobject:
        return torch.from_numpy(a).to("cuda")
    dt = torch.from_numpy(a[:0].reshape(-1)).dtype
    ab = a.reshape(-1).view(np.uint8)
    if _is_pinned(ab):
        # already page-locked: one DMA, no staging copy, on the copy stream (its
        # buffer allocated there), so it runs beside the kernels already queued on
        # the current stream (jpeg_encode: the next plane's upload beside this one's
        # RLE); the current stream waits for it, the host too (`a` is free on return)
        s, cur = _copy_stream(), torch.cuda.current_stream()
        with torch.cuda.stream(s):
            out = torch.empty(tuple(a.shape), dtype=dt, device="cuda")
            out.reshape(-1).view(torch.uint8).copy_(torch.from_numpy(ab), non_blocking=True)
            done = torch.cuda.Event()
            done.record(s)
        cur.wait_event(done)
        out.record_stream(cur)
        if wait:
            done.synchronize()
        return out
    out = torch.empty(tuple(a.shape), dtype=dt, device="cuda")
    ob = out.reshape(-1).view(torch.uint8)
    with _staging_lock:
        s = _copy_stream()
        s.wait_stream(torch.cuda.current_stream())  # `out` was allocated on the current stream
        done = [None, None]
        for i, (o, n) in enumerate(_chunks(a.nbytes)):
            st = _stage(i % 2, n)
            if done[i % 2] is not None:
                done[i % 2].synchronize()  # the buffer's previous DMA has read it
            _par_copy(st.numpy(), ab[o:o + n])
            with torch.cuda.stream(s):
                ob[o:o + n].copy_(st, non_blocking=True)
                done[i % 2] = torch.cuda.Event()
                done[i % 2].record(s)
        torch.cuda.current_stream().wait_stream(s)
        for e in done:
            if e is not None:
                e.synchronize()  # the staging buffers are free for the next caller
    return out


def to_device_parts(parts, offsets, nbytes):
    """One new uint8 device tensor of nbytes holding host uint8 array parts[i] at
    byte offsets[i] (ascending, non-overlapping) and zeros elsewhere: the parts go
    straight into the pinned staging buffers (one host copy; to_device of a
    concatenation would copy twice)."""
    require_gpu()
    spans = [(int(o), np.ascontiguousarray(a).reshape(-1).view(np.uint8)) for o, a in zip(offsets, parts)]
    if spans and all(a.size == 0 or _is_pinned(a) for _, a in spans):
        # every part already page-locked (jpeg_encode's packed bits handed to
        # jpeg_decode): zeros, then one DMA per part, no staging copy
        out = torch.zeros((max(int(nbytes), 1),), dtype=torch.uint8, device="cuda")
        for o, a in spans:
            if a.size:
                out[o:o + a.size].copy_(torch.from_numpy(a), non_blocking=True)
        torch.cuda.current_stream().synchronize()  # the parts are free on return
        return out
    out = torch.empty((max(int(nbytes), 1),), dtype=torch.uint8, device="cuda")
    with _staging_lock:
        s = _copy_stream()
        s.wait_stream(torch.cuda.current_stream())
        done = [None, None]
        for i, (c0, n) in enumerate(_chunks(int(nbytes))):
            st = _stage(i % 2, n)
            if done[i % 2] is not None:
                done[i % 2].synchronize()
            sn = st.numpy()
            pos = c0  # bytes of this chunk before `pos` are written
            for o, a in spans:
                a0, a1 = max(o, c0), min(o + a.size, c0 + n)
                if a1 <= c0 or a0 >= c0 + n:
                    continue
                if a0 > pos:
                    sn[pos - c0:a0 - c0] = 0
                _par_copy(sn[a0 - c0:a1 - c0], a[a0 - o:a1 - o])
                pos = a1
            if pos < c0 + n:
                sn[pos - c0:] = 0
            with torch.cuda.stream(s):
                out[c0:c0 + n].copy_(st, non_blocking=True)
                done[i % 2] = torch.cuda.Event()
                done[i % 2].record(s)
        torch.cuda.current_stream().wait_stream(s)
        for e in done:
            if e is not None:
                e.synchronize()
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


def _d2h_chunks(src_u8, nbytes, host_copy):
    """DMA src_u8 (a flat uint8 device view) into the two pinned buffers chunk by
    chunk on the copy stream, and hand each landed chunk to host_copy(offset, n,
    pinned uint8 numpy view) while the next chunk's DMA runs (call with
    _staging_lock held)."""
    s = _copy_stream()
    s.wait_stream(torch.cuda.current_stream())
    chunks = _chunks(nbytes)
    ev = [None, None]

    def issue(i):
        o, n = chunks[i]
        with torch.cuda.stream(s):
            _stage(i % 2, n).copy_(src_u8[o:o + n], non_blocking=True)
            ev[i % 2] = torch.cuda.Event()
            ev[i % 2].record(s)

    issue(0)
    for i, (o, n) in enumerate(chunks):
        if i + 1 < len(chunks):
            issue(i + 1)  # its buffer's previous chunk (i - 1) was copied out below
        ev[i % 2].synchronize()
        host_copy(o, n, _stage(i % 2, n).numpy())


def to_host(t):
    """A device tensor as a new numpy array (through the pinned buffers when large:
    each chunk's host copy overlaps the next chunk's DMA)."""
    sync()
    nbytes = t.numel() * t.element_size()
    if nbytes < _PIN_MIN or not t.is_cuda:
        return t.cpu().numpy()
    t = t.contiguous()
    out = host_empty(tuple(t.shape), torch.empty(0, dtype=t.dtype).numpy().dtype)
    tb, ob = t.reshape(-1).view(torch.uint8), out.reshape(-1).view(np.uint8)
    if _is_pinned(ob):  # a pinned pool buffer: the DMA writes the result in place
        torch.from_numpy(ob).copy_(tb)
        return out
    with _staging_lock:
        _d2h_chunks(tb, nbytes, lambda o, n, st: _par_copy(ob[o:o + n], st))
    return out


def to_host_f64(t):
    """A device int32 tensor as a new float64 numpy array (the reference's planes are
    float64): DMA into the pinned buffers, the cast split over host threads and
    overlapped with the next chunk's DMA.  A pageable copy runs at ~4 GB/s here and
    the single-threaded cast after it doubled the time (8K luma: 48 vs 17 ms)."""
    assert t.dtype == torch.int32 and t.is_cuda
    sync()
    t = t.contiguous()
    n = t.numel()
    out = host_empty((n,), np.float64)
    if n and _is_pinned(out):
        # a pinned pool buffer: widen on the device and DMA the float64 values in
        # place (CPU writes into pinned memory run at ~0.73x of pageable here, so
        # the host-side cast below would cost more than the doubled bytes)
        torch.from_numpy(out).copy_(t.reshape(-1).to(torch.float64))
        return out.reshape(tuple(t.shape))
    with _staging_lock:
        _d2h_chunks(t.reshape(-1).view(torch.uint8), 4 * n,
                    lambda o, nb, st: _par_copy(out[o // 4:(o + nb) // 4], st.view(np.int32)))
    return out.reshape(tuple(t.shape))


def to_host_f64_many(tensors):
    """[to_host_f64(t)] with one wait: each plane widened on the device and copied
    straight into its pinned pool buffer, all queued before the host waits."""
    outs = [host_empty((t.numel(),), np.float64) for t in tensors]
    if not all(t.numel() and _is_pinned(o) for t, o in zip(tensors, outs)):
        return [to_host_f64(t) for t in tensors]
    for t, o in zip(tensors, outs):
        torch.from_numpy(o).copy_(t.contiguous().reshape(-1).to(torch.float64), non_blocking=True)
    torch.cuda.current_stream().synchronize()
    return [o.reshape(tuple(t.shape)) for t, o in zip(tensors, outs)]


def to_device_i32(a, nonint_msg, range_msg, wait=True):
    """A host array of integer values as a new int32 device tensor, refusing
    non-integer (ValueError(nonint_msg)) or out-of-int32 (ValueError(range_msg))
    values as the host checks did.  Large float arrays (the reference's float64
    planes) are checked and cast on the GPU after one pinned copy: np.mod, min / max
    and two casts of an 8K float64 plane took ~0.2 s on the host."""
    a = np.asarray(a)
    if a.dtype == np.int32:  # already in range
        return to_device(a, wait=wait)
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


# two pinned host staging buffers of _CHUNK bytes (reused; callers on several
# threads take turns under _staging_lock), a copy stream for their DMAs, and a small
# thread pool for the host side of the copies
_PIN_MIN = 4 << 20
_HOST_THREADS = int(os.environ.get("HICCUP_HOST_THREADS", "8"))  # host copy threads
_CHUNK = 32 << 20
_staging = [None, None]
_staging_lock = threading.Lock()
_cstream = None
_pool = None


def _chunks(nbytes, chunk=None):
    """(offset, length) pieces of a copy of nbytes, each <= _CHUNK (a multiple of 8)."""
    c = _CHUNK if chunk is None else chunk
    return [(o, min(c, nbytes - o)) for o in range(0, nbytes, c)]


def _stage(k, nbytes):
    """The first nbytes (<= _CHUNK) of pinned buffer k (call with _staging_lock held)."""
    assert nbytes <= _CHUNK
    if _staging[k] is None:
        _staging[k] = torch.empty(_CHUNK, dtype=torch.uint8, pin_memory=True)
    return _staging[k][:nbytes]


# Host result arrays.  A fresh numpy array of a few hundred MB costs its page faults
# on first touch (~11 ms per 133 MB single-threaded on the GPU box, ~22 ms when eight
# copy threads fault it together; the DMA itself is 2.3 ms): the large results of
# to_host / to_host_f64 are views of pooled buffers instead, and the pool's buffers
# are pinned, so a result the DMA writes needs no staging copy, and a result handed
# back (jpeg_compression's planes into jpeg_encode, jpeg_decode's into
# jpeg_decompression) goes up without one either.  A pooled buffer is handed out
# again only when nothing but the pool references it (a caller's result, or any view
# of it, keeps it out of the pool).
_HOST_POOL_MAX = 4 << 30  # bytes the pool may hold
_host_pool = []
_pinned_spans = []  # [start, end) addresses of the pool's pinned buffers
_host_pool_lock = threading.Lock()


def host_empty(shape, dtype):
    """np.empty(shape, dtype) from the pool of faulted buffers when large."""
    dt = np.dtype(dtype)
    nbytes = int(np.prod(shape, dtype=np.int64)) * dt.itemsize
    if nbytes < _PIN_MIN:
        return np.empty(shape, dt)
    with _host_pool_lock:
        best = None
        for b in _host_pool:
            # referenced only by the list, the loop variable and getrefcount's argument
            if b.nbytes >= nbytes and sys.getrefcount(b) <= 3 and (best is None or b.nbytes < best.nbytes):
                best = b
        if best is None:
            if sum(b.nbytes for b in _host_pool) + nbytes <= _HOST_POOL_MAX:
                # pinned (page-locked, so also faulted in): DMA reaches it directly
                best = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True).numpy()
                _host_pool.append(best)
                _pinned_spans.append((best.ctypes.data, best.ctypes.data + nbytes))
            else:
                best = np.empty(nbytes, np.uint8)
                _fault_in(best)
        return best[:nbytes].view(dt).reshape(shape)


def _is_pinned(a):
    """Whether host array a lies inside a pinned pool buffer (a result of to_host /
    to_host_f64 or a view of one): the DMA can then read / write it in place."""
    lo = a.ctypes.data
    hi = lo + a.nbytes
    return any(s <= lo and hi <= e for s, e in _pinned_spans)


def _fault_in(buf):
    """Touch every page of a new host buffer on the worker threads, 2 MiB apart."""
    step = 2 << 20
    n = buf.size
    bounds = [(o, min(n, o + step)) for o in range(0, n, step)]
    _ensure_pool()
    list(_pool.map(lambda ab: buf[ab[0]:ab[1]].fill(0), bounds))


def _ensure_pool():
    global _pool
    if _pool is None:
        from concurrent.futures import ThreadPoolExecutor
        _pool = ThreadPoolExecutor(_HOST_THREADS)


def _copy_stream():
    global _cstream
    if _cstream is None:
        _cstream = torch.cuda.Stream()
    return _cstream


def _par_copy(dst, src):
    """dst[...] = src (same shape; a cast if the dtypes differ) in 8 row ranges on
    host threads (numpy releases the GIL while it copies)."""
    _ensure_pool()
    d, s_ = dst.reshape(-1), src.reshape(-1)
    n = d.size
    k = _HOST_THREADS if n >= (1 << 20) else 1
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
