"""Subprocess bodies of the allocator hazard tests (tests/test_gpu_kernels.py).

Each runs in a fresh process because the pool's knobs (ELX_POOL_CACHE, H_CUB_DEBUG)
are read once, when the library first touches the GPU.  ELX_POOL_CACHE=0 is the
regime round 4's release threshold 0 stood for: every freed block goes back to
the driver (hipFree) at once, so a premature reuse is as likely as it gets.  `python tests/_pool_workers.py <case>` prints "OK <case>" on success.

The hazard (round 4's wrong GEMMs): a block whose last reader runs on a stream
that is not ordered before the stream it is freed on.  A spin kernel delays the
reader by ~0.2 s, so a block handed out early is overwritten before the reader
runs -- deterministically, not by chance.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from elemental_amd import _lib as L  # noqa: E402
from elemental_amd import el  # noqa: E402

SPIN_CYCLES = 400_000_000  # torch.cuda._sleep: ~0.2 s of s_memtime cycles on gfx950


def _stream():
    s = ctypes.c_void_p()
    L.call("elx_stream_create", ctypes.byref(s))
    return s


def _spin(stream):
    with torch.cuda.stream(torch.cuda.ExternalStream(stream.value)):
        torch.cuda._sleep(SPIN_CYCLES)


def pool_free_after_delayed_reader():
    """Pool level: X is read on s_read behind a spin; the caller orders the free
    (on s_free) after the reader with an event, as the pool contract asks; a new
    request of the same bin on a third stream must not see X's memory change
    before the reader ran (cached: it waits on the free's event; uncached: the
    block returns to the driver only once idle)."""
    n = (64 << 20) // 8
    s_read, s_free, s_new = _stream(), _stream(), _stream()
    Y = torch.zeros(n, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    X = ctypes.c_void_p()
    L.call("elx_pool_alloc", ctypes.byref(X), n * 8, s_free)
    L.call("elx_fill2d", L.F64, n, 1, 1.0, X, n, s_free)
    L.call("elx_stream_synchronize", s_free)
    _spin(s_read)
    L.call("elx_copy2d", L.F64, n, 1, X, 1, n, ctypes.c_void_p(Y.data_ptr()), 1, n, s_read)
    ev = ctypes.c_void_p()
    L.call("elx_event_create", ctypes.byref(ev))
    L.call("elx_event_record", ev, s_read)
    L.call("elx_stream_wait_event", s_free, ev)
    L.call("elx_pool_free", X, s_free)
    X2 = ctypes.c_void_p()
    L.call("elx_pool_alloc", ctypes.byref(X2), n * 8, s_new)
    L.call("elx_fill2d", L.F64, n, 1, 2.0, X2, n, s_new)
    el.device_synchronize()
    y = Y.cpu().numpy()
    bad = int(np.count_nonzero(y != 1.0))
    assert bad == 0, f"{bad} of {n} entries changed under the delayed reader (reused: {X2.value == X.value})"
    L.call("elx_pool_free", X2, s_new)
    L.call("elx_event_destroy", ev)
    el.device_synchronize()


def view_on_other_stream():
    """DistMatrix level (the SetStream / shared-view hazard): a view of O moved
    to stream s2 is read there behind a spin; the view and then O are dropped
    (O's storage is returned on O's stream) and a new matrix of the same size
    is allocated and overwritten on O's stream at once.  ~DistMatrix orders O's
    stream after the view's work, so the reader still sees O's values."""
    g = el.Grid()
    m, n = 2048, 1024
    O = el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU, height=m, width=n).fill_hash(5, -1.0, 1.0)
    want = O.get_local()
    s2 = _stream()
    V = O(None, None)
    V.set_stream(s2.value)
    D = el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU)
    D.set_stream(s2.value)
    D.Resize(m, n)
    _spin(s2)
    el.Copy(V, D)  # on D's stream (s2), behind the spin
    del V
    del O
    N = el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU, height=m, width=n)
    N.fill_hash(6, 10.0, 1.0)  # on the library's stream, where O's block went back
    got = D.get_local()
    el.device_synchronize()
    assert np.array_equal(got, want), f"{int(np.count_nonzero(got != want))} entries differ"
    del N, D


def set_stream_owned():
    """SetStream on a matrix that owns allocated pool storage (the reference
    refuses it, Memory/impl.hpp:305-316; here it fences and rebinds): work
    queued on the old stream before the move (a spin, then a fill) is complete
    before work on the new stream reads the matrix."""
    g = el.Grid()
    m, n = 1024, 512
    A = el.DistMatrix(g, el.F64, el.MC, el.MR, el.GPU, height=m, width=n).fill_hash(7, 0.0, 1.0)
    want = A.get_local()
    s_old, s_new = _stream(), _stream()
    A.set_stream(s_old.value)
    _spin(s_old)
    el.Fill(A, 3.0)  # on s_old, behind the spin
    A.set_stream(s_new.value)
    el.Scale(2.0, A)  # on s_new: must see the fill
    got = A.get_local()
    assert np.all(got == 6.0), (got.min(), got.max(), np.array_equal(got, want))
    del A
    el.device_synchronize()


def debug_trace_cross_stream():
    """H_CUB_DEBUG=1 (cub.cpp:45-50): every allocation, cache return and reuse is
    logged; a block freed on one stream and requested on another shows up as a
    cross-stream reuse naming both streams and the event."""
    s1, s2 = _stream(), _stream()
    p = ctypes.c_void_p()
    L.call("elx_pool_alloc", ctypes.byref(p), 3 << 20, s1)
    _spin(s1)
    L.call("elx_pool_free", p, s1)
    q = ctypes.c_void_p()
    L.call("elx_pool_alloc", ctypes.byref(q), 3 << 20, s2)
    assert q.value == p.value
    L.call("elx_pool_free", q, s2)
    el.device_synchronize()


def release_off_the_lock():
    """Run with H_CUB_MAX_CACHED_SIZE=0, so every free is over the cap and its
    block goes back to the driver.  A block freed behind a ~0.2 s spin returns
    to the host at once (the event wait and hipFree happen on the allocator's
    release thread, never under its lock), a second thread's Alloc / Free
    completes while the spin still runs, and once the device is idle the
    bytes are back with the driver."""
    import threading
    import time
    s1, s2 = _stream(), _stream()
    base = el.pool_backing_reserved()
    n = (64 << 20) // 8
    X = ctypes.c_void_p()
    L.call("elx_pool_alloc", ctypes.byref(X), n * 8, s1)
    L.call("elx_fill2d", L.F64, n, 1, 1.0, X, n, s1)
    L.call("elx_stream_synchronize", s1)
    _spin(s1)
    spun = torch.cuda.Event()
    with torch.cuda.stream(torch.cuda.ExternalStream(s1.value)):
        spun.record()
    t0 = time.perf_counter()
    L.call("elx_pool_free", X, s1)
    dt_free = time.perf_counter() - t0
    other = {}

    def second_thread():
        t = time.perf_counter()
        q = ctypes.c_void_p()
        L.call("elx_pool_alloc", ctypes.byref(q), 32 << 20, s2)
        L.call("elx_pool_free", q, s2)
        other["dt"] = time.perf_counter() - t

    th = threading.Thread(target=second_thread)
    th.start()
    th.join(timeout=10)
    spin_running = not spun.query()
    el.device_synchronize()
    back = el.pool_backing_reserved()
    print(f"free {dt_free * 1e3:.3f} ms, second thread alloc+free {other.get('dt', -1) * 1e3:.3f} ms, "
          f"spin still running after it: {spin_running}, backing {base} -> {back}", flush=True)
    assert dt_free < 0.010, dt_free
    assert "dt" in other and spin_running, (other, spin_running)
    assert back == base, (base, back)


CASES = {f.__name__: f for f in (pool_free_after_delayed_reader, view_on_other_stream, set_stream_owned,
                                  debug_trace_cross_stream, release_off_the_lock)}

if __name__ == "__main__":
    for name in sys.argv[1:]:
        CASES[name]()
        print("OK", name, flush=True)
