"""Output recycling of the host-buffer entry points (Engine.outputs): a set of output arrays
is handed out again only when the caller holds no reference to any of them (CPU test: the
pool logic needs no device)."""
import sys
import threading

import numpy as np

from stereovision_amd import engine as EN


class _Pool:
    outputs = EN.Engine.outputs
    _register = EN.Engine._register      # no library: registration is skipped
    _unregister = EN.Engine._unregister

    def __init__(self):
        self._recycle = {}
        self._out_lock = threading.Lock()


SPEC = (((6, 5), np.float32), ((6, 5), np.float32), ((6, 5, 3), np.uint8))


def _ids(arrs):
    return [id(a) for a in arrs]


def test_released_set_is_reused():
    p = _Pool()
    a = p.outputs(SPEC)
    ids = _ids(a)
    assert [x.shape for x in a] == [(6, 5), (6, 5), (6, 5, 3)]
    assert [x.dtype for x in a] == [np.float32, np.float32, np.uint8]
    del a
    assert _ids(p.outputs(SPEC)) == ids


def test_held_arrays_views_and_buffers_block_reuse():
    p = _Pool()
    a = p.outputs(SPEC)
    ids = _ids(a)
    view = a[0][2:]           # a view keeps its base alive
    del a
    assert _ids(p.outputs(SPEC)) != ids
    del view
    b = p.outputs(SPEC)
    assert _ids(b) == ids
    mv = memoryview(b[2])      # an exported buffer too
    del b
    assert _ids(p.outputs(SPEC)) != ids
    del mv


def test_pool_is_bounded_and_keyed_by_shape():
    p = _Pool()
    held = [p.outputs(SPEC) for _ in range(5)]
    assert len(p._recycle[next(iter(p._recycle))]) == 3
    other = p.outputs((((2, 2), np.float32),))
    assert other[0].shape == (2, 2) and len(p._recycle) == 2
    assert len({id(h[0]) for h in held}) == 5   # every held set distinct


class _FakeLib:
    def __init__(self):
        self.registered = {}

    def sv_host_register(self, ptr, nbytes):
        self.registered[ptr] = nbytes
        return 0

    def sv_host_unregister(self, ptr):
        self.registered.pop(ptr)
        return 0


class _RegPool(_Pool):
    def __init__(self):
        super().__init__()
        self.lib = _FakeLib()


def test_registered_set_is_reused_every_call():
    """A set page-locked on its first reuse must keep being handed out: the registry may not
    hold a reference that makes the set look referenced (round 5: it did, so every other
    call allocated, page-faulted and registered a fresh 20 MB set and took the host
    expansion path)."""
    p = _RegPool()
    ids = _ids(p.outputs(SPEC))          # fresh set (not registered yet)
    for _ in range(6):                   # released every time: the same set, registered once
        got = p.outputs(SPEC)
        assert _ids(got) == ids
        del got
    assert len(p._recycle[next(iter(p._recycle))]) == 1
    assert len(p.lib.registered) == 3
    # popping a set from a full slot unregisters it
    held = [p.outputs(SPEC) for _ in range(4)]
    assert len(p.lib.registered) <= 9
    del held


def test_full_slot_never_evicts_a_held_set():
    """Eviction from a full slot takes the oldest RELEASED set only: a set another call still
    holds is never unregistered from under it (its DMA may be in flight)."""
    p = _RegPool()
    held = [p.outputs(SPEC) for _ in range(3)]        # fills the slot, all held
    for _ in range(3):
        extra = p.outputs(SPEC)                       # untracked: the slot keeps the held sets
        assert all(_ids(extra) != _ids(h) for h in held)
        del extra
    assert [_ids(s) for s in p._recycle[next(iter(p._recycle))]] == [_ids(h) for h in held]
    del held[1]
    new = p.outputs(SPEC)                             # the released one is reused
    assert _ids(new) not in [_ids(h) for h in held]


def test_concurrent_callers_never_share_a_set(monkeypatch):
    """Two threads taking and releasing output sets (the reference's 2-worker pool): no set is
    ever handed to both at once.  The check is widened on purpose (a thread switch right after
    a set is found released) so that an unlocked check-and-take would be caught."""
    import time
    orig = EN._set_unreferenced

    def slow(arrs):
        free = orig(arrs)
        if free:
            time.sleep(0.0002)
        return free
    monkeypatch.setattr(EN, "_set_unreferenced", slow)
    p = _Pool()
    in_use, lock, errors = set(), threading.Lock(), []
    old = sys.getswitchinterval()
    sys.setswitchinterval(1e-6)

    def worker():
        for _ in range(300):
            got = p.outputs(SPEC)
            key = id(got[0])
            with lock:
                if key in in_use:
                    errors.append(key)
                in_use.add(key)
            time.sleep(0.0001)                        # hold it for a moment
            with lock:
                in_use.discard(key)
            del got

    try:
        ts = [threading.Thread(target=worker) for _ in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    finally:
        sys.setswitchinterval(old)
    assert not errors


def test_pipeline_depth_is_capped_at_two_contexts_per_hardware_queue(monkeypatch):
    """DepthMapPipeline keeps at most 2 x GPU_MAX_HW_QUEUES (8 by default)
    frames in flight — past that the per-call staging time grows and the rate falls
    (profiles/r06_pipeline/sweep.txt); cap=False keeps the request (the measurement)."""
    from stereovision_amd import pipeline as P

    class _E:
        device = 0

        def __init__(self, *a):
            pass

        def close(self):
            pass
    monkeypatch.setattr(P, "get_engine", lambda d=None: _E())
    monkeypatch.setattr(P, "Engine", _E)
    monkeypatch.delenv("GPU_MAX_HW_QUEUES", raising=False)
    assert P.max_in_flight() == 8
    for req, exp in ((1, 1), (3, 3), (4, 4), (8, 8), (12, 8), (24, 8)):
        p = P.DepthMapPipeline(64, 9, depth=req)
        assert (p.requested_depth, p.depth, len(p._engines)) == (req, exp, exp)
        p.close()
    p = P.DepthMapPipeline(64, 9, depth=12, cap=False)
    assert p.depth == 12
    p.close()
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "8")
    assert P.max_in_flight() == 16
    p = P.DepthMapPipeline(64, 9, depth=12)
    assert p.depth == 12
    p.close()
