"""PinnedPool bookkeeping on the CPU (no page-locked memory is allocated: the blocks are
fake addresses and stay under keep_bytes, so the library is never called).

ADVICE r5: the release callback runs from weakref.finalize, which a cyclic collection can
start in the middle of an allocation made while the same thread holds the pool's lock; it must
then not wait on that lock."""

import threading

from sctools_amd import _lib


def test_release_while_lock_held_does_not_block():
    pool = _lib.PinnedPool(keep_bytes=1 << 30, max_bytes=1 << 30)
    c = _lib.PinnedPool.MIN_BYTES
    pool._held = 2 * c
    done = threading.Event()
    with pool._mu:  # this thread holds the lock, as inside empty() / trim()
        t = threading.Thread(target=lambda: (pool._release(0x1000, c), done.set()))
        t.start()
        t.join(5)
        assert done.is_set(), "release waited on the pool lock"
        pool._release(0x2000, c)  # same thread, lock held: queued, not a deadlock
        assert len(pool._pending) == 2 and pool._idle == 0
    pool._drain()
    assert not pool._pending
    assert sorted(pool._free[c]) == [0x1000, 0x2000] and pool._idle == 2 * c and pool._held == 2 * c


def test_trim_files_pending_blocks_first():
    pool = _lib.PinnedPool(keep_bytes=1 << 30, max_bytes=1 << 30)
    c = _lib.PinnedPool.MIN_BYTES
    pool._held = c
    with pool._mu:
        pool._release(0x3000, c)
    freed = []

    class FakeLib:
        def sct_host_free(self, p):
            freed.append(p.value)

    real = _lib.lib
    _lib.lib = lambda: FakeLib()
    try:
        pool.trim()
    finally:
        _lib.lib = real
    assert freed == [0x3000] and pool._held == 0 and pool._idle == 0 and not pool._pending


def test_idle_blocks_make_room_for_the_latest():
    """A block handed back stays idle when it fits keep_bytes on its own; the longest-idle blocks are
    freed to make room for it (so a repeated large call reuses its block instead of page-locking a
    new one), and a block larger than keep_bytes is freed at once."""
    MB = _lib.PinnedPool.MIN_BYTES
    pool = _lib.PinnedPool(keep_bytes=4 * MB, max_bytes=1 << 30)
    pool._held = 1 * MB + 2 * MB + 4 * MB + 8 * MB
    freed = []

    class FakeLib:
        def sct_host_free(self, p):
            freed.append(p.value)

    real = _lib.lib
    _lib.lib = lambda: FakeLib()
    try:
        pool._release(0x10, MB)
        pool._release(0x20, 2 * MB)
        assert pool._idle == 3 * MB and not freed
        pool._release(0x40, 4 * MB)  # both older blocks go
        assert sorted(freed) == [0x10, 0x20] and pool._idle == 4 * MB and pool._free[4 * MB] == [0x40]
        pool._release(0x80, 8 * MB)  # larger than keep_bytes: freed, the idle one stays
        assert freed[-1] == 0x80 and pool._free[4 * MB] == [0x40]
        assert pool._held == 4 * MB and list(pool._order) == [(4 * MB, 0x40)]
    finally:
        _lib.lib = real
