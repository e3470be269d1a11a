"""parallel.ThreadLoopback, the host transport of the one-GPU multi-rank
tests, on CPU: rank-order sums (u32 wraps like RCCL), min / max,
all-gather-v with uneven and empty segments, and the failure paths (a
mismatched collective or a failing rank ends every rank, none waits)."""
import threading

import numpy as np
import pytest

from pynbodyext.parallel import OP_MAX, OP_MIN, OP_SUM, ThreadLoopback


def _run(world, fn, timeout=30):
    lb = ThreadLoopback(world, timeout=timeout)
    out = [None] * world
    errs = [None] * world

    def body(r):
        lb._rank.value = r
        try:
            out[r] = fn(lb, r)
        except BaseException as e:  # noqa: BLE001
            errs[r] = e
            lb.abort()

    ts = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout + 5)
    assert not any(t.is_alive() for t in ts)
    return out, errs


def test_allreduce_ops_and_dtypes():
    def fn(lb, r):
        f = np.array([0.1 * (r + 1), -1.0, r], dtype=np.float64)
        lb.allreduce(f, OP_SUM)
        u = np.full(3, 0xFFFFFFF0 + r, dtype=np.uint32)
        lb.allreduce(u, OP_SUM)
        k = np.array([r, 10 - r], dtype=np.uint64)
        lo, hi = k.copy(), k.copy()
        lb.allreduce(lo, OP_MIN)
        lb.allreduce(hi, OP_MAX)
        return f, u, lo, hi

    out, errs = _run(4, fn)
    assert errs == [None] * 4
    want_f = ((0.1 + 0.2) + 0.30000000000000004) + 0.4  # rank order
    for f, u, lo, hi in out:
        assert f[0] == want_f and f[1] == -4.0 and f[2] == 6.0
        assert np.all(u == (sum(0xFFFFFFF0 + r for r in range(4)) & 0xFFFFFFFF))
        assert list(lo) == [0, 7] and list(hi) == [3, 10]


def test_allgatherv_uneven_and_empty():
    counts, displs = [3, 0, 5, 1], [0, 3, 3, 8]

    def fn(lb, r):
        buf = np.zeros(9, dtype=np.uint8)
        buf[displs[r]:displs[r] + counts[r]] = r + 1
        lb.allgatherv(buf, counts, displs)
        return buf

    out, errs = _run(4, fn)
    assert errs == [None] * 4
    for b in out:
        assert list(b) == [1, 1, 1, 3, 3, 3, 3, 3, 4]


def test_mismatched_allreduce_fails_every_rank():
    def fn(lb, r):
        lb.allreduce(np.zeros(2 + r), OP_SUM)

    _, errs = _run(3, fn)
    assert all(isinstance(e, RuntimeError) for e in errs)


def test_failing_rank_releases_the_others():
    def fn(lb, r):
        if r == 1:
            raise ValueError("rank 1 fails before the collective")
        lb.allreduce(np.zeros(4), OP_SUM)

    _, errs = _run(3, fn, timeout=60)
    assert isinstance(errs[1], ValueError)
    assert all(isinstance(errs[r], threading.BrokenBarrierError) for r in (0, 2))


def test_run_requires_the_library():
    """run() creates pbx_comm_init_host communicators: on a machine without a
    GPU that fails loudly (no CPU fallback)."""
    from pynbodyext import _native as nat

    try:
        n = nat.device_count()
    except RuntimeError:
        n = 0
    if n:
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        ThreadLoopback(2).run(lambda comm: None)
