"""The multi-device group's failure protocol (sctools_amd.multigpu.GroupRun), on CPU threads.

The group's one collective is the gene-partial all-reduce that replaces MergeGeneMetrics
(merge.py:74-191).  A rank that fails before it must not leave its peers blocked in a collective
whose peers never come; a rank that fails while a collective is in flight must cancel it
(ncclCommAbort on the devices; here a stub abort).  The stub collective below is a threading
barrier, which blocks exactly as an all-reduce with a missing peer does.
"""

import ctypes
import threading
import time

import pytest

from sctools_amd.multigpu import GroupAborted, GroupRun, parse_devices


class StubComms:
    """An 'all-reduce' that returns only when both ranks called it, and an abort that releases it."""

    def __init__(self, size=2):
        self.barrier = threading.Barrier(size)
        self.aborts = 0
        self.sums = [None] * size

    def allreduce(self, rank, value, timeout=30.0):
        self.sums[rank] = value
        self.barrier.wait(timeout)  # blocks while a peer is missing (BrokenBarrierError on abort)
        return sum(self.sums)

    def abort(self):
        self.aborts += 1
        self.barrier.abort()


def _run(g, fn, limit=10.0):
    t0 = time.monotonic()
    try:
        return g.run(fn)
    finally:
        assert time.monotonic() - t0 < limit, "the group did not return promptly"


def test_success_sums_on_every_rank():
    c = StubComms()
    g = GroupRun(2, abort_fn=c.abort, timeout=10)

    def fn(r):
        g.before_collective(r)
        return c.allreduce(r, r + 1)

    assert _run(g, fn) == [3, 3]
    assert c.aborts == 0


def test_rank_failing_before_the_collective_raises_instead_of_hanging():
    c = StubComms()
    g = GroupRun(2, abort_fn=c.abort, timeout=30)

    def fn(r):
        if r == 1:
            time.sleep(0.2)  # rank 0 is already waiting at the collective
            raise RuntimeError("rank 1: decode error")
        g.before_collective(r)
        return c.allreduce(r, 1)  # never reached

    with pytest.raises(RuntimeError, match="decode error"):
        _run(g, fn)
    assert c.aborts == 1
    assert c.sums == [None, None], "no rank issued the collective"


def test_rank_failing_during_the_collective_cancels_it():
    c = StubComms()
    g = GroupRun(2, abort_fn=c.abort, timeout=30)
    issued = threading.Event()

    def fn(r):
        g.before_collective(r)
        if r == 1:
            issued.wait(5)
            raise MemoryError("rank 1: out of device memory")  # after rank 0 issued its all-reduce
        done = threading.Event()

        def device():  # the collective in flight: completes only if rank 1 joins (or is aborted)
            try:
                c.allreduce(r, 1)
            except threading.BrokenBarrierError:
                pass
            done.set()

        threading.Thread(target=device, daemon=True).start()
        issued.set()
        g.wait(r, lambda: False)  # the stream never completes on its own

    with pytest.raises(MemoryError):
        _run(g, fn)
    assert c.aborts == 1


def test_collective_that_never_completes_times_out():
    c = StubComms()
    g = GroupRun(2, abort_fn=c.abort, timeout=0.3)

    def fn(r):
        g.before_collective(r)
        g.wait(r, lambda: False)

    with pytest.raises(TimeoutError):
        _run(g, fn)
    assert c.aborts == 1


def test_rank_that_never_arrives_times_out():
    c = StubComms()
    g = GroupRun(2, abort_fn=c.abort, timeout=0.3)

    def fn(r):
        if r == 1:
            time.sleep(1.0)  # returns without reaching the collective
            return None
        g.before_collective(r)

    with pytest.raises(TimeoutError):
        _run(g, fn)


def test_group_aborted_is_reported_only_without_a_root_cause():
    g = GroupRun(3, timeout=10)

    def fn(r):
        if r == 2:
            raise ValueError("root cause")
        g.before_collective(r)

    with pytest.raises(ValueError, match="root cause"):
        _run(g, fn)


def test_parse_devices_allows_shards_sharing_a_device():
    assert parse_devices(3) == [0, 1, 2]
    assert parse_devices([0, 0, 1]) == [0, 0, 1]
    with pytest.raises(ValueError):
        parse_devices(0)
    with pytest.raises(ValueError):
        parse_devices([])


def test_device_group_stays_aborted():
    """after abort() a rank reaching its communicator raises GroupAborted; neither it nor
    comms() re-initialises communicators (a fresh ncclCommInitAll from a late rank would issue an
    all-reduce whose peers never come).  CPU: a DeviceGroup shell with a stub library."""
    from sctools_amd.multigpu import DeviceGroup

    class Lib:
        def __init__(self):
            self.aborted, self.inits = [], 0

        def sct_comm_abort(self, c):
            self.aborted.append(c.value)

        def sct_comm_init_all(self, *a):
            self.inits += 1
            return 0

    g = object.__new__(DeviceGroup)
    g.devices, g.shared, g.lib, g._run, g._aborted = [0, 1], False, Lib(), None, False
    g._comms = (ctypes.c_void_p * 2)(11, 12)
    assert g._rank_comm(1) == 12
    g.abort()
    assert g.lib.aborted == [11, 12]
    with pytest.raises(GroupAborted):
        g._rank_comm(0)
    with pytest.raises(GroupAborted):
        g.comms()
    assert g.lib.inits == 0
    g.abort()  # idempotent: nothing left to abort
    assert g.lib.aborted == [11, 12]
