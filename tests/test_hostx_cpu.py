"""pe_host_exchange (include/placement.h): the shared-memory all-gather the sharded greedy uses when
RCCL cannot be set up.  CPU only: 2 and 3 processes, many calls of varying size, every rank's
result checked; the name is gone from /dev/shm once every rank attached; a missing peer times out."""
import multiprocessing as mp
import os
import sys
import time
import uuid

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "training-operator_amd")]


def _worker(name, rank, world, calls, q):
    try:
        from placement import HostExchange
        hx = HostExchange(name, rank, world, 4096)
        bad = 0
        for k in range(calls):
            n = (k * 37) % 4097          # 0 .. 4096 bytes, identical on every rank
            blob = bytes(((rank * 131 + k + i) & 0xFF) for i in range(n))
            out = hx.allgather(blob)
            want = b"".join(bytes(((r * 131 + k + i) & 0xFF) for i in range(n)) for r in range(world))
            bad += out != want
        hx.close()
        q.put((rank, bad))
    except Exception as ex:  # noqa: BLE001
        q.put((rank, repr(ex)))


@pytest.mark.parametrize("world", [2, 3])
def test_host_exchange_allgather(world):
    name = f"/pe_hx_test_{uuid.uuid4().hex[:12]}"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(name, r, world, 300, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert res == {r: 0 for r in range(world)}, res
    assert not os.path.exists("/dev/shm" + name)


def test_host_exchange_peer_missing_times_out():
    from placement import HostExchange, PlacementError
    os.environ["PE_HX_TIMEOUT_S"] = "1"
    try:
        name = f"/pe_hx_test_{uuid.uuid4().hex[:12]}"
        hx = HostExchange(name, 0, 2, 64)
        t0 = time.time()
        with pytest.raises(PlacementError) as ei:
            hx.allgather(b"x" * 8)
        assert ei.value.code == -5 and time.time() - t0 < 30
        hx.close()
        assert not os.path.exists("/dev/shm" + name)
        with pytest.raises(PlacementError):      # rank 1 with no rank 0: the segment never appears
            HostExchange(f"/pe_hx_test_{uuid.uuid4().hex[:12]}", 1, 2, 64)
    finally:
        del os.environ["PE_HX_TIMEOUT_S"]
