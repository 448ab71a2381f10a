import threading
import time

import pytest

from distributed_compute_pytorch_amd._ext import C
from distributed_compute_pytorch_amd.distributed.launch import free_port


def test_set_get_add_check_delete():
    s = C.TCPStore("127.0.0.1", 0, 1, True, 5000, True)
    s.set("k", b"v1")
    assert s.get("k") == b"v1"
    assert s.add("ctr", 3) == 3 and s.add("ctr", -1) == 2
    assert s.check(["k", "ctr"]) and not s.check(["nope"])
    assert s.delete_key("k") and not s.check(["k"])
    assert s.num_keys() >= 1
    assert s.compare_set("cas", b"", b"a") == b"a"
    assert s.compare_set("cas", b"x", b"b") == b"a"
    assert s.compare_set("cas", b"a", b"b") == b"b"
    s.set("bin", bytes(range(256)))
    assert s.get("bin") == bytes(range(256))


def test_get_blocks_until_set_and_times_out():
    port = free_port()
    master = C.TCPStore("127.0.0.1", port, 2, True, 3000, False)
    client = C.TCPStore("127.0.0.1", port, 2, False, 3000, False)

    def setter():
        time.sleep(0.3)
        client.set("late", b"ok")

    t = threading.Thread(target=setter)
    t.start()
    assert master.get("late") == b"ok"
    t.join()
    master.timeout_ms = 200
    with pytest.raises(TimeoutError):
        master.get("never")
    with pytest.raises(TimeoutError):
        master.wait(["never2"], 100)


def test_barrier_threads():
    port = free_port()
    n = 4
    stores = [None] * n
    errs = []

    def mk(i):
        try:
            stores[i] = C.TCPStore("127.0.0.1", port, n, i == 0, 10000, True)
            stores[i].barrier("b")
            stores[i].barrier("b")
        except Exception as e:  # pragma: no cover
            errs.append(e)

    ts = [threading.Thread(target=mk, args=(i,)) for i in range(n)]
    [t.start() for t in ts]
    [t.join(20) for t in ts]
    assert not errs
