"""CPU tests of ecamd_host_copy (host/copy_pool.cpp, include/ecamd_host.h): the batched host copies
the per-call staging and liberasurecode.so.1 run through helper threads.  Byte-exact for ragged
batches on both sides of the 1 MiB parallel threshold, from many caller threads at once (one gets
the helpers, the others copy alone), with the helpers disabled, and in a forked child (which must
copy alone without touching the parent's locks)."""
import ctypes as C
import os
import subprocess
import sys
import threading

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "liberasurecode_amd", "lib", "libecamd_host.so")


def lib():
    h = C.CDLL(LIB)
    h.ecamd_host_copy.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
    h.ecamd_host_copy.restype = C.c_int
    return h


def run_copy(h, srcs, dsts):
    n = len(srcs)
    d = (C.c_void_p * n)(*[x.ctypes.data for x in dsts])
    s = (C.c_void_p * n)(*[x.ctypes.data for x in srcs])
    ln = (C.c_int64 * n)(*[x.nbytes for x in srcs])
    return h.ecamd_host_copy(n, d, s, ln)


@pytest.mark.parametrize("sizes", [[0], [1], [17, 0, 5], [1 << 20], [(1 << 20) - 1, 1],
                                   [(256 << 10) + 3] * 7, [3 << 20, 5, (1 << 20) + 17, 0, 999_999],
                                   [10 << 20]])
def test_copy_exact(sizes):
    h = lib()
    rng = np.random.default_rng(len(sizes) * 31 + sum(sizes) % 1000)
    srcs = [rng.integers(0, 256, n, dtype=np.uint8) for n in sizes]
    dsts = [np.full(n + 64, 0xEE, np.uint8) for n in sizes]  # guard bytes after each region
    assert run_copy(h, srcs, [d[:len(s)] for d, s in zip(dsts, srcs)]) == 0
    for s, d in zip(srcs, dsts):
        assert np.array_equal(d[:len(s)], s)
        assert (d[len(s):] == 0xEE).all()


def test_copy_bad_arguments():
    h = lib()
    assert h.ecamd_host_copy(0, None, None, None) == 0
    assert h.ecamd_host_copy(2, None, None, None) == -22


def test_copy_concurrent_callers():
    h = lib()
    errors = []

    def job(t):
        rng = np.random.default_rng(t)
        for it in range(6):
            sizes = [int(x) for x in rng.integers(0, 700_000, 1 + (t + it) % 6)]
            srcs = [rng.integers(0, 256, n, dtype=np.uint8) for n in sizes]
            dsts = [np.zeros(n, np.uint8) for n in sizes]
            if run_copy(h, srcs, dsts) != 0 or not all(np.array_equal(a, b) for a, b in zip(srcs, dsts)):
                errors.append((t, it))

    threads = [threading.Thread(target=job, args=(t,)) for t in range(8)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert errors == []


_CHILD = r"""
import ctypes as C, os, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import test_host_copy as T
h = T.lib()
src = [np.arange(3 << 20, dtype=np.uint8), np.arange(5, dtype=np.uint8)]
dst = [np.zeros(3 << 20, np.uint8), np.zeros(5, np.uint8)]
assert T.run_copy(h, src, dst) == 0 and all(np.array_equal(a, b) for a, b in zip(src, dst))
if os.environ.get("ECAMD_TEST_FORK"):
    pid = os.fork()
    if pid == 0:  # the helpers live in the parent: the child copies alone
        dst2 = [np.zeros(3 << 20, np.uint8), np.zeros(5, np.uint8)]
        ok = T.run_copy(h, src, dst2) == 0 and all(np.array_equal(a, b) for a, b in zip(src, dst2))
        os._exit(0 if ok else 1)
    _, status = os.waitpid(pid, 0)
    assert os.waitstatus_to_exitcode(status) == 0
print("OK")
"""


@pytest.mark.parametrize("env", [{"ECAMD_COPY_THREADS": "0"}, {"ECAMD_COPY_THREADS": "2"},
                                 {"ECAMD_TEST_FORK": "1"}])
def test_copy_helpers_off_and_fork(env):
    e = dict(os.environ, **env)
    r = subprocess.run([sys.executable, "-c", _CHILD, os.path.dirname(os.path.abspath(__file__))],
                       capture_output=True, text=True, timeout=120, env=e)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().endswith("OK")


@pytest.mark.parametrize("sizes", [[0], [1], [17, 0, 5], [(256 << 10) + 3] * 7, [3 << 20, 5, (1 << 20) + 17],
                                   [10 << 20]])
@pytest.mark.parametrize("second", ["all", "some"])
def test_copy2_exact(sizes, second):
    """ecamd_host_copy2: every copy lands in dst and -- where a second destination is given -- in
    dst2 too, byte-exact, guard bytes intact (the per-call staging pack with frontend tees)."""
    h = lib()
    h.ecamd_host_copy2.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    rng = np.random.default_rng(len(sizes) * 7 + sum(sizes) % 997)
    srcs = [rng.integers(0, 256, n, dtype=np.uint8) for n in sizes]
    d1 = [np.full(n + 64, 0xEE, np.uint8) for n in sizes]
    d2 = [np.full(n + 64, 0xDD, np.uint8) for n in sizes]
    use2 = [second == "all" or i % 2 == 0 for i in range(len(sizes))]
    n = len(sizes)
    dst = (C.c_void_p * n)(*[x.ctypes.data for x in d1])
    dst2 = (C.c_void_p * n)(*[x.ctypes.data if u else None for x, u in zip(d2, use2)])
    src = (C.c_void_p * n)(*[x.ctypes.data for x in srcs])
    ln = (C.c_int64 * n)(*[x.nbytes for x in srcs])
    assert h.ecamd_host_copy2(n, dst, dst2, src, ln) == 0
    for s, a, b, u in zip(srcs, d1, d2, use2):
        assert np.array_equal(a[:len(s)], s) and (a[len(s):] == 0xEE).all()
        if u:
            assert np.array_equal(b[:len(s)], s)
            assert (b[len(s):] == 0xDD).all()
        else:
            assert (b == 0xDD).all()
    assert h.ecamd_host_copy2(1, None, None, None, None) == -22
