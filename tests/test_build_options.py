"""CPU: build-time options of the drop-in libraries.

LIBERASURECODE_SO_SUFFIX (include/erasurecode/erasurecode_version.h:35-37 of the reference): every
backend library name the frontend dlopen()s carries the suffix
(src/backends/rs_vand/liberasurecode_rs_vand.c:43, src/backends/xor/flat_xor_hd.c:45), and this
build's codec libraries carry it in their sonames, so a deployment that ships suffixed libraries
switches by path alone."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "liberasurecode_amd", "csrc")
LIB = os.path.join(ROOT, "liberasurecode_amd", "lib")
SFX = "-amdtest"


def _readelf(path):
    return subprocess.run(["readelf", "-d", path], capture_output=True, text=True, check=True).stdout


@pytest.fixture(scope="module")
def suffixed(tmp_path_factory):
    out = tmp_path_factory.mktemp("sfx")
    for name in ("libecamd.so", "libecamd_host.so"):  # reuse this build's device libraries
        os.symlink(os.path.join(LIB, name), out / name)
    targets = [str(out / f"liberasurecode_rs_vand{SFX}.so.1"), str(out / f"libXorcode{SFX}.so.1"),
               str(out / "liberasurecode.so.1")]
    subprocess.run(["make", "-s", "-C", CSRC, f"OUT={out}", f"SO_SUFFIX={SFX}"] + targets,
                   check=True)
    return out


def test_sonames_and_needed_carry_suffix(suffixed):
    assert f"[liberasurecode_rs_vand{SFX}.so.1]" in _readelf(
        str(suffixed / f"liberasurecode_rs_vand{SFX}.so.1"))
    assert f"[libXorcode{SFX}.so.1]" in _readelf(str(suffixed / f"libXorcode{SFX}.so.1"))
    assert f"NEEDED)             Shared library: [libXorcode{SFX}.so.1]" in _readelf(
        str(suffixed / "liberasurecode.so.1"))
    strings = subprocess.run(["strings", str(suffixed / "liberasurecode.so.1")],
                             capture_output=True, text=True, check=True).stdout.split()
    assert f"liberasurecode_rs_vand{SFX}.so.1" in strings
    assert "liberasurecode_rs_vand.so.1" not in strings


_PROBE = r"""
import ctypes as C, sys
lib = C.CDLL(sys.argv[1])
class A(C.Structure):
    _fields_ = [("k", C.c_int), ("m", C.c_int), ("w", C.c_int), ("hd", C.c_int),
                ("p1", C.c_uint64 * 4), ("p2", C.c_void_p), ("ct", C.c_int)]
lib.liberasurecode_instance_create.argtypes = [C.c_int, C.POINTER(A)]
a = A(k=4, m=2, w=16, hd=3, ct=1)
print(lib.liberasurecode_instance_create(6, C.byref(a)), lib.liberasurecode_backend_available(6))
"""


def _create_rc(frontend):
    r = subprocess.run([sys.executable, "-c", _PROBE, frontend], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    rc, avail = map(int, r.stdout.split())
    return rc, avail


def test_frontend_dlopens_the_suffixed_name(suffixed):
    front = str(suffixed / "liberasurecode.so.1")
    rc, avail = _create_rc(front)
    # the suffixed codec library is found; without a GPU its init fails (no CPU fallback)
    assert avail == 1
    assert rc > 0 or rc == -202, rc  # -EBACKENDINITERR
    # remove it: the unsuffixed name next to it is NOT a substitute
    hidden = suffixed / "hidden"
    hidden.mkdir(exist_ok=True)
    shutil.move(str(suffixed / f"liberasurecode_rs_vand{SFX}.so.1"), str(hidden))
    os.symlink(os.path.join(LIB, "liberasurecode_rs_vand.so.1"),
               suffixed / "liberasurecode_rs_vand.so.1")
    try:
        rc, avail = _create_rc(front)
        assert avail == 0 and rc == -204, rc  # -EBACKENDNOTAVAIL
    finally:
        os.unlink(suffixed / "liberasurecode_rs_vand.so.1")
        shutil.move(str(hidden / f"liberasurecode_rs_vand{SFX}.so.1"), str(suffixed))
