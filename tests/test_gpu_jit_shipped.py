"""GPU: the bitsliced kernels shipped with the library (lib/jit/, written by build() through
ecamd_bitslice_prebuild, liberasurecode_amd/prebuild.py) make the headline path independent of
first-use compiles.  Each case runs tests/jit_shipped_run.py in a FRESH process with an empty
$ECAMD_JIT_CACHE and the default knob (bitslice 1: never waits for a compile):

* the built library: C3 encode and the bench's decode {0,1,2,3} report ECAMD_FORM_BITSLICED and run
  the bitsliced kernel at their first launch; a map not shipped reports ECAMD_FORM_COMPILING and
  runs on the LDS tables meanwhile;
* a copy of the libraries WITHOUT ecamd_jitc but with jit/: the shipped maps still run bitsliced at
  once, the other reports ECAMD_FORM_UNAVAILABLE and runs on the tables;
* a copy without ecamd_jitc and without jit/: every map reports UNAVAILABLE and runs on the tables.
Every result byte-exact against the oracle.  (The reference builds its matrix at instance creation,
src/backends/rs_vand/liberasurecode_rs_vand.c:147-249; this is the GPU counterpart of "ready at
create".)"""
import json
import os
import shutil
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(os.path.dirname(HERE), "liberasurecode_amd", "lib")
TABLES, BITSLICED, COMPILING, UNAVAILABLE = 0, 1, 2, 3


def _run(tmp_path, libdir):
    cache = tmp_path / "jitcache"
    cache.mkdir(mode=0o700)
    env = dict(os.environ, ECAMD_JIT_CACHE=str(cache))
    if libdir:
        env["LIBERASURECODE_AMD_LIBDIR"] = libdir
    r = subprocess.run([sys.executable, os.path.join(HERE, "jit_shipped_run.py")], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def _copy_libs(tmp_path, with_jit):
    dst = tmp_path / "lib"
    dst.mkdir()
    for name in os.listdir(LIB):
        src = os.path.join(LIB, name)
        if name == "ecamd_jitc" or os.path.isdir(src):
            continue
        shutil.copy2(src, dst / name)
    if with_jit:
        shutil.copytree(os.path.join(LIB, "jit"), dst / "jit")
    return str(dst)


def test_shipped_objects_exist():
    assert os.path.isdir(os.path.join(LIB, "jit")), "build() did not prebuild lib/jit"
    assert any(n.endswith(".co") for n in os.listdir(os.path.join(LIB, "jit")))


def test_fresh_process_runs_shipped_bitsliced_at_first_launch(tmp_path):
    out = _run(tmp_path, None)
    assert out["encode_form"] == BITSLICED and out["encode_bitsliced_launches"] > 0, out
    assert out["decode_shipped_form"] == BITSLICED and out["decode_shipped_bitsliced_launches"] > 0, out
    assert out["decode_other_form"] == COMPILING and out["decode_other_bitsliced_launches"] == 0, out
    assert out["encode_exact"] and out["decode_shipped_exact"] and out["decode_other_exact"], out
    assert out["frame_bitsliced_launches"] > 0 and out["frame_exact"], out  # ecamd_frame_prebuild
    for name in ("reconstruct6", "decode_2_7"):  # rebuild traffic's maps, never benched (prebuild.rebuild_ops)
        assert out[name + "_form"] == BITSLICED and out[name + "_bitsliced_launches"] > 0, out
        assert out[name + "_exact"], out
    # a small one-stripe operation: gf16_small_kernel, reported as such (no compile started for it)
    assert out["small16k_form"] == TABLES and out["small16k_bitsliced_launches"] == 0, out
    assert out["small16k_exact"], out


def test_without_helper_shipped_maps_still_bitsliced(tmp_path):
    out = _run(tmp_path, _copy_libs(tmp_path, True))
    assert out["available"] == 0, out
    assert out["encode_form"] == BITSLICED and out["encode_bitsliced_launches"] > 0, out
    assert out["decode_shipped_form"] == BITSLICED and out["decode_shipped_bitsliced_launches"] > 0, out
    assert out["decode_other_form"] == UNAVAILABLE and out["decode_other_bitsliced_launches"] == 0, out
    assert out["encode_exact"] and out["decode_shipped_exact"] and out["decode_other_exact"], out
    assert out["frame_bitsliced_launches"] > 0 and out["frame_exact"], out
    for name in ("reconstruct6", "decode_2_7"):
        assert out[name + "_form"] == BITSLICED and out[name + "_bitsliced_launches"] > 0, out
        assert out[name + "_exact"], out


def test_without_helper_or_shipped_objects_tables_serve(tmp_path):
    out = _run(tmp_path, _copy_libs(tmp_path, False))
    for name in ("encode", "decode_shipped", "decode_other", "frame", "reconstruct6", "decode_2_7"):
        assert out[name + "_bitsliced_launches"] == 0, out
    for name in ("encode", "decode_shipped", "decode_other", "reconstruct6", "decode_2_7"):
        assert out[name + "_form"] == UNAVAILABLE, out
        assert out[name + "_exact"], out
    assert out["frame_exact"], out
