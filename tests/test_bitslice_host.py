"""CPU: the bitsliced GF(2^16) network (liberasurecode_amd/csrc/host/bitslice.cpp).

Multiplication by a constant is GF(2)-linear (rs_galois_mult == carry-less multiply mod 0x1100b,
src/builtin/rs_vand/rs_galois.c:90-100), so an output word is an XOR of input bits.  The network
built for a matrix -- bit planes, distance-guided temporaries, three-input accumulation -- is evaluated on
the host and compared with the numpy GF(2^16) products and, for the reference generators, with the
oracle's encode; the generated kernel source must compile for gfx950."""
import ctypes as C
import os
import shutil
import subprocess

import numpy as np
import pytest

import gfnp
import oracle_lib as orc
from liberasurecode_amd import _lib


def evaluate(coeff, R, K, cap, words):
    out = np.zeros((R, 32), np.uint16)
    ops = C.c_int()
    assert _lib.host().ecamd_bitslice_eval(_lib.ints(coeff), R, K, cap, words.ctypes.data,
                                           out.ctypes.data, C.byref(ops)) == 0
    return out, ops.value


@pytest.mark.parametrize("R,K", [(1, 1), (5, 3), (8, 20), (8, 32), (6, 17), (7, 1)])
@pytest.mark.parametrize("cap", [0, 8, 24])
def test_network_matches_gf_products(R, K, cap):
    rng = np.random.default_rng(R * 100 + K + cap)
    coeff = rng.integers(0, 65536, R * K).tolist()
    coeff[0] = 0
    coeff[-1] = 1
    words = rng.integers(0, 65536, (K, 32), dtype=np.uint16)
    got, ops = evaluate(coeff, R, K, cap, words)
    want = gfnp.apply_map(np.array(coeff).reshape(R, K).tolist(), [w.view(np.uint8) for w in words])
    assert (got.view(np.uint8) == np.stack(want)).all()
    assert ops > 0


@pytest.mark.parametrize("k,m", [(20, 8), (10, 6), (12, 5)])
def test_network_of_reference_generator(k, m):
    G = orc.generator(k, m)
    data = np.random.default_rng(k).integers(0, 256, (k, 64), dtype=np.uint8)
    got, ops = evaluate(G[k * k:], m, k, 24, data.view(np.uint16).copy())
    assert (got.view(np.uint8) == orc.encode(k, m, data)).all()


def test_shared_pairs_cut_the_work():
    G = orc.generator(20, 8)
    words = np.zeros((20, 32), np.uint16)
    _, plain = evaluate(G[400:], 8, 20, 0, words)
    _, cse = evaluate(G[400:], 8, 20, 24, words)
    assert cse < 0.7 * plain


@pytest.mark.skipif(not shutil.which("/opt/rocm/bin/hipcc"), reason="needs hipcc")
@pytest.mark.parametrize("depth,cap", [(0, 64), (2, 96), (4, 96)])
def test_generated_source_compiles_for_gfx950(tmp_path, depth, cap):
    """C5 encode: both forms fit without spills at the caps the JIT tries first; it steps down
    through its caps when the compiler spills (hip/ecamd_jit.hip)."""
    G = orc.generator(20, 8)
    h = _lib.host()
    n = h.ecamd_bitslice_source(_lib.ints(G[400:]), 8, 20, cap, depth, None, 0)
    buf = C.create_string_buffer(n + 1)
    h.ecamd_bitslice_source(_lib.ints(G[400:]), 8, 20, cap, depth, buf, n + 1)
    src = tmp_path / "bs.hip"
    src.write_text("#include <hip/hip_runtime.h>\n" + buf.value.decode())
    out = tmp_path / "bs.s"
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "--cuda-device-only",
                        "-S", "-o", str(out), str(src)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    asm = out.read_text()
    assert "ScratchSize: 0" in asm          # the network fits the registers: no spills
    assert "Occupancy: 2" in asm            # 2 waves per SIMD
    if depth:
        assert " lds" in asm and "ds_read_b128" in asm   # LDS-DMA ring


JITC = os.path.join(os.path.dirname(_lib.__file__), "lib", "ecamd_jitc")


@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/libhiprtc.so"), reason="needs hiprtc")
def test_jitc_builds_a_request(tmp_path):
    """The child-process compiler (csrc/jit/jitc.cpp) libecamd starts for each new matrix: the
    network search and the hiprtc compile both run there; the code object appears whole."""
    G = orc.generator(12, 5)
    req = tmp_path / "bs.req"
    rows = [" ".join(str(c) for c in G[12 * 12 + 12 * r:12 * 12 + 12 * (r + 1)]) for r in range(5)]
    req.write_text("ecamd-bitslice-request 1\n5 12 40 0\n" + "\n".join(rows) + "\n")
    out = tmp_path / "bs.co"
    env = dict(os.environ, ECAMD_JIT_KEEP_SOURCE="1")
    r = subprocess.run([JITC, str(req), str(out)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert out.read_bytes()[:4] == b"\x7fELF"
    assert "5 outputs x 12 inputs" in (tmp_path / "bs.hip").read_text()
    assert not req.exists()  # the request is consumed
    assert not [p for p in os.listdir(tmp_path) if ".tmp." in p]
    bad = tmp_path / "bad.req"
    for text in ("nonsense\n", "ecamd-bitslice-request 1\n9 12 40 0\n", "ecamd-bitslice-request 1\n1 1 40 0\n70000\n"):
        bad.write_text(text)
        assert subprocess.run([JITC, str(bad), str(tmp_path / "bad.co")], capture_output=True).returncode == 2
    assert not (tmp_path / "bad.co").exists()


@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/libhiprtc.so") or not shutil.which("/opt/rocm/bin/hipcc"),
                    reason="needs hiprtc and hipcc")
@pytest.mark.parametrize("flags,tag", [(19, "crc"), (193, "wave_copy")])
def test_jitc_builds_realigned_inputs(tmp_path, flags, tag):
    """Version-3 requests (round 4): copy-through inputs at offsets that are not multiples of 16 --
    Swift's object chunks j*104858 -- get aligned loads + the neighbour lane's chunk, realigned with
    a compile-time shift (BitsliceStyle::in_shift); the crc variant and the one-wave copy form both
    build, the crc one without scratch.  Malformed shift lines are refused."""
    G = orc.generator(10, 4)
    shifts = [(j * 104858) % 16 for j in range(10)]
    rows = [" ".join(str(c) for c in G[100 + 10 * r:100 + 10 * (r + 1)]) for r in range(4)]
    head = f"ecamd-bitslice-request 3\n4 10 16 0 {flags}\n"  # cap 16: the step the JIT reaches (40 spills)
    req = tmp_path / "bs.req"
    req.write_text(head + " ".join(map(str, shifts)) + "\n" + "\n".join(rows) + "\n")
    out = tmp_path / "bs.co"
    env = dict(os.environ, ECAMD_JIT_KEEP_SOURCE="1")
    r = subprocess.run([JITC, str(req), str(out)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert out.read_bytes()[:4] == b"\x7fELF"
    src = (tmp_path / "bs.hip").read_text()
    assert "rlg<10>(" in src and "rlg<4>(" in src and "l63 ?" in src
    assert "a.in_off[0] + off" in src  # input 0 (shift 0) keeps its plain loads
    if tag == "crc":
        hip = tmp_path / "k.hip"
        hip.write_text("#include <hip/hip_runtime.h>\n" + src)
        r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "--cuda-device-only", "-S",
                            "-o", str(tmp_path / "k.s"), str(hip)], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        assert "ScratchSize: 0" in (tmp_path / "k.s").read_text()
    bad = tmp_path / "bad.req"
    body = "\n".join(rows) + "\n"
    for text in (head + "16 " + " ".join(map(str, shifts[1:])) + "\n" + body,  # shift out of range
                 head + " ".join("0" for _ in shifts) + "\n" + body,          # no shift: version 2's job
                 "ecamd-bitslice-request 3\n4 10 40 0 64\n" + " ".join(map(str, shifts)) + "\n" + body):  # no copy
        bad.write_text(text)
        assert subprocess.run([JITC, str(bad), str(tmp_path / "bad.co")], capture_output=True).returncode == 2


@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/libhiprtc.so") or not shutil.which("/opt/rocm/bin/hipcc"),
                    reason="needs hiprtc and hipcc")
def test_jitc_realign_lane_experiment(tmp_path):
    """Experiment flag ECAMD_BS_RLANE (round 4, profiles/r04_rlane_ab.log): the one-wave copy-through
    form takes the last lane's next chunk of chunks 0-2 from lane 0 of the following chunk by
    v_readlane and loads only chunk 3's; the kernel builds without scratch and issues fewer loads."""
    G = orc.generator(10, 4)
    shifts = [(j * 104858) % 16 for j in range(10)]
    rows = [" ".join(str(c) for c in G[100 + 10 * r:100 + 10 * (r + 1)]) for r in range(4)]
    req_text = f"ecamd-bitslice-request 3\n4 10 96 0 {1 | 192 | (2 << 8)}\n" + " ".join(map(str, shifts)) + "\n" + \
        "\n".join(rows) + "\n"
    loads = {}
    for rl in ("0", "1"):
        req = tmp_path / f"rl{rl}.req"
        req.write_text(req_text)
        out = tmp_path / f"rl{rl}.co"
        env = dict(os.environ, ECAMD_JIT_KEEP_SOURCE="1", ECAMD_BS_RLANE=rl)
        r = subprocess.run([JITC, str(req), str(out)], capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stderr[-2000:]
        src = (tmp_path / f"rl{rl}.hip").read_text()
        assert ("xh[c] = lane0(xa[c + 1]);" in src) == (rl == "1")
        hip = tmp_path / f"k{rl}.hip"
        hip.write_text("#include <hip/hip_runtime.h>\n" + src)
        asm = tmp_path / f"k{rl}.s"
        r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "--cuda-device-only", "-S",
                            "-o", str(asm), str(hip)], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        text = asm.read_text()
        assert "ScratchSize: 0" in text
        loads[rl] = sum(1 for ln in text.splitlines() if ln.strip().startswith("buffer_load"))
    assert loads["1"] < loads["0"], loads


@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/libhiprtc.so") or not shutil.which("/opt/rocm/bin/hipcc"),
                    reason="needs hiprtc and hipcc")
@pytest.mark.parametrize("depth", [2, 4])
def test_jitc_copy_ring_form(tmp_path, depth):
    """Round 6 (knob bs_copy_ring): the one-wave copy-through form reads its inputs through
    an LDS ring of `depth` slots; realigned inputs get the aligned 4 KiB + 16 B of the tile per slot (one
    more LDS-DMA load, by lane 0) and realign on the LDS read (rl2<d>).  Builds without scratch; the ring
    is refused for the 16 KiB-tile copy form and the crc variant."""
    G = orc.generator(10, 4)
    shifts = [(j * 104858) % 16 for j in range(10)]
    rows = "\n".join(" ".join(str(c) for c in G[100 + 10 * r:100 + 10 * (r + 1)]) for r in range(4)) + "\n"
    wave_copy = 1 | 64 | (2 << 11) | (2 << 15)
    req = tmp_path / "ring.req"
    req.write_text(f"ecamd-bitslice-request 3\n4 10 0 {depth} {wave_copy}\n" + " ".join(map(str, shifts)) + "\n" + rows)
    out = tmp_path / "ring.co"
    env = dict(os.environ, ECAMD_JIT_KEEP_SOURCE="1")
    r = subprocess.run([JITC, str(req), str(out)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    src = (tmp_path / "ring.hip").read_text()
    assert f"ring[{depth} * 5120]" in src and "rl2<10>(" in src and "threadIdx.x == 0u ?" in src
    assert src.count("// copy-through") == 40  # 4 chunks of each of the 10 inputs
    hip = tmp_path / "k.hip"
    hip.write_text("#include <hip/hip_runtime.h>\n" + src)
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "--cuda-device-only", "-S",
                        "-o", str(tmp_path / "k.s"), str(hip)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "ScratchSize: 0" in (tmp_path / "k.s").read_text()
    bad = tmp_path / "bad.req"
    for flags in (1, 1 | 2 | 16 | (1 << 22) | (2 << 23)):  # 16 KiB-tile copy form; the one-wave crc variant
        bad.write_text(f"ecamd-bitslice-request 2\n4 10 0 {depth} {flags}\n" + rows)
        assert subprocess.run([JITC, str(bad), str(tmp_path / "bad.co")], capture_output=True).returncode == 2


@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/libhiprtc.so"), reason="needs hiprtc")
def test_jitc_prefetch_flag(tmp_path):
    """Flag bits 8-10 (round 4): the one-wave form loads the first 2 / 4 chunks of the next input before
    the current input's network (BitsliceStyle::prefetch); other values, or the flag without one-wave
    tiles, are refused."""
    G = orc.generator(10, 4)
    rows = "\n".join(" ".join(str(c) for c in G[100 + 10 * r:100 + 10 * (r + 1)]) for r in range(4)) + "\n"
    env = dict(os.environ, ECAMD_JIT_KEEP_SOURCE="1")
    for pf in (2, 4):
        req = tmp_path / f"pf{pf}.req"
        req.write_text(f"ecamd-bitslice-request 2\n4 10 96 0 {192 | (pf << 8)}\n" + rows)
        out = tmp_path / f"pf{pf}.co"
        r = subprocess.run([JITC, str(req), str(out)], capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stderr[-2000:]
        src = (tmp_path / f"pf{pf}.hip").read_text()
        assert f"v4u xn[{pf}];" in src and "xn[c] = __builtin_amdgcn_raw_buffer_load_b128" in src
    bad = tmp_path / "bad.req"
    for flags in (192 | (3 << 8), 1 | (4 << 8), 192 | (6 << 8)):
        bad.write_text(f"ecamd-bitslice-request 2\n4 10 96 0 {flags}\n" + rows)
        assert subprocess.run([JITC, str(bad), str(tmp_path / "bad.co")], capture_output=True).returncode == 2


@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/libhiprtc.so"), reason="needs hiprtc")
@pytest.mark.parametrize("pos,mb,mix,shifted,l1", [(2, 4, 0, False, 0), (1, 4, 0, False, 0), (4, 4, 0, False, 0),
                                                    (2, 3, 1, False, 0), (2, 4, 0, True, 0), (2, 4, 0, False, 1)])
def test_jitc_crc_wave_form(tmp_path, pos, mb, mix, shifted, l1):
    """Flag bit 22 (round 5): the crc variant in one-wave 4 KiB tiles -- workgroups of W waves (bits
    23-26) sharing one table image of `pos` position sets for pieces 1 KiB apart (bits 2-3), byte
    piece tables for the first mb dwords (bits 28-29: 4 - mb), the lane-shift fold (bit 4), the next
    input prefetched (bits 8-10), occupancy in bits 11-18, bit 27 no barrier between lookups and
    network, bit 30 (round 6) dword 3 of each piece looked up in the image in global memory.  The kernel
    builds without scratch, its static LDS is the image (the piece sets, 4 KiB of maps, 32 KiB of lane
    tables), the tile loop carries no atomics; malformed requests are refused."""
    G = orc.generator(10, 4)
    rows = "\n".join(" ".join(str(c) for c in G[100 + 10 * r:100 + 10 * (r + 1)]) for r in range(4)) + "\n"
    pcode = {1: 0, 2: 1, 4: 2}[pos]
    flags = (1 | 2 | (pcode << 2) | 16 | (4 << 8) | (3 << 11) | (3 << 15) | (1 << 22) | (4 << 23) | (mix << 27) |
             ((4 - mb) << 28) | (l1 << 30))
    shifts = [(j * 104858) % 16 for j in range(10)]
    head = (f"ecamd-bitslice-request 3\n4 10 40 0\n{flags}\n" + " ".join(map(str, shifts)) + "\n") if shifted \
        else f"ecamd-bitslice-request 2\n4 10 40 0\n{flags}\n"
    req = tmp_path / "cw.req"
    req.write_text(head + rows)
    out = tmp_path / "cw.co"
    env = dict(os.environ, ECAMD_JIT_KEEP_SOURCE="1")
    r = subprocess.run([JITC, str(req), str(out)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    src = (tmp_path / "cw.hip").read_text()
    words = pos * (mb * 1024 + (4 - mb) * 128) + 8 * 128 + 8 * 16 * 64
    assert f"u32 ctab[{words}];" in src
    assert "__launch_bounds__(256)" in src and "amdgpu_waves_per_eu(3, 3)" in src
    assert "atomic" not in src
    assert ("piece_r0m<" in src) == (mb < 4)
    assert ("piece_r0g(ctab" in src) == bool(l1)
    assert ("rlg<10>(" in src) == shifted
    notes = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", str(out)], capture_output=True,
                           text=True).stdout
    assert ".private_segment_fixed_size: 0" in notes
    assert f".group_segment_fixed_size: {4 * words}" in notes
    bad = tmp_path / "bad.req"
    for f in (flags & ~2 & ~1,                      # the form without crc
              flags & ~(15 << 23),                  # no waves per workgroup
              flags | 32,                           # nibble-table variant bit
              (flags & ~(1 << 22) & ~(15 << 23)) | (1 << 27),  # bit 27 without the form
              flags | (1 << 28) | (1 << 30)):       # global-memory lookups with nibble tables
        bad.write_text(f"ecamd-bitslice-request 2\n4 10 40 0\n{f}\n" + rows)
        assert subprocess.run([JITC, str(bad), str(tmp_path / "bad.co")], capture_output=True).returncode == 2
