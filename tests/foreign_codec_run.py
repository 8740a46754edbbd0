"""Runner (a subprocess of tests/test_foreign_codec.py): drives this repo's liberasurecode.so.1
through its C API for one backend and prints one JSON line -- digests of every fragment, the
decode / reconstruct / fragments_needed results, and which codec libraries the process mapped.

Started with LD_LIBRARY_PATH=oracle/_ref (the REFERENCE codec libraries compiled from
/root/reference by oracle/Makefile) the frontend's DT_NEEDED libXorcode.so.1 and its
dlopen("liberasurecode_rs_vand.so.1") resolve to the reference's own CPU codecs (RUNPATH $ORIGIN is
searched after LD_LIBRARY_PATH): BASELINE configs[0] -- "CPU reference backend, plumbing, no GPU"
-- and the foreign-codec path of the frontend (no ecamd hooks, checksums from host zlib).
Test infrastructure only; the product never links oracle/_ref.

usage: foreign_codec_run.py xor|rs [checksum]"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ec_api as E  # noqa: E402

SHAPES = {  # backend, k, m, hd, object bytes: C1 (flat_xor_hd 3,3,3, 4 KiB fragments), rs_vand 10+4
    "xor": (E.EC_BACKEND_FLAT_XOR_HD, 3, 3, 3, 3 * 4096),
    "rs": (E.EC_BACKEND_LIBERASURECODE_RS_VAND, 10, 4, 0, 10 * 4096 - 6),
}


def sha(b):
    return hashlib.sha256(b).hexdigest()


def mapped_codecs():
    libs = set()
    for line in open("/proc/self/maps"):
        path = line.split()[-1] if "/" in line else ""
        base = os.path.basename(path)
        if base.startswith(("libecamd", "liberasurecode", "libXorcode")):
            libs.add(os.path.relpath(os.path.realpath(path), os.path.dirname(HERE)))
    return sorted(libs)


def direct_free(desc, k, m):
    """Fragments freed with libc free() instead of liberasurecode_encode_cleanup, as the reference's
    own tests do (test/liberasurecode_test.c:1110, test/libec_slap.c:224,300).  glibc then hands
    the same addresses to smaller requests; the frontend's recycled-buffer pool must not take such a
    smaller block for the large one it once was (a later large encode would overflow it).
    Returns one [round, encode rc, exact round trip] per large encode."""
    import ctypes as C
    libc = C.CDLL(None)
    libc.free.argtypes = [C.c_void_p]
    res = []
    for rnd in range(3):
        big = bytes((j * 7 + rnd * 11 + (j >> 10)) & 0xFF for j in range(k * (96 << 10) + 5))
        rc, d, p, fl = E.encode(desc, big)
        fr = E.fragments(d, k, fl) + E.fragments(p, m, fl)
        ok = rc == 0 and E.decode(desc, fr[1:], fl) == (0, big)
        res.append([rnd, rc, ok])
        for i in range(k):
            libc.free(d[i])
        for i in range(m):
            libc.free(p[i])
        # smaller objects (fragments under the pool's 64 KiB floor) returned through the cleanup
        for j in range(2 * (k + m)):
            sm = bytes(((j + 1) * (i + 3)) & 0xFF for i in range(k * (8 << 10) + j))
            rc2, d2, p2, fl2 = E.encode(desc, sm)
            fr2 = E.fragments(d2, k, fl2) + E.fragments(p2, m, fl2)
            E.lib().liberasurecode_encode_cleanup(desc, d2, p2)
            res.append([rnd, rc2, rc2 == 0 and E.decode(desc, fr2[1:], fl2) == (0, sm)])
    return res


def main():
    name = sys.argv[1]
    ct = int(sys.argv[2]) if len(sys.argv) > 2 else E.CHKSUM_NONE
    be, k, m, hd, size = SHAPES[name]
    desc = E.create(be, k, m, hd=hd, ct=ct)
    out = {"backend": name, "k": k, "m": m, "hd": hd, "size": size, "ct": ct, "create": desc}
    if desc <= 0:
        out["libs"] = mapped_codecs()
        print(json.dumps(out))
        return
    obj = bytes((i * 131 + (i >> 7) * 17 + 5) & 0xFF for i in range(size))
    rc, d, p, flen = E.encode(desc, obj)
    out["encode_rc"] = rc
    frags = E.fragments(d, k, flen) + E.fragments(p, m, flen)
    E.lib().liberasurecode_encode_cleanup(desc, d, p)
    out["fragment_len"] = flen
    out["fragments_sha256"] = [sha(f) for f in frags]
    out["fragments_hex_head"] = [f[:96].hex() for f in frags]
    # decode every erasure pattern of up to (hd - 1 or m) lost fragments, first few
    import itertools
    n = k + m
    lim = (hd - 1) if name == "xor" else m
    dec = []
    for r in range(0, lim + 1):
        for lost in itertools.islice(itertools.combinations(range(n), r), 40):
            have = [f for i, f in enumerate(frags) if i not in lost]
            rc, data = E.decode(desc, have, flen)
            dec.append([list(lost), rc, rc == 0 and data == obj])
    out["decode"] = dec
    rec = []
    for dest in range(n):
        lost = [dest, (dest + 1) % n] if lim >= 2 else [dest]
        have = [f for i, f in enumerate(frags) if i not in lost]
        rc, got = E.reconstruct(desc, have, flen, dest)
        rec.append([dest, rc, rc == 0 and got == frags[dest]])
    out["reconstruct"] = rec
    need = []
    for dest in range(n):
        rc, idx = E.fragments_needed(desc, [dest], [], n)
        need.append([dest, rc, idx])
    out["fragments_needed"] = need
    # recycled buffers (frontend.cpp BufferPool): objects of different sizes and contents in turn,
    # each encoded twice with other calls between; digests must repeat and every decode round-trip
    pool = []
    sizes = [(1 << 20) + 13, (3 << 20) - 7, (256 << 10) + 1, 2 << 20]
    for rep in range(2):
        for i, sz in enumerate(sizes):
            o2 = bytes((j * 29 + i * 7 + (j >> 9)) & 0xFF for j in range(sz))
            rc, d, p, fl = E.encode(desc, o2)
            fr = E.fragments(d, k, fl) + E.fragments(p, m, fl)
            E.lib().liberasurecode_encode_cleanup(desc, d, p)
            rc2, back = E.decode(desc, fr[1:], fl)  # fragment 0 lost
            rc3, sysd = E.decode(desc, fr[:k], fl)
            pool.append([rep, sz, rc, sha(b"".join(fr)), rc2 == 0 and back == o2, rc3 == 0 and sysd == o2])
    out["pool"] = pool
    out["direct_free"] = direct_free(desc, k, m)
    out["libs"] = mapped_codecs()  # before destroy: the backend library is dlclose()d there
    out["destroy"] = E.lib().liberasurecode_instance_destroy(desc)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
