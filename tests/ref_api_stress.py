"""test/liberasure_rs_isal_stress_test.c restated for liberasurecode_rs_vand.

The reference's stress test takes any backend id (main, :346-380) and, for nb_iter random sets of m
erased fragments (create_skips_array + rand() % (k + m), :204-240 and :305-344):

* encode_decode_test_impl (:111-201): instance_create, encode of a 1 KiB buffer (create_buffer,
  /dev/urandom), every fragment's header checked (idx, size, orig_data_size, backend_id,
  chksum_mismatch) and every data payload against the object, then liberasurecode_decode
  (force_metadata_checks = 1) from the fragments not skipped -- data first, then parity, in index
  order (create_frags_array, :71-109) -- must return the object;
* reconstruct_test_impl (:242-303): encode of a 1 MiB buffer, liberasurecode_reconstruct_fragment of
  destination `i` from the same fragment set, compared with the encoded fragment.  `i` is declared
  0 and never changes, so the reference always rebuilds fragment 0 (which the frontend copies when
  it is available, src/erasurecode.c:857-867).  Here destination 0 is run as written AND every
  erased index (what the test means to do).

Pattern sets (the reference draws random ones; these are fixed so that runs compare):
* (10, 4): EVERY erasure set of 1 .. 4 fragments -- all 1,470;
* (20, 8): 2,000 random sets of exactly 8 (the reference's count = m), drawn as the reference does
  (rand() % (k + m) until m distinct) from a seeded generator.

Buffers come from a seeded generator instead of /dev/urandom.  Every call's output is checked as the
reference checks it, and all outputs (encoded fragments, decoded objects, rebuilt fragments) go
into one SHA-256 per code, so the GPU codec and the REFERENCE codec (oracle/_ref, on the CPU,
tests/ref_api_stress_run.py) can be compared byte for byte: tests/golden/rs_stress.json holds the
reference's digests (tests/golden/make_stress_golden.py)."""
import ctypes as C
import hashlib
import itertools
import random

import numpy as np

import ec_api as E

BE = E.EC_BACKEND_LIBERASURECODE_RS_VAND
HDR = 80
DEC_SIZE = 1024  # encode_decode_test_impl, :118
REC_SIZE = 1 << 20  # reconstruct_test_impl, :248


def patterns(k, m, n_random=2000, seed=20260101):
    """(10, 4): every 1..m erasure set; otherwise n_random sets of m, drawn as main's loops draw them."""
    if (k, m) == (10, 4):
        return [list(c) for r in range(1, m + 1) for c in itertools.combinations(range(k + m), r)]
    rng = random.Random(seed)
    out = []
    for _ in range(n_random):
        skip = set()
        while len(skip) < m:
            skip.add(rng.randrange(k + m))
        out.append(sorted(skip))
    return out


def _frag_set(frags, skip):
    return [f for i, f in enumerate(frags) if i not in skip]


def _check_headers(frags, data, k, m, flen):
    """The header and payload checks of encode_decode_test_impl (:149-174)."""
    remaining, off = len(data), 0
    for i in range(k + m):
        meta = E.FragmentMetadata.from_buffer_copy(frags[i][:C.sizeof(E.FragmentMetadata)])
        assert meta.idx == i, ("idx", i, meta.idx)
        assert meta.size == flen - HDR - meta.frag_backend_metadata_size, ("size", i)
        assert meta.orig_data_size == len(data), ("orig_data_size", i)
        assert meta.backend_id == BE and meta.chksum_mismatch == 0, ("backend / chksum", i)
        cmp = min(remaining, meta.size)
        assert frags[i][HDR:HDR + cmp] == data[off:off + cmp], ("payload", i)
        remaining -= cmp
        off += meta.size


def _encode(desc, data, k, m):
    rc, d, p, flen = E.encode(desc, data)
    assert rc == 0, ("encode", rc)
    frags = E.fragments(d, k, flen) + E.fragments(p, m, flen)
    assert E.lib().liberasurecode_encode_cleanup(desc, d, p) == 0
    return frags, flen


def stress(k, m, n_random=2000, seed=1, limit=None, reencode=50):
    """Runs both halves over the pattern set of (k, m); returns {"decode": sha256, "reconstruct":
    sha256, "patterns": n, "reconstructs": n}.  Raises AssertionError on the first mismatch.

    The reconstruct half keeps one instance and re-encodes a fresh 1 MiB buffer every `reencode`
    patterns (the reference encodes one per iteration: the same calls, at a fraction of the CPU time
    on the reference codec); (10, 4) rebuilds destination 0 and every erased index, (20, 8) destination
    0 and one erased index drawn per pattern."""
    pats = patterns(k, m, n_random)[:limit]
    rng = np.random.default_rng(seed * 1000 + k * 10 + m)
    pick = random.Random(seed)
    lib = E.lib()
    hdec, hrec = hashlib.sha256(), hashlib.sha256()
    nrec = 0
    rdesc = E.create(BE, k, m)
    assert rdesc > 0, ("instance_create", rdesc)
    try:
        for n, skip in enumerate(pats):
            # encode_decode_test_impl: one instance per iteration, as the reference creates it
            desc = E.create(BE, k, m)
            assert desc > 0, ("instance_create", desc)
            try:
                data = rng.integers(0, 256, DEC_SIZE, dtype=np.uint8).tobytes()
                frags, flen = _encode(desc, data, k, m)
                _check_headers(frags, data, k, m, flen)
                rc, out = E.decode(desc, _frag_set(frags, skip), flen, force=1)
                assert rc == 0 and out == data, ("decode", skip, rc)
                for f in frags:
                    hdec.update(f)
                hdec.update(out)
            finally:
                assert lib.liberasurecode_instance_destroy(desc) == 0
            # reconstruct_test_impl: destination 0 as written, then the erased indices
            if n % reencode == 0:
                rdata = rng.integers(0, 256, REC_SIZE, dtype=np.uint8).tobytes()
                rfrags, rflen = _encode(rdesc, rdata, k, m)
                hrec.update(hashlib.sha256(b"".join(rfrags)).digest())
            avail = _frag_set(rfrags, skip)
            lost = [i for i in skip if i != 0]
            if (k, m) != (10, 4) and lost:
                lost = [pick.choice(lost)]
            for dest in [0] + lost:
                rc, out = E.reconstruct(rdesc, avail, rflen, dest)
                assert rc == 0 and out == rfrags[dest], ("reconstruct", skip, dest, rc)
                hrec.update(out)
                nrec += 1
    finally:
        assert lib.liberasurecode_instance_destroy(rdesc) == 0
    return {"decode": hdec.hexdigest(), "reconstruct": hrec.hexdigest(), "patterns": len(pats),
            "reconstructs": nrec}


CODES = [(10, 4), (20, 8)]
