"""test/libec_slap.c restated: the reference's one API-level stress test of flat_xor_hd.

For each (k, m, hd) the reference runs (libec_slap.c:464-495: (6..15, 6, 3), (5..10, 5, 3),
(6..20, 6, 4), (5..10, 5, 4)) -- plus (3, 3, 3), BASELINE configs[0] -- through
liberasurecode_instance_create / encode / fragments_needed / decode (libec_slap.c:153-344):

* 999 encodes of a 32 KiB-per-fragment object (fill_buffer, :146-151), each cleaned up, then one
  kept;
* every failure combination of 1 .. hd-1 fragments (test_xor_hd_code.h's failure_combs_N_hd are
  all such subsets of the k + m fragments, in that order): fragments_needed for the combination's
  highest index -- missing_mask_to_array (:67-77) keeps only the last set bit -- must succeed and
  not name it; then a decode (force_metadata_checks = 1) must return the object;
* 1000 random decodes of hd-1 consecutive indices from a random start (:318-336; the reference's
  `mi + 1 % (k + m)` is `mi + 1`, so indices past the last fragment simply name nothing).

The reference builds its fragment sets with `(missing_mask | 1L << i) == 1` (create_frags_array_set,
:101-136), which drops a fragment only for mask 0 / 1 at i = 0 -- so as written its decodes see
(almost) every fragment.  Both sets are run here: `literal` (that expression, the reference's
behaviour) and `excluded` (the missing fragments really left out, what the test means to do), and
every decode's output is compared with the object (the reference checks the combinations' output
and only the return code of the random ones).

Runs in-process on the GPU (tests/test_gpu_reference_api.py, this repo's codecs) and, through
tests/ref_api_slap_run.py, on the CPU in front of the REFERENCE codec libraries (oracle/_ref)."""
import itertools
import random

import numpy as np

import ec_api as E

BLOCKSIZE = 32768  # libec_slap.c:160
CODES = ([(k, 6, 3) for k in range(6, 16)] + [(k, 5, 3) for k in range(5, 11)] +
         [(k, 6, 4) for k in range(6, 21)] + [(k, 5, 4) for k in range(5, 11)] + [(3, 3, 3)])


def fill_buffer(size, seed=0):
    """fill_buffer (:146-151): buf[i] = (char)(seed += i)."""
    i = np.arange(size, dtype=np.int64)
    return ((seed + i * (i + 1) // 2) & 0xFF).astype(np.uint8).tobytes()


def _frag_set(frags, k, m, mask, literal):
    out = []
    for i in range(k + m):
        if literal:
            if (mask | (1 << i)) == 1:  # the reference's expression (data loop; parity never matches)
                continue
        elif mask & (1 << i):
            continue
        out.append(frags[i])
    return out


def slap(k, m, hd, encodes=1000, decodes=1000, seed=8262014):
    """libec_slap.c test_hd_code for one code; raises AssertionError on the first failure."""
    data = fill_buffer(BLOCKSIZE * k)
    desc = E.create(E.EC_BACKEND_FLAT_XOR_HD, k, m, hd=hd)
    assert desc > 0, ("instance_create", desc)
    lib = E.lib()
    try:
        for _ in range(encodes - 1):
            rc, d, p, flen = E.encode(desc, data)
            assert rc == 0, ("encode", rc)
            assert lib.liberasurecode_encode_cleanup(desc, d, p) == 0
        rc, d, p, flen = E.encode(desc, data)
        assert rc == 0, ("encode", rc)
        frags = E.fragments(d, k, flen) + E.fragments(p, m, flen)
        assert lib.liberasurecode_encode_cleanup(desc, d, p) == 0
        n = k + m
        for size in range(1, hd):
            for comb in itertools.combinations(range(n), size):
                mask = 0
                for idx in comb:
                    mask |= 1 << idx
                hi = max(comb)  # missing_mask_to_array keeps the last set bit only
                rc, needed = E.fragments_needed(desc, [hi], [], n)
                assert rc >= 0, ("fragments_needed", comb, rc)
                assert hi not in needed, ("needed names a missing fragment", comb, needed)
                for literal in (True, False):
                    rc, out = E.decode(desc, _frag_set(frags, k, m, mask, literal), flen, force=1)
                    assert rc == 0 and out == data, ("decode", comb, literal, rc)
        rng = random.Random(seed)  # srand(time(NULL)) in the reference
        for _ in range(decodes):
            mi = rng.randrange(n)
            mask = 0
            for j in range(hd - 1):
                mask |= 1 << (mi + j)
            for literal in (True, False):
                rc, out = E.decode(desc, _frag_set(frags, k, m, mask, literal), flen, force=1)
                assert rc == 0 and out == data, ("random decode", mi, literal, rc)
    finally:
        assert lib.liberasurecode_instance_destroy(desc) == 0
