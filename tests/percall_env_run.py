"""Child process of tests/test_gpu_percall_env.py: the per-call API (liberasurecode_encode / _decode /
_reconstruct_fragment through this repo's liberasurecode.so.1) under whatever ECAMD_PERCALL_* settings
the parent put in the environment (they are read once per process).  RS(10,4) and flat_xor_hd (10,6,4)
objects of 4 KiB,
64 KiB and 1 MiB (+5 bytes), CHKSUM_NONE and CHKSUM_CRC32: every fragment compared with the restated
framing over the oracle codec (test_gpu_frontend.rs_expected), a decode of 4 lost data fragments and a
reconstruct of a lost parity.  Prints one JSON line {"ok": true, "digest": sha256 of all outputs}."""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
import torch  # noqa: E402,F401  (one HIP runtime per process: torch's)

import ec_api as E  # noqa: E402
from test_gpu_frontend import payload_bytes, rs_expected, xor_expected  # noqa: E402


def main():
    h = hashlib.sha256()
    # liberasurecode_rs_vand (10, 4) and flat_xor_hd (10, 6, 4): 4 / 3 data fragments lost
    for be, k, m, hd, lost in ((E.EC_BACKEND_LIBERASURECODE_RS_VAND, 10, 4, 4, 4), (E.EC_BACKEND_FLAT_XOR_HD, 10, 6, 4, 3)):
        for ct in (E.CHKSUM_NONE, E.CHKSUM_CRC32):
            desc = E.create(be, k, m, hd=hd, ct=ct)
            assert desc > 0, desc
            for size in (4096, 65536 + 5, (1 << 20) + 5):
                data = payload_bytes(size, size * 3 + ct)
                rc, dp, pp, flen = E.encode(desc, data)
                assert rc == 0, ("encode", size, rc)
                frags = E.fragments(dp, k, flen) + E.fragments(pp, m, flen)
                E.lib().liberasurecode_encode_cleanup(desc, dp, pp)
                want = rs_expected(k, m, data, ct) if be == E.EC_BACKEND_LIBERASURECODE_RS_VAND \
                    else xor_expected(k, m, hd, data, ct)
                assert frags == want, ("fragments", be, ct, size)
                rc, out = E.decode(desc, frags[lost:], flen, force=1)
                assert rc == 0 and out == data, ("decode", be, ct, size, rc)
                rc, rec = E.reconstruct(desc, frags[:k] + frags[k + 1:], flen, k)
                assert rc == 0 and rec == frags[k], ("reconstruct", be, ct, size, rc)
                for f in frags:
                    h.update(f)
            assert E.lib().liberasurecode_instance_destroy(desc) == 0
    print(json.dumps({"ok": True, "digest": h.hexdigest()}))


if __name__ == "__main__":
    main()
