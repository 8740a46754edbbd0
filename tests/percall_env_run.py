"""Child process of tests/test_gpu_percall_env.py: the per-call API (liberasurecode_encode / _decode /
_reconstruct_fragment through this repo's liberasurecode.so.1) under whatever ECAMD_PERCALL_* settings
the parent put in the environment (they are read once per process).  RS(10,4) objects of 4 KiB,
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
from test_gpu_frontend import payload_bytes, rs_expected  # noqa: E402


def main():
    h = hashlib.sha256()
    for ct in (E.CHKSUM_NONE, E.CHKSUM_CRC32):
        desc = E.create(E.EC_BACKEND_LIBERASURECODE_RS_VAND, 10, 4, hd=4, ct=ct)
        assert desc > 0, desc
        for size in (4096, 65536 + 5, (1 << 20) + 5):
            data = payload_bytes(size, size * 3 + ct)
            rc, dp, pp, flen = E.encode(desc, data)
            assert rc == 0, ("encode", size, rc)
            frags = E.fragments(dp, 10, flen) + E.fragments(pp, 4, flen)
            E.lib().liberasurecode_encode_cleanup(desc, dp, pp)
            assert frags == rs_expected(10, 4, data, ct), ("fragments", ct, size)
            rc, out = E.decode(desc, frags[4:], flen, force=1)
            assert rc == 0 and out == data, ("decode", ct, size, rc)
            rc, rec = E.reconstruct(desc, frags[:10] + frags[11:], flen, 10)
            assert rc == 0 and rec == frags[10], ("reconstruct", ct, size, rc)
            for f in frags:
                h.update(f)
        assert E.lib().liberasurecode_instance_destroy(desc) == 0
    print(json.dumps({"ok": True, "digest": h.hexdigest()}))


if __name__ == "__main__":
    main()
