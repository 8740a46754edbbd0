"""Runner (a subprocess of tests/test_gpu_frontend.py::test_decode_direct_matches_general_path):
liberasurecode_decode over rs_vand (10,4) and (4,2) for every erasure pattern of up to m lost
fragments on a few object sizes -- plus irregular inputs: a surviving data fragment whose header
claims another payload size or orig_data_size (libec_version below 1.2.0, so its header checksum is
not consulted, src/erasurecode.c:1126-1128), duplicate fragments, fewer than k distinct ones --
and prints one JSON line of [case, rc, sha256 of the object] (and of every encode's fragments).
Run with ECAMD_FRONTEND_DECODE_DIRECT / ECAMD_FRONTEND_TEE on and off (decode straight into the
object, frontend.cpp decode_direct; object <-> payload copies on the codec's staging pack,
TeeCopies) and with both off (the reference's order of operations): the lines must be equal."""
import hashlib
import itertools
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ec_api as E  # noqa: E402


def sha(b):
    return hashlib.sha256(b).hexdigest() if b is not None else None


def main():
    out = []
    for k, m in ((10, 4), (4, 2)):
        desc = E.create(E.EC_BACKEND_LIBERASURECODE_RS_VAND, k, m, hd=m)
        assert desc > 0, desc
        for size in (1, 4096 * k - 3, (1 << 20) + 7, 3 * (1 << 20)):
            obj = bytes((i * 197 + (i >> 8) * 13 + size) & 0xFF for i in range(size))
            rc, d, p, flen = E.encode(desc, obj)
            assert rc == 0
            frags = E.fragments(d, k, flen) + E.fragments(p, m, flen)
            E.lib().liberasurecode_encode_cleanup(desc, d, p)
            out.append([f"{k},{m},{size},encode", rc, sha(b"".join(frags)), None])
            pats = [c for r in range(1, m + 1) for c in itertools.combinations(range(k + m), r)]
            for lost in pats[:: max(1, len(pats) // 60)]:
                have = [f for i, f in enumerate(frags) if i not in lost]
                rc, data = E.decode(desc, have, flen)
                out.append([f"{k},{m},{size},{list(lost)}", rc, sha(data), rc == 0 and data == obj])
            # irregular survivors: the direct path must hand them to the general one
            lost = [0, k]  # a data and a parity fragment gone: the codec runs
            bs = flen - 80
            # a claimed payload size beyond the real one would make the reference read past the
            # fragments (prepare_fragments_for_decode takes it for the blocksize): only smaller ones
            cases = ([("size", bs - 2)] if bs > 2 else []) + [("orig", size + 5), ("orig", max(0, size - 9))]
            for field, val in cases:
                bad = bytearray(frags[1])
                if field == "size":
                    bad[4:8] = val.to_bytes(4, "little")
                else:
                    bad[12:20] = val.to_bytes(8, "little")
                bad[63:67] = (1).to_bytes(4, "little")  # libec_version 0.0.1: metadata CRC not checked
                have = [bytes(bad)] + [f for i, f in enumerate(frags) if i not in lost and i != 1]
                rc, data = E.decode(desc, have, flen)
                out.append([f"{k},{m},{size},{field}={val}", rc, sha(data), None])
            have = [f for i, f in enumerate(frags) if i not in (0, 1)] + [frags[2]]  # a duplicate
            rc, data = E.decode(desc, have, flen)
            out.append([f"{k},{m},{size},dup", rc, sha(data), rc == 0 and data == obj])
        E.lib().liberasurecode_instance_destroy(desc)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
