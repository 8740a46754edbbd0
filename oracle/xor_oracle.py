"""xor_oracle.py -- TEST INFRASTRUCTURE ONLY (the checker for the flat-XOR path; never shipped).

A numpy restatement of the reference's flat-XOR HD codec operating on real byte buffers, in the
same order the reference touches them:
  code tables ..................... include/xor_codes/xor_hd_code_defs.h:29-173
  valid (k, m, hd) ................ src/builtin/xor_codes/xor_hd_code.c:664-693
  encode / selective_encode ....... src/builtin/xor_codes/xor_code.c:180-207
  failure pattern ................. xor_code.c:74-128
  connected parity ................ xor_code.c:316-371
  decode_one/two/three, decode .... xor_hd_code.c:418-662
  reconstruct_one ................. xor_code.c:248-314
Parity pinning: tests/test_xor_oracle.py checks it against tests/golden/xor_codes.json, produced by
the reference libXorcode.so.1 compiled from its own sources (oracle/Makefile).
"""
import numpy as np

PARITY_BMS = {
    (12, 6, 4): [1649, 3235, 2375, 718, 1436, 2872], (10, 5, 3): [163, 300, 337, 582, 664],
    (3, 3, 3): [5, 6, 3], (6, 6, 3): [3, 48, 36, 24, 9, 6], (7, 6, 3): [67, 112, 36, 24, 9, 6],
    (8, 6, 3): [67, 112, 164, 152, 9, 6], (9, 6, 3): [67, 112, 164, 152, 265, 262],
    (10, 6, 3): [579, 112, 676, 152, 265, 262], (11, 6, 3): [579, 1136, 676, 152, 1289, 262],
    (12, 6, 3): [579, 1136, 676, 2200, 1289, 2310], (13, 6, 3): [4675, 1136, 676, 6296, 1289, 2310],
    (14, 6, 3): [4675, 9328, 676, 6296, 1289, 10502],
    (15, 6, 3): [4675, 9328, 17060, 6296, 17673, 10502], (6, 6, 4): [7, 56, 56, 11, 21, 38],
    (7, 6, 4): [71, 120, 120, 11, 21, 38], (8, 6, 4): [71, 120, 120, 139, 149, 166],
    (9, 6, 4): [327, 376, 120, 395, 149, 166], (10, 6, 4): [327, 376, 632, 395, 661, 678],
    (11, 6, 4): [1351, 1400, 632, 395, 1685, 678], (13, 6, 4): [5447, 5496, 2680, 2443, 1685, 6822],
    (14, 6, 4): [5447, 5496, 10872, 10635, 9877, 6822],
    (15, 6, 4): [21831, 5496, 27256, 27019, 9877, 6822],
    (16, 6, 4): [21831, 38264, 27256, 27019, 42645, 39590],
    (17, 6, 4): [87367, 38264, 92792, 27019, 108181, 39590],
    (18, 6, 4): [87367, 169336, 92792, 158091, 108181, 170662],
    (19, 6, 4): [349511, 169336, 354936, 158091, 108181, 432806],
    (20, 6, 4): [349511, 693624, 354936, 682379, 632469, 432806],
    (5, 5, 3): [3, 12, 17, 6, 24], (6, 5, 3): [35, 44, 17, 6, 24], (7, 5, 3): [35, 44, 81, 70, 24],
    (8, 5, 3): [163, 44, 81, 70, 152], (9, 5, 3): [163, 300, 337, 70, 152],
    (5, 5, 4): [7, 25, 14, 19, 28], (6, 5, 4): [39, 57, 46, 19, 28], (7, 5, 4): [103, 57, 46, 83, 92],
    (8, 5, 4): [103, 185, 174, 211, 92], (9, 5, 4): [359, 441, 174, 211, 348],
    (10, 5, 4): [359, 441, 686, 723, 860],
}


def valid(k, m, hd):
    if hd == 3:
        return (m == 6 and 6 <= k <= 15) or (m == 5 and 5 <= k <= 10) or (m == 3 and k == 3)
    if hd == 4:
        return (m == 6 and 6 <= k <= 20) or (m == 5 and 5 <= k <= 10)
    return False


class XorCode:
    def __init__(self, k, m, hd):
        assert valid(k, m, hd)
        self.k, self.m, self.hd = k, m, hd
        self.pbm = PARITY_BMS[(k, m, hd)]
        self.dbm = [sum(1 << j for j in range(m) if self.pbm[j] >> i & 1) for i in range(k)]

    # ---- index logic ----
    def pattern(self, missing):
        """get_failure_pattern as (ndata, nparity) or None for 'too many'."""
        nd = npar = 0
        for n, idx in enumerate(missing, 1):
            if n >= self.hd:
                return None
            if idx < self.k:
                nd += 1
            else:
                npar += 1
            if nd + npar >= 4 or (nd == 3 and npar) or (nd and npar >= 2 and nd + npar > 2 and nd >= 2):
                return None
        return nd, npar

    def missing_in_parity(self, p_abs, md):
        if md is None:
            return 0
        return sum(1 for d in md if self.dbm[d] >> (p_abs - self.k) & 1)

    def connected(self, d, mp, md):
        for i in range(self.m):
            if self.missing_in_parity(i + self.k, md) > 1:
                continue
            if not self.pbm[i] >> d & 1:
                continue
            if mp is None or (self.k + i) not in mp:
                return i + self.k
        return -1

    # ---- byte work on buffers (list of k data + m parity uint8 arrays, modified in place) ----
    def encode(self, bufs):
        k = self.k
        for i in range(k):
            for j in range(self.m):
                if self.pbm[j] >> i & 1:
                    bufs[k + j] ^= bufs[i]

    def _selective(self, bufs, mp):
        for i in range(self.k):
            for p in mp:
                if self.pbm[p - self.k] >> i & 1:
                    bufs[p] ^= bufs[i]

    def _one(self, bufs, md, mp):
        d = md[0]
        p = self.connected(d, mp, md)
        bufs[d][:] = bufs[p]
        for i in range(self.k):
            if i != d and self.pbm[p - self.k] >> i & 1:
                bufs[d] ^= bufs[i]

    def _two(self, bufs, md, mp):
        d = md[0]
        p = self.connected(d, mp, md)
        if p < 0:
            d = md[1]
            p = self.connected(d, mp, md)
            if p < 0:
                return -2
            rest = [md[0]]
        else:
            rest = [md[1]]
        bufs[d][:] = bufs[p]
        for i in range(self.k):
            if i != d and self.pbm[p - self.k] >> i & 1:
                bufs[d] ^= bufs[i]
        self._one(bufs, rest, mp)
        return 0

    def _three(self, bufs, md, mp):
        d, p, src, bm = -1, -1, None, None
        for x in md:
            p = self.connected(x, mp, md)
            if p > -1:
                d, src, bm = x, bufs[p].copy(), self.pbm[p - self.k]
                break
        if p < 0:
            c2 = c3 = -1
            for i in range(self.m):
                n = self.missing_in_parity(self.k + i, md)
                if n == 2 and c2 < 0:
                    c2 = i
                elif n == 3 and c3 < 0:
                    c3 = i
            if c2 < 0 or c3 < 0:
                return -2
            bm = self.pbm[c2] ^ self.pbm[c3]
            src = bufs[self.k + c2] ^ bufs[self.k + c3]
            d = next((x for x in md if bm >> x & 1), -1)
            if d < 0:
                return -2
        bufs[d][:] = src
        for i in range(self.k):
            if i != d and bm >> i & 1:
                bufs[d] ^= bufs[i]
        rest = [x for x in md if x != d]
        return self._two(bufs, rest, mp)

    def decode(self, bufs, missing, decode_parity=1):
        pat = self.pattern(missing)
        md = [x for x in missing if x < self.k]
        mp = [x for x in missing if x >= self.k]
        if pat is None:
            return -1
        nd, npar = pat
        ret = 0
        if nd == 1:
            self._one(bufs, md, mp if npar else None)
        elif nd == 2:
            ret = self._two(bufs, md, mp if npar else None)
        elif nd == 3:
            ret = self._three(bufs, md, None)
        if npar and decode_parity:
            self._selective(bufs, mp)
        return ret

    def reconstruct_one(self, bufs, missing, idx):
        md = [x for x in missing if x < self.k]
        mp = [x for x in missing if x >= self.k]
        if idx < self.k:
            p = self.connected(idx, mp, md)
            if p >= 0:
                bufs[idx][:] = bufs[p]
                for i in range(self.k):
                    if self.pbm[p - self.k] >> i & 1 and i != idx:
                        bufs[idx] ^= bufs[i]
                return 0
            return self.decode(bufs, missing, 1)
        if self.missing_in_parity(idx, md) == 0:
            bufs[idx][:] = 0
            for i in range(self.k):
                if self.pbm[idx - self.k] >> i & 1:
                    bufs[idx] ^= bufs[i]
            return 0
        return self.decode(bufs, missing, 1)


def encode_bytes(k, m, hd, data: np.ndarray) -> np.ndarray:
    """(k, bs) data -> (m, bs) parity (parity starts zeroed, as the frontend allocates it)."""
    c = XorCode(k, m, hd)
    bufs = [np.array(x) for x in data] + [np.zeros(data.shape[1], np.uint8) for _ in range(m)]
    c.encode(bufs)
    return np.stack(bufs[k:])
