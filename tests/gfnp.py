"""numpy GF(2^16) helpers for tests (independent of the product and of the C oracle)."""
import numpy as np

POLY = 0x1100B


def _tables():
    log = np.zeros(65536, dtype=np.int64)
    exp = np.zeros(2 * 65535, dtype=np.int64)
    v = 1
    for e in range(65535):
        log[v] = e
        exp[e] = v
        exp[e + 65535] = v
        v <<= 1
        if v & 0x10000:
            v ^= POLY
    return log, exp


LOG, EXP = _tables()


def mul_vec(c: int, words: np.ndarray) -> np.ndarray:
    """c * words (uint16 array) over GF(2^16)."""
    if c == 0:
        return np.zeros_like(words)
    w = words.astype(np.int64)
    out = EXP[LOG[w] + LOG[c]]
    out[w == 0] = 0
    return out.astype(np.uint16)


def apply_map(coeff, inputs):
    """coeff: R x K ints; inputs: list of K byte arrays (even length or odd with tail byte).
    Returns R byte arrays: sum_j coeff[r][j] * inputs[j] on little-endian 16-bit words."""
    bs = inputs[0].shape[0]
    nw = bs // 2
    outs = []
    for row in coeff:
        acc = np.zeros(nw, dtype=np.uint16)
        tail = 0
        for c, x in zip(row, inputs):
            acc ^= mul_vec(int(c), x[:2 * nw].view("<u2"))
            if bs & 1:
                tail ^= int(mul_vec(int(c), np.array([x[-1]], dtype=np.uint16))[0]) & 0xFF
        o = np.empty(bs, dtype=np.uint8)
        o[:2 * nw] = acc.view(np.uint8)
        if bs & 1:
            o[-1] = tail
        outs.append(o)
    return outs
