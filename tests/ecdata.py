"""Deterministic synthetic fragment data shared by tests, golden generation and bench checks.

splitmix64 counter stream: 64-bit word i of a fragment = mix(seed + (i+1) * 0x9E3779B97F4A7C15),
emitted little-endian.  Fragment j of stripe s uses seed 0xEC0DE ^ (s << 8) ^ j.
The same stream is produced on the GPU by ecamd_fill_splitmix (liberasurecode_amd/csrc/hip).
"""
import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)


def frag_seed(stripe: int, frag: int, base: int = 0xEC0DE) -> int:
    return (base ^ (stripe << 8) ^ frag) & 0xFFFFFFFFFFFFFFFF


def splitmix_bytes(seed: int, nbytes: int) -> np.ndarray:
    nw = (nbytes + 7) // 8
    with np.errstate(over="ignore"):
        i = np.arange(1, nw + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * GOLDEN
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").view(np.uint8)[:nbytes].copy()


def stripe_fragments(stripe: int, count: int, nbytes: int, base: int = 0xEC0DE) -> np.ndarray:
    """(count, nbytes) uint8 array of fragments 0..count-1 of `stripe`."""
    out = np.empty((count, nbytes), dtype=np.uint8)
    for j in range(count):
        out[j] = splitmix_bytes(frag_seed(stripe, j, base), nbytes)
    return out


EDGE_PATTERNS = {
    "zeros": lambda n: np.zeros(n, dtype=np.uint8),
    "ones": lambda n: np.full(n, 0xFF, dtype=np.uint8),
    "u16_0001": lambda n: np.tile(np.array([0x01, 0x00], dtype=np.uint8), (n + 1) // 2)[:n],
    "u16_8000": lambda n: np.tile(np.array([0x00, 0x80], dtype=np.uint8), (n + 1) // 2)[:n],
}
