"""Test infrastructure: a numpy restatement of the device dropout generator
(spotv2net_amd/csrc/sv2n_rng.hip, sv2n_dropout_uniform): Philox4x32-10
(Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as 1, 2, 3",
SC'11; the Random123 known-answer vectors pin it in test_rng.py), key =
seed, counter = (i/4 low, i/4 high, salt, step), element i = word i%4,
u = (word >> 8)·2^-24.  Used by the tests to rebuild the product's dropout
masks for the oracle; never imported by the product."""
import numpy as np

M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
_M32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised over the counter words (uint32 arrays or ints); returns the
    four output words as uint64 arrays holding 32-bit values."""
    c = [np.asarray(x, dtype=np.uint64) & _M32 for x in (c0, c1, c2, c3)]
    k0, k1 = np.uint64(k0 & 0xFFFFFFFF), np.uint64(k1 & 0xFFFFFFFF)
    for _ in range(10):
        p0 = np.uint64(M0) * c[0]
        p1 = np.uint64(M1) * c[2]
        c = [(p1 >> np.uint64(32)) ^ c[1] ^ k0, p1 & _M32, (p0 >> np.uint64(32)) ^ c[3] ^ k1,
             p0 & _M32]
        k0 = (k0 + np.uint64(W0)) & _M32
        k1 = (k1 + np.uint64(W1)) & _M32
    return c


def dropout_uniform_ref(n: int, seed: int, step: int, salt: int) -> np.ndarray:
    """the n uniforms sv2n_dropout_uniform writes (float32)"""
    nb = (n + 3) // 4
    b = np.arange(nb, dtype=np.uint64)
    w = philox4x32_10(b & _M32, b >> np.uint64(32), np.full(nb, salt, np.uint64),
                      np.full(nb, step, np.uint64), seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    words = np.stack(w, axis=1).reshape(-1)[:n]
    return (words >> np.uint64(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
