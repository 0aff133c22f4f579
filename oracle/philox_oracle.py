"""CPU restatement of the training-noise generator (TEST INFRASTRUCTURE ONLY: imported by tests/, never by the
product path).

Philox4x32-10 (Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as 1, 2, 3", SC'11; the
Random123 library's philox4x32 with 10 rounds, multipliers 0xD2511F53 / 0xCD9E8D57, Weyl key increments
0x9E3779B9 / 0xBB67AE85), pinned by the Random123 known-answer vectors in tests/test_noise_cpu.py.

The product kernel (csrc/entropy.hip uniform_noise_kernel, replacing the reference's
``torch.empty_like(x).uniform_(-0.5, 0.5)`` at entropy_models.py:170) draws element i of draw d with seed s as
  c = philox4x32_10(ctr = (q lo, q hi, d lo, d hi), key = (s lo, s hi)),  q = i // 4
  u_i = (c[i % 4] >> 8) * 2^-24 - 1/2.
"""
import numpy as np

M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF


def philox4x32_10(ctr, key):
    """ctr: 4 uint32, key: 2 uint32 (Python ints) -> 4 uint32."""
    c0, c1, c2, c3 = (int(v) & MASK for v in ctr)
    k0, k1 = (int(v) & MASK for v in key)
    for _ in range(10):
        p0, p1 = M0 * c0, M1 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & MASK, p1 & MASK, ((p0 >> 32) ^ c3 ^ k1) & MASK, p0 & MASK
        k0, k1 = (k0 + W0) & MASK, (k1 + W1) & MASK
    return c0, c1, c2, c3


def uniform_noise(n, seed, draw, start=0):
    """Elements [start, start + n) of draw `draw` of the generator seeded with `seed` (fp32 numpy)."""
    out = np.empty(n, dtype=np.float32)
    for i in range(start, start + n):
        q = i // 4
        c = philox4x32_10((q & MASK, q >> 32, draw & MASK, draw >> 32), (seed & MASK, (seed >> 32) & MASK))
        out[i - start] = np.float32((c[i % 4] >> 8) * 2.0 ** -24 - 0.5)
    return out
