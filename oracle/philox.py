"""Philox4x32-10 (oracle — test infrastructure only).

Restated from the Random123 paper / reference implementation (Salmon et al.,
SC'11), the counter-based generator named by the north star. Constants
M0=0xD2511F53, M1=0xCD9E8D57, W0=0x9E3779B9, W1=0xBB67AE85 (the same values
as /opt/rocm/include/rocrand/rocrand_philox4x32_10.h).  Pinned by the
Random123 ``kat_vectors`` entries for philox4x32_10 (tests/golden/philox_kat.json).

The draw schedule of the simulator (isim semantics v1):
  error draw of the invocation with hop id h of trace t:
      word (h & 3) of philox(ctr=(t_lo, t_hi, h >> 2, 0), key=(seed_lo, seed_hi))
  probability draw of the k-th call command of that invocation:
      word (k & 3) of philox(ctr=(t_lo, t_hi, h, 1 + (k >> 2)), key)
"""
M32 = 0xFFFFFFFF
M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85


def philox4x32_10(ctr, key):
    c0, c1, c2, c3 = (x & M32 for x in ctr)
    k0, k1 = key[0] & M32, key[1] & M32
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & M32, p1 & M32, ((p0 >> 32) ^ c3 ^ k1) & M32, p0 & M32
        k0 = (k0 + W0) & M32
        k1 = (k1 + W1) & M32
    return (c0, c1, c2, c3)


def err_draw(seed: int, t: int, h: int) -> int:
    blk = philox4x32_10((t & M32, t >> 32, h >> 2, 0), (seed & M32, seed >> 32))
    return blk[h & 3]


def prob_draw(seed: int, t: int, h: int, k: int) -> int:
    blk = philox4x32_10((t & M32, t >> 32, h, 1 + (k >> 2)), (seed & M32, seed >> 32))
    return blk[k & 3]
