"""Philox-4x32-10 counter RNG in numpy -- TEST INFRASTRUCTURE (oracle).

The reference draws its sampling noise from numpy's global MT19937
(`distributions.py:11-12` categorical, `core.py:432-435` DiagGauss) and re-seeds
it per episode (`core.py:215`); the env RNG is never seeded, so reference
trajectories are not reproducible.  The batched collector instead
uses a counter-based stream so that every (env, step) draw is addressable; this
file is the bit-exact CPU twin of ``modular_rl_amd/csrc/mrl_common.h`` used to
check the GPU collector.  Stream layout (shared with the HIP code):

  key      = (seed & 0xffffffff, (seed >> 32) ^ (0x9E3779B9 * domain))
  counter  = (env_global_id, word1, word2, call)   -- meaning per domain:
     domain 0 (action noise): word1/word2 = lo/hi of the global step index
     domain 1 (reset noise):  word1/word2 = lo/hi of the env's episode counter
  doubles  = ((x0 >> 5) * 2**26 + (x1 >> 6)) * 2**-53, same for (x2, x3)
"""
import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint64(0x9E3779B9)
W1 = np.uint64(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 (Salmon et al. 2011). All args uint32 arrays."""
    c0, c1, c2, c3 = (np.asarray(v, dtype=np.uint64) & MASK for v in (c0, c1, c2, c3))
    k0 = np.asarray(k0, dtype=np.uint64) & MASK
    k1 = np.asarray(k1, dtype=np.uint64) & MASK
    for r in range(10):
        if r > 0:
            k0 = (k0 + W0) & MASK
            k1 = (k1 + W1) & MASK
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & MASK, lo1, (hi0 ^ c3 ^ k1) & MASK, lo0
    return [v.astype(np.uint32) for v in (c0, c1, c2, c3)]


def key_for(seed, domain):
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    k0 = seed & 0xFFFFFFFF
    k1 = ((seed >> 32) ^ ((0x9E3779B9 * int(domain)) & 0xFFFFFFFF)) & 0xFFFFFFFF
    return np.uint32(k0), np.uint32(k1)


def _u01(a, b):
    a = a.astype(np.float64)
    b = b.astype(np.float64)
    return (np.floor(a / 32.0) * 67108864.0 + np.floor(b / 64.0)) * (1.0 / 9007199254740992.0)


def uniform2(seed, domain, gid, w, call):
    """Two U[0,1) doubles per (gid, w, call); w is a 64-bit word (lo/hi)."""
    k0, k1 = key_for(seed, domain)
    gid = np.asarray(gid, dtype=np.uint64)
    w = np.asarray(w, dtype=np.uint64)
    x0, x1, x2, x3 = philox4x32_10(gid & MASK, w & MASK, (w >> np.uint64(32)) & MASK,
                                   np.broadcast_to(np.uint64(call), np.broadcast(gid, w).shape), k0, k1)
    return _u01(x0, x1), _u01(x2, x3)


def normals(seed, domain, gid, w, d):
    """d standard normals per (gid, w) via Box-Muller on successive calls."""
    outs = []
    for call in range((d + 1) // 2):
        u1, u2 = uniform2(seed, domain, gid, w, call)
        rad = np.sqrt(-2.0 * np.log(1.0 - u1))
        ang = 2.0 * np.pi * u2
        outs.append(rad * np.cos(ang))
        outs.append(rad * np.sin(ang))
    return np.stack(outs[:d], axis=-1)


def uniforms(seed, domain, gid, w, n):
    """n U[0,1) doubles per (gid, w)."""
    outs = []
    for call in range((n + 1) // 2):
        a, b = uniform2(seed, domain, gid, w, call)
        outs += [a, b]
    return np.stack(outs[:n], axis=-1)
