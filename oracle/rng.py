"""Counter-based random stream used for stochastic actions in batched rollouts.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

The reference samples actions with torch ``Categorical(probs).sample()`` /
``Normal(mean, std).sample()`` (policies/discrete.py:21-22, policies/mujoco.py:20-21),
whose CPU generator streams cannot be reproduced on a GPU.  The build therefore
defines its own stream (DESIGN.md "Random streams"): a splitmix64 counter hash.
The HIP kernels (dfd-starter_amd/csrc/fdr_common.h) compute exactly the same
integers; the float transforms below are the same f32 formulas, so GPU and oracle
agree to a few ulp (transcendentals) and bit-exactly on the integer draws.

    key      = mix64(seed)
    h(c)     = mix64(key + c * GOLDEN)                (mod 2^64)
    c        = (lane << 32) | (t << 4) | k            t < 2^28, k < 16
    uniform  = (h >> 40) * 2^-24                       in [0, 1)
    normal   = sqrt(-2 ln u1) * cos(2 pi u2),  u1 = ((h >> 40) + 1) * 2^-24,
                                               u2 = ((h >> 16) & 0xFFFFFF) * 2^-24
    jiggle   = +1e-12 if (h(lane, JIGGLE_T, 15) & 1) else -1e-12
"""
import numpy as np

M64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15
JIGGLE_T = (1 << 28) - 1


def mix64(z):
    """splitmix64 finaliser on numpy uint64 arrays (wrapping arithmetic)."""
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def counter(lane, t, k):
    lane = np.asarray(lane, dtype=np.uint64)
    t = np.asarray(t, dtype=np.uint64)
    k = np.asarray(k, dtype=np.uint64)
    return (lane << np.uint64(32)) | (t << np.uint64(4)) | k


def hash_bits(seed, lane, t, k):
    key = mix64(np.uint64(seed & M64))
    c = counter(lane, t, k)
    with np.errstate(over="ignore"):
        return mix64(key + c * np.uint64(GOLDEN))


def uniform(seed, lane, t, k):
    h = hash_bits(seed, lane, t, k)
    return ((h >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)).astype(np.float32)


def normal(seed, lane, t, k):
    h = hash_bits(seed, lane, t, k)
    u1 = (((h >> np.uint64(40)) + np.uint64(1)).astype(np.float32) * np.float32(2.0 ** -24)).astype(np.float32)
    u2 = (((h >> np.uint64(16)) & np.uint64(0xFFFFFF)).astype(np.float32) * np.float32(2.0 ** -24)).astype(np.float32)
    r = np.sqrt(np.float32(-2.0) * np.log(u1, dtype=np.float32), dtype=np.float32)
    c = np.cos(np.float32(2.0 * np.pi) * u2, dtype=np.float32)
    return (r * c).astype(np.float32)


def jiggle(seed, lane):
    h = hash_bits(seed, lane, JIGGLE_T, 15)
    return np.where((h & np.uint64(1)) == 1, 1e-12, -1e-12)
