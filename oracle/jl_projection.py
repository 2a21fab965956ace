"""CPU restatement of DrQ.compute_weights' random projection -- TEST INFRASTRUCTURE ONLY (the
checker for drq_project_task_gradients, include/drq.h).

Reference: project_grad (mtrl/rl/algorithms/drqeps.py:428-448): for block c of 500 000 parameters,
jax.random.normal(jax.random.PRNGKey(seed + c), (rows, proj_dim)) / sqrt(proj_dim), accumulated
as chunk @ proj_chunk.  JAX itself is not in this image; its published algorithm (jax 0.5.3 as
pinned in the reference's uv.lock) is restated here:
  * PRNGKey(seed) for threefry = (seed >> 32, seed & 0xffffffff) = (0, seed) for 32-bit seeds;
  * jax_threefry_partitionable = True (the default since jax 0.5.0): element i of a random_bits
    array is threefry2x32(key, (i >> 32, i & 0xffffffff)), output words XORed (32-bit draws);
  * threefry2x32 with 20 rounds and rotations (13, 15, 26, 6) / (17, 29, 16, 24) (Salmon et al.
    2011, Random123) -- pinned by the Random123 known-answer vectors in tests/test_drq_cpu.py;
  * _uniform: float32 from (bits >> 9) | 0x3f800000, minus 1, scaled to [nextafter(-1, 0), 1);
  * normal = sqrt(2) * erf_inv(u) with XLA's single-precision erf_inv (Giles' polynomial).
The uniform / erf_inv steps are not pinned by any JAX output here (parity unpinned beyond the
threefry bits): the device path is compared with this restatement."""

from __future__ import annotations

import numpy as np

_ROT = ((13, 15, 26, 6), (17, 29, 16, 24))


def _rotl(x, r):
    return ((x << np.uint32(r)) | (x >> np.uint32(32 - r))).astype(np.uint32)


def threefry2x32(k0, k1, c0, c1):
    """threefry2x32_20 on uint32 arrays -> (x0, x1)."""
    with np.errstate(over="ignore"):
        k0, k1 = np.uint32(k0), np.uint32(k1)
        ks = (k0, k1, np.uint32(k0 ^ k1 ^ np.uint32(0x1BD11BDA)))
        x0 = (np.asarray(c0, np.uint32) + ks[0]).astype(np.uint32)
        x1 = (np.asarray(c1, np.uint32) + ks[1]).astype(np.uint32)
        for g in range(5):
            for r in _ROT[g % 2]:
                x0 = (x0 + x1).astype(np.uint32)
                x1 = _rotl(x1, r)
                x1 = (x1 ^ x0).astype(np.uint32)
            x0 = (x0 + ks[(g + 1) % 3]).astype(np.uint32)
            x1 = (x1 + ks[(g + 2) % 3] + np.uint32(g + 1)).astype(np.uint32)
    return x0, x1


_LT5 = (2.81022636e-08, 3.43273939e-07, -3.5233877e-06, -4.39150654e-06, 0.00021858087, -0.00125372503,
        -0.00417768164, 0.246640727, 1.50140941)
_GE5 = (-0.000200214257, 0.000100950558, 0.00134934322, -0.00367342844, 0.00573950773, -0.0076224613,
        0.00943887047, 1.00167406, 2.83297682)


def erf_inv32(x):
    x = np.asarray(x, np.float32)
    w = -np.log1p(-x * x)
    lt = w < np.float32(5.0)
    w = np.where(lt, w - np.float32(2.5), np.sqrt(w) - np.float32(3.0)).astype(np.float32)
    p = np.where(lt, np.float32(_LT5[0]), np.float32(_GE5[0])).astype(np.float32)
    for a, b in zip(_LT5[1:], _GE5[1:]):
        p = (np.where(lt, np.float32(a), np.float32(b)) + p * w).astype(np.float32)
    return (p * x).astype(np.float32)


def normal(seed: int, lin) -> np.ndarray:
    """jax.random.normal(PRNGKey(seed), shape).ravel()[lin], float32."""
    lin = np.asarray(lin, np.uint64)
    x0, x1 = threefry2x32(0, seed, (lin >> np.uint64(32)).astype(np.uint32), (lin & np.uint64(0xFFFFFFFF)).astype(np.uint32))
    bits = x0 ^ x1
    f = ((bits >> np.uint32(9)) | np.uint32(0x3F800000)).view(np.float32) - np.float32(1.0)
    lo = np.nextafter(np.float32(-1.0), np.float32(0.0))
    scale = np.float32(1.0) - lo  # rounds to 2.0
    u = np.maximum(lo, f * scale + lo).astype(np.float32)
    return (np.float32(np.sqrt(2)) * erf_inv32(u)).astype(np.float32)


def project(G: np.ndarray, proj_dim: int, chunk: int, seed: int) -> np.ndarray:
    """project_grad for every row of G [T][P] in float64 (small P x proj_dim only)."""
    G = np.asarray(G, np.float64)
    T, P = G.shape
    out = np.zeros((T, proj_dim))
    j = np.arange(proj_dim, dtype=np.uint64)
    for c0 in range(0, P, chunk):
        rows = min(chunk, P - c0)
        c = c0 // chunk
        lin = np.arange(rows, dtype=np.uint64)[:, None] * np.uint64(proj_dim) + j[None, :]
        N = normal(seed + c, lin).astype(np.float64) / np.sqrt(proj_dim)
        out += G[:, c0:c0 + rows] @ N
    return out
