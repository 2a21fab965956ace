"""ImpalaDQN parameters for the DrQ-eps engine, in flax ravel order (include/drq.h).

Layout: ImpalaDQN.init (mtrl/rl/networks.py:127-149) flattened with dict keys sorted at every
level -- DistributionalDense_0 (Dense_0, Dense_1 = advantage, Dense_2 = value, LayerNorm_0),
ImpalaEncoder_0 (stack_s / Conv_0..Conv_4, kernel [3][3][Cin][Cout]), LayerNorm_0,
TaskEmbedding_0/Embed_0/embedding.  Initialisers as the reference's modules: xavier_uniform for
each stack's first conv and the head's Dense layers (impala.py:17, networks.py:109), flax's
lecun_normal (truncated normal) for the residual convs, zero biases, LayerNorm scale 1, Embed variance_scaling(1,
fan_in, normal).  DrQ.initialize's shrink-and-perturb (drqeps.py:182-197): encoder leaves are the
mean of two independent draws, everything else the second draw.  The numpy stream replaces JAX's
threefry (not reproducible)."""

from __future__ import annotations

import math

import numpy as np


def param_spec(num_tasks=26, n_actions=18, n_atoms=51, in_ch=4, hw=84, scale=1, embed_dim=32, n_hidden=512,
               stacks=(8, 16, 16), blocks=2):
    h, c, convs = hw, in_ch, []
    for si, s in enumerate(stacks):
        co = scale * s
        for k in range(1 + 2 * blocks):
            cin = c if k == 0 else co
            convs += [(f"ImpalaEncoder_0/stack_{si}/Conv_{k}/bias", (co,)),
                      (f"ImpalaEncoder_0/stack_{si}/Conv_{k}/kernel", (3, 3, cin, co))]
        h, c = (h + 1) // 2, co
    F = h * h * c + embed_dim
    H = n_hidden * scale
    A, Z = n_actions, n_atoms
    d = "DistributionalDense_0/"
    return ([(d + "Dense_0/bias", (H,)), (d + "Dense_0/kernel", (F, H)), (d + "Dense_1/bias", (A * Z,)),
             (d + "Dense_1/kernel", (H, A * Z)), (d + "Dense_2/bias", (Z,)), (d + "Dense_2/kernel", (H, Z)),
             (d + "LayerNorm_0/bias", (H,)), (d + "LayerNorm_0/scale", (H,))] + convs +
            [("LayerNorm_0/bias", (F,)), ("LayerNorm_0/scale", (F,)),
             ("TaskEmbedding_0/Embed_0/embedding", (num_tasks, embed_dim))])


def truncated_lecun_normal(rng: np.random.Generator, shape, fan_in: int) -> np.ndarray:
    """flax's default kernel init lecun_normal = jax variance_scaling(1, "fan_in",
    "truncated_normal"): a standard normal truncated to [-2, 2], scaled by
    sqrt(1 / fan_in) / 0.87962566103423978 (the std of that truncated normal), so the leaf has
    variance 1 / fan_in.  Rejection sampling on the numpy stream (threefry is not reproduced)."""
    z = rng.standard_normal(shape)
    bad = np.abs(z) > 2.0
    while bad.any():
        z[bad] = rng.standard_normal(int(bad.sum()))
        bad = np.abs(z) > 2.0
    return z * (math.sqrt(1.0 / fan_in) / 0.87962566103423978)


def _draw(spec, rng):
    out = []
    for path, shape in spec:
        leaf = path.rsplit("/", 1)[1]
        if leaf == "bias":
            v = np.zeros(shape)
        elif leaf == "scale":
            v = np.ones(shape)
        elif leaf == "embedding":
            v = rng.normal(0.0, 1.0 / math.sqrt(shape[1]), shape)
        elif "/Conv_" in path and not path.endswith("Conv_0/kernel"):
            v = truncated_lecun_normal(rng, shape, shape[0] * shape[1] * shape[2])
        else:
            fi, fo = ((shape[0] * shape[1] * shape[2], shape[0] * shape[1] * shape[3]) if len(shape) == 4 else shape)
            lim = math.sqrt(6.0 / (fi + fo))
            v = rng.uniform(-lim, lim, shape)
        out.append(np.asarray(v, np.float64).ravel())
    return out


def init_drq(seed: int = 1, shrink_rate: float = 0.5, **geometry) -> np.ndarray:
    spec = param_spec(**geometry)
    rng = np.random.default_rng(seed)
    first, fresh = _draw(spec, rng), _draw(spec, rng)
    parts = [(a * (1 - shrink_rate) + b * shrink_rate) if p.startswith("ImpalaEncoder_0") else b
             for (p, _), a, b in zip(spec, first, fresh)]
    return np.concatenate(parts).astype(np.float32)


def shrink_and_perturb(params: np.ndarray, rng: np.random.Generator, shrink_rate: float = 0.5,
                       **geometry) -> np.ndarray:
    """DrQ.shrink_and_perturb (drqeps.py:212-245) on a flat parameter vector: one fresh draw; the
    ImpalaEncoder leaves become old (1 - rate) + fresh rate (float32, as jax computes them), every
    other leaf the fresh draw."""
    spec = param_spec(**geometry)
    fresh = _draw(spec, rng)
    old = np.asarray(params, np.float32)
    out, o = [], 0
    r = np.float32(shrink_rate)
    for (path, shape), new in zip(spec, fresh):
        n = int(np.prod(shape))
        new = new.astype(np.float32)
        out.append(old[o:o + n] * (np.float32(1) - r) + new * r if path.startswith("ImpalaEncoder_0") else new)
        o += n
    assert o == old.size, (o, old.size)
    return np.concatenate(out)
