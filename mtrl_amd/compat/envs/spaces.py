"""Box space: gymnasium's when installed, else a minimal stand-in with the same fields."""

from __future__ import annotations

import numpy as np

try:  # pragma: no cover - depends on the environment
    from gymnasium.spaces import Box  # noqa: F401
except ImportError:  # gymnasium is not part of this image

    class Box:  # type: ignore[no-redef]
        def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
            low = np.asarray(low, dtype=dtype)
            high = np.asarray(high, dtype=dtype)
            if shape is not None:
                low = np.broadcast_to(low, shape).astype(dtype)
                high = np.broadcast_to(high, shape).astype(dtype)
            self.low, self.high, self.dtype = low, high, np.dtype(dtype)
            self.shape = tuple(low.shape)
            self._rng = np.random.default_rng(seed)

        def sample(self):
            lo = np.where(np.isfinite(self.low), self.low, -1.0)
            hi = np.where(np.isfinite(self.high), self.high, 1.0)
            return self._rng.uniform(lo, hi).astype(self.dtype)

        def seed(self, seed=None):
            self._rng = np.random.default_rng(seed)


try:  # pragma: no cover - depends on the environment
    from gymnasium.spaces import Discrete  # noqa: F401
except ImportError:

    class Discrete:  # type: ignore[no-redef]
        def __init__(self, n, seed=None):
            self.n = int(n)
            self.shape = ()
            self._rng = np.random.default_rng(seed)

        def sample(self):
            return int(self._rng.integers(0, self.n))
