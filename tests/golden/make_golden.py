"""Regenerate the golden fixtures under tests/golden/ from the oracle.

    python tests/golden/make_golden.py

update_small.npz: one MTSAC step (T=3, W=16, B=12, float64) -- inputs, injected
noise, the 10 logs and the post-update actor vector.  index_streams.npz: replay
index vectors drawn by numpy.random.default_rng (the reference's dependency) for
seeds {0, 1, 42} and highs {7, 128, 4001, 100000}, n = 128, three consecutive
draws each.  These are self-generated (parity unpinned for the update math,
see oracle/mtsac.py); the index streams are numpy's own output.
"""

import pathlib
import sys

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
sys.path.insert(0, str(HERE.parent))

from helpers import synthetic_batch, synthetic_eps  # noqa: E402
from oracle import mtsac as om  # noqa: E402


def main():
    T, W, B, seed = 3, 16, 12, 7
    cfg = om.OracleConfig(num_tasks=T, obs_dim=39 + T, actor_width=W, critic_width=W)
    st = om.initialize(cfg, seed=seed)
    batch = synthetic_batch(T, B, seed=1)
    en, ec = synthetic_eps(B, seed=2)
    new, logs = om.update(cfg, st, batch, en, ec)
    np.savez_compressed(
        HERE / "update_small.npz", T=T, D=39 + T, W=W, seed=seed, obs=batch[0], act=batch[1], nobs=batch[2],
        done=batch[3], rew=batch[4], eps_next=en, eps_cur=ec,
        logs=np.array([logs[k] for k in om.LOG_KEYS]), actor_after=new.actor,
    )
    streams = {}
    for s in (0, 1, 42):
        for high in (7, 128, 4001, 100000):
            r = np.random.default_rng(s)
            streams[f"s{s}_h{high}"] = np.stack([r.integers(0, high, size=128) for _ in range(3)])
    np.savez_compressed(HERE / "index_streams.npz", **streams)


if __name__ == "__main__":
    main()
