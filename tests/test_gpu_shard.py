"""Task-sharded update (the multi-GPU decomposition) on one device.

Two engines own tasks [0,3) and [3,5) of a T=5 problem and sum their trunk
gradients through the bring-your-own all-reduce hook (include/mtsac.h,
mtsac_set_allreduce_hook) -- the same reduction points and scalar tail the RCCL
path uses.  The sharded run must reproduce the single-engine run and the oracle.
"""

from __future__ import annotations

import threading

import numpy as np
import pytest

from helpers import synthetic_batch, synthetic_eps
from oracle import mtsac as om

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("T,W,n,world", [(5, 32, 4, 2), (50, 2048, 2, 8)],
                         ids=["t5_w32_x2", "mt50_w2048_x8"])  # the second is the 8-GPU task split (7,7,6,...)
def test_sharded_update_matches_single_and_oracle(T, W, n, world):
    from mtrl_amd import _lib as L
    from mtrl_amd.engine import MTSACEngine, make_config
    from mtrl_amd.init import init_mtsac, leaf_shapes
    from mtrl_amd.shard import InProcessAllReduce, local_rows, shard_tasks

    D = 39 + T
    B = n * T
    cfgo = om.OracleConfig(num_tasks=T, obs_dim=D, actor_width=W, critic_width=W)
    a_full, c_full = init_mtsac(T, D, 4, W, 3, W, 3, 2, seed=3)
    st = om.initialize(cfgo, seed=0)
    st.actor, st.critic, st.critic_target = (a_full.astype(np.float64), c_full.astype(np.float64),
                                             c_full.astype(np.float64))

    def mk(begin, count):
        e = MTSACEngine(make_config(num_tasks=T, task_begin=begin, task_count=count, obs_dim=D, actor_width=W,
                                    critic_width=W, batch_per_task=n, capacity=16))
        a, c = init_mtsac(T, D, 4, W, 3, W, 3, 2, seed=3, task_begin=begin, task_count=count)
        e.set_params(L.ACTOR, a)
        e.set_params(L.CRITIC, c)
        e.set_params(L.CRITIC_TARGET, c)
        return e

    single = mk(0, T)
    shards = [mk(*shard_tasks(T, world, r)) for r in range(world)]
    group = InProcessAllReduce(world)
    for r, e in enumerate(shards):
        e.set_allreduce_hook(group.hook(r))

    for step in range(2):
        batch = synthetic_batch(T, B, seed=50 + step, dtype=np.float32)
        en, ec = synthetic_eps(B, seed=60 + step, dtype=np.float32)
        single.update(batch, en, ec)
        want1 = single.logs()
        st, want = om.update(cfgo, st, [b.astype(np.float64) for b in batch], en.astype(np.float64),
                             ec.astype(np.float64))
        errs = []

        def run(r):
            try:
                b0, c0 = shard_tasks(T, world, r)
                rows = local_rows(T, n, b0, c0)
                shards[r].update(tuple(x[rows] for x in batch), en[rows], ec[rows])
            except Exception as ex:  # pragma: no cover
                errs.append(ex)

        th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
        [t.start() for t in th]
        [t.join() for t in th]
        assert not errs, errs
        logs = [e.logs() for e in shards]
        assert all(lg == logs[0] for lg in logs)  # every scalar is reduced, so the ranks agree bitwise
        for k in ("losses/qf_loss", "losses/actor_loss", "losses/qf_values"):
            assert abs(logs[0][k] - want[k]) <= 1e-5 * max(abs(want[k]), 1e-3), (step, k, logs[0][k], want[k])
            assert abs(logs[0][k] - want1[k]) <= 1e-5 * max(abs(want1[k]), 1e-3)
        for k in ("metrics/critic_grad_magnitude", "metrics/actor_grad_magnitude", "metrics/critic_params_norm",
                  "metrics/actor_params_norm", "alpha", "losses/alpha_loss"):
            assert abs(logs[0][k] - want1[k]) <= 1e-4 * max(abs(want1[k]), 1e-3), (step, k, logs[0][k], want1[k])

    # trunks identical across shards; heads partition the single engine's heads
    for which, hd, ens in ((L.ACTOR, 8, None), (L.CRITIC, 1, 2)):
        full = single.get_params(which)
        parts = [e.get_params(which) for e in shards]
        in_dim = D if which == L.ACTOR else D + 4
        sh_full = leaf_shapes(in_dim, W, 3, T, hd, ens)
        def leaves(vec, T_l):
            out, o = {}, 0
            for k, s in leaf_shapes(in_dim, W, 3, T_l, hd, ens):
                m = int(np.prod(s)); out[k] = vec[o:o + m].reshape(s); o += m
            return out
        lf = leaves(full, T)
        lp = [leaves(p, shard_tasks(T, world, r)[1]) for r, p in enumerate(parts)]
        for k, _ in sh_full:
            if k.startswith("head"):
                got = np.concatenate([x[k] for x in lp], axis=0 if ens is None else 1)
            else:
                for x in lp[1:]:
                    np.testing.assert_array_equal(lp[0][k], x[k])
                got = lp[0][k]
            d = np.abs(got.astype(np.float64) - lf[k])
            # Adam can flip the sign of a ~0 gradient's update: median tight, max <= 2 * lr * steps
            assert np.median(d) < 1e-6 and d.max() < 2 * 3e-4 * 2 + 1e-6, (which, k, np.median(d), d.max())
    for e in shards + [single]:
        e.close()
