"""ORACLE-SIDE CPU BASELINE (test/measurement infrastructure only).

Only ``bench.py``'s ``cpu_baseline`` leg (and tests) may import this module.

A PyTorch-CPU fp32 restatement of the reference's update (XLA:CPU cannot run
here: jax absent, Python 3.10 -- SURVEY.md §8c/§8d), structured like the
reference program rather than like the HIP engine: all T heads are evaluated on
every row and the row's head is selected afterwards (``nn.vmap(nn.Dense)`` +
``x[arange(B), task]``, mtrl/nn/multi_head.py:50-66), gradients come from
autograd (``jax.value_and_grad``, mtsac.py:587-596, 689-691, 723-725), and the
optimizer is optax clip_by_global_norm + adam restated (config/optim.py:26-43).
Replay sampling uses numpy's ``default_rng`` exactly like buffers.py:523-548.
It uses every thread it is given (``torch.set_num_threads``).
"""

from __future__ import annotations

import math

import numpy as np
import torch


class CPUMTSAC:
    def __init__(self, num_tasks, obs_dim, width, batch_per_task, capacity, seed=1, action_dim=4, depth=3,
                 num_critics=2, dtype=torch.float32, clip=False):
        self.T, self.D, self.W, self.A = num_tasks, obs_dim, width, action_dim
        self.n, self.cap, self.C, self.depth = batch_per_task, capacity, num_critics, depth
        self.clip = clip
        self.dt = dtype
        g = torch.Generator().manual_seed(seed)

        def he(fan_in, shape):
            lim = math.sqrt(6.0 / fan_in)
            return ((torch.rand(shape, generator=g, dtype=dtype) * 2 - 1) * lim).requires_grad_(True)

        def uni(b, shape):
            return ((torch.rand(shape, generator=g, dtype=dtype) * 2 - 1) * b).requires_grad_(True)

        def net(in_dim, hd, bound, ens):
            pre = () if ens is None else (ens,)
            p = {}
            fan = in_dim
            for i in range(depth):
                p[f"W{i}"] = he(fan, pre + (fan, width))
                p[f"b{i}"] = torch.zeros(pre + (width,), dtype=dtype, requires_grad=True)
                fan = width
            p["head_W"] = uni(bound, pre + (num_tasks, width, hd))
            p["head_b"] = uni(bound, pre + (num_tasks, hd))
            return p

        self.actor = net(obs_dim, 2 * action_dim, 1e-3, None)
        self.critic = net(action_dim + obs_dim, 1, 3e-3, num_critics)
        self.target = {k: v.detach().clone() for k, v in self.critic.items()}
        self.log_alpha = torch.zeros(num_tasks, dtype=dtype, requires_grad=True)
        self.opt = {}
        for name, p in (("actor", self.actor), ("critic", self.critic), ("alpha", {"la": self.log_alpha})):
            self.opt[name] = ({k: torch.zeros_like(v) for k, v in p.items()},
                              {k: torch.zeros_like(v) for k, v in p.items()}, [0])
        # replay buffer (cap, T, dim) float32 filled per SURVEY.md §8d
        r = np.random.default_rng(1234)
        F = obs_dim - num_tasks
        self.obs = np.zeros((capacity, num_tasks, obs_dim), np.float32)
        self.obs[:, :, :F] = r.standard_normal((capacity, num_tasks, F), dtype=np.float32)
        self.obs[:, np.arange(num_tasks), F + np.arange(num_tasks)] = 1.0
        self.nobs = self.obs.copy()
        self.nobs[:, :, :F] = r.standard_normal((capacity, num_tasks, F), dtype=np.float32)
        self.act = r.uniform(-1, 1, (capacity, num_tasks, action_dim)).astype(np.float32)
        self.rew = r.uniform(0, 10, (capacity, num_tasks, 1)).astype(np.float32)
        self.done = (r.uniform(size=(capacity, num_tasks, 1)) < 1 / 500).astype(np.float32)
        self.rng = np.random.default_rng(seed)
        self.noise = torch.Generator().manual_seed(2)

    # --------------------------------------------------------------- networks
    def _mh(self, p, x, sel=None):
        t = torch.argmax(x[:, -self.T:], dim=1)
        h = x
        for i in range(self.depth):
            w, b = (p[f"W{i}"], p[f"b{i}"]) if sel is None else (p[f"W{i}"][sel], p[f"b{i}"][sel])
            h = torch.relu(h @ w + b)
        hw, hb = (p["head_W"], p["head_b"]) if sel is None else (p["head_W"][sel], p["head_b"][sel])
        allh = torch.einsum("bw,twk->btk", h, hw) + hb[None]
        return allh[torch.arange(x.shape[0]), t]

    def _q(self, p, x):
        return torch.stack([self._mh(p, x, c) for c in range(self.C)])

    def _pi(self, x, eps):
        out = self._mh(self.actor, x)
        mu, ls = out[:, : self.A], torch.clamp(out[:, self.A:], -20.0, 2.0)
        sig = torch.exp(ls)
        z = mu + sig * eps
        a = torch.tanh(z)
        lp = (-0.5 * eps**2 - 0.5 * math.log(2 * math.pi) - torch.log(sig)).sum(1) - (
            2.0 * (math.log(2.0) - z - torch.nn.functional.softplus(-2.0 * z))).sum(1)
        return a, lp

    def _apply(self, name, params, max_norm):
        m, v, cnt = self.opt[name]
        with torch.no_grad():
            if max_norm is not None:
                gn = torch.sqrt(sum((p.grad.double() ** 2).sum() for p in params.values())).float()
                if not bool(gn < max_norm):
                    for p in params.values():
                        p.grad.copy_((p.grad / gn) * max_norm)
            cnt[0] += 1
            bc1, bc2 = 1 - 0.9 ** cnt[0], 1 - 0.999 ** cnt[0]
            for k, p in params.items():
                m[k].mul_(0.9).add_(p.grad, alpha=0.1)
                v[k].mul_(0.999).addcmul_(p.grad, p.grad, value=0.001)
                p.add_((m[k] / bc1) / (torch.sqrt(v[k] / bc2) + 1e-5), alpha=-3e-4)
                p.grad = None

    # --------------------------------------------------------------- one step
    def step(self):
        idx = self.rng.integers(0, self.cap, size=self.n)  # buffers.py:523-527 (buffer full)
        B = self.n * self.T
        obs = torch.from_numpy(self.obs[idx].reshape(B, -1))
        nobs = torch.from_numpy(self.nobs[idx].reshape(B, -1))
        act = torch.from_numpy(self.act[idx].reshape(B, -1))
        rew = torch.from_numpy(self.rew[idx].reshape(B, 1))
        done = torch.from_numpy(self.done[idx].reshape(B, 1))
        tid = obs[:, -self.T:]
        alpha = torch.exp(tid @ self.log_alpha.detach().reshape(-1, 1))
        en = torch.randn((B, self.A), generator=self.noise, dtype=self.dt)
        ec = torch.randn((B, self.A), generator=self.noise, dtype=self.dt)
        with torch.no_grad():
            an, lpn = self._pi(nobs, en)
            qt = torch.stack([self._mh({k: v for k, v in self.target.items()}, torch.cat([an, nobs], 1), c)
                              for c in range(self.C)])
            y = rew + (1 - done) * 0.99 * (qt.min(0).values - alpha * lpn.reshape(-1, 1))
        q = self._q(self.critic, torch.cat([act, obs], 1))
        if self.clip:
            y, q = torch.clamp(y, -5000, 5000), torch.clamp(q, -5000, 5000)
        qf_loss = ((q - y[None]) ** 2).mean()
        qf_loss.backward()
        self._apply("critic", self.critic, 1.0)
        with torch.no_grad():
            for k in self.target:
                self.target[k].mul_(0.995).add_(self.critic[k], alpha=0.005)
        a, lp = self._pi(obs, ec)
        qpi = self._q(self.critic, torch.cat([a, obs], 1))
        actor_loss = (alpha * lp.reshape(-1, 1) - qpi.min(0).values).mean()
        for p in self.critic.values():
            p.requires_grad_(False)
        actor_loss.backward()
        for p in self.critic.values():
            p.requires_grad_(True)
        self._apply("actor", self.actor, 1.0)
        alpha_loss = (-(tid @ self.log_alpha.reshape(-1, 1)) * (lp.detach().reshape(-1, 1) - self.A)).mean()
        alpha_loss.backward()
        self._apply("alpha", {"la": self.log_alpha}, None)
        return float(qf_loss), float(actor_loss)
