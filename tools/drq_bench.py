"""DrQ-eps gradient steps/s on one MI355X (experiments/atari.py: 26 games, IMPALA scale 1, 51 atoms,
batch 256), the batch resident on the device; next to the PyTorch-CPU fp32 restatement
(oracle/drq.py) on the host's cores.  Prints one JSON line.
usage: python tools/drq_bench.py [--steps K] [--warmup W] [--batch B] [--cpu-steps N]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=200)
ap.add_argument("--warmup", type=int, default=20)
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--cpu-steps", type=int, default=3)
ap.add_argument("--capacity", type=int, default=1000, help="device buffer slots per task for the sample+update leg")
args = ap.parse_args()

from mtrl_amd import _lib as L  # noqa: E402
from mtrl_amd.drq import DrQEngine, DrQSettings  # noqa: E402
from oracle import drq as od  # noqa: E402  (CPU baseline leg only)

B = args.batch
cfg = od.DrQConfig()
rng = np.random.default_rng(0)
obs = rng.integers(0, 256, (B, 4, 84, 84), dtype=np.uint8)
nobs = rng.integers(0, 256, (B, 4, 84, 84), dtype=np.uint8)
act = rng.integers(0, 18, B).astype(np.int32)
done = (rng.random(B) < 0.05).astype(np.float32)
rew = rng.standard_normal(B).astype(np.float32)
task = (np.arange(B) % 26).astype(np.int32)
co, cn = rng.integers(0, 8, (B, 2)).astype(np.int32), rng.integers(0, 8, (B, 2)).astype(np.int32)
no = (1 + 0.05 * np.clip(rng.standard_normal(B), -2, 2)).astype(np.float32)
nn = (1 + 0.05 * np.clip(rng.standard_normal(B), -2, 2)).astype(np.float32)
p0 = od.initialize(cfg, 0)

e = DrQEngine(DrQSettings(batch=B))
e.set_params(L.DRQ_PARAMS, p0)
e.set_params(L.DRQ_TARGET, p0)
e.update((obs, act, nobs, done, rew, task), (co, no, cn, nn))
e.update_resident(args.warmup)
e.synchronize()
t0 = time.perf_counter()
e.update_resident(args.steps)
e.synchronize()
dt = time.perf_counter() - t0
logs = e.logs()
e.close()

# sample_unbalanced + update from the device Atari buffer (MemoryEfficientAtariMultiTaskReplayBuffer,
# what OffPolicyAlgorithm.train calls), filled past capacity so the guard window is in play; the
# Dirichlet / index draws on the host are inside the timed region
import dataclasses  # noqa: E402

eb = DrQEngine(dataclasses.replace(DrQSettings(batch=B), capacity=args.capacity))
eb.set_params(L.DRQ_PARAMS, p0)
eb.set_params(L.DRQ_TARGET, p0)
eb.seed_rng(1)
T = 26
a0 = time.perf_counter()
for i in range(args.capacity + 8):
    o = np.roll(obs[:T], i, axis=-1)
    eb.buffer_add(o, o, act[:T], rew[:T], np.zeros(T, np.float32), done[:T])
eb.synchronize()
add_dt = time.perf_counter() - a0
eb.seed_augment(2)
eb.sample_unbalanced_update(args.warmup)
eb.synchronize()
t0 = time.perf_counter()
eb.sample_unbalanced_update(args.steps)
eb.synchronize()
sdt = time.perf_counter() - t0
eb.close()

import torch  # noqa: E402

threads = torch.get_num_threads()
st = od.init_state(cfg, 0)
ob, nb = od.augment(obs, co, no), od.augment(nobs, cn, nn)
batch = (ob, act, nb, done, rew, task)
st, _ = od.update(cfg, st, batch, dtype=torch.float32)  # warm-up
c0 = time.perf_counter()
for _ in range(args.cpu_steps):
    st, _ = od.update(cfg, st, batch, dtype=torch.float32)
cdt = time.perf_counter() - c0
print(json.dumps({
    "metric": "DrQ-eps gradient steps/sec, 26 Atari games, IMPALA (scale 1) + dueling C51 (51 atoms), batch %d" % B,
    "value": args.steps / dt, "unit": "gradient steps/sec", "ms_per_step": 1e3 * dt / args.steps,
    "steps": args.steps, "warmup": args.warmup, "dtype": "fp32", "data": "synthetic uint8 frames, resident batch",
    "logs": logs,
    "sample_update": {"value": args.steps / sdt, "unit": "gradient steps/sec", "ms_per_step": 1e3 * sdt / args.steps,
                      "sampler": "sample_unbalanced (host draws, device gather + augmentation draws)",
                      "capacity_per_task": args.capacity, "buffer_full": True,
                      "add_ms_per_env_step": 1e3 * add_dt / (args.capacity + 8)},
    "cpu_baseline": {"value": args.cpu_steps / cdt, "unit": "gradient steps/sec", "cores": threads, "kind": "port",
                     "sample": f"{args.cpu_steps} steps of the PyTorch-CPU fp32 restatement (oracle/drq.py), batch {B}"},
}), flush=True)
