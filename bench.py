#!/usr/bin/env python3
"""bench.py -- SAC gradient-steps/sec of the MI355X MTSAC engine (BASELINE.json metric).

One "step" = one complete MTSAC gradient step (reference MTSAC.update,
mtrl/rl/algorithms/mtsac.py:1173-1251) on one batch of 128 rows per task drawn
from the device-resident replay buffer: index stream + gather, actor forward on s',
target critic, critic forward/backward + clip/Adam/Polyak, actor forward, critic
with the updated params, actor backward + clip/Adam, temperature update.  Nothing
is skipped inside the timed region; inputs are resident in HBM.

Default workload (N=1): MT50 MTMHSAC-v2 at width 2048 (experiments/width_scaling/
mt50_mtmhsac_v2_2048.py): T=50, B=6400, fp32-accurate arithmetic: the trunk GEMMs on fp16 MFMA as
two power-of-two-scaled fp16 planes per operand and three products (precision split2h, held to the
fp32-GEMM error bound and the 1e-5 loss bar by tests/; --precision split3 is the 3-plane bf16 form).  With --gpus N (torchrun, or N rank
processes spawned here before anything touches a GPU; one rank per GPU) the 50 tasks are sharded contiguously over the ranks and the trunk gradients
are all-reduced over RCCL; the problem size is fixed, so scaling is "strong".

Prints ONE JSON line on rank 0 (keys per the driver contract, plus roofline and
cpu_baseline).
"""

from __future__ import annotations

import argparse
import json
import math
import re
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

WORKLOADS = {
    # name: (T, width, clip, description)
    "mt50_w2048": (50, 2048, False, "MT50 MTMHSAC-v2 width=2048 (experiments/width_scaling/mt50_mtmhsac_v2_2048.py)"),
    "mt10_w2048": (10, 2048, True, "MT10 MTMHSAC width=2048 clip (experiments/width_scaling/mt10_mtmhsac_v2_2048.py)"),
    "mt10_w400": (10, 400, False, "MT10 MTMHSAC width=400 (experiments/mt10_mtmhsac.py)"),
    "mt50_w400": (50, 400, False, "MT50 MTMHSAC-v2 width=400 (experiments/mt50_mtmhsac_v2.py)"),
}
FP32_MFMA_PEAK_TF = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
BF16_MFMA_PEAK_TF = 2500.0  # MI355X_MICROARCH.md: bf16 dense MFMA peak (no sparsity)
PRECISIONS = {"fp32": 0, "split3": 1, "bf16": 2, "split2h": 3}
HBM_PEAK_GBS = 8000.0
# enum mtsac_gemm_family (include/mtsac.h) -> the rocprof kernel(s) of that family, per precision
GEMM_FAMILIES = {
    "split3": {
        0: "gemm_x3f_kernel<208, 1, *, *, false, 0, 3> (hidden-layer forward, planes, bias+ReLU)",
        1: "gemm_x3f_kernel<208, 2, *, *, true, 0, 3> (hidden-layer data grad, planes, ReLU mask from the bf16 high plane)",
        2: "gemm_x3p_kernel<Geo<256, 256, 2, 4, 3, 16, 0>, true, true, 0, false, 3> (hidden-layer weight grad, k-major planes, split-K)",
        3: "gemm_x3f_kernel<208, 1, false, true, false, 8, 3> (input-layer forward, planes, K = in_dim padded to 64)",
        4: "gemm_x3_kernel<true, false, 0> (input-layer weight grad, on-the-fly split, split-K)",
    },
    "split2h": {
        0: "gemm_x3f_kernel<208, 1, *, *, false, 0, 2> (hidden-layer forward, fp16 planes, bias+ReLU)",
        1: "gemm_x3f_kernel<208, 2, *, *, true, 0, 2> (hidden-layer data grad, fp16 planes, ReLU mask from the planes)",
        2: "gemm_x3p_kernel<Geo<256, 128, 4, 2, 4, 16, 0>, true, true, 0, false, 2> (hidden-layer weight grad, k-major fp16 planes, 256 x 128 k16 tiles; the critic's without split-K)",
        3: "gemm_x3f_kernel<208, 1, false, true, false, 8, 2> (input-layer forward, fp16 planes, K = in_dim padded to 64)",
        4: "gemm_x3p_kernel<Geo<256, 128, 4, 2, 4, 16, 0>, true, true, 0, false, 2> (input-layer weight grad, k-major fp16 planes of dz0, split-K)",
    },
    "fp32": {
        0: "gemm_f32_kernel<false, true, 1> (hidden-layer forward, NT vs transposed kernel)",
        1: "gemm_f32_kernel<false, true, 2> (hidden-layer data grad)",
        2: "gemm_f32_kernel<true, false, 0> (hidden-layer weight grad)",
        3: "gemm_f32_kernel<false, false, 1> (input-layer forward)",
        4: "gemm_f32_kernel<true, false, 0> (input-layer weight grad, split-K)",
    },
}
METRIC = "SAC gradient-steps/sec, MT50 width-2048 batch=128/task, 1/2/4/8 MI355X"
# BASELINE.json configs[4] (experiments/atari.py): the reference's Atari agent is DrQ-eps, not PPO
# 
DRQ_WORKLOAD = "atari_drq"
DRQ_METRIC = "DrQ-eps gradient-steps/sec, experiments/atari.py (26 games, IMPALA scale 1, dueling C51, batch 256), 1 MI355X"
FP32_VALU_PEAK_TF = 157.3  # MI355X_MICROARCH.md: peak FP32 (vector)


def _recency(path):  # r<round><letters>_...: rounds in order, then a..z, aa..zz (the naming used here)
    m = re.match(r"r(\d+)([a-z]*)", os.path.basename(path))
    return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")


def pmc_clock(precision, family, workload):
    """The shader clock the chip held under a GEMM family in the newest committed clock pass of the
    default workload (profiles/*_clock.json, tools/pmc_clock.py: GRBM_GUI_ACTIVE / 8 / duration), and
    the family's fraction of the peak at that clock there; None for other workloads."""
    import glob

    if workload != "mt50_w2048":
        return None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_clock.json")), key=_recency, reverse=True):
        try:
            with open(path) as f:
                v = json.load(f).get(precision, {}).get(str(family))
            if v is not None:
                return {"clock_ghz": v["clock_ghz"], "frac_nominal": v["frac_nominal"],
                        "frac_at_clock": v["frac_at_clock"], "source": os.path.relpath(path, ROOT),
                        "basis": "eager pass under rocprofv3 --pmc GRBM_GUI_ACTIVE; peak x clock / 2.4 GHz"}
        except (OSError, ValueError, KeyError):
            continue
    return None


def pmc_traffic(precision, family, workload):
    """HBM bytes per launch of a GEMM family from the committed rocprofv3 PMC summary of THIS
    workload (profiles/*_pmc_traffic.json, written by tools/pmc_traffic.py; a file without a
    "workload" key is the default mt50_w2048 run), or None."""
    import glob

    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")), key=_recency, reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
            if d.get("workload", "mt50_w2048") != workload:
                continue
            v = d.get(precision, {}).get(str(family))
            if v is not None:
                return v["hbm_bytes_per_launch"], os.path.relpath(path, ROOT)
        except (OSError, ValueError, KeyError):
            continue
    return None, None


def build_stamps():
    """Provenance of the measured library: the source hash stamped into libmtsac.so at link time and
    the hash of the sources in this tree (mtrl_amd/_lib.py refuses a library whose stamp differs)."""
    try:
        from mtrl_amd import _lib as L

        return {"lib_stamp": L.load().mtsac_build_stamp().decode(), "source_stamp": L.source_stamp()}
    except Exception as e:  # pragma: no cover - reported, not fatal for a dry run
        return {"error": str(e)}


def algorithmic_flops(T, W, n=128, A=4):
    """GEMM flops of one step counting only each row's own head."""
    B = n * T
    Ia, Ic = 39 + T, 39 + T + A
    Af = 2 * B * (Ia * W + 2 * W * W + 8 * W)
    Cf = 2 * B * (Ic * W + 2 * W * W + W)
    return (Af + 2 * Cf + 2 * (3 * Cf - 2 * B * Ic * W) + (3 * Af - 2 * B * Ia * W)
            + 2 * (2 * Cf - 2 * B * Ic * W + 2 * B * 4 * W))


def available_cores():
    """Cores this process may run on: the affinity mask, capped by a cgroup CPU quota when
    one is set (the GPU box grants a share of a larger host)."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, math.ceil(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    return (min(n, quota) if quota else n), n, quota


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            return next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), "")
    except OSError:
        return ""


def cpu_time_steps(T, W, clip, steps, threads):
    import torch
    from oracle.cpu_baseline import CPUMTSAC

    torch.set_num_threads(threads)
    m = CPUMTSAC(T, 39 + T, W, 128, 100_000, clip=clip)
    m.step()  # warm-up
    t0 = time.perf_counter()
    for _ in range(steps):
        m.step()
    return steps / (time.perf_counter() - t0), time.perf_counter() - t0


def cpu_baseline(T, W, clip, steps, c0_steps):
    """The oracle-side PyTorch-CPU restatement on this host's cores: the bench
    workload on a bounded sample of steps, plus C0 (MT10/W400, the reference's own config)."""
    threads, affinity, quota = available_cores()
    sps, dt = cpu_time_steps(T, W, clip, steps, threads)
    out = {"value": sps, "unit": "SAC gradient-steps/sec", "cores": threads, "kind": "port",
           "sample": f"{steps} full steps (B={128 * T}, W={W}, fp32 PyTorch-CPU autograd restatement, "
                     f"oracle/cpu_baseline.py) after 1 warm-up step, {dt:.1f}s on {threads} threads; "
                     f"affinity {affinity} cpus, cgroup quota {quota or 'none'}; {cpu_model()}"}
    if c0_steps > 0:
        c0, dt0 = cpu_time_steps(10, 400, False, c0_steps, threads)
        out["c0_mt10_w400"] = {"value": c0, "unit": "SAC gradient-steps/sec", "cores": threads,
                               "sample": f"{c0_steps} steps of C0 (MT10 W=400 B=1280, experiments/mt10_mtmhsac.py), "
                                         f"{dt0:.1f}s"}
    return out


def bench_drq(args, world, rank, local_rank, dist):
    """configs[4]: one DrQ-eps training step = sample_unbalanced(256) from a full device Atari
    buffer (host Dirichlet / index draws included) + augmentation + the three ImpalaDQN passes,
    C51 loss, backward, AdamW, Polyak (mtrl/rl/algorithms/drqeps.py:268-351, base.py:213-221).
    The agent does not shard: with --gpus N every rank runs its own replica ("replicas only")."""
    import dataclasses

    import torch

    from mtrl_amd import _lib as L
    from mtrl_amd.drq import DrQEngine, DrQSettings
    from mtrl_amd.drq_init import init_drq

    s = dataclasses.replace(DrQSettings(batch=256), capacity=args.drq_capacity, normalize_rewards=1)
    e = DrQEngine(s, device=local_rank)
    p = init_drq(1)
    e.set_params(L.DRQ_PARAMS, p)
    e.set_params(L.DRQ_TARGET, p)
    e.seed_rng(1 + rank)
    e.seed_augment(2 + rank)
    rng = np.random.default_rng(rank)
    T = s.num_tasks
    frames = rng.integers(0, 256, (T, 4, 84, 84), dtype=np.uint8)
    for i in range(s.capacity + s.nstep + 8):  # past capacity: the guard window is in play
        o = np.roll(frames, i, axis=-1)
        e.buffer_add(o, np.roll(o, 1, axis=-1), rng.integers(0, 18, T), rng.standard_normal(T).astype(np.float32),
                     np.zeros(T, np.float32), (rng.random(T) < 0.01).astype(np.float32))
    e.sample_unbalanced_update(args.warmup)
    e.synchronize()
    settle = 0
    if args.settle_s > 0:
        a = time.perf_counter()
        e.sample_unbalanced_update(20)
        e.synchronize()
        settle = [int(args.settle_s / max((time.perf_counter() - a) / 20, 1e-4))]
        if dist:
            dist.broadcast_object_list(settle, src=0)
        settle = settle[0]
        e.sample_unbalanced_update(settle)
        e.synchronize()
    e.set_timing(False)  # the timed steps run without events (as the SAC bench); then an events pass
    if dist:
        dist.barrier()
    torch.cuda.synchronize(local_rank)
    t0 = time.perf_counter()
    e.sample_unbalanced_update(args.steps)
    e.synchronize()
    torch.cuda.synchronize(local_rank)
    elapsed = time.perf_counter() - t0
    if dist:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    e.set_timing(True)
    e.sample_unbalanced_update(args.steps)
    e.synchronize()
    ms, nl, fl = e.timing()
    e.set_timing(False)
    logs = e.logs()
    e.close()
    assert all(math.isfinite(v) for v in logs.values()), logs
    achieved = (fl / nl) / (ms / nl * 1e-3) / 1e12 if nl else 0.0
    out = {
        "metric": DRQ_METRIC, "value": world * args.steps / elapsed, "unit": "DrQ gradient-steps/sec",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps,
        "settle_steps": settle, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
        "data": f"synthetic uint8 frame stacks in a full device MemoryEfficientAtariMultiTaskReplayBuffer "
                f"({s.capacity} slots/task), random-init ImpalaDQN",
        "config": {"workload": "experiments/atari.py DrQ-eps: 26 games, 4x84x84 uint8, IMPALA 8/16/16 scale 1, "
                               "task embedding 32, dense 512, 18 actions x 51 atoms, 3-step returns",
                   "global_batch": 256 * world, "batch_per_replica": 256, "sampler": "sample_unbalanced",
                   "parallelism": f"replicas{world}" if world > 1 else "single"},
        "roofline": {"bound": "valu", "kernel": "conv_fwd_kernel<ci, co, *, *> (IMPALA 3x3 convs, direct fp32 FMA "
                                                "on the vector ALUs; an MFMA implicit GEMM is not built, DESIGN 6b)",
                     "achieved": achieved, "peak": FP32_VALU_PEAK_TF, "peak_basis": "FP32 vector peak",
                     "unit": "TFLOP/s", "frac": achieved / FP32_VALU_PEAK_TF, "traffic": None,
                     "launches": nl, "avg_launch_us": 1e3 * ms / max(nl, 1),
                     "algorithmic_flops_per_launch": fl / max(nl, 1),
                     "timing": "HIP events per launch on the engine stream, every 8th update of a second pass of "
                               "the timed steps (the timed pass runs without events)"},
        "logs": logs,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import drq as od  # the cpu_baseline leg only

        threads, affinity, quota = available_cores()
        torch.set_num_threads(threads)
        cfg = od.DrQConfig()
        st = od.init_state(cfg, 0)
        B = 256
        obs = rng.integers(0, 256, (B, 4, 84, 84), dtype=np.uint8)
        crop = rng.integers(0, 8, (B, 2)).astype(np.int32)
        noise = (1 + 0.05 * np.clip(rng.standard_normal(B), -2, 2)).astype(np.float32)
        batch = (od.augment(obs, crop, noise), rng.integers(0, 18, B).astype(np.int32),
                 od.augment(np.roll(obs, 1, -1), crop, noise), np.zeros(B, np.float32),
                 rng.standard_normal(B).astype(np.float32), (np.arange(B) % 26).astype(np.int32))
        st, _ = od.update(cfg, st, batch, dtype=torch.float32)
        a = time.perf_counter()
        for _ in range(args.cpu_steps):
            st, _ = od.update(cfg, st, batch, dtype=torch.float32)
        dt = time.perf_counter() - a
        out["cpu_baseline"] = {"value": args.cpu_steps / dt, "unit": "DrQ gradient-steps/sec", "cores": threads,
                               "kind": "port",
                               "sample": f"{args.cpu_steps} DrQ updates at batch {B} (augmentation, 3 ImpalaDQN passes, "
                                         f"C51, autograd backward, AdamW) of the PyTorch-CPU fp32 restatement "
                                         f"oracle/drq.py, {dt:.1f}s on {threads} threads; {cpu_model()}"}
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n):
    """`bench.py --gpus N` outside torchrun: start N fresh rank processes (nothing here has
    touched the GPU), forward rank 0's output, exit with the worst return code."""
    import subprocess

    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="mt50_w2048", choices=sorted(WORKLOADS) + [DRQ_WORKLOAD])
    ap.add_argument("--drq-capacity", type=int, default=2000, help="atari_drq: device buffer slots per task")
    ap.add_argument("--no-graph", action="store_true", help="same as --exec eager")
    ap.add_argument("--exec", default="auto", choices=["auto", "graph", "eager", "pipelined"],
                    help="hipGraph replay, eager steps, or eager steps with cross-step pipelining (the next "
                         "step's gather + critic forward beside the previous step's tail); auto = the fastest "
                         "(task shards: pipelined)")
    ap.add_argument("--precision", default="split2h", choices=sorted(PRECISIONS),
                    help="fp32: f32-input MFMA; split3: fp32-accurate 3-way bf16 split on bf16 MFMA; "
                         "split2h: fp32-accurate 2-way fp16 split (per-tensor power-of-two scale) on fp16 MFMA; "
                         "bf16: perf-only, trunk GEMM operands rounded to bf16 (one MFMA per product)")
    ap.add_argument("--settle-s", type=float, default=6.0,
                    help="untimed steady-state seconds after the warm-up (DVFS settles under load; long enough "
                         "for a once-per-second utilisation sampler to see the GPU busy)")
    ap.add_argument("--cpu-steps", type=int, default=5)
    ap.add_argument("--cpu-c0-steps", type=int, default=50)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dry-run", action="store_true",
                    help="control plane only (ranks, shards, timing reduction) on CPU/gloo; no engine")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo")  # host-side control plane only; gradients go over RCCL

    if args.workload == DRQ_WORKLOAD:
        if not args.dry_run:
            bench_drq(args, world, rank, local_rank, dist)
        if dist:
            dist.destroy_process_group()
        return

    from mtrl_amd.shard import allreduce_floats_per_step, shard_tasks

    T, W, clip, desc = WORKLOADS[args.workload]
    shards = [list(shard_tasks(T, world, r)) for r in range(world)]
    tb, tc = shards[rank]
    ar_bytes = 4 * allreduce_floats_per_step(39 + T, 4, W, 3, W, 3, 2) if world > 1 else 0
    base = {
        "metric": METRIC,
        "unit": "SAC gradient-steps/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": {"fp32": "fp32", "split3": "fp32 (3xbf16 split MFMA, fp32-accurate)",
                  "split2h": "fp32 (2xfp16 split, per-tensor power-of-two scaled, 3 fp16 MFMA products, fp32-accurate)",
                  "bf16": "bf16 trunk GEMMs (fp32 accumulate, fp32 master weights / Adam / heads)"}[args.precision],
        "data": "synthetic (SURVEY.md §8d recipe, device-filled full buffer, cap=100000/task; random-init weights)",
        "config": {"workload": desc, "num_tasks": T, "width": W, "batch_per_task": 128, "global_batch": 128 * T,
                   "parallelism": f"task-shard{world}" if world > 1 else "single", "precision": args.precision,
                   "task_shards": shards, "allreduce_bytes_per_step": ar_bytes},
        "build": build_stamps(),
    }
    if args.dry_run:
        import torch

        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        if dist:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if rank == 0:
            print(json.dumps(dict(base, value=None, dry_run=True, nranks=world, max_over_ranks=float(t.item()))),
                  flush=True)
        if dist:
            dist.destroy_process_group()
        return

    from mtrl_amd import _lib as L
    from mtrl_amd.engine import MTSACEngine, make_config
    from mtrl_amd.init import init_mtsac

    cfg = make_config(num_tasks=T, task_begin=tb, task_count=tc, obs_dim=39 + T, actor_width=W, critic_width=W,
                      batch_per_task=128, capacity=100_000, clip=int(clip), precision=PRECISIONS[args.precision])
    eng = MTSACEngine(cfg, device=local_rank)
    actor, critic = init_mtsac(T, 39 + T, 4, W, 3, W, 3, 2, seed=1, task_begin=tb, task_count=tc)
    eng.set_params(L.ACTOR, actor)
    eng.set_params(L.CRITIC, critic)
    eng.set_params(L.CRITIC_TARGET, critic)
    eng.buffer_fill_synthetic(1234)
    eng.seed_rng(1)  # every rank draws the same index vector (buffers.py:523-527)
    nranks = 1
    if world > 1:
        uid = [MTSACEngine.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        eng.comm_init(uid[0], world, rank, timeout_s=600.0)  # a rank that never joins ends the run
        nranks = eng.comm_nranks()

    import torch

    mode = "eager" if args.no_graph else args.exec
    if mode == "auto" and world > 1:
        # task shards run eager (profiles/r2c_shard_steps.txt: 25 / 13 / 7 tasks 4.83 / 3.21 / 2.38 ms
        # eager vs 4.88 / 3.38 / 2.60 graph), where the per-layer all-reduce buckets on the collective
        # stream overlap the rest of the backward, and pipelined: the actor's all-reduce and Adam overlap
        # the next step's gather and critic forward; no RCCL collective is captured in a graph
        mode = "pipelined"

    def set_mode(m):
        eng.enable_graph(m == "graph")
        eng.lib.mtsac_debug_set_pipeline(eng._h, 1 if m == "pipelined" else 0)

    set_mode(mode if mode != "auto" else "eager")
    eng.update_many(args.warmup)
    eng.synchronize()
    if mode == "auto":  # pick the fastest execution mode on rank 0, same choice everywhere
        trial = {}
        for m in ("graph", "eager", "pipelined"):
            set_mode(m)
            eng.update_many(1)
            eng.synchronize()
            if dist:
                dist.barrier()
            a = time.perf_counter()
            eng.update_many(3)
            eng.synchronize()
            trial[m] = time.perf_counter() - a
        choice = [min(trial, key=trial.get)]
        if dist:
            dist.broadcast_object_list(choice, src=0)
        mode = choice[0]
        set_mode(mode)
        eng.update_many(1)
        eng.synchronize()
    # steady state: run untimed for --settle-s seconds (the same count on every rank)
    settle = 0
    if args.settle_s > 0:
        a = time.perf_counter()
        eng.update_many(5)
        eng.synchronize()
        per = max((time.perf_counter() - a) / 5, 1e-4)
        settle = [int(args.settle_s / per)]
        if dist:
            dist.broadcast_object_list(settle, src=0)
        settle = settle[0]
        eng.update_many(settle)
        eng.synchronize()
    # The timed steps run uninstrumented: an event pair around every GEMM launch costs a few us of
    # stream time per record, 0.2 ms per step at MT10/W400 (787 vs 587 us per step).  Eager: the
    # kernel timing comes from HIP events around every GEMM launch on the stream it runs on, over a
    # second pass of the same number of steps right after; a graph replay cannot carry events, so
    # then it comes from one extra serialised step.
    live = mode != "graph"
    eng.set_timing(False)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(local_rank)
    t0 = time.perf_counter()
    eng.update_many(args.steps)
    eng.synchronize()
    torch.cuda.synchronize(local_rank)
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = t1 - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    logs = eng.logs()
    assert all(math.isfinite(v) for v in logs.values()), logs
    events_ms = None
    if live:  # the events pass: the same steps again, every GEMM launch bracketed by HIP events
        eng.set_timing(True)
        a = time.perf_counter()
        eng.update_many(args.steps)
        eng.synchronize()
        events_ms = 1e3 * (time.perf_counter() - a) / args.steps
        eng.set_timing(False)

    # dominant-kernel roofline from the per-launch HIP events
    names = dict(GEMM_FAMILIES["split3" if args.precision == "bf16" else args.precision])
    fam = {f: eng.timing(f) for f in names} if live else None
    # the same kernels solo: one extra step serialised on one stream.  Eager: context for the
    # fraction (under the step's concurrency a launch shares the CUs with its neighbours).
    # Graph: the replays carry no events, so this IS the measurement (rocprof's mean over the
    # replays agrees within a few %).
    eng.set_timing(True, serial=True)
    eng.update_many(1)
    eng.synchronize()
    solo = {f: eng.timing(f) for f in names}
    eng.set_timing(False)
    for f in names:  # the kernel the engine actually launched for each family
        k = eng.timing_kernel(f)
        if k and k != "gemm_x3p_kernel":
            names[f] = k + " (" + names[f].split(" (", 1)[1]
    if fam is None:
        fam = solo
    timed_steps = args.steps if live else 1
    dom = max(fam, key=lambda f: fam[f][0])
    ms, nl, fl = fam[dom]
    gemm_ms = sum(v[0] for v in fam.values()) / timed_steps
    gemm_fl = sum(v[2] for v in fam.values()) / timed_steps
    achieved = (fl / nl) / (ms / nl * 1e-3) / 1e12 if nl else 0.0
    traffic, traffic_src = pmc_traffic(args.precision, dom, args.workload)
    if args.precision == "split3":  # 6 bf16 MFMA products per fp32 multiply-add
        peak, basis = BF16_MFMA_PEAK_TF / 6.0, "bf16 dense MFMA peak / 6 products (fp32-accurate split)"
    elif args.precision == "split2h":  # 3 fp16 MFMA products (fp16 runs at the bf16 rate)
        peak, basis = BF16_MFMA_PEAK_TF / 3.0, "fp16 dense MFMA peak / 3 products (fp32-accurate 2xfp16 split)"
    elif args.precision == "bf16":
        peak, basis = BF16_MFMA_PEAK_TF, "bf16 dense MFMA peak"
    else:
        peak, basis = FP32_MFMA_PEAK_TF, "f32-input MFMA dense peak"

    flops = algorithmic_flops(T, W)
    sps = args.steps / elapsed
    out = dict(base)
    out.update({
        "value": sps,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "settle_steps": settle,
        "nranks": nranks,
        "roofline": {"bound": "mfma", "kernel": names[dom], "achieved": achieved,
                     "peak": peak, "peak_basis": basis, "unit": "TFLOP/s", "frac": achieved / peak,
                     "traffic": traffic, "traffic_unit": "HBM bytes per launch (rocprofv3 PMC, gfx950-corrected)",
                     "traffic_source": traffic_src, "launches": nl, "avg_launch_us": 1e3 * ms / max(nl, 1),
                     "algorithmic_flops_per_launch": fl / max(nl, 1),
                     "timing": "HIP events per launch over a second pass of the timed eager steps (the "
                               "timed pass runs without events)" if live
                     else "graph replays carry no events: HIP events per launch in one serialised step",
                     "events_pass_ms_per_step": events_ms,
                     "clock": pmc_clock(args.precision, dom, args.workload),
                     "solo": {"achieved": (solo[dom][2] / max(solo[dom][1], 1)) / (solo[dom][0] / max(solo[dom][1], 1) * 1e-3) / 1e12
                              if solo[dom][0] else None,
                              "avg_launch_us": 1e3 * solo[dom][0] / max(solo[dom][1], 1),
                              "frac": ((solo[dom][2] / (solo[dom][0] * 1e-3) / 1e12) / peak) if solo[dom][0] else None,
                              "timing": "one extra step with every kernel serialised on one stream"}},
        "step_flops": flops,
        "step_tflops_per_s": flops * sps / world / 1e12,
        "gemm_kernel_ms_per_step": gemm_ms,  # sum of GEMM launch durations (they overlap across streams)
        "gemm_tflops_per_s": gemm_fl / (gemm_ms * 1e-3) / 1e12 if gemm_ms else 0.0,
        "gemm_families": {names[f]: {"ms_per_step": v[0] / timed_steps, "launches_per_step": v[1] / timed_steps,
                                     "avg_launch_us": 1e3 * v[0] / max(v[1], 1),
                                     "tflops": v[2] / (v[0] * 1e-3) / 1e12 if v[0] else 0.0}
                          for f, v in fam.items()},
        "logs": logs,
    })
    out["config"] = dict(out["config"], exec=mode)
    eng.close()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(T, W, clip, args.cpu_steps, args.cpu_c0_steps)
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
