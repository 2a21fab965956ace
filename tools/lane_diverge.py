"""Localise the 5-lane reproducibility failure ("Lanes and hardware queues").

Each fresh child process (GPU_MAX_HW_QUEUES=16, MTSAC_LANES=1) runs three engines from the same
start state on the same device-sampled stream:
  A: 5 lanes, whole steps (update_many(1) per step)
  B: one stream (mtsac_debug_force_one_stream), whole steps -- the reference issue
  C: 5 lanes, pipelined (update_many(4))
and compares A and C against B bitwise after every step (every 4 steps for C): logs, parameters,
Adam moments.  The first mismatch is printed with the leaves that differ (nu = the squared-gradient
moment names the gradient leaf that went wrong first).  usage: lane_diverge.py CHILDREN STEPS [ENV=VAL ...]
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import sys
sys.path.insert(0, {root!r})
import numpy as np
from mtrl_amd import _lib as L
from mtrl_amd.engine import MTSACEngine, make_config
from mtrl_amd.init import init_mtsac
T, tc, W, prec, STEPS = 10, 10, 400, 1, {steps}
a0, c0 = init_mtsac(T, 39 + T, 4, W, 3, W, 3, 2, seed=4, task_begin=0, task_count=tc)
def mk(one, pipe):
    e = MTSACEngine(make_config(num_tasks=T, task_begin=0, task_count=tc, obs_dim=39 + T, actor_width=W,
                                critic_width=W, batch_per_task=128, capacity=512, precision=prec))
    if one:
        e.lib.mtsac_debug_force_one_stream(e._h, 1)
    e.set_params(L.ACTOR, a0); e.set_params(L.CRITIC, c0); e.set_params(L.CRITIC_TARGET, c0)
    e.buffer_fill_synthetic(77); e.seed_rng(5); e.enable_graph(False)
    e.lib.mtsac_debug_set_pipeline(e._h, pipe)
    return e
B = mk(True, 0)
A = mk(False, 0)
C = mk(False, 1)
print("lane modes A/B/C", [e.lib.mtsac_debug_lane_mode(e._h) for e in (A, B, C)], flush=True)
WH = [L.ACTOR, L.CRITIC, L.CRITIC_TARGET, L.LOG_ALPHA, L.ACTOR_ADAM_MU, L.ACTOR_ADAM_NU, L.CRITIC_ADAM_MU,
      L.CRITIC_ADAM_NU]
NAMES = ["actor", "critic", "critic_target", "log_alpha", "actor_mu", "actor_nu", "critic_mu", "critic_nu"]
def leaves(which, n):
    # flax leaf order: head bias, head kernel, then (bias, kernel) per layer; critic leaves x2
    hd, E, I = (8, 1, 39 + T) if which in (L.ACTOR, L.ACTOR_ADAM_MU, L.ACTOR_ADAM_NU) else (1, 2, 43 + T)
    sizes = [T * hd * E, T * W * hd * E]
    fan = I
    for i in range(3):
        sizes += [W * E, fan * W * E]
        fan = W
    names = ["head_b", "head_W"] + [f"{{k}}{{i}}" for i in range(3) for k in ("b", "W")]
    out, o = [], 0
    for nm, s in zip(names, sizes):
        out.append((nm, o, o + s)); o += s
    assert o == n, (o, n)
    return out
def snap(e):
    return e.logs(), [e.get_params(w) for w in WH], e.get_rng_state()
def diff(tag, step, x, y):
    bad = []
    if x[0] != y[0]:
        bad.append("logs " + str({{k: (x[0][k], y[0][k]) for k in x[0] if x[0][k] != y[0][k]}}))
    for nm, w, p, q in zip(NAMES, WH, x[1], y[1]):
        if not np.array_equal(p, q):
            if w == L.LOG_ALPHA:
                bad.append(f"{{nm}}: {{int((p != q).sum())}} differ")
                continue
            for lf, b, e in leaves(w, p.size):
                d = p[b:e] != q[b:e]
                if d.any():
                    rel = np.abs(p[b:e] - q[b:e]).max() / max(np.abs(q[b:e]).max(), 1e-30)
                    bad.append(f"{{nm}}.{{lf}}: {{int(d.sum())}}/{{e - b}} differ, max rel {{rel:.2e}}")
    if x[2] != y[2]:
        bad.append("rng state")
    if bad:
        print(f"MISMATCH {{tag}} after step {{step}}:", flush=True)
        for s in bad:
            print("   ", s, flush=True)
        return True
    return False
first = {{}}
for s in range(1, STEPS + 1):
    B.update_many(1); A.update_many(1)
    sb = snap(B)
    if "A" not in first and diff("A(lanes, whole)", s, snap(A), sb):
        first["A"] = s
    if s % 4 == 0:
        C.update_many(4)
        if "C" not in first and diff("C(lanes, pipelined)", s, snap(C), sb):
            first["C"] = s
print("first mismatch", first, flush=True)
"""
K, STEPS = int(sys.argv[1]), int(sys.argv[2])
extra = dict(kv.split("=", 1) for kv in sys.argv[3:])
env = dict(os.environ, GPU_MAX_HW_QUEUES="16", MTSAC_LANES="1", **extra)
for k in range(K):
    r = subprocess.run([sys.executable, "-u", "-c", CHILD.format(root=ROOT, steps=STEPS)], capture_output=True,
                       text=True, timeout=300, env=env)
    print(f"== child {k} {extra} rc={r.returncode}", flush=True)
    print(r.stdout[-6000:], flush=True)
    if r.returncode != 0:
        print(r.stderr[-3000:], flush=True)
        break
