"""Race hunt: churn device memory with big S3 / 7-task-shard engines (as the GPU suite does before
the W400 case), then repeat whole-step W400 runs (one update_many(1) per step, logs per step) and
pipelined runs, reporting the first step at which a run leaves the first whole-step run."""
import sys
import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from mtrl_amd import _lib as L  # noqa: E402
from mtrl_amd.engine import MTSACEngine, make_config  # noqa: E402
from mtrl_amd.init import init_mtsac  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6


def make(T, tc, W, prec=1):
    e = MTSACEngine(make_config(num_tasks=T, task_begin=0, task_count=tc, obs_dim=39 + T, actor_width=W,
                                critic_width=W, batch_per_task=128, capacity=512, precision=prec))
    a, c = init_mtsac(T, 39 + T, 4, W, 3, W, 3, 2, seed=4, task_begin=0, task_count=tc)
    e.set_params(L.ACTOR, a)
    e.set_params(L.CRITIC, c)
    e.set_params(L.CRITIC_TARGET, c)
    e.buffer_fill_synthetic(77)
    e.seed_rng(5)
    e.enable_graph(False)
    return e


for T, tc, W in ((50, 50, 2048), (50, 7, 2048)):  # what the suite runs just before
    for pipe in (0, 1):
        e = make(T, tc, W)
        e.lib.mtsac_debug_set_pipeline(e._h, pipe)
        e.update_many(4)
        e.logs()
        e.close()


def whole():
    e = make(10, 10, 400)
    e.lib.mtsac_debug_set_pipeline(e._h, 0)
    out = []
    for s in range(4):
        e.update_many(1)
        out.append(e.logs())
    p = [e.get_params(w) for w in (L.ACTOR, L.CRITIC)]
    e.close()
    return out, p


def piped():
    e = make(10, 10, 400)
    e.lib.mtsac_debug_set_pipeline(e._h, 1)
    e.update_many(4)
    out = e.logs()
    p = [e.get_params(w) for w in (L.ACTOR, L.CRITIC)]
    e.close()
    return out, p


ref, refp = whole()
for r in range(reps):
    for kind in ("whole", "piped"):
        if kind == "whole":
            lg, p = whole()
            bad = [(s, [k for k in lg[s] if lg[s][k] != ref[s][k]]) for s in range(4)]
            bad = [(s, k) for s, k in bad if k]
        else:
            lg, p = piped()
            k = [k for k in lg if lg[k] != ref[3][k]]
            bad = [(3, k)] if k else []
        pd = [i for i in range(2) if not np.array_equal(p[i], refp[i])]
        print(f"rep {r} {kind}: {'OK' if not bad and not pd else f'DIFF steps/keys {bad} params {pd}'}", flush=True)
print("done", flush=True)
