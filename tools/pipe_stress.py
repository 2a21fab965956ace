"""Repeat 4 device-sampled steps at one config in whole-step and pipelined issue and compare every
run's logs / parameters with the first whole-step run (race hunting)."""
import sys
import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from mtrl_amd import _lib as L  # noqa: E402
from mtrl_amd.engine import MTSACEngine, make_config  # noqa: E402
from mtrl_amd.init import init_mtsac  # noqa: E402

T, tc, W, prec, reps = (int(a) for a in sys.argv[1:6])
steps = int(sys.argv[6]) if len(sys.argv) > 6 else 4
a0, c0 = init_mtsac(T, 39 + T, 4, W, 3, W, 3, 2, seed=4, task_begin=0, task_count=tc)


def run(pipe):
    e = MTSACEngine(make_config(num_tasks=T, task_begin=0, task_count=tc, obs_dim=39 + T, actor_width=W,
                                critic_width=W, batch_per_task=128, capacity=512, precision=prec))
    e.set_params(L.ACTOR, a0)
    e.set_params(L.CRITIC, c0)
    e.set_params(L.CRITIC_TARGET, c0)
    e.buffer_fill_synthetic(77)
    e.seed_rng(5)
    e.enable_graph(False)
    e.lib.mtsac_debug_set_pipeline(e._h, pipe)
    e.update_many(steps)
    out = (e.logs(), [e.get_params(w) for w in (L.ACTOR, L.CRITIC, L.ACTOR_ADAM_NU, L.CRITIC_ADAM_MU)])
    e.close()
    return out


ref = run(0)
bad = 0
for r in range(reps):
    for pipe in (0, 1):
        lg, ps = run(pipe)
        diff = [k for k in lg if lg[k] != ref[0][k]]
        pd = [i for i, (x, y) in enumerate(zip(ps, ref[1])) if not np.array_equal(x, y)]
        if diff or pd:
            bad += 1
            print(f"rep {r} pipe {pipe}: logs differ {diff} params differ {pd}", flush=True)
print(f"T={T} tc={tc} W={W} prec={prec}: {bad} of {2 * reps} runs differ from the first whole-step run", flush=True)
