import sys, faulthandler
faulthandler.enable()
sys.path[:0] = ['.', 'tests']
import numpy as np
from mtrl_amd.engine import MTSACEngine, make_config
from mtrl_amd.init import init_mtsac
from mtrl_amd import _lib as L
mode = sys.argv[1]
T, W, n = 3, 32, 4
c = make_config(num_tasks=T, task_count=T, obs_dim=39 + T, actor_width=W, critic_width=W, batch_per_task=n, capacity=64)
e = MTSACEngine(c)
a, q = init_mtsac(T, 39 + T, 4, W, 3, W, 3, 2)
e.set_params(L.ACTOR, a); e.set_params(L.CRITIC, q); e.set_params(L.CRITIC_TARGET, q)
e.buffer_fill_synthetic(1); e.seed_rng(1)
e.enable_graph(mode == 'graph')
print('start', mode, flush=True)
e.update_many(1); print('1 ok', flush=True)
e.update_many(3); print('3 ok', e.logs(), flush=True)
