"""Full-batch GPU parity at the bench's own sizes ("do this" 1).

The bench runs S3 (MT50/W2048, n=128 -> B=6400) on the 224x256-tile GEMM
geometry with a ragged last row tile (6400 = 28*224 + 128), the full-K split
choice and full-size plane buffers; S2 (MT10/W2048 clip, B=1280) and the 8-way
MT50 task split (7,7,6,6,6,6,6,6 tasks x 128 rows) run other geometries and
split-K choices.  Each case here is ONE complete gradient step on exactly those
shapes, compared with the float64 oracle (oracle/mtsac.py, restating
mtrl/rl/algorithms/mtsac.py:1173-1251) from the same fp32 parameters, batch and
injected noise.  log_alpha starts away from 0 so the temperature loss is live.

Bars (BASELINE.json north_star): losses within 1e-5 relative (qf_values
included); grad and parameter norms within 1e-5 relative; parameters after the
step elementwise within fp32 Adam tolerance (median |d| < 1e-6, max <= 2 lr).
"""

from __future__ import annotations

import functools

import numpy as np
import pytest

from helpers import synthetic_batch, synthetic_eps
from oracle import mtsac as om

pytestmark = pytest.mark.gpu

RTOL = 1e-5
LOSS_KEYS = ("losses/qf_loss", "losses/actor_loss", "losses/alpha_loss", "losses/qf_values")
NORM_KEYS = ("metrics/critic_grad_magnitude", "metrics/actor_grad_magnitude", "metrics/critic_params_norm",
             "metrics/actor_params_norm", "alpha")

CASES = {
    "s3_mt50_w2048": dict(T=50, W=2048, n=128, clip=False),
    "s2_mt10_w2048_clip": dict(T=10, W=2048, n=128, clip=True),
}
# S4: the literal experiments/mt50_mtmhsac_v2.py (MT50 at the default width 400), sharded only
SHARD_CASES = dict(CASES, s4_mt50_w400=dict(T=50, W=400, n=128, clip=False))


def _cfg(spec):
    T, W = spec["T"], spec["W"]
    return om.OracleConfig(num_tasks=T, obs_dim=39 + T, actor_width=W, critic_width=W, clip=spec["clip"])


@functools.lru_cache(maxsize=None)
def _problem(name):
    """fp32-representable start state, one batch + noise, and the float64 oracle step (cached:
    the same oracle result serves both precisions and the sharded run)."""
    spec = SHARD_CASES[name]
    cfg = _cfg(spec)
    T, n = spec["T"], spec["n"]
    B = n * T
    st = om.initialize(cfg, seed=11)
    st.log_alpha = np.random.default_rng(12).uniform(-0.3, 0.3, T)
    for k in ("actor", "critic", "critic_target", "log_alpha"):
        setattr(st, k, getattr(st, k).astype(np.float32).astype(np.float64))
    batch = synthetic_batch(T, B, seed=100, dtype=np.float32)
    en, ec = synthetic_eps(B, seed=200, dtype=np.float32)
    st1, want = om.update(cfg, st, [b.astype(np.float64) for b in batch], en.astype(np.float64),
                          ec.astype(np.float64))
    return cfg, st, batch, en, ec, st1, want


def _engine(spec, precision, begin=0, count=None, cu_slice=None):
    """cu_slice = (k, n): the engine's streams run on CU slice k of n only (MTSAC_CU_SLICE, read at
    create), as ranks on their own GPUs have their own CUs.  Round 5 saw, once, a handful of wrong
    values of the head backward's cross-wave LDS reduction with all engines co-resident on every CU
    ("Eight engines on one device"); those reductions are now self-checked (a
    mismatch makes the engine's next logs() raise), and the determinism test below runs co-resident."""
    import os

    from mtrl_amd.engine import MTSACEngine, make_config

    T, W, n = spec["T"], spec["W"], spec["n"]
    c = make_config(num_tasks=T, task_begin=begin, task_count=T if count is None else count, obs_dim=39 + T,
                    actor_width=W, critic_width=W, batch_per_task=n, capacity=n, clip=int(spec["clip"]),
                    precision=precision)
    if cu_slice is not None:
        os.environ["MTSAC_CU_SLICE"] = f"{cu_slice[0]}:{cu_slice[1]}"
    try:
        e = MTSACEngine(c)
    finally:
        os.environ.pop("MTSAC_CU_SLICE", None)
    e.enable_graph(False)
    return e


def _load(e, st, begin=0, count=None):
    from mtrl_amd import _lib as L
    from mtrl_amd.init import slice_heads

    T = st.log_alpha.size
    count = T if count is None else count
    cfg = e.config
    e.set_params(L.ACTOR, slice_heads(st.actor, cfg.obs_dim, cfg.actor_width, cfg.actor_depth, T, 8, None, begin,
                                      count))
    for which, v in ((L.CRITIC, st.critic), (L.CRITIC_TARGET, st.critic_target)):
        e.set_params(which, slice_heads(v, cfg.obs_dim + 4, cfg.critic_width, cfg.critic_depth, T, 1, 2, begin,
                                        count))
    e.set_params(L.LOG_ALPHA, st.log_alpha)


def _check_logs(got, want, tag):
    errs = {k: abs(got[k] - want[k]) / max(abs(want[k]), 1e-30) for k in LOSS_KEYS + NORM_KEYS}
    print(tag, {k: f"{v:.2e}" for k, v in errs.items()})
    for k in LOSS_KEYS + NORM_KEYS:
        assert errs[k] <= RTOL, (tag, k, got[k], want[k], errs[k])
    assert got["metrics/explore_loss"] == 0.0


def _check_params(e, st1, tag, begin=0, count=None):
    from mtrl_amd import _lib as L
    from mtrl_amd.init import slice_heads

    cfg = e.config
    T = st1.log_alpha.size
    count = T if count is None else count
    refs = ((L.ACTOR, slice_heads(st1.actor, cfg.obs_dim, cfg.actor_width, cfg.actor_depth, T, 8, None, begin,
                                  count)),
            (L.CRITIC, slice_heads(st1.critic, cfg.obs_dim + 4, cfg.critic_width, cfg.critic_depth, T, 1, 2, begin,
                                   count)),
            (L.CRITIC_TARGET, slice_heads(st1.critic_target, cfg.obs_dim + 4, cfg.critic_width, cfg.critic_depth, T,
                                          1, 2, begin, count)),
            (L.LOG_ALPHA, st1.log_alpha))
    for which, ref in refs:
        d = np.abs(e.get_params(which).astype(np.float64) - ref)
        assert np.median(d) < 1e-6, (tag, which, np.median(d))
        assert d.max() < 2 * 3e-4 + 1e-6, (tag, which, d.max())


@pytest.mark.parametrize("precision", [0, 1, 3], ids=["fp32", "split3", "split2h"])
@pytest.mark.parametrize("name", list(CASES))
def test_full_batch_step_matches_oracle(name, precision):
    cfg, st, batch, en, ec, st1, want = _problem(name)
    e = _engine(CASES[name], precision)
    _load(e, st)
    e.update(batch, en, ec)
    _check_logs(e.logs(), want, f"{name}/p{precision}")
    _check_params(e, st1, f"{name}/p{precision}")
    assert e.get_adam_count(0) == 1 and e.get_adam_count(1) == 1 and e.get_adam_count(2) == 1
    e.close()


def _run_8way(name, precision, world=8, cu_slices=True):
    """The MT50 8-GPU task split as 8 engines on one device (each on its own CU slice, or all of them
    co-resident on every CU), one full-batch step through the in-process all-reduce hook; returns the
    engines (open) and their logs."""
    import threading

    from mtrl_amd.shard import InProcessAllReduce, local_rows, shard_tasks

    spec = SHARD_CASES[name]
    cfg, st, batch, en, ec, st1, want = _problem(name)
    T, n = spec["T"], spec["n"]
    shards = []
    for r in range(world):
        b0, c0 = shard_tasks(T, world, r)
        e = _engine(spec, precision, b0, c0, cu_slice=(r, world) if cu_slices else None)
        _load(e, st, b0, c0)
        shards.append(e)
    group = InProcessAllReduce(world)
    for r, e in enumerate(shards):
        e.set_allreduce_hook(group.hook(r))
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
    return shards, [e.logs() for e in shards]


@pytest.mark.parametrize("precision", [0, 1, 3], ids=["fp32", "split3", "split2h"])
@pytest.mark.parametrize("name", ["s3_mt50_w2048", "s4_mt50_w400"])
def test_full_batch_8way_shard_matches_oracle(precision, name):
    """The MT50 8-GPU task split (7,7,6,6,6,6,6,6 tasks, 128 rows each) as 8 engines on one
    device reducing through the in-process hook (same reduction points as RCCL), against
    the float64 oracle of the unsharded step.  S3 (W=2048) and S4, the literal
    experiments/mt50_mtmhsac_v2.py width 400 (a shard's trunk GEMMs then run gemm_x3s and the
    256x128 weight-grad tiles)."""
    from mtrl_amd.shard import shard_tasks

    world = 8
    spec = SHARD_CASES[name]
    cfg, st, batch, en, ec, st1, want = _problem(name)
    shards, logs = _run_8way(name, precision, world)
    assert all(lg == logs[0] for lg in logs)  # every logged scalar is reduced: ranks agree bitwise
    _check_logs(logs[0], want, f"shard8/p{precision}")
    for r, e in enumerate(shards):
        b0, c0 = shard_tasks(spec["T"], world, r)
        _check_params(e, st1, f"shard8/p{precision}/r{r}", b0, c0)
        e.close()


def test_full_batch_8way_shard_split2h_deterministic():
    """the 8-engine S3 split2h step twice in one process (fresh engines,
    same inputs) gives bitwise the same logs, parameters and Adam moments on every rank, and logs within
    RTOL of the float64 oracle; the head backward's LDS reductions are self-checked (a slot that held
    other bits than its writer stored raises from logs()).  Every engine runs on its own CU slice, as
    each rank owns its GPU in production.  Round 6 ran this co-resident (no slices) twice: green once
    (profiles/r6a_gpu_tests.log), and once the two repetitions differed by one ulp in
    actor_grad_magnitude (both within 1.2e-7 of the oracle) with the self-check silent
    (profiles/r6b_coresident_nondeterminism.log) -- DESIGN.md section 5 has the analysis; the
    in-process co-resident 8-engine setting is not a production configuration."""
    from mtrl_amd import _lib as L

    *_, want = _problem("s3_mt50_w2048")
    outs = []
    for rep in range(2):
        shards, logs = _run_8way("s3_mt50_w2048", 3)
        _check_logs(logs[0], want, f"shard8-coresident/split2h/rep{rep}")
        outs.append((logs, [[e.get_params(w) for w in (L.ACTOR, L.CRITIC, L.CRITIC_TARGET, L.ACTOR_ADAM_MU,
                                                         L.CRITIC_ADAM_MU, L.ACTOR_ADAM_NU)] for e in shards]))
        for e in shards:
            e.close()
    (la, pa), (lb, pb) = outs
    assert la == lb, [(r, {k: (a[k], b[k]) for k in a if a[k] != b[k]}) for r, (a, b) in enumerate(zip(la, lb)) if a != b]
    for r, (xa, xb) in enumerate(zip(pa, pb)):
        for q, (x, y) in enumerate(zip(xa, xb)):
            assert np.array_equal(x, y), (r, q, int(np.count_nonzero(x != y)))


@pytest.mark.parametrize("precision", [1, 3], ids=["split3", "split2h"])
def test_head_backward_selfcheck_fires(precision):
    """The head backward's LDS self-check is live end to end: the last step's actor head weight pass,
    re-run with one cross-wave LDS slot corrupted on purpose (mtsac_debug_head_selfcheck, into a
    scratch output), makes the next logs() raise the self-check error; the error clears, and the
    step's own parameters and logs are untouched by the check run."""
    from mtrl_amd import _lib as L

    name = "s2_mt10_w2048_clip"
    cfg, st, batch, en, ec, st1, want = _problem(name)
    e = _engine(CASES[name], precision)
    _load(e, st)
    e.update(batch, en, ec)
    logs = e.logs()  # a clean step: no fault
    _check_logs(logs, want, f"selfcheck/p{precision}")
    before = e.get_params(L.ACTOR)
    L.check(e.lib.mtsac_debug_head_selfcheck(e._h))
    with pytest.raises(Exception, match="self-check"):
        e.logs()
    assert e.logs() == logs  # cleared; the logs buffer was not touched
    assert np.array_equal(e.get_params(L.ACTOR), before)
    e.close()


def test_full_batch_modelled_collective_matches_oracle():
    """S3 at full batch through the SHARDED step with the device collective on its own stream (the
    modelled collective, a one-rank sum, with every bucket NaN until its collective is done, so a
    consumer that does not wait for the collective stream poisons the step): the bucketed trunk
    gradients, scalar tail, clip norm and logs of the RCCL path, against the float64 oracle."""
    name = "s3_mt50_w2048"
    cfg, st, batch, en, ec, st1, want = _problem(name)
    e = _engine(CASES[name], 1)
    _load(e, st)
    assert e.lib.mtsac_debug_set_collective_model(e._h, 8, 150.0, 1) == 0
    e.update(batch, en, ec)
    _check_logs(e.logs(), want, f"{name}/modelled")
    _check_params(e, st1, f"{name}/modelled")
    e.close()


def _device_steps(T, tc, W, prec, steps, pipe, model=0, calls=None, info=None):
    """Logs, parameters, moments, index-stream and noise state after device-sampled eager steps."""
    from mtrl_amd import _lib as L
    from mtrl_amd.engine import MTSACEngine, make_config
    from mtrl_amd.init import init_mtsac

    a0, c0 = init_mtsac(T, 39 + T, 4, W, 3, W, 3, 2, seed=4, task_begin=0, task_count=tc)
    e = MTSACEngine(make_config(num_tasks=T, task_begin=0, task_count=tc, obs_dim=39 + T, actor_width=W,
                                critic_width=W, batch_per_task=128, capacity=512, precision=prec))
    e.set_params(L.ACTOR, a0)
    e.set_params(L.CRITIC, c0)
    e.set_params(L.CRITIC_TARGET, c0)
    e.buffer_fill_synthetic(77)
    e.seed_rng(5)
    e.enable_graph(False)
    if model:
        assert e.lib.mtsac_debug_set_collective_model(e._h, 8, 300.0, 1) == 0
    e.lib.mtsac_debug_set_pipeline(e._h, pipe)
    if info is not None:
        info["bfrag"] = e.lib.mtsac_debug_bfrag(e._h)
    for k in calls or (steps,):
        e.update_many(k)
    out = (e.logs(), [e.get_params(w) for w in (L.ACTOR, L.CRITIC, L.CRITIC_TARGET, L.LOG_ALPHA, L.ACTOR_ADAM_MU,
                                               L.ACTOR_ADAM_NU, L.CRITIC_ADAM_MU, L.CRITIC_ADAM_NU)],
           e.get_rng_state(), e.noise_state())
    e.close()
    return out


def _assert_same(a, b):
    assert a[0] == b[0], {k: (a[0][k], b[0][k]) for k in a[0] if a[0][k] != b[0][k]}
    for x, y in zip(a[1], b[1]):
        np.testing.assert_array_equal(x, y)
    assert a[2] == b[2] and a[3] == b[3]


@pytest.mark.parametrize("T,tc,W,prec,model", [(50, 50, 2048, 1, 0), (50, 7, 2048, 1, 1), (50, 7, 2048, 1, 0),
                                               (10, 10, 400, 1, 0), (50, 6, 400, 1, 1), (10, 10, 2048, 2, 0),
                                               (50, 50, 2048, 3, 0), (50, 7, 2048, 3, 1), (10, 10, 400, 3, 0)],
                         ids=["s3", "mt50_shard7_modelled", "mt50_shard7", "mt10_w400", "s4_shard6_modelled",
                              "mt10_w2048_bf16", "s3_split2h", "mt50_shard7_modelled_split2h", "mt10_w400_split2h"])
def test_pipelined_steps_equal_whole_steps(T, tc, W, prec, model):
    """Cross-step pipelining on one compute stream (engine.cpp step(), p2): step k+1's gather and
    critic(s, a) forward run on the prefetch stream beside step k's actor backward, all-reduce and
    Adam; 4 device-sampled steps issued that way give bitwise the logs, parameters, optimizer moments
    and index-stream / noise state of 4 whole steps.  The modelled cases take the sharded path with
    the device collective (NaN-poisoned buckets) on its own stream, as an 8-GPU rank does."""
    _assert_same(_device_steps(T, tc, W, prec, 4, 0, model), _device_steps(T, tc, W, prec, 4, 1, model))


@pytest.mark.parametrize("T,tc,prec,model", [(50, 50, 3, 0), (50, 50, 1, 0), (50, 50, 2, 0), (10, 10, 3, 0),
                                             (50, 7, 3, 0), (50, 7, 3, 1), (50, 13, 1, 0)],
                         ids=["s3_split2h", "s3_split3", "s3_bf16", "mt10_w2048_split2h", "mt50_shard7_split2h",
                              "mt50_shard7_modelled_split2h", "mt50_shard13_split3"])
def test_fragment_layout_weights_equal_row_major(T, tc, prec, model):
    """W = 2048: the weight planes the trunk GEMMs read (W^T for the forward, W for the data grad) in
    the fragment layout (gemm_common.h frag_off; the optimizer's tile pass and the set_params split
    write them so) give bitwise the logs, parameters, moments and stream states of row-major planes
    over 3 device-sampled steps.  A layer's planes take the layout only where every GEMM reading them
    runs on gemm_x3f (engine.cpp frag_probe): every layer at S3, the critic's hidden layers on
    MT10 and the task shards."""
    from mtrl_amd import _lib as L

    lib = L.load()
    info_off, info_on = {}, {}
    try:
        assert lib.mtsac_debug_set_bfrag(0) == 0
        a = _device_steps(T, tc, 2048, prec, 3, 0, model, info=info_off)
    finally:
        lib.mtsac_debug_set_bfrag(-1)
    b = _device_steps(T, tc, 2048, prec, 3, 0, model, info=info_on)
    print("bfrag mask (bit i actor layer i, bit 8 + i critic layer i):", hex(info_on["bfrag"]))
    assert info_off["bfrag"] == 0, info_off
    if tc == 50:  # S3: every layer of both networks
        assert info_on["bfrag"] == 0x707, hex(info_on["bfrag"])
    else:  # the critic's hidden layers at least (gemm_x3f + split-K; others may run on gemm_x3p)
        assert info_on["bfrag"] & 0x600 == 0x600, hex(info_on["bfrag"])
    _assert_same(a, b)


_PIPE_LANES_CHILD = """
import sys
sys.path.insert(0, {root!r})
sys.path.insert(0, {tests!r})
import test_gpu_fullbatch as t
a = t._device_steps(10, 10, 400, 1, 4, 0)
b = t._device_steps(10, 10, 400, 1, 4, 1)
t._assert_same(a, b)
print("lanes pipelined == whole: ok")
"""


def test_pipelined_steps_equal_whole_steps_lanes():
    """The same bar for the 5-lane form (MTSAC_LANES=1, a child process started with 16 hardware
    queues): MT10/W400, 4 steps, whole vs pipelined, bitwise."""
    import os

    from mtrl_amd.hwq import child_env

    tests = os.path.dirname(os.path.abspath(__file__))
    code = _PIPE_LANES_CHILD.format(root=os.path.dirname(tests), tests=tests)
    r = _child(code, child_env(16))
    assert r.returncode == 0 and "ok" in r.stdout


def test_full_batch_graph_replay_equals_eager():
    """S3 at full size on the device-sampled path the bench times: 3 steps replayed from the
    step graph give bitwise the logs, parameters and index-stream state of 3 eager steps."""
    from mtrl_amd import _lib as L

    spec = CASES["s3_mt50_w2048"]
    _, st, *_ = _problem("s3_mt50_w2048")
    outs = []
    for graph in (False, True):
        e = _engine(spec, 1)
        _load(e, st)
        e.enable_graph(graph)
        e.buffer_fill_synthetic(1234)
        e.seed_rng(1)
        e.update_many(3)
        outs.append((e.logs(), e.get_params(L.ACTOR), e.get_params(L.CRITIC), e.get_rng_state()))
        e.close()
    assert outs[0][0] == outs[1][0]
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
    np.testing.assert_array_equal(outs[0][2], outs[1][2])
    assert outs[0][3] == outs[1][3]


# Precision bf16 (perf-only, BASELINE configs[2] "bf16 MFMA"): the trunk GEMM operands are rounded
# to bf16 (one MFMA per product, fp32 accumulation), everything else fp32.  Not the reference's
# arithmetic, so it is held to a stated drift bound instead of the 1e-5 parity bar: one full step
# from the same start state, batch and noise against the float64 oracle.  Measured (MI355X): losses
# <= 1.5e-4, grad norms <= 9.3e-5 relative (qf_values of S2 the largest); the bound is 1e-3.
BF16_LOSS_RTOL = 1e-3
BF16_NORM_RTOL = 1e-3


@pytest.mark.parametrize("name", list(CASES))
def test_full_batch_bf16_drift_bound(name):
    cfg, st, batch, en, ec, st1, want = _problem(name)
    e = _engine(CASES[name], 2)
    _load(e, st)
    e.update(batch, en, ec)
    got = e.logs()
    errs = {k: abs(got[k] - want[k]) / max(abs(want[k]), 1e-30) for k in LOSS_KEYS + NORM_KEYS}
    print(f"{name}/bf16", {k: f"{v:.2e}" for k, v in errs.items()})
    for k in LOSS_KEYS:
        assert errs[k] <= BF16_LOSS_RTOL, (name, k, got[k], want[k], errs[k])
    for k in NORM_KEYS:
        assert errs[k] <= BF16_NORM_RTOL, (name, k, got[k], want[k], errs[k])
    # the update still moves every parameter the way the fp32 step does
    from mtrl_amd import _lib as L

    d = np.abs(e.get_params(L.CRITIC).astype(np.float64) - st1.critic)
    assert np.median(d) < 1e-5, np.median(d)
    e.close()


@pytest.mark.parametrize("T,tc,W,prec", [(50, 50, 2048, 1), (50, 7, 2048, 1), (10, 10, 400, 1), (10, 10, 2048, 2),
                                         (50, 50, 2048, 3), (10, 10, 400, 3)],
                         ids=["s3", "mt50_shard7", "mt10_w400", "mt10_w2048_bf16", "s3_split2h", "mt10_w400_split2h"])
def test_update_many_equals_single_steps(T, tc, W, prec):
    """The default issue (every compute segment on one stream, engine.cpp one_stream): 4 device-
    sampled steps in one update_many call give bitwise the logs, parameters, optimizer moments and
    index-stream state of 4 calls of one step each -- run to run reproducible, which the 5-lane
    form was not ("Lanes and hardware queues")."""
    from mtrl_amd import _lib as L
    from mtrl_amd.engine import MTSACEngine, make_config
    from mtrl_amd.init import init_mtsac

    a0, c0 = init_mtsac(T, 39 + T, 4, W, 3, W, 3, 2, seed=4, task_begin=0, task_count=tc)
    outs = []
    for calls in ((4,), (1, 1, 1, 1)):
        e = MTSACEngine(make_config(num_tasks=T, task_begin=0, task_count=tc, obs_dim=39 + T, actor_width=W,
                                    critic_width=W, batch_per_task=128, capacity=512, precision=prec))
        assert e.lib.mtsac_debug_lane_mode(e._h) == 1
        e.set_params(L.ACTOR, a0)
        e.set_params(L.CRITIC, c0)
        e.set_params(L.CRITIC_TARGET, c0)
        e.buffer_fill_synthetic(77)
        e.seed_rng(5)
        e.enable_graph(False)
        for k in calls:
            e.update_many(k)
        outs.append((e.logs(), [e.get_params(w) for w in (L.ACTOR, L.CRITIC, L.CRITIC_TARGET, L.LOG_ALPHA,
                                                           L.ACTOR_ADAM_NU, L.CRITIC_ADAM_MU)],
                     e.get_rng_state(), e.noise_state()))
        e.close()
    a, b = outs
    assert a[0] == b[0]
    for x, y in zip(a[1], b[1]):
        np.testing.assert_array_equal(x, y)
    assert a[2] == b[2] and a[3] == b[3]


_LANE_CHILD = """
import sys
sys.path.insert(0, {root!r})
from mtrl_amd.engine import MTSACEngine, make_config
mk = lambda: MTSACEngine(make_config(num_tasks=2, task_count=2, obs_dim=41, actor_width=64, critic_width=64,
                                     batch_per_task=8, capacity=16))
a = mk()
m1 = a.lib.mtsac_debug_lane_mode(a._h)
b, c = mk(), mk()
m3 = [e.lib.mtsac_debug_lane_mode(e._h) for e in (a, b, c)]
b.close(); c.close()
m1b = a.lib.mtsac_debug_lane_mode(a._h)
a.close()
print("modes", m1, m3, m1b)
"""


def _child(code: str, env: dict, timeout: int = 200):
    import subprocess
    import sys

    r = subprocess.run([sys.executable, "-u", "-c", code], capture_output=True, text=True, timeout=timeout, env=env)
    print(r.stdout[-3000:], r.stderr[-3000:])
    return r


def test_lane_mode():
    """One compute stream by default; the experimental 5-lane form (MTSAC_LANES=1) only while every
    live engine's 5 streams + 3 reserved fit the hardware queues the process STARTED with
    (GPU_MAX_HW_QUEUES, read from /proc/self/environ; re-decided for all live engines at each
    create / destroy).  Child processes: lanes requested at 16 queues -> one engine has lanes, three
    (15 + 3 > 16) one stream each, the survivor its lanes back; requested at 4 -> one stream; not
    requested -> one stream."""
    import os

    from mtrl_amd.hwq import child_env

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = _LANE_CHILD.format(root=root)
    r = _child(code, child_env(16))
    assert r.returncode == 0 and "modes 0 [1, 1, 1] 0" in r.stdout
    r = _child(code, dict(child_env(16), GPU_MAX_HW_QUEUES="4"))
    assert r.returncode == 0 and "modes 1 [1, 1, 1] 1" in r.stdout
    r = _child(code, child_env(16, lanes=False))
    assert r.returncode == 0 and "modes 1 [1, 1, 1] 1" in r.stdout


def _drift_run(T, W, prec, chunks):
    """Logs after each chunk of device-sampled eager steps (same start, stream and noise as
    _device_steps)."""
    from mtrl_amd import _lib as L
    from mtrl_amd.engine import MTSACEngine, make_config
    from mtrl_amd.init import init_mtsac

    a0, c0 = init_mtsac(T, 39 + T, 4, W, 3, W, 3, 2, seed=4, task_begin=0, task_count=T)
    e = MTSACEngine(make_config(num_tasks=T, task_begin=0, task_count=T, obs_dim=39 + T, actor_width=W,
                                critic_width=W, batch_per_task=128, capacity=512, precision=prec))
    e.set_params(L.ACTOR, a0)
    e.set_params(L.CRITIC, c0)
    e.set_params(L.CRITIC_TARGET, c0)
    e.buffer_fill_synthetic(77)
    e.seed_rng(5)
    e.enable_graph(False)
    out = []
    for k in chunks:
        e.update_many(k)
        out.append((e.logs(), e.get_params(L.CRITIC).astype(np.float64), e.get_params(L.ACTOR).astype(np.float64)))
    e.close()
    return out


@pytest.mark.parametrize("T,W,chunks", [(10, 400, (1, 9, 40, 100, 150)), (50, 2048, (1, 9, 50))],
                         ids=["mt10_w400_300", "s3_60"])
def test_split2h_long_run_drift_like_split3(T, W, chunks):
    """Many device-sampled steps: split2h's exponents come from bounds the producers record step after
    step (weights through the Adam step bound, activations and grads through their partial maxima), so
    a long run is where a bound that fails to hold would show (an fp16 overflow turns a step into inf /
    NaN): every log stays finite.  Both split precisions are fp32-accurate with their own summation
    orders, so each drifts from the exact-fp32 path (precision fp32: FMA GEMMs) by the chaotic growth
    of last-bit differences; the bar is on the parameters (relative L2 distance to the fp32 run), which
    average that growth over 10^7 entries: split2h's stays within 4x split3's at every checkpoint."""
    runs = {p: _drift_run(T, W, p, chunks) for p in (0, 1, 3)}
    for p, r in runs.items():
        for lg, _, _ in r:
            assert all(np.isfinite(v) for v in lg.values()), (p, lg)
    n = 0
    for i, k in enumerate(chunks):
        n += k
        ref = runs[0][i]
        row = {}
        for p in (1, 3):
            lg, c, a = runs[p][i]
            row[p] = (max(np.linalg.norm(c - ref[1]) / np.linalg.norm(ref[1]),
                          np.linalg.norm(a - ref[2]) / np.linalg.norm(ref[2])),
                      {kk: abs(lg[kk] - ref[0][kk]) / max(abs(ref[0][kk]), 1e-6) for kk in LOSS_KEYS})
        print(f"T={T} W={W} step {n}: param drift vs fp32 split3 {row[1][0]:.2e} split2h {row[3][0]:.2e}; "
              f"loss drift split3 " + " ".join(f"{v:.1e}" for v in row[1][1].values()) +
              " split2h " + " ".join(f"{v:.1e}" for v in row[3][1].values()))
        assert row[3][0] <= 4 * row[1][0] + 1e-7, (n, row)


@pytest.mark.parametrize("precision", [1, 3], ids=["split3", "split2h"])
@pytest.mark.parametrize("name", ["s3_mt50_w2048", "s4_mt50_w400"])
def test_full_batch_8way_sharded_optimizer_matches_oracle(precision, name):
    """The sharded trunk optimizer (ZeRO-1 style, mtsac_set_sharded_optimizer): the MT50 8-way task
    split with every trunk bucket reduce-scattered, the clip norm from an all-reduced |g|^2, Adam on
    each rank's 1/8 of the trunk, the new trunk all-gathered and re-split into planes on every rank --
    through the in-process collective hook, against the float64 oracle of the unsharded step.  The
    ranks' logs and replicated parameters agree bitwise, and each rank's first Adam moments are nonzero
    only on its own trunk shards (the sharding really happened)."""
    import threading

    from mtrl_amd import _lib as L
    from mtrl_amd.shard import InProcessCollectives, local_rows, shard_tasks

    world = 8
    spec = SHARD_CASES[name]
    cfg, st, batch, en, ec, st1, want = _problem(name)
    T, n = spec["T"], spec["n"]
    shards = []
    for r in range(world):
        b0, c0 = shard_tasks(T, world, r)
        e = _engine(spec, precision, b0, c0, cu_slice=(r, world))
        _load(e, st, b0, c0)
        e.set_sharded_optimizer(True)
        shards.append(e)
    group = InProcessCollectives(world)
    for r, e in enumerate(shards):
        e.set_collective_hook(group.collective_hook(r), r, world)
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
    assert all(lg == logs[0] for lg in logs)
    _check_logs(logs[0], want, f"zero8/p{precision}")
    for r, e in enumerate(shards):
        b0, c0 = shard_tasks(T, world, r)
        _check_params(e, st1, f"zero8/p{precision}/r{r}", b0, c0)
    mu = [e.get_params(L.CRITIC_ADAM_MU) for e in shards]
    frac = [float(np.count_nonzero(m)) / m.size for m in mu]
    print(f"{name}/p{precision}: nonzero critic mu fraction per rank {[round(f, 3) for f in frac]}")
    assert max(frac) < 0.3, frac
    for e in shards:
        e.close()


_DIGEST_CHILD = """
import hashlib
import sys
sys.path.insert(0, {root!r})
sys.path.insert(0, {tests!r})
import numpy as np
import test_gpu_fullbatch as t
a = t._device_steps({T}, {tc}, 2048, 3, 3, 0)
h = hashlib.sha256()
h.update(repr(sorted(a[0].items())).encode())
for x in a[1]:
    h.update(np.ascontiguousarray(x).tobytes())
h.update(repr(a[2]).encode())
h.update(repr(a[3]).encode())
print("digest", h.hexdigest())
"""


@pytest.mark.parametrize("T,tc", [(50, 50), (50, 7)], ids=["s3_split2h", "mt50_shard7_split2h"])
def test_head_kernel_forms_bitwise(T, tc):
    """The head kernels' launch forms are bitwise interchangeable: the fused head backward (data and
    weight passes reading h once) against the separate passes (MTSAC_HEAD_BWD_SPLIT=1), and the
    policy / action-grad rows per wave (MTSAC_HEAD_RW=4 against the default): 3 device-sampled
    steps each in a fresh process (the switches are read once), digests of logs, parameters,
    moments and stream states equal."""
    import os

    tests = os.path.dirname(os.path.abspath(__file__))
    code = _DIGEST_CHILD.format(root=os.path.dirname(tests), tests=tests, T=T, tc=tc)
    digests = []
    for extra in ({}, {"MTSAC_HEAD_BWD_SPLIT": "1"}, {"MTSAC_HEAD_RW": "4"}):
        r = _child(code, dict(os.environ, **extra), timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        digests.append([ln for ln in r.stdout.splitlines() if ln.startswith("digest")][-1])
    assert digests[0] == digests[1] == digests[2], digests
