"""Non-blocking replay add (engine.cpp mtsac_buffer_add; buffers.py:426-474).

The add is staged through a pinned ring and committed on the engine stream, so the host
returns at once and the order against updates is the stream order: adds interleaved with
device-sampled updates, with no host synchronisation between them, must give bitwise the
state of the fully serialised order.  Device (torch) arrays are accepted as well.
"""

from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

T, W, n, CAP = 3, 32, 4, 64


def _engine(normalize=0):
    from mtrl_amd import _lib as L
    from mtrl_amd.engine import MTSACEngine, make_config
    from mtrl_amd.init import init_mtsac

    e = MTSACEngine(make_config(num_tasks=T, task_count=T, obs_dim=39 + T, actor_width=W, critic_width=W,
                                batch_per_task=n, capacity=CAP, normalize_rewards=normalize))
    a, c = init_mtsac(T, 39 + T, 4, W, 3, W, 3, 2, seed=2)
    e.set_params(L.ACTOR, a)
    e.set_params(L.CRITIC, c)
    e.set_params(L.CRITIC_TARGET, c)
    e.seed_rng(1)
    return e


def _rows(rng):
    o = np.zeros((T, 39 + T), np.float32)
    o[:, :39] = rng.standard_normal((T, 39))
    o[np.arange(T), 39 + np.arange(T)] = 1
    no = o.copy()
    no[:, :39] = rng.standard_normal((T, 39))
    return (o, no, rng.uniform(-1, 1, (T, 4)).astype(np.float32), rng.uniform(0, 10, T).astype(np.float32),
            (rng.uniform(size=T) < 0.2).astype(np.float32))


@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
def test_interleaved_adds_equal_serial_order(graph):
    from mtrl_amd import _lib as L

    outs = []
    for serial in (True, False):
        e = _engine()
        e.enable_graph(graph)
        rng = np.random.default_rng(7)
        for _ in range(20):
            e.buffer_add(*_rows(rng))
        e.synchronize()
        for _ in range(40):  # > the 32-slot staging ring
            e.buffer_add(*_rows(rng))
            if serial:
                e.synchronize()
            e.update_many(1)
            if serial:
                e.synchronize()
        outs.append((e.logs(), e.get_params(L.ACTOR), e.get_params(L.CRITIC), e.buffer_read(0, CAP),
                     e.buffer_state(), e.get_rng_state()))
        e.close()
    a, b = outs
    assert a[0] == b[0]
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[2], b[2])
    for x, y in zip(a[3], b[3]):
        np.testing.assert_array_equal(x, y)
    assert a[4] == b[4] == (60, False) and a[5] == b[5]


def test_device_array_add_and_reward_stats():
    import torch

    rng = np.random.default_rng(3)
    host, dev = _engine(normalize=1), _engine(normalize=1)
    want_min, want_max = np.full(T, np.inf), np.full(T, -np.inf)
    for _ in range(70):  # wraps the 64-slot buffer
        rows = _rows(rng)
        host.buffer_add(*rows)
        dev.buffer_add(*[torch.from_numpy(x).cuda() for x in rows])
        want_min = np.minimum(want_min, rows[3].astype(np.float64))
        want_max = np.maximum(want_max, rows[3].astype(np.float64))
    for x, y in zip(host.buffer_read(0, CAP), dev.buffer_read(0, CAP)):
        np.testing.assert_array_equal(x, y)
    assert host.buffer_state() == dev.buffer_state() == (70 % CAP, True)
    for e in (host, dev):
        mn, mx = e.reward_stats()
        np.testing.assert_array_equal(mn, want_min)
        np.testing.assert_array_equal(mx, want_max)
    # reads into device memory too
    obs = torch.empty((CAP, T, 39 + T), device="cuda")
    from mtrl_amd import _lib as L

    L.check(host.lib.mtsac_buffer_read(host._h, 0, CAP, obs.data_ptr(), None, None, None, None))
    np.testing.assert_array_equal(obs.cpu().numpy(), host.buffer_read(0, CAP)[0])
    host.close()
    dev.close()


@pytest.mark.parametrize("side_stream", [False, True], ids=["default_stream", "side_stream"])
def test_device_add_from_one_reused_tensor(side_stream):
    """The producer overwrites ONE device tensor per field right after every add (and frees
    temporaries): each add must still store the rows it was given (the pack kernel
    runs on the engine stream; the producer stream is made to wait for it)."""
    import torch

    rng = np.random.default_rng(11)
    host, dev = _engine(), _engine()
    stream = torch.cuda.Stream() if side_stream else torch.cuda.current_stream()
    with torch.cuda.stream(stream):
        bufs = [torch.empty(x.shape, device="cuda") for x in _rows(rng)]
        for _ in range(50):
            rows = _rows(rng)
            host.buffer_add(*rows)
            for b, x in zip(bufs, rows):
                b.copy_(torch.from_numpy(x).cuda(non_blocking=True))
            dev.buffer_add(*bufs)
            for b in bufs:  # the very next producer work clobbers the arrays
                b.fill_(-7.0)
            junk = torch.full((4096,), 3.0, device="cuda")  # reuses freed blocks on this stream
            del junk
    torch.cuda.synchronize()
    for x, y in zip(host.buffer_read(0, CAP), dev.buffer_read(0, CAP)):
        np.testing.assert_array_equal(x, y)
    host.close()
    dev.close()


def test_mixed_host_device_add_is_rejected():
    import torch

    from mtrl_amd._lib import MTSACError

    e = _engine()
    rows = list(_rows(np.random.default_rng(0)))
    rows[0] = torch.from_numpy(rows[0]).cuda()
    with pytest.raises(MTSACError):
        e.buffer_add(*rows)
    e.close()
