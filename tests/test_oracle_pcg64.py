"""Pin the oracle's index-stream restatement to numpy itself (the reference's own
dependency: ``np.random.default_rng(seed).integers`` at mtrl/rl/buffers.py:260,523-527)."""

import numpy as np
import pytest

from oracle.pcg64 import MASK128, PCG_MULT, PCG64State, lcg_jump_table


@pytest.mark.parametrize("seed", [0, 1, 42, 1234, 2**63 + 5])
@pytest.mark.parametrize("high", [1, 2, 7, 128, 4001, 100000, 2**31 - 1, 2**31 + 5, 2**32])
def test_integers_match_numpy(seed, high):
    r = np.random.default_rng(seed)
    s = PCG64State.from_seed(seed)
    for n in (1, 5, 128, 3):  # consecutive calls keep the buffered high half between calls
        np.testing.assert_array_equal(s.integers(high, n), r.integers(0, high, size=n))
        assert s.to_numpy_state() == r.bit_generator.state


def test_state_round_trip_and_raw_stream():
    r = np.random.default_rng(9)
    s = PCG64State.from_numpy_state(r.bit_generator.state)
    raw = r.bit_generator.random_raw(10)
    s2 = PCG64State.from_seed(9)
    assert [s2.next64() for _ in range(10)] == [int(x) for x in raw]
    assert s.copy().to_numpy_state() == s.to_numpy_state()


def test_jump_table_advances_lcg():
    s = PCG64State.from_seed(3)
    tab = lcg_jump_table(65)
    for j in (0, 1, 2, 17, 64):
        a, c = tab[j]
        want = s.copy()
        for _ in range(j):
            want.state = (want.state * PCG_MULT + want.inc) & MASK128
        assert (a * s.state + c * s.inc) & MASK128 == want.state


def test_golden_index_streams():
    """tests/golden/index_streams.npz holds numpy's own output (make_golden.py)."""
    import pathlib

    z = np.load(pathlib.Path(__file__).parent / "golden" / "index_streams.npz", allow_pickle=False)
    for key in z.files:
        s, h = key[1:].split("_h")
        st = PCG64State.from_seed(int(s))
        got = np.stack([st.integers(int(h), 128) for _ in range(3)])
        np.testing.assert_array_equal(got, z[key])
