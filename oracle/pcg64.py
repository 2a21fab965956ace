"""ORACLE (test infrastructure only) -- CPU restatement of the replay-index stream.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module, and only as the checker.  The product path
(``mtrl_amd``) never routes through it.

What it restates
----------------
``MultiTaskReplayBuffer.sample`` draws its shared index vector with
``self._rng.integers(low=0, high=max(...), size=(n,))`` where
``self._rng = np.random.default_rng(seed)`` (reference ``mtrl/rl/buffers.py:260``,
``:523-527``).  The arithmetic therefore lives in numpy (pinned 2.2.4 at
``uv.lock:1078``; 2.2.6 in this container -- same stream):

* bit generator: PCG64 = PCG "XSL RR 128/64" with a 128-bit LCG
  ``s <- s * 0x2360ED051FC65DA44385DF649FCCF645 + inc``; the step happens
  BEFORE the output, output ``rotr64(hi(s) ^ lo(s), s >> 122)``
  (numpy ``random/src/pcg64/pcg64.h``: ``pcg_setseq_128_xsl_rr_64_random_r``).
* ``next_uint32``: if a buffered high half exists return it, else draw a
  64-bit word, return its LOW 32 bits and buffer the HIGH 32 bits
  (``pcg64_next32``; state fields ``has_uint32`` / ``uinteger``).
* ``integers(0, high, size=n)`` with int64 dtype and ``high <= 2**32``:
  ``random_bounded_uint64_fill`` -> ``buffered_bounded_lemire_uint32``
  with ``rng = high - 1``: ``m = u32 * high``; if ``lo32(m) < high`` then
  reject while ``lo32(m) < (2**32 - high) % high``; result ``m >> 32``.
  ``high == 1`` (rng == 0) returns zeros WITHOUT consuming the stream.
  ``high == 2**32`` (rng == 0xFFFFFFFF) returns raw ``next_uint32``.

Pinning: ``tests/test_oracle_pcg64.py`` checks this restatement against
``numpy.random.default_rng(seed).integers`` itself (the reference's own
dependency) for many seeds / highs / sizes, bit for bit, including the
generator state afterwards.
"""

from __future__ import annotations

import numpy as np

MASK32 = (1 << 32) - 1
MASK64 = (1 << 64) - 1
MASK128 = (1 << 128) - 1
PCG_MULT = 0x2360ED051FC65DA44385DF649FCCF645


class PCG64State:
    """Mutable PCG64 state in the same four fields numpy exposes."""

    __slots__ = ("state", "inc", "has_uint32", "uinteger")

    def __init__(self, state: int, inc: int, has_uint32: int = 0, uinteger: int = 0):
        self.state = state & MASK128
        self.inc = inc & MASK128
        self.has_uint32 = int(has_uint32)
        self.uinteger = int(uinteger) & MASK32

    @classmethod
    def from_seed(cls, seed) -> "PCG64State":
        """Initial state exactly as ``np.random.default_rng(seed)`` builds it.

        Seeding goes through numpy's SeedSequence (hash-based); that part is
        taken from numpy directly -- it runs once per buffer, on the host.
        """
        st = np.random.default_rng(seed).bit_generator.state
        return cls.from_numpy_state(st)

    @classmethod
    def from_numpy_state(cls, st: dict) -> "PCG64State":
        assert st["bit_generator"] == "PCG64", st["bit_generator"]
        return cls(st["state"]["state"], st["state"]["inc"], st["has_uint32"], st["uinteger"])

    def to_numpy_state(self) -> dict:
        return {
            "bit_generator": "PCG64",
            "state": {"state": self.state, "inc": self.inc},
            "has_uint32": self.has_uint32,
            "uinteger": self.uinteger,
        }

    def copy(self) -> "PCG64State":
        return PCG64State(self.state, self.inc, self.has_uint32, self.uinteger)

    # -- raw stream -------------------------------------------------------
    def next64(self) -> int:
        self.state = (self.state * PCG_MULT + self.inc) & MASK128
        hi = self.state >> 64
        lo = self.state & MASK64
        x = hi ^ lo
        rot = self.state >> 122
        return ((x >> rot) | (x << ((64 - rot) & 63))) & MASK64

    def next32(self) -> int:
        if self.has_uint32:
            self.has_uint32 = 0
            return self.uinteger
        w = self.next64()
        self.has_uint32 = 1
        self.uinteger = w >> 32
        return w & MASK32

    # -- bounded draws ------------------------------------------------------
    def bounded(self, high: int) -> int:
        """One ``integers(0, high)`` draw (``1 <= high <= 2**32``)."""
        rng = high - 1
        if rng == 0:
            return 0
        if rng == MASK32:
            return self.next32()
        rng_excl = high
        m = self.next32() * rng_excl
        leftover = m & MASK32
        if leftover < rng_excl:
            threshold = (MASK32 - rng) % rng_excl
            while leftover < threshold:
                m = self.next32() * rng_excl
                leftover = m & MASK32
        return m >> 32

    def integers(self, high: int, n: int) -> np.ndarray:
        if not (1 <= high <= (1 << 32)):
            raise ValueError("high must be in [1, 2**32] for the 32-bit Lemire path")
        return np.array([self.bounded(high) for _ in range(n)], dtype=np.int64)


def lcg_jump_table(n: int) -> list[tuple[int, int]]:
    """(A_j, C_j) with state_{i+j} = A_j * state_i + C_j * inc (mod 2**128).

    ``C_j`` multiplies the increment, so the table is seed independent.
    Used by the device index generator to let lane j advance j steps in one
    multiply-add (restated here so the tests can check the C-ABI's table).
    """
    out = []
    a, c = 1, 0
    for _ in range(n):
        out.append((a, c))
        a = (a * PCG_MULT) & MASK128
        c = (c * PCG_MULT + 1) & MASK128
    return out
