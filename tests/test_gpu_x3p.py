"""Pre-split-plane GEMM (gemm_x3p.hip): device split (natural / transposed) + LDS-DMA
pipelined bf16x6 MFMA GEMM vs a float64 product of the same fp32 inputs."""

import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[0, 1], ids=["geo128x128", "geo256x128"])
def geo(request):
    from mtrl_amd import _lib as L

    lib = L.load()
    old = lib.mtsac_debug_x3p_geo(request.param)
    yield request.param
    lib.mtsac_debug_x3p_geo(old)


def _run(epi, M, N, K, A, a_kmajor, B, b_kmajor, bias=None, mask=None):
    from mtrl_amd import _lib as L

    lib = L.load()
    A = np.ascontiguousarray(A, np.float32)
    B = np.ascontiguousarray(B, np.float32)
    C = np.zeros((M, N), np.float32)
    bias = None if bias is None else np.ascontiguousarray(bias, np.float32)
    mask = None if mask is None else np.ascontiguousarray(mask, np.float32)
    L.check(lib.mtsac_debug_gemm_x3p(epi, M, N, K, A.ctypes.data, a_kmajor, B.ctypes.data, b_kmajor, C.ctypes.data,
                                     None if bias is None else bias.ctypes.data,
                                     None if mask is None else mask.ctypes.data))
    return C


@pytest.mark.parametrize("shape", [(200, 136, 93), (128, 128, 32), (64, 400, 400), (257, 132, 260), (8, 4, 4),
                                   (6400, 256, 96)])
@pytest.mark.parametrize("layout", [(0, 0), (0, 1), (1, 1)])  # (A k-major?, B k-major?): NT-, NN-, TN-forms
def test_x3p_matches_fp64(shape, layout, geo):
    M, N, K = shape
    rng = np.random.default_rng(1)
    A = rng.standard_normal((K, M) if layout[0] else (M, K)).astype(np.float32)
    B = rng.standard_normal((K, N) if layout[1] else (N, K)).astype(np.float32)
    C = _run(0, M, N, K, A, layout[0], B, layout[1])
    A64 = A.astype(np.float64).T if layout[0] else A.astype(np.float64)
    B64 = B.astype(np.float64) if layout[1] else B.astype(np.float64).T
    ref, mag = A64 @ B64, np.abs(A64) @ np.abs(B64)
    err = np.abs(C - ref)
    assert np.all(err <= 4e-6 * mag + 1e-30), float((err / mag).max())


def test_x3p_epilogues(geo):
    M, N, K = 300, 200, 96
    rng = np.random.default_rng(2)
    A = rng.standard_normal((M, K)).astype(np.float32)
    B = rng.standard_normal((K, N)).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32)
    C = _run(1, M, N, K, A, 0, B, 1, bias=bias)
    np.testing.assert_allclose(C, np.maximum(A.astype(np.float64) @ B + bias, 0), rtol=1e-5, atol=1e-4)
    H = rng.standard_normal((M, N)).astype(np.float32)
    C = _run(2, M, N, K, A, 0, B, 1, mask=H)
    np.testing.assert_allclose(C, (A.astype(np.float64) @ B) * (H > 0), rtol=1e-5, atol=1e-4)
