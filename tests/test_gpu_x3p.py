"""Pre-split-plane GEMM (gemm_x3p.hip): device split in the stored orientation, LDS-DMA
pipeline, row-major (ds_read_b128) and k-major (ds_read_b64_tr_b16) operand images, split-K
and the plane-writing epilogue -- against a float64 product of the same fp32 inputs."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[0, 1, 2, 3, 4, 5], ids=["geo128x128k32", "geo256x128k32", "geo256x128k16", "geo256x256k16",
                                             "geo128x128k16", "geo224x256k16"])
def geo(request):
    from mtrl_amd import _lib as L

    lib = L.load()
    old = lib.mtsac_debug_x3p_geo(request.param)
    yield request.param
    lib.mtsac_debug_x3p_geo(old)


def _run(epi, M, N, K, A, a_kmajor, B, b_kmajor, bias=None, mask=None, splits=1, want_planes=False):
    from mtrl_amd import _lib as L

    lib = L.load()
    A = np.ascontiguousarray(A, np.float32)
    B = np.ascontiguousarray(B, np.float32)
    C = np.zeros((M, N), np.float32)
    S = np.zeros((M, N), np.float32) if want_planes else None
    bias = None if bias is None else np.ascontiguousarray(bias, np.float32)
    mask = None if mask is None else np.ascontiguousarray(mask, np.float32)
    L.check(lib.mtsac_debug_gemm_x3p(epi | (splits << 8), M, N, K, A.ctypes.data, a_kmajor, B.ctypes.data, b_kmajor,
                                     C.ctypes.data, None if bias is None else bias.ctypes.data,
                                     None if mask is None else mask.ctypes.data,
                                     None if S is None else S.ctypes.data))
    return (C, S) if want_planes else C


def _operands(M, N, K, layout, seed=1):
    rng = np.random.default_rng(seed)
    A = rng.standard_normal((K, M) if layout[0] else (M, K)).astype(np.float32)
    B = rng.standard_normal((K, N) if layout[1] else (N, K)).astype(np.float32)
    A64 = A.astype(np.float64).T if layout[0] else A.astype(np.float64)
    B64 = B.astype(np.float64) if layout[1] else B.astype(np.float64).T
    return A, B, A64 @ B64, np.abs(A64) @ np.abs(B64)


# (A k-major?, B k-major?): NT (forward / data grad), TN (weight grad) and the mixed forms
LAYOUTS = [(0, 0), (0, 1), (1, 0), (1, 1)]


@pytest.mark.parametrize("shape", [(200, 136, 93), (128, 128, 32), (64, 400, 400), (257, 132, 260), (8, 8, 4),
                                   (6400, 256, 96), (300, 520, 64)])
@pytest.mark.parametrize("layout", LAYOUTS)
def test_x3p_matches_fp64(shape, layout, geo):
    M, N, K = shape
    A, B, ref, mag = _operands(M, N, K, layout)
    C = _run(0, M, N, K, A, layout[0], B, layout[1])
    err = np.abs(C - ref)
    assert np.all(err <= 4e-6 * mag + 1e-30), float((err / mag).max())


@pytest.mark.parametrize("splits", [2, 3, 8, 16])
@pytest.mark.parametrize("shape", [(256, 128, 6400), (100, 300, 1000), (8, 8, 33), (400, 400, 1280)])
def test_x3p_splitk_weight_grad(shape, splits, geo):
    M, N, K = shape
    A, B, ref, mag = _operands(M, N, K, (1, 1), seed=2)
    C = _run(0, M, N, K, A, 1, B, 1, splits=splits)
    err = np.abs(C - ref)
    assert np.all(err <= 4e-6 * mag + 1e-30), float((err / mag).max())


def test_x3p_epilogues(geo):
    M, N, K = 300, 200, 96
    rng = np.random.default_rng(2)
    A = rng.standard_normal((M, K)).astype(np.float32)
    Bt = rng.standard_normal((N, K)).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32)
    C, S = _run(1, M, N, K, A, 0, Bt, 0, bias=bias, want_planes=True)
    np.testing.assert_allclose(C, np.maximum(A.astype(np.float64) @ Bt.T + bias, 0), rtol=1e-5, atol=1e-4)
    # the planes written beside C reconstruct it to ~2^-24 relative
    np.testing.assert_allclose(S, C, rtol=1e-7, atol=1e-30)
    H = rng.standard_normal((M, N)).astype(np.float32)
    C, S = _run(2, M, N, K, A, 0, Bt, 0, mask=H, want_planes=True)
    np.testing.assert_allclose(C, (A.astype(np.float64) @ Bt.T) * (H > 0), rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(S, C, rtol=1e-7, atol=1e-30)
    assert np.all(S[H <= 0] == 0)


@pytest.mark.parametrize("splits", [2, 4])
def test_x3p_splitk_epilogues(splits, geo):
    """Split-K on the forward / data-grad forms: partial slabs, then the finishing pass applies
    bias+ReLU or the ReLU mask and writes the planes."""
    M, N, K = 300, 200, 512
    rng = np.random.default_rng(5)
    A = rng.standard_normal((M, K)).astype(np.float32)
    Bt = rng.standard_normal((N, K)).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32)
    ref = A.astype(np.float64) @ Bt.T.astype(np.float64)
    C, S = _run(1, M, N, K, A, 0, Bt, 0, bias=bias, splits=splits, want_planes=True)
    np.testing.assert_allclose(C, np.maximum(ref + bias, 0), rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(S, C, rtol=1e-7, atol=1e-30)
    H = rng.standard_normal((M, N)).astype(np.float32)
    C, S = _run(2, M, N, K, A, 0, Bt, 0, mask=H, splits=splits, want_planes=True)
    np.testing.assert_allclose(C, ref * (H > 0), rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(S, C, rtol=1e-7, atol=1e-30)
