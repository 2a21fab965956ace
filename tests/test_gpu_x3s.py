"""gemm_x3s (mtrl_amd/csrc/gemm_x3s.hip): the small-row-count plane GEMM of the trunk forward and
data grad (task shards, MT10), 16 TI x 64 tiles with the K range split over the 4 waves of a
workgroup.  Checked against float64 numpy with the fp32-GEMM bound |err| <= 4e-6 sum|a b|, on the
shapes a rank of the 8-way MT50 job and MT10 run (B = 768 / 896 / 1280, W = 2048 and 400), every
tile height (TI = 4..8), ragged edges (rows past M, a partial column tile, odd K-step counts: the
phantom step) and every epilogue."""

from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SMALL = 512  # epi bit 9: gemm_x3s
M16 = 256    # epi bit 8: ReLU mask from the bf16 high plane


def _run(epi, A, B, bias=None, mask=None, planes=True):
    from mtrl_amd import _lib as L

    lib = L.load()
    E, M, K = A.shape
    N = B.shape[1]
    C = np.zeros((E, M, N), np.float32)
    Cs = np.zeros((E, M, N), np.float32) if planes else None
    p = lambda a: None if a is None else np.ascontiguousarray(a, np.float32).ctypes.data
    rc = lib.mtsac_debug_gemm_x3f(epi | SMALL, E, M, N, K, p(A), p(B), C.ctypes.data, p(bias), p(mask),
                                  None if Cs is None else Cs.ctypes.data)
    L.check(rc)
    return C, Cs


def _ref(A, B):
    A64, B64 = A.astype(np.float64), B.astype(np.float64)
    return np.einsum("emk,enk->emn", A64, B64), np.einsum("emk,enk->emn", np.abs(A64), np.abs(B64))


SHAPES = [(1, 896, 2048, 2048), (2, 768, 2048, 256), (1, 1280, 400, 416), (2, 1280, 2048, 128), (1, 100, 64, 96),
          (1, 3200, 512, 192), (2, 640, 2048, 64)]
IDS = ["shard7_w2048", "shard6_e2", "mt10_w400_oddK", "mt10_input_e2", "tiny", "shard25", "k64_two_waves_idle"]


@pytest.mark.parametrize("E,M,N,K", SHAPES, ids=IDS)
def test_bias_relu_with_planes(E, M, N, K):
    rng = np.random.default_rng(M + N + K)
    A = rng.standard_normal((E, M, K)).astype(np.float32)
    B = (rng.standard_normal((E, N, K)) / np.sqrt(K)).astype(np.float32)
    bias = rng.standard_normal((E, N)).astype(np.float32) * 0.1
    C, Cs = _run(1, A, B, bias=bias)
    acc, scale = _ref(A, B)
    want = np.maximum(acc + bias[:, None, :], 0)
    err = np.abs(C - want)
    assert np.all(err <= 4e-6 * (scale + np.abs(bias[:, None, :])) + 1e-30), float((err / (scale + 1e-30)).max())
    np.testing.assert_array_equal(Cs, C)  # the planes sum back to the fp32 output exactly


@pytest.mark.parametrize("E,M,N,K", SHAPES[:4], ids=IDS[:4])
def test_relu_mask_bf16_high_plane(E, M, N, K):
    rng = np.random.default_rng(7 + M)
    A = rng.standard_normal((E, M, K)).astype(np.float32)
    B = rng.standard_normal((E, N, K)).astype(np.float32)
    mask = np.maximum(rng.standard_normal((E, M, N)), 0).astype(np.float32)  # a ReLU output: >= 0
    mask[:, :, :7] = 1e-30  # tiny positive activations still pass through the bf16 high plane
    C, Cs = _run(2 | M16, A, B, mask=mask)
    acc, scale = _ref(A, B)
    want = np.where(mask > 0, acc, 0.0)
    assert np.all(np.abs(C - want) <= 4e-6 * scale + 1e-30)
    np.testing.assert_array_equal(Cs, C)


def test_fp32_only_output():
    rng = np.random.default_rng(3)
    A = rng.standard_normal((1, 896, 2048)).astype(np.float32)
    B = rng.standard_normal((1, 2048, 2048)).astype(np.float32)
    C, _ = _run(1, A, B, bias=np.zeros((1, 2048), np.float32), planes=False)
    acc, scale = _ref(A, B)
    assert np.all(np.abs(C - np.maximum(acc, 0)) <= 4e-6 * scale + 1e-30)


def test_tile_heights():
    """gemm_x3s_ti: every tile height the cost model picks is exercised above."""
    from mtrl_amd import _lib as L

    lib = L.load()
    got = {lib.mtsac_debug_x3s_ti(M, N, E) for E, M, N, _ in SHAPES}
    assert got >= {5, 7}, got


def test_fp32_mask_rejected():
    from mtrl_amd import _lib as L

    lib = L.load()
    A = np.zeros((1, 896, 64), np.float32)
    B = np.zeros((1, 256, 64), np.float32)
    C = np.zeros((1, 896, 256), np.float32)
    assert lib.mtsac_debug_gemm_x3f(2 | SMALL, 1, 896, 256, 64, A.ctypes.data, B.ctypes.data, C.ctypes.data, None,
                                    A.ctypes.data, None) == -95


BF16 = 1024  # epi bit 10: precision bf16 (the operands' high planes only, one MFMA per product)


@pytest.mark.parametrize("E,M,N,K", SHAPES[:3], ids=IDS[:3])
def test_bf16_products(E, M, N, K):
    """Precision bf16: C = sum_k bf16(a) bf16(b) in fp32, i.e. exactly the product of the
    rounded operands up to fp32 accumulation."""
    rng = np.random.default_rng(21 + M)
    A = rng.standard_normal((E, M, K)).astype(np.float32)
    B = (rng.standard_normal((E, N, K)) / np.sqrt(K)).astype(np.float32)
    bias = rng.standard_normal((E, N)).astype(np.float32) * 0.1
    C, _ = _run(1 | BF16, A, B, bias=bias)
    import torch

    Ar = torch.from_numpy(A).to(torch.bfloat16).to(torch.float64).numpy()
    Br = torch.from_numpy(B).to(torch.bfloat16).to(torch.float64).numpy()
    acc, scale = _ref(Ar, Br)
    want = np.maximum(acc + bias[:, None, :], 0)
    assert np.all(np.abs(C - want) <= 4e-6 * (scale + np.abs(bias[:, None, :])) + 1e-30)
