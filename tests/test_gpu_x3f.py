"""gemm_x3f (mtrl_amd/csrc/gemm_x3f.hip): the row-major x row-major plane GEMM of the trunk
forward and data grad, 16x16x32 MFMA, 208 x 256 tiles, A through LDS in full lines, B straight
to registers.  Checked against float64 numpy with the fp32-GEMM bound |err| <= 4e-6 sum|a b|
(what an fp32 GEMM with fp32 accumulation meets at these K), on the bench's own shape and on
ragged ones (rows past M, a partial last column tile, batch > 1), every epilogue."""

from __future__ import annotations

import ctypes
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(epi, A, B, bias=None, mask=None, planes=True, m16=False):
    from mtrl_amd import _lib as L

    lib = L.load()
    E, M, K = A.shape
    N = B.shape[1]
    C = np.zeros((E, M, N), np.float32)
    Cs = np.zeros((E, M, N), np.float32) if planes else None
    p = lambda a: None if a is None else np.ascontiguousarray(a, np.float32).ctypes.data
    rc = lib.mtsac_debug_gemm_x3f(epi | (256 if m16 else 0), E, M, N, K, p(A), p(B), C.ctypes.data, p(bias), p(mask),
                                  None if Cs is None else Cs.ctypes.data)
    L.check(rc)
    return C, Cs


def _ref(A, B):
    A64, B64 = A.astype(np.float64), B.astype(np.float64)
    acc = np.einsum("emk,enk->emn", A64, B64)
    scale = np.einsum("emk,enk->emn", np.abs(A64), np.abs(B64))
    return acc, scale


@pytest.mark.parametrize("E,M,N,K", [(1, 6400, 2048, 2048), (2, 6300, 2040, 192), (1, 6240, 2048, 128)],
                         ids=["s3_fwd", "ragged_e2", "exact_rows"])
def test_bias_relu_with_planes(E, M, N, K):
    rng = np.random.default_rng(M + K)
    A = rng.standard_normal((E, M, K)).astype(np.float32)
    B = (rng.standard_normal((E, N, K)) / np.sqrt(K)).astype(np.float32)
    bias = rng.standard_normal((E, N)).astype(np.float32) * 0.1
    C, Cs = _run(1, A, B, bias=bias)
    acc, scale = _ref(A, B)
    want = np.maximum(acc + bias[:, None, :], 0)
    err = np.abs(C - want)
    assert np.all(err <= 4e-6 * (scale + np.abs(bias[:, None, :])) + 1e-30), float((err / (scale + 1e-30)).max())
    np.testing.assert_array_equal(Cs, C)  # the planes sum back to the fp32 output exactly


@pytest.mark.parametrize("m16", [False, True], ids=["mask_f32", "mask_bf16_hi"])
def test_relu_mask(m16):
    rng = np.random.default_rng(7)
    E, M, N, K = 2, 6400, 2048, 256
    A = rng.standard_normal((E, M, K)).astype(np.float32)
    B = rng.standard_normal((E, N, K)).astype(np.float32)
    mask = np.maximum(rng.standard_normal((E, M, N)), 0).astype(np.float32)  # a ReLU output: >= 0
    mask[:, :, :7] = 1e-30  # tiny positive activations still pass through the bf16 high plane
    C, Cs = _run(2, A, B, mask=mask, m16=m16)
    acc, scale = _ref(A, B)
    want = np.where(mask > 0, acc, 0.0)
    assert np.all(np.abs(C - want) <= 4e-6 * scale + 1e-30)
    np.testing.assert_array_equal(Cs, C)


def test_fp32_only_output():
    rng = np.random.default_rng(3)
    A = rng.standard_normal((1, 6400, 64)).astype(np.float32)
    B = rng.standard_normal((1, 2048, 64)).astype(np.float32)
    C, _ = _run(1, A, B, bias=np.zeros((1, 2048), np.float32), planes=False)
    acc, scale = _ref(A, B)
    assert np.all(np.abs(C - np.maximum(acc, 0)) <= 4e-6 * scale + 1e-30)


def test_rejects_small_grids():
    from mtrl_amd import _lib as L

    lib = L.load()
    A = np.zeros((1, 416, 64), np.float32)
    B = np.zeros((1, 256, 64), np.float32)
    C = np.zeros((1, 416, 256), np.float32)
    assert lib.mtsac_debug_gemm_x3f(1, 1, 416, 256, 64, A.ctypes.data, B.ctypes.data, C.ctypes.data, None, None,
                                    None) == -95



@pytest.mark.parametrize("E,M,N,K,epi,m16", [(2, 6400, 2048, 256, 1, False), (2, 6300, 2040, 192, 2, True),
                                             (1, 12800, 2048, 128, 1, False), (1, 6400, 2048, 128, 2, False),
                                             (2, 1280, 2048, 512, 2, True), (1, 1270, 2040, 256, 1, False)],
                         ids=["s3_critic_fwd", "ragged_mask16", "merged_actor_fwd", "e1_208rows", "c2_critic_80rows",
                              "c2_e1_48rows_ragged"])
def test_bf16_products(E, M, N, K, epi, m16):
    """Precision bf16 on gemm_x3f: exactly the products of the bf16-rounded operands, fp32 sums.
    Each shape runs the row tile the bf16 cost model picks (gemm_x3f.hip bf16_bm): 400 rows for
    the S3 critic / merged actor forward, 208 for single-member 6400-row grads, 80 / 48 for MT10's
    1280 rows -- ragged rows and columns included, every tile height's epilogue image in LDS."""
    import torch

    rng = np.random.default_rng(31 + M + K)
    A = rng.standard_normal((E, M, K)).astype(np.float32)
    B = (rng.standard_normal((E, N, K)) / 16).astype(np.float32)
    Ar = torch.from_numpy(A).to(torch.bfloat16).to(torch.float64).numpy()
    Br = torch.from_numpy(B).to(torch.bfloat16).to(torch.float64).numpy()
    acc, scale = _ref(Ar, Br)
    if epi == 1:
        bias = rng.standard_normal((E, N)).astype(np.float32) * 0.1
        C, _ = _run(1 | 1024, A, B, bias=bias)
        want = np.maximum(acc + bias[:, None, :], 0)
        assert np.all(np.abs(C - want) <= 4e-6 * (scale + np.abs(bias[:, None, :])) + 1e-30)
    else:
        mask = np.maximum(rng.standard_normal((E, M, N)), 0).astype(np.float32)
        C, _ = _run(2 | 1024 | (256 if m16 else 0), A, B, mask=mask, m16=m16)
        want = np.where(mask > 0, acc, 0.0)
        assert np.all(np.abs(C - want) <= 4e-6 * scale + 1e-30)


@pytest.mark.parametrize("E,M,N,K,epi,m16,bf16", [(2, 896, 2048, 2048, 1, False, False),
                                                  (2, 768, 2048, 2048, 2, True, False),
                                                  (2, 1280, 2040, 512, 2, False, False),
                                                  (1, 1800, 2048, 1024, 1, False, False),
                                                  (2, 300, 2048, 2048, 1, False, True),
                                                  (2, 320, 2048, 2048, 2, True, True)],
                         ids=["shard7_fwd", "shard6_dgrad_m16", "mt10_ragged_dgrad", "e1_ragged_fwd", "bf16_split_fwd",
                              "bf16_split_dgrad_m16"])
def test_split_k_task_shards(E, M, N, K, epi, m16, bf16):
    """Few rows (task shards): K split over workgroups, raw partial slabs, then the finishing
    pass applies bias+ReLU or the ReLU mask (fp32 or the bf16 high plane) and writes the planes."""
    from mtrl_amd import _lib as L

    lib = L.load()
    rng = np.random.default_rng(M + K + epi)
    A = rng.standard_normal((E, M, K)).astype(np.float32)
    B = (rng.standard_normal((E, N, K)) / np.sqrt(K)).astype(np.float32)
    bias = rng.standard_normal((E, N)).astype(np.float32) * 0.1
    mask = np.maximum(rng.standard_normal((E, M, N)), 0).astype(np.float32)
    C = np.zeros((E, M, N), np.float32)
    Cs = np.zeros((E, M, N), np.float32)
    p = lambda a: np.ascontiguousarray(a, np.float32).ctypes.data
    L.check(lib.mtsac_debug_gemm_x3f(epi | (256 if m16 else 0) | 2048 | (1024 if bf16 else 0), E, M, N, K, p(A),
                                     p(B), C.ctypes.data, p(bias), p(mask), Cs.ctypes.data))
    if bf16:  # the products of the bf16-rounded operands
        import torch

        A = torch.from_numpy(A).to(torch.bfloat16).to(torch.float64).numpy()
        B = torch.from_numpy(B).to(torch.bfloat16).to(torch.float64).numpy()
    acc, scale = _ref(A, B)
    if epi == 1:
        want = np.maximum(acc + bias[:, None, :], 0)
        tol = 4e-6 * (scale + np.abs(bias[:, None, :])) + 1e-30
    else:
        want = np.where(mask > 0, acc, 0.0)  # h > 0 <=> its bf16 high plane > 0
        tol = 4e-6 * scale + 1e-30
    err = np.abs(C - want)
    assert np.all(err <= tol), float((err / (scale + 1e-30)).max())
    if bf16:  # precision bf16 keeps (and its GEMMs read) the high plane only
        import torch

        np.testing.assert_array_equal(Cs, torch.from_numpy(C).to(torch.bfloat16).float().numpy())
    else:
        np.testing.assert_array_equal(Cs, C)


@pytest.mark.parametrize("E,M,N,K,epi,m16,planes,h2", [(2, 896, 2048, 2048, 1, False, True, False),
                                                       (2, 896, 2048, 2048, 1, False, False, False),
                                                       (2, 768, 2048, 2048, 2, True, True, False),
                                                       (1, 1792, 2048, 2048, 1, False, True, False),
                                                       (2, 1280, 2040, 512, 2, True, True, False),
                                                       (2, 300, 2048, 2048, 2, True, False, False),
                                                       (2, 896, 2048, 2048, 1, False, True, True),
                                                       (1, 1792, 2048, 2048, 1, False, False, True),
                                                       (2, 768, 2048, 2048, 2, True, True, True),
                                                       (2, 1664, 2048, 2048, 2, True, True, True)],
                         ids=["shard7_fwd_planes", "shard7_fwd_top_fp32", "shard6_dgrad_m16", "shard7_actor_2b",
                              "mt10_ragged_dgrad_m16", "short_dgrad_fp32_only", "h2_shard7_fwd_planes",
                              "h2_shard7_actor_top_fp32", "h2_shard6_dgrad_m16", "h2_shard13_dgrad_m16"])
def test_split_k_in_launch_finish_bitwise(E, M, N, K, epi, m16, planes, h2):
    """The in-launch split-K finish gives the separate finishing pass's bits exactly and meets the fp32
    bound against float64.  split3: every slice writes its slab and draws a ticket, the last one adds
    the slabs in slice order with its own partial in its place.  split2h (the default precision, two
    slices): the pair hand-off -- the ticket first, the first slice publishes its partial with the
    unscale factor 2^-(eA + eB) already applied,
    the second adds it to its own (fp32 addition commutes) and applies the epilogue; C and the output
    planes equal the finishing pass's bit for bit."""
    from mtrl_amd import _lib as L

    lib = L.load()
    rng = np.random.default_rng(M + 3 * K + epi)
    A = rng.standard_normal((E, M, K)).astype(np.float32)
    B = (rng.standard_normal((E, N, K)) / np.sqrt(K)).astype(np.float32)
    bias = rng.standard_normal((E, N)).astype(np.float32) * 0.1
    mask = np.maximum(rng.standard_normal((E, M, N)), 0).astype(np.float32)
    p = lambda a: np.ascontiguousarray(a, np.float32).ctypes.data
    out = []
    for fin in (0, 4096):
        C = np.zeros((E, M, N), np.float32)
        Cs = np.zeros((E, M, N), np.float32) if planes else None
        L.check(lib.mtsac_debug_gemm_x3f(epi | (256 if m16 else 0) | 2048 | fin | (8192 if h2 else 0), E, M, N, K,
                                         p(A), p(B), C.ctypes.data, p(bias), p(mask),
                                         None if Cs is None else Cs.ctypes.data))
        out.append((C, Cs))
    np.testing.assert_array_equal(out[1][0], out[0][0])
    if planes:
        np.testing.assert_array_equal(out[1][1], out[0][1])
        if not h2:  # split3 planes sum to C exactly (split2h's carry 22 bits: test_split2h_products)
            np.testing.assert_array_equal(out[1][1], out[1][0])
    acc, scale = _ref(A, B)
    if epi == 1:
        want = np.maximum(acc + bias[:, None, :], 0)
        tol = 4e-6 * (scale + np.abs(bias[:, None, :])) + 1e-30
    else:
        want = np.where(mask > 0, acc, 0.0)
        tol = 4e-6 * scale + 1e-30
    assert np.all(np.abs(out[1][0] - want) <= tol)


@pytest.mark.parametrize("E,M,N,K,epi,m16,scale_a,spread", [(1, 6400, 2048, 2048, 1, False, 1.0, 0),
                                                            (2, 6300, 2040, 192, 1, False, 37.0, 0),
                                                            (2, 6400, 2048, 256, 2, True, 1e-6, 0),
                                                            (2, 6400, 2048, 512, 2, False, 3e3, 0),
                                                            (1, 6400, 2048, 2048, 2, True, 1.0, 6)],
                         ids=["s3_fwd", "ragged_e2_large", "dgrad_m16_tiny_grads", "dgrad_f32mask_large",
                              "dgrad_rows_spread_1e6"])
def test_split2h_products(E, M, N, K, epi, m16, scale_a, spread):
    """Precision split2h on gemm_x3f: operands as two fp16 planes of x 2^e (e per tensor from its
    max), 3 products (h*l, l*h, h*h) unscaled by 2^-(eA + eB); the output planes at the exponent of
    the bound K max|A| max|B| + max|bias|.  The fp32-GEMM bound |err| <= 4e-6 sum|a b| holds at
    operand magnitudes from gradients (1e-6) to large activations; the planes carry the output to
    22 bits (|planes - C| <= 2^-21 |C| + 2^-24 2^-e: the low plane's subnormal spacing in the scaled
    unit -- half of it from rounding, all of it where the sticky subnormal keeps a positive value
    nonzero -- e the output exponent from the device's bound K max|A| mB + mB, mB = max(max|B|,
    max|bias|): a weight record covers the trunk's kernels and biases alike), and the ReLU mask read from the planes is
    exactly 'x > 0' down to the tiniest positive activation.  rows_spread: row magnitudes over six
    decades under one tensor exponent, each element still within 4e-6 of its own row's sum |a b|."""
    rng = np.random.default_rng(M + K + epi)
    A = rng.standard_normal((E, M, K)) * scale_a
    if spread:  # row magnitudes over `spread` decades (per-row TD errors of a data grad): the planes'
        A *= 10.0 ** (-spread * rng.random((E, M, 1)))  # per-tensor exponent serves every row
    A = A.astype(np.float32)
    B = (rng.standard_normal((E, N, K)) / np.sqrt(K)).astype(np.float32)
    acc, scale = _ref(A, B)
    if epi == 1:
        bias = (rng.standard_normal((E, N)) * 0.1 * scale_a).astype(np.float32)
        C, Cs = _run(1 | 8192, A, B, bias=bias)
        want = np.maximum(acc + bias[:, None, :], 0)
        tol = 4e-6 * (scale + np.abs(bias[:, None, :])) + 1e-30
        mB = max(float(np.abs(B).max()), float(np.abs(bias).max()))
        bound = K * float(np.abs(A).max()) * mB + mB
    else:
        mask = np.maximum(rng.standard_normal((E, M, N)), 0).astype(np.float32)
        mask[:, :, :7] = 1e-30  # tiny positive activations: the planes' sticky subnormal keeps them active
        C, Cs = _run(2 | 8192 | (256 if m16 else 0), A, B, mask=mask, m16=m16)
        want = np.where(mask > 0, acc, 0.0)
        tol = 4e-6 * scale + 1e-30
        bound = K * float(np.abs(A).max()) * float(np.abs(B).max())
    err = np.abs(C - want)
    print("max err / sum|ab|", float((err / (scale + 1e-30)).max()))
    assert np.all(err <= tol), float((err / (scale + 1e-30)).max())
    e = 15 - math.frexp(bound * 1.00390625)[1]
    dev = np.abs(Cs.astype(np.float64) - C)
    lim = 2.0 ** -21 * np.abs(C) + 1.01 * 2.0 ** (-24 - e)
    print("planes: e", e, "worst |planes - C| / limit", float((dev / lim).max()))
    assert np.all(dev <= lim)


@pytest.mark.parametrize("E,M,N,K,epi,m16,prec,split", [(1, 6400, 2048, 2048, 1, False, "split2h", False),
                                                        (2, 6400, 2048, 256, 2, True, "split2h", False),
                                                        (2, 6300, 2032, 192, 1, False, "split3", False),
                                                        (2, 6400, 2048, 512, 2, True, "bf16", False),
                                                        (2, 896, 2048, 2048, 1, False, "split2h", True),
                                                        (2, 768, 2048, 2048, 2, True, "split3", True)],
                         ids=["s3_fwd_h2", "dgrad_m16_h2", "ragged_split3", "dgrad_bf16", "shard7_splitk_h2",
                              "shard6_splitk_split3_dgrad"])
def test_fragment_layout_b_bitwise(E, M, N, K, epi, m16, prec, split):
    """B planes in the fragment layout (gemm_common.h frag_off: each 16-row x 32-k MFMA fragment 1 KB
    contiguous, the engine's weight planes at S3) give the row-major planes' outputs bit for bit:
    the same products in the same order, only the addresses differ."""
    from mtrl_amd import _lib as L

    lib = L.load()
    rng = np.random.default_rng(M + K + N)
    A = rng.standard_normal((E, M, K)).astype(np.float32)
    B = (rng.standard_normal((E, N, K)) / np.sqrt(K)).astype(np.float32)
    bias = rng.standard_normal((E, N)).astype(np.float32) * 0.1
    mask = np.maximum(rng.standard_normal((E, M, N)), 0).astype(np.float32)
    p = lambda a: np.ascontiguousarray(a, np.float32).ctypes.data
    flags = {"split2h": 8192, "split3": 0, "bf16": 1024}[prec] | (256 if m16 else 0) | (2048 if split else 0)
    out = []
    for frag in (0, 16384):
        C = np.zeros((E, M, N), np.float32)
        Cs = np.zeros((E, M, N), np.float32)
        L.check(lib.mtsac_debug_gemm_x3f(epi | flags | frag, E, M, N, K, p(A), p(B), C.ctypes.data, p(bias), p(mask),
                                         Cs.ctypes.data))
        out.append((C, Cs))
    np.testing.assert_array_equal(out[1][0], out[0][0])
    np.testing.assert_array_equal(out[1][1], out[0][1])
    assert np.abs(out[1][0]).max() > 0
