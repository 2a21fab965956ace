/*
 * mtsac_debug.h -- test-only entry points of libmtsac.so (not part of the drop-in
 * boundary).  They expose single device kernels so the parity tests can check a
 * kernel in isolation against the oracle / a torch fp32 reference.
 */
#ifndef MTSAC_DEBUG_H_
#define MTSAC_DEBUG_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One batched fp32 MFMA GEMM with epilogue on device 0 (host pointers in/out):
 *   kind 0 NN: C = A[M][K] . B[K][N]   kind 1 NT: C = A[M][K] . B[N][K]^T
 *   kind 2 TN: C = A[K][M]^T . B[K][N]
 *   epi 0 store (+ db = column sums of B when kind 2 and db != NULL),
 *   epi 1 relu(acc + bias[n]), epi 2 acc * (mask[m][n] > 0).
 * Every operand is dense with the given leading dimension; batch strides are the
 * dense matrix sizes (A shared across the batch when a_shared != 0). */
int mtsac_debug_gemm(int precision, int kind, int epi, int batch, int M, int N, int K, const float* A, int lda, int a_shared,
                     const float* B, int ldb, float* C, int ldc, const float* bias, const float* mask, int ldm,
                     float* db);

#ifdef __cplusplus
}
#endif
#endif
