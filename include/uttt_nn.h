/*
 * uttt_nn.h — C ABI of the DualNetwork leaf-evaluator kernels (dual_network.py:89-121,
 * inference form: BatchNorm folded into each convolution, activations NHWC f32,
 * 128 channels). The 3x3 128->128 convolutions themselves are computed by the
 * caller (MIOpen through PyTorch-ROCm); these kernels replace everything else.
 */
#ifndef UTTT_NN_H
#define UTTT_NN_H

#include <stdint.h>

#include "uttt_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Layout of the packed head-weight block (floats), all BN-folded:
 *   policy 1x1 conv W[2][128], b[2]; value 1x1 conv W[128], b[1];
 *   policy FC W^T[162][81] (input-major; input index = plane*81 + position, torch.flatten
 *   of NCHW), b[81]; value FC1 W^T[81][256], b[256]; value FC2 W[256], b[1]. */
#define UTTT_HEAD_PCONV_W 0
#define UTTT_HEAD_PCONV_B (UTTT_HEAD_PCONV_W + 2 * 128)
#define UTTT_HEAD_VCONV_W (UTTT_HEAD_PCONV_B + 2)
#define UTTT_HEAD_VCONV_B (UTTT_HEAD_VCONV_W + 128)
#define UTTT_HEAD_PFC_W (UTTT_HEAD_VCONV_B + 1)
#define UTTT_HEAD_PFC_B (UTTT_HEAD_PFC_W + 81 * 162)
#define UTTT_HEAD_VFC1_W (UTTT_HEAD_PFC_B + 81)
#define UTTT_HEAD_VFC1_B (UTTT_HEAD_VFC1_W + 256 * 81)
#define UTTT_HEAD_VFC2_W (UTTT_HEAD_VFC1_B + 256)
#define UTTT_HEAD_VFC2_B (UTTT_HEAD_VFC2_W + 256)
#define UTTT_HEAD_SIZE (UTTT_HEAD_VFC2_B + 1)

/* Stem from the engine's pending leaves (slot order, after uttt_search_select):
 * out[n][81][128] = relu(conv3x3(planes, w) + b) with w[27][128] = folded
 * conv_input weight laid out [in_plane*9 + ky*3 + kx][out_channel]
 * (dual_network.py:89-92; planes of uttt_game.cpp:244-280). Engine stream. */
int uttt_nn_stem(uttt_engine_t *eng, const float *w, const float *b, float *out);
/* y = relu(x + bias[c] (+ residual)) over rows x channels (NHWC); residual may be NULL
 * (ResidualBlock, dual_network.py:36-45, minus the convolutions). */
int uttt_nn_epilogue(const float *x, const float *bias, const float *residual, float *y, int64_t rows,
                     int32_t channels, void *stream);
/* Policy softmax (n,81) (logits if softmax == 0) and tanh value (n) from the final
 * activation (n,81,128) (dual_network.py:106-121). */
int uttt_nn_heads(const float *act, const float *head_weights, int32_t n, float *policy, float *value,
                  int32_t softmax, void *stream);

/* Residual-tower 3x3 conv (128->128, pad 1, 9x9 boards) + bias (+ residual) + ReLU as one
 * Winograd F(2x2,3x3) f32-MFMA kernel (csrc/wino_conv.hip). x, residual, y: [n_boards][81][128]
 * NHWC; y must not alias x or residual. u: 16*128*128 transformed weights U[xi][ci][co] = G g G^T
 * from uttt_nn_wino_weights (host) of a folded conv weight w[128 co][128 ci][3][3], stored in the
 * kernel's B-fragment order U[xi][ci/16][co][ci%2][(ci%16)/2]. */
int uttt_nn_wino_weights(const float *w, float *u);
int uttt_nn_conv3x3_wino(const float *x, const float *u, const float *bias, const float *residual, float *y,
                         int32_t n_boards, void *stream);

/* The same conv as Winograd F(3x3,3x3) (csrc/wino3_conv.hip): a 9x9 board is exactly 3x3 tiles
 * of 3x3 outputs, 25 transform points (Toom-Cook on {0,1,-1,2,inf}). u: 25*128*128 floats,
 * U[xi][ci][co] = G g G^T from uttt_nn_wino3_weights, stored as U[xi][ci/16][co][ci%4][(ci%16)/4].
 * Same argument rules as uttt_nn_conv3x3_wino. */
int uttt_nn_wino3_weights(const float *w, float *u);
int uttt_nn_conv3x3_wino3(const float *x, const float *u, const float *bias, const float *residual, float *y,
                          int32_t n_boards, void *stream);

/* The same F(3x3,3x3) conv with its point GEMMs on the f16 matrix cores at f32-level accuracy
 * (csrc/wino3h_conv.hip): V and U are each split into f16 hi + lo halves (power-of-two scaled into
 * f16 range) and M = Vhi Uhi + Vhi Ulo + Vlo Uhi accumulates in f32.
 * uttt_nn_wino3h_weights: u receives 25*128*128*2 f16 (hi, lo) in the kernel's B-fragment order
 * U[xi][ci/32][hi|lo][co][(ci%32)/8][ci%8], *u_scale the power of two U was scaled by.
 * uttt_nn_conv3x3_wino3h: x_amax (required) points at max|x| as u32 float bits (e.g. from
 * uttt_nn_amax, or the y_amax of the conv that produced x); y_amax (optional) receives
 * max(y) by atomic max (the caller zeroes it). Other rules as uttt_nn_conv3x3_wino. */
int uttt_nn_wino3h_weights(const float *w, uint16_t *u, float *u_scale);
int uttt_nn_conv3x3_wino3h(const float *x, const uint16_t *u, float u_scale, const float *bias,
                           const float *residual, float *y, const uint32_t *x_amax, uint32_t *y_amax,
                           int32_t n_boards, void *stream);
/* *amax = max(*amax, max |x[i]|) over count floats, as u32 float bits (zero *amax first). */
int uttt_nn_amax(const float *x, int64_t count, uint32_t *amax, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* UTTT_NN_H */
