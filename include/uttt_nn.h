/*
 * uttt_nn.h — C ABI of the DualNetwork leaf-evaluator kernels (dual_network.py:89-121,
 * inference form: BatchNorm folded into each convolution, activations NHWC f32,
 * 128 channels): stem, residual-tower convolutions (Winograd F(3x3,3x3) on the
 * matrix cores) and the two heads. Every kernel computes each board from that
 * board's inputs only, so outputs do not depend on batch size or composition.
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

/* Stem from the engine's pending leaves (slot order, after uttt_search_select, or after
 * uttt_search_select_async with the count read on the device):
 * out[n][81][128] = relu(conv3x3(planes, w) + b) with w[27][128] = folded
 * conv_input weight laid out [in_plane*9 + ky*3 + kx][out_channel]
 * (dual_network.py:89-92; planes of uttt_game.cpp:244-280). Engine stream. */
int uttt_nn_stem(uttt_engine_t *eng, const float *w, const float *b, float *out);
/* The same stem from n packed states (any states, e.g. the uttt_cpp.State objects of a
 * pv_mcts_scores flush), on `stream`. */
int uttt_nn_stem_states(const uttt_state_t *states, int32_t n, const float *w, const float *b, float *out,
                        void *stream);
/* Policy softmax (n,81) (logits if softmax == 0) and tanh value (n) from the final
 * activation (n,81,128) (dual_network.py:106-121). */
int uttt_nn_heads(const float *act, const float *head_weights, int32_t n, float *policy, float *value,
                  int32_t softmax, void *stream);
/* The same for a device-resident count *n_dev <= max_n (uttt_search_select_async): the grid is
 * sized for max_n and rows past *n_dev are not touched. */
int uttt_nn_heads_dev(const float *act, const float *head_weights, const int32_t *n_dev, int32_t max_n,
                      float *policy, float *value, int32_t softmax, void *stream);

/* Residual-tower 3x3 conv (128->128, pad 1, 9x9 boards) + bias (+ residual) + ReLU as one
 * Winograd F(3x3,3x3) kernel (csrc/wino3h_conv.hip; dual_network.py:28-45): a 9x9 board is
 * exactly 3x3 tiles of 3x3 outputs, 25 transform points (Toom-Cook on {0,1,-1,2,inf}). The point
 * GEMMs run on the f16 matrix cores at f32-level accuracy: V and U are each split into f16
 * hi + lo halves (power-of-two scaled into f16 range) and M = Vhi Uhi + Vhi Ulo + Vlo Uhi
 * accumulates in f32. x, residual, y: [n_boards][81][128] NHWC; y must not alias x or residual.
 * uttt_nn_wino3h_weights: U = G g G^T (host, double) of a folded conv weight w[128 co][128 ci][3][3];
 * u receives 25*128*128*2 f16 (hi, lo) in the kernel's A-fragment order
 * U[xi][ci/32][hi|lo][co/16][(ci%32)/8][co%16][ci%8], *u_scale the power of two U was scaled by.
 * uttt_nn_conv3x3_wino3h: V is scaled per board, so a board's outputs depend on its own inputs only.
 * x_amax (required): max|x| as u32 float bits, one per board when x_amax_per_board != 0 (e.g. the
 * y_amax row of the conv that produced x), else one bound x_amax[0] for every board (the stem).
 * y_amax (optional): receives max(y) of each board by atomic max (the row must be zero on entry).
 * amax_clear (optional): the kernel zeroes amax_clear[0 .. clear_count), for a later conv's y_amax;
 * it must not be x_amax or y_amax. */
int uttt_nn_wino3h_weights(const float *w, uint16_t *u, float *u_scale);
int uttt_nn_conv3x3_wino3h(const float *x, const uint16_t *u, float u_scale, const float *bias,
                           const float *residual, float *y, const uint32_t *x_amax, int32_t x_amax_per_board,
                           uint32_t *y_amax, uint32_t *amax_clear, int32_t clear_count, int32_t n_boards,
                           void *stream);
/* The same conv on min(*n_dev, max_boards) boards, the count read on the device. */
int uttt_nn_conv3x3_wino3h_dev(const float *x, const uint16_t *u, float u_scale, const float *bias,
                               const float *residual, float *y, const uint32_t *x_amax, int32_t x_amax_per_board,
                               uint32_t *y_amax, uint32_t *amax_clear, int32_t clear_count, const int32_t *n_dev,
                               int32_t max_boards, void *stream);
/* f16 mode (not f32-level; the optional fast evaluator of SURVEY §8(f) rank 1): the same conv with
 * M = Vhi Uhi alone (one f16 MFMA product instead of three, U's hi plane only), the same u buffer,
 * scales and argument meaning. Outputs within ~1e-3 relative of the f32 conv; a board's
 * outputs still depend on its own inputs only. */
int uttt_nn_conv3x3_wino3h_f16(const float *x, const uint16_t *u, float u_scale, const float *bias,
                               const float *residual, float *y, const uint32_t *x_amax, int32_t x_amax_per_board,
                               uint32_t *y_amax, uint32_t *amax_clear, int32_t clear_count, int32_t n_boards,
                               void *stream);
int uttt_nn_conv3x3_wino3h_f16_dev(const float *x, const uint16_t *u, float u_scale, const float *bias,
                                   const float *residual, float *y, const uint32_t *x_amax, int32_t x_amax_per_board,
                                   uint32_t *y_amax, uint32_t *amax_clear, int32_t clear_count, const int32_t *n_dev,
                                   int32_t max_boards, void *stream);
/* The whole residual tower (n_layers convs = 2 per block of dual_network.py:28-45, n_layers a multiple
 * of 4) as ONE persistent dataflow launch (csrc/wino3h_impl.h k_wino3t_tower): the same per-set
 * arithmetic as uttt_nn_conv3x3_wino3h, so the same output bits, on min(*n_dev, max_boards) boards
 * (n_dev may be NULL: max_boards boards). act: three [max_boards][81][128] activation buffers act_stride
 * floats apart, X_even = act, t = act + act_stride, X_odd = act + 2 act_stride; block b reads X_b
 * (X_even for even b): conv 2b: X_b -> t, conv 2b+1: t + X_b -> X_{b+1}; the final activation is
 * X_{n_layers/2} (X_even: n_layers is a multiple of 4). The stem writes X_even.
 * u_all: n_layers U buffers of uttt_nn_wino3h_weights back to back; u_scale_all[n_layers] (device);
 * bias_all[n_layers][128]. stem_amax: the stem output's one bound (u32 float bits). rows: four per-board
 * max rows of row_stride >= max_boards u32, row 0 zero on entry (left zero on exit; the per-conv
 * kernels' rotation leaves it so too). ctl: two blocks of uttt_nn_tower_ctl_words(row_stride) u32
 * launch counters, zero before the first launch; consecutive launches on one ctl alternate parity 0, 1
 * (a launch resets the other block for the next). One launch at a time per ctl. Workgroups run at most
 * UTTT_TOWER_ITEMS work items each (default 0: persistent, one workgroup per CU). */
int uttt_nn_tower_wino3h_dev(float *act, int64_t act_stride, const uint16_t *u_all, const float *u_scale_all,
                             const float *bias_all, int32_t n_layers, const uint32_t *stem_amax, uint32_t *rows,
                             int32_t row_stride, uint32_t *ctl, int32_t parity, const int32_t *n_dev,
                             int32_t max_boards, void *stream);
int32_t uttt_nn_tower_ctl_words(int32_t max_boards);
/* Small batches: the conv's 128 output channels split over 2 workgroups per set (same output bits
 * as the persistent kernel). split: -1 automatic (default: up to 28 boards), 0 or 1 never, 2 always. */
int uttt_nn_wino3h_set_split(int32_t split);
/* *amax = max(*amax, max |x[i]|) over count floats, as u32 float bits (zero *amax first). */
int uttt_nn_amax(const float *x, int64_t count, uint32_t *amax, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* UTTT_NN_H */
