// wino3h_conv.hip — the residual tower's 3x3 convolution (dual_network.py:28-45,
// 128 -> 128 channels on 9x9 boards) as Winograd F(3x3, 3x3) whose point GEMMs
// run on the f16 matrix cores with f32-level accuracy (split-f16 products).
//
// Same algorithm as wino3_conv.hip (Toom-Cook points {0, 1, -1, 2, inf}: V =
// B^T d B, M = V (.) U per point, Y = A^T M A), different arithmetic for M:
// every operand is split into two f16 halves, v = v_hi + v_lo (v_hi = v rounded
// to f16, v_lo = the remainder rounded to f16: 21-22 significant bits), and
//
//   M = V_hi U_hi + V_hi U_lo + V_lo U_hi     (each product exact in f32,
//                                              accumulated in f32 by the MFMA)
//
// i.e. three v_mfma_f32_16x16x32_f16 per 32-channel k-step where the f32 form
// needs eight v_mfma_f32_16x16x4_f32 per 16 channels: 16.5 against 32 cycles
// per instruction on gfx950 (tools/diag/mfma_rate.hip), 5.2x fewer MFMA cycles
// per MAC. The dropped V_lo U_lo term is ~2^-22 relative (both splits round to nearest). To keep both halves
// in f16's range, V is scaled by a power of two sv chosen PER BOARD from that
// board's input maximum (|V| <= 36 max|x|, so 36 max|x| sv <= 2^15) and U by su
// from its own maximum (host); the epilogue multiplies each tile's results by
// 1/(sv su) of its board (exact). A board's outputs therefore depend on that
// board's inputs only, never on the other boards of the batch (the evaluation
// cache replays outputs across forwards, engine.hip). The per-board maxima come
// from the producer: every conv's epilogue atomically maxes its outputs into a
// u32 slot per board (the stem output uses one weight-derived bound for all
// boards), so no extra pass is needed. Error against an f64 direct conv:
// DESIGN.md §5.
//
// Workgroup = 8 waves, one set = 32 tile slots x 128 output channels; wave w owns
// channels 16w..16w+15. The 63 tiles of 7 consecutive boards are two sets (tiles
// 0-31: boards 0-3; tiles 32-62: boards 3-6), so 63 of 64 MFMA rows carry a tile, and
// a set's inputs are 4 boards staged per chunk in rows of 10 (one zero column shared
// by neighbouring rows) under shared zero rows: every 5x5 window reads its zero
// border from the layout. Per 32-channel chunk: all waves transform (one tile x
// channel-pair item per thread, split to f16 hi/lo, into LDS in fragment order),
// barrier, then all waves run the 25 point GEMMs M^T = U^T V^T (U fragments from
// L2 a few points ahead as the A operand, V from LDS as the B operand, so a lane's
// four results are four consecutive output channels of one tile) with the previous
// point's fold (S[a][v] += A^T[a][u] M) spread over the next point's MFMAs (points
// u = 0 and 4 accumulate into S on the MFMA itself); the
// next chunk's inputs are in flight meanwhile. Y = S A after a set's last chunk,
// then scale, bias, residual, ReLU, and one 16-byte store per output position
// straight from registers, output max.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "uttt_nn.h"
#include "wino3h_impl.h"

namespace uttt {
void set_error(const char *fmt, ...);
}

namespace uttt {
namespace wino3h {
// |x| maximum into *amax (u32 float bits; the caller zeroes it first)
__global__ __launch_bounds__(256) void k_amax(const float *__restrict__ x, int64_t count, uint32_t *__restrict__ amax) {
    float m = 0.0f;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < count; i += (int64_t)gridDim.x * 256)
        m = fmaxf(m, fabsf(x[i]));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
    if ((threadIdx.x & 63) == 0) atomicMax(amax, __builtin_bit_cast(uint32_t, m));
}

}  // namespace wino3h
}  // namespace uttt

using namespace uttt;

extern "C" {

int uttt_nn_wino3h_weights(const float *w, uint16_t *u, float *u_scale) {
    // U[xi=(p,q)][ci][co] = (G g G^T)[p][q] in double, scaled by su = 2^k (max |U| su <= 2^15),
    // split hi = f16(U su) (round to nearest), lo = f16(U su - hi), stored as
    // U[xi][ci/32][hi|lo][co/16][(ci%32)/8][co%16][ci%8] (the kernel's A-fragment order)
    if (!w || !u || !u_scale) {
        set_error("uttt_nn_wino3h_weights: null pointer");
        return UTTT_ERR_ARG;
    }
    static const double G[5][3] = {{0.5, 0, 0},
                                   {-0.5, -0.5, -0.5},
                                   {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                                   {1.0 / 6, 1.0 / 3, 2.0 / 3},
                                   {0, 0, 1}};
    using namespace wino3h;
    double *U = new double[(size_t)NP * C * C];
    double umax = 0.0;
    for (int co = 0; co < C; ++co)
        for (int ci = 0; ci < C; ++ci) {
            const float *g = w + ((size_t)co * C + ci) * 9;
            double tg[5][3];
            for (int p = 0; p < 5; ++p)
                for (int k = 0; k < 3; ++k)
                    tg[p][k] = G[p][0] * g[0 * 3 + k] + G[p][1] * g[1 * 3 + k] + G[p][2] * g[2 * 3 + k];
            for (int p = 0; p < 5; ++p)
                for (int q = 0; q < 5; ++q) {
                    const double v = tg[p][0] * G[q][0] + tg[p][1] * G[q][1] + tg[p][2] * G[q][2];
                    U[((size_t)(p * 5 + q) * C + ci) * C + co] = v;
                    umax = fabs(v) > umax ? fabs(v) : umax;
                }
        }
    if (!std::isfinite(umax)) {
        delete[] U;
        set_error("uttt_nn_wino3h_weights: non-finite weights");
        return UTTT_ERR_ARG;
    }
    int e = 0;
    if (umax > 0.0) {
        frexp(umax, &e);  // 2^(e-1) <= umax < 2^e
        e = 15 - e;
    }
    const double su = ldexp(1.0, e);
    for (int xi = 0; xi < NP; ++xi)
        for (int ci = 0; ci < C; ++ci)
            for (int co = 0; co < C; ++co) {
                const double v = U[((size_t)xi * C + ci) * C + co] * su;
                const _Float16 hi = (_Float16)v;
                const _Float16 lo = (_Float16)(v - (double)hi);
                // lane (co % 16, kq) of wave co / 16 reads 16 bytes at wave * 1 KB + lane * 16:
                // lane-linear, 1.6x the per-CU rate of the permuted order (tools/diag/u_stream.hip)
                const size_t o = ((size_t)xi * NCH + ci / KC) * 2 * C * 32 +
                                 ((((co / 16) * 4 + (ci % KC) / 8) * 16 + co % 16) * 8 + ci % 8);
                u[o] = __builtin_bit_cast(uint16_t, hi);
                u[o + C * 4 * 8] = __builtin_bit_cast(uint16_t, lo);
            }
    delete[] U;
    *u_scale = (float)su;
    return UTTT_OK;
}

static int conv3x3_wino3h(const float *x, const uint16_t *u, float u_scale, const float *bias, const float *residual,
                          float *y, const uint32_t *x_amax, int32_t x_amax_per_board, uint32_t *y_amax,
                          uint32_t *amax_clear, int32_t clear_count, int32_t n_boards, const int32_t *n_dev,
                          void *stream, bool f16 = false) {
    if (!x || !u || !bias || !y || !x_amax || n_boards < 0 || x == y || (residual && residual == y) ||
        !(u_scale > 0.0f) || clear_count < 0 || (clear_count > 0 && !amax_clear) ||
        (amax_clear && (amax_clear == y_amax || amax_clear == x_amax))) {
        set_error("uttt_nn_conv3x3_wino3h: bad arguments (x_amax required; output must not alias input or residual; "
                  "the cleared max row must differ from x_amax and y_amax)");
        return UTTT_ERR_ARG;
    }
    if (n_boards == 0 && clear_count == 0) return UTTT_OK;
    const int pb = x_amax_per_board ? 1 : 0;
    const int split = wino3h::split_for(n_boards > 0 ? n_boards : 1);
    if (split > 1) {
        const dim3 sgrid((unsigned)(wino3h::n_sets(n_boards > 0 ? n_boards : 1) * split));
        const hipStream_t s = (hipStream_t)stream;
#define UTTT_WINO3S(RES, SP, R, M)                                                                                 \
    hipLaunchKernelGGL((wino3h::k_wino3s_conv<RES, SP, 3, M>), sgrid, dim3(64 * (8 / SP)), 0, s, x, u, u_scale, bias, R, \
                       y, x_amax, pb, y_amax, amax_clear, clear_count, n_boards, n_dev)
        if (f16) {
            if (residual) UTTT_WINO3S(true, 2, residual, wino3h::kF16);
            else UTTT_WINO3S(false, 2, nullptr, wino3h::kF16);
        } else {
            if (residual) UTTT_WINO3S(true, 2, residual, 0);
            else UTTT_WINO3S(false, 2, nullptr, 0);
        }
#undef UTTT_WINO3S
        hipError_t r = hipGetLastError();
        if (r != hipSuccess) {
            set_error("k_wino3s_conv launch: %s", hipGetErrorString(r));
            return UTTT_ERR_HIP;
        }
        return UTTT_OK;
    }
    const dim3 grid(wino3h::grid_size(n_boards > 0 ? n_boards : 1));
    const hipStream_t st = (hipStream_t)stream;
    using wino3h::k_wino3h_conv;
    if (f16) {
        if (residual)
            hipLaunchKernelGGL((k_wino3h_conv<true, wino3h::kF16>), grid, dim3(wino3h::NT), 0, st, x, u, u_scale, bias,
                               residual, y, x_amax, pb, y_amax, amax_clear, clear_count, n_boards, n_dev);
        else
            hipLaunchKernelGGL((k_wino3h_conv<false, wino3h::kF16>), grid, dim3(wino3h::NT), 0, st, x, u, u_scale, bias,
                               nullptr, y, x_amax, pb, y_amax, amax_clear, clear_count, n_boards, n_dev);
    } else if (residual) {
        hipLaunchKernelGGL(k_wino3h_conv<true>, grid, dim3(wino3h::NT), 0, st, x, u, u_scale, bias, residual, y, x_amax,
                           pb, y_amax, amax_clear, clear_count, n_boards, n_dev);
    } else {
        hipLaunchKernelGGL(k_wino3h_conv<false>, grid, dim3(wino3h::NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax,
                           pb, y_amax, amax_clear, clear_count, n_boards, n_dev);
    }
    hipError_t r = hipGetLastError();
    if (r != hipSuccess) {
        set_error("k_wino3h_conv launch: %s", hipGetErrorString(r));
        return UTTT_ERR_HIP;
    }
    return UTTT_OK;
}

int uttt_nn_conv3x3_wino3h(const float *x, const uint16_t *u, float u_scale, const float *bias, const float *residual,
                           float *y, const uint32_t *x_amax, int32_t x_amax_per_board, uint32_t *y_amax,
                           uint32_t *amax_clear, int32_t clear_count, int32_t n_boards, void *stream) {
    return conv3x3_wino3h(x, u, u_scale, bias, residual, y, x_amax, x_amax_per_board, y_amax, amax_clear, clear_count,
                          n_boards, nullptr, stream);
}

int uttt_nn_conv3x3_wino3h_dev(const float *x, const uint16_t *u, float u_scale, const float *bias,
                               const float *residual, float *y, const uint32_t *x_amax, int32_t x_amax_per_board,
                               uint32_t *y_amax, uint32_t *amax_clear, int32_t clear_count, const int32_t *n_dev,
                               int32_t max_boards, void *stream) {
    if (!n_dev) {
        set_error("uttt_nn_conv3x3_wino3h_dev: n_dev required");
        return UTTT_ERR_ARG;
    }
    return conv3x3_wino3h(x, u, u_scale, bias, residual, y, x_amax, x_amax_per_board, y_amax, amax_clear, clear_count,
                          max_boards, n_dev, stream);
}

int uttt_nn_conv3x3_wino3h_f16(const float *x, const uint16_t *u, float u_scale, const float *bias,
                               const float *residual, float *y, const uint32_t *x_amax, int32_t x_amax_per_board,
                               uint32_t *y_amax, uint32_t *amax_clear, int32_t clear_count, int32_t n_boards,
                               void *stream) {
    return conv3x3_wino3h(x, u, u_scale, bias, residual, y, x_amax, x_amax_per_board, y_amax, amax_clear, clear_count,
                          n_boards, nullptr, stream, true);
}

int uttt_nn_conv3x3_wino3h_f16_dev(const float *x, const uint16_t *u, float u_scale, const float *bias,
                                   const float *residual, float *y, const uint32_t *x_amax, int32_t x_amax_per_board,
                                   uint32_t *y_amax, uint32_t *amax_clear, int32_t clear_count, const int32_t *n_dev,
                                   int32_t max_boards, void *stream) {
    if (!n_dev) {
        set_error("uttt_nn_conv3x3_wino3h_f16_dev: n_dev required");
        return UTTT_ERR_ARG;
    }
    return conv3x3_wino3h(x, u, u_scale, bias, residual, y, x_amax, x_amax_per_board, y_amax, amax_clear, clear_count,
                          max_boards, n_dev, stream, true);
}

int uttt_nn_tower_wino3h_dev(float *act, int64_t act_stride, const uint16_t *u_all, const float *u_scale_all,
                             const float *bias_all, int32_t n_layers, const uint32_t *stem_amax, uint32_t *rows,
                             int32_t row_stride, uint32_t *ctl, int32_t parity, const int32_t *n_dev,
                             int32_t max_boards, void *stream) {
    if (!act || act_stride < (int64_t)max_boards * 81 * 128 || !u_all || !u_scale_all || !bias_all || !stem_amax ||
        !rows || !ctl || n_layers <= 0 || n_layers % 4 != 0 || max_boards < 0 || row_stride < max_boards ||
        (parity != 0 && parity != 1)) {
        set_error("uttt_nn_tower_wino3h_dev: bad arguments (three activation buffers of max_boards boards act_stride "
                  "floats apart, n_layers a positive multiple of 4, row_stride >= max_boards, parity 0 or 1)");
        return UTTT_ERR_ARG;
    }
    if (max_boards == 0) return UTTT_OK;
    // items per workgroup (UTTT_TOWER_ITEMS; 0: one persistent workgroup per CU, every item)
    static int items = -1, cus = 0;
    if (items < 0) {
        const char *e = getenv("UTTT_TOWER_ITEMS");
        items = (e && *e) ? atoi(e) : 0;
        if (items < 0) items = 0;
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        // persistent workgroups (items 0): UTTT_TOWER_CUS of them (default every CU; fewer leave CUs to the
        // other lane's kernels)
        const char *g = getenv("UTTT_TOWER_CUS");
        if (g && *g && atoi(g) > 0 && atoi(g) < cus) cus = atoi(g);
    }
    const int max_items = n_layers * wino3h::n_sets(max_boards);
    int per = items, wgs;
    if (per == 0) {
        wgs = max_items < cus ? max_items : cus;
        per = 1 << 30;
    } else {
        wgs = (max_items + per - 1) / per;
    }
    hipLaunchKernelGGL((wino3h::k_wino3t_tower<wino3h::kHandoff>), dim3((unsigned)wgs), dim3(wino3h::NT), 0,
                       (hipStream_t)stream, act, (int64_t)act_stride, u_all, u_scale_all, bias_all, (int)n_layers,
                       stem_amax, rows, (int)row_stride, ctl, (int)uttt_nn_tower_ctl_words(row_stride), (int)parity, per,
                       (int)max_boards, n_dev);
    hipError_t r = hipGetLastError();
    if (r != hipSuccess) {
        set_error("k_wino3t_tower launch: %s", hipGetErrorString(r));
        return UTTT_ERR_HIP;
    }
    return UTTT_OK;
}

int32_t uttt_nn_tower_ctl_words(int32_t max_boards) {
    // one block: ticket [0], items done [32], done[g] [64 + g] for ceil(max_boards / 7) groups; padded to 32
    const int32_t w = wino3h::kTowerCtlDone + (max_boards + wino3h::GB - 1) / wino3h::GB;
    return (w + 31) / 32 * 32;
}

int uttt_nn_wino3h_set_split(int32_t split) {
    if (split < -1 || split > 2) {
        set_error("uttt_nn_wino3h_set_split: split must be -1 (automatic), 0/1 (the persistent kernel) or 2");
        return UTTT_ERR_ARG;
    }
    wino3h::g_split = split;
    return UTTT_OK;
}

int uttt_nn_amax(const float *x, int64_t count, uint32_t *amax, void *stream) {
    if (!x || !amax || count < 0) {
        set_error("uttt_nn_amax: bad arguments");
        return UTTT_ERR_ARG;
    }
    if (count == 0) return UTTT_OK;
    int64_t blocks = (count + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(wino3h::k_amax, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, x, count, amax);
    hipError_t r = hipGetLastError();
    if (r != hipSuccess) {
        set_error("k_amax launch: %s", hipGetErrorString(r));
        return UTTT_ERR_HIP;
    }
    return UTTT_OK;
}

}  // extern "C"
