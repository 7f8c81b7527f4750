// nn_kernels.hip — the DualNetwork leaf evaluator's non-GEMM parts on gfx950
// (dual_network.py:89-121 with BatchNorm folded into the convolutions; NHWC f32):
//
//   k_stem      leaf bitboards -> relu(conv3x3(3->128) + b), written NHWC. The input
//               planes (own, opponent, legal; uttt_game.cpp:244-280) are 0/1, so the
//               conv is a masked sum of 27 weight rows; no NCHW tensor is built.
//   k_heads     1x1 convs (128->2, 128->1) + ReLU, policy FC 162->81 + softmax,
//               value FC 81->256 + ReLU + FC 256->1 + tanh: one position per workgroup.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "uttt_bits.h"
#include "uttt_engine.h"
#include "uttt_nn.h"

namespace uttt {

void set_error(const char *fmt, ...);
int engine_pending_view(uttt_engine_t *e, const uttt_state_t **leaf, const int32_t **tree_of, int32_t *n,
                        const int32_t **n_dev, int32_t *max_n, hipStream_t *stream);

namespace nn {

constexpr int C = 128;  // DN_FILTERS

// out[s][pos][c] = relu(b[c] + sum_{ch,ky,kx} w[ch*9+ky*3+kx][c] * in_ch(R+ky-1, C+kx-1))
// SB leaves per workgroup: the 27x128 weights go to LDS once for all of them, and
// per (leaf, output position) the 27-bit mask of set input taps; then each thread
// sums the weight rows of the set taps for (leaf, position, 4 channels) items and
// stores float4s (a wave covers two positions: little divergence in the tap loop).
constexpr int SB = 2;  // round 5: 4 -> 2 (a 1,370-leaf launch is 685 workgroups, at most 6 leaves per CU instead of 8)
__device__ __forceinline__ uint32_t bit3(uint32_t w0, uint32_t w1, uint32_t w2, int a) {
    // bit a of a 81-bit board held in three 27-bit words, without indexing an array
    // (a dynamically indexed local array lands in scratch memory)
    const uint32_t w = a < 27 ? w0 : (a < 54 ? w1 : w2);
    return (w >> (a % 27)) & 1u;
}
__global__ __launch_bounds__(256) void k_stem(const uttt_state_t *__restrict__ leaf, const int32_t *__restrict__ tree_of,
                                              int n, const int32_t *__restrict__ n_dev, const float *__restrict__ w,
                                              const float *__restrict__ b, float *__restrict__ out) {
    __shared__ float4 s_w[27 * (C / 4)];
    __shared__ uint32_t s_mask[SB * 81];
    const int s0 = blockIdx.x * SB;
    if (n_dev) n = min(n, *n_dev);  // the count k_scan left on the device (grid sized for the maximum n)
    if (s0 >= n) return;
    const int nb = n - s0 < SB ? n - s0 : SB;
    const int t = threadIdx.x;
    for (int i = t; i < 27 * (C / 4); i += 256) s_w[i] = reinterpret_cast<const float4 *>(w)[i];
    for (int i = t; i < nb * 81; i += 256) {
        const uttt_state_t s = leaf[tree_of ? tree_of[s0 + i / 81] : s0 + i / 81];
        uint32_t lm[3];
        legal_mask(s, lm);
        const int pos = i % 81, R = pos / 9, Cc = pos % 9;
        uint32_t m = 0u;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
                const int r = R + ky - 1, c = Cc + kx - 1;
                if (r < 0 || r > 8 || c < 0 || c > 8) continue;
                const int a = action_at(r * 9 + c), tap = ky * 3 + kx;
                m |= bit3(s.own[0], s.own[1], s.own[2], a) << tap;
                m |= bit3(s.opp[0], s.opp[1], s.opp[2], a) << (9 + tap);
                m |= bit3(lm[0], lm[1], lm[2], a) << (18 + tap);
            }
        s_mask[i] = m;
    }
    __syncthreads();
    constexpr int CG = C / 4;
    float4 *o = reinterpret_cast<float4 *>(out) + (size_t)s0 * 81 * CG;
    const float4 bias = reinterpret_cast<const float4 *>(b)[t % CG];  // 256 % CG == 0: fixed per thread
    for (int i = t; i < nb * 81 * CG; i += 256) {
        const int cg = i % CG;
        float4 acc = bias;
        for (uint32_t m = s_mask[i / CG]; m; m &= m - 1u) {
            const float4 wv = s_w[__builtin_ctz(m) * CG + cg];
            acc.x += wv.x;
            acc.y += wv.y;
            acc.z += wv.z;
            acc.w += wv.w;
        }
        acc.x = fmaxf(acc.x, 0.0f);
        acc.y = fmaxf(acc.y, 0.0f);
        acc.z = fmaxf(acc.z, 0.0f);
        acc.w = fmaxf(acc.w, 0.0f);
        o[i] = acc;
    }
}

// Head weight block (uttt_nn.h UTTT_HEAD_*): folded 1x1 convs, then the FC layers with
// their weights stored input-major (consecutive threads = consecutive outputs read
// consecutive floats). The two FC weight matrices (132 KB) are staged in LDS once per
// workgroup and shared by its HB boards: with HB = 1 every board streamed them from L2 in
// chains of dependent loads (84 us for 1,380 boards in the bench, round 3). Each board's
// arithmetic - order of every sum included - is the same for any HB.
constexpr int HB = 8;
constexpr int HT = 1024;  // threads: 1x1 convs in 64 groups of 16 lanes, FC1 as 4 board groups x 256 units
__global__ __launch_bounds__(HT) void k_heads(const float *__restrict__ act, const float *__restrict__ hw, int n,
                                              const int32_t *__restrict__ n_dev, float *__restrict__ policy,
                                              float *__restrict__ value, int softmax) {
    __shared__ float s_pw[162 * 81];   // policy FC W^T [162][81]
    __shared__ float s_w1[81 * 256];   // value FC1 W^T [81][256]
    __shared__ float s_h[HB][3 * 81];  // relu(1x1 conv): [p0 | p1 | v] x 81 (NCHW flatten order)
    __shared__ float s_z[HB][81];      // policy logits
    __shared__ float s_v[HB][4];       // value FC2 partial sums, one per 64 units
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int b0 = blockIdx.x * HB;
    if (n_dev) n = min(n, *n_dev);
    if (b0 >= n) return;
    const int nb = n - b0 < HB ? n - b0 : HB;
#pragma unroll 4
    for (int i = t; i < 162 * 81; i += HT) s_pw[i] = hw[UTTT_HEAD_PFC_W + i];
#pragma unroll 4
    for (int i = t; i < 81 * 256; i += HT) s_w1[i] = hw[UTTT_HEAD_VFC1_W + i];
    // 1x1 convs (128 -> 2 policy planes, 128 -> 1 value plane) + ReLU: 16 lanes per
    // (position, board), 8 channels per lane, 16-lane shuffle reduction
    {
        const int g = t & 15;
        float w0[8], w1[8], w2[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            w0[k] = hw[UTTT_HEAD_PCONV_W + 8 * g + k];
            w1[k] = hw[UTTT_HEAD_PCONV_W + C + 8 * g + k];
            w2[k] = hw[UTTT_HEAD_VCONV_W + 8 * g + k];
        }
        const float c0 = hw[UTTT_HEAD_PCONV_B], c1 = hw[UTTT_HEAD_PCONV_B + 1], c2 = hw[UTTT_HEAD_VCONV_B];
        for (int i = t >> 4; i < nb * 81; i += HT / 16) {
            const float4 *src = reinterpret_cast<const float4 *>(act + ((size_t)b0 * 81 + i) * C + 8 * g);
            const float4 xa = src[0], xb = src[1];
            const float x[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
            float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                a0 += w0[k] * x[k];
                a1 += w1[k] * x[k];
                a2 += w2[k] * x[k];
            }
#pragma unroll
            for (int off = 8; off > 0; off >>= 1) {
                a0 += __shfl_xor(a0, off);
                a1 += __shfl_xor(a1, off);
                a2 += __shfl_xor(a2, off);
            }
            if (g == 0) {
                const int bi = i / 81, pos = i % 81;
                s_h[bi][pos] = fmaxf(a0 + c0, 0.0f);
                s_h[bi][81 + pos] = fmaxf(a1 + c1, 0.0f);
                s_h[bi][162 + pos] = fmaxf(a2 + c2, 0.0f);
            }
        }
    }
    __syncthreads();
    // value FC1 (81 -> 256) + ReLU: unit u = t % 256 of boards q, q + 4 (q = t / 256); FC2
    // (256 -> 1) partial sums per 64 units, combined in the same order for every board
    {
        const int u = t & 255, q = t >> 8;
        constexpr int BQ = HB / 4;
        float acc[BQ];
        const float bt = hw[UTTT_HEAD_VFC1_B + u];
#pragma unroll
        for (int r = 0; r < BQ; ++r) acc[r] = bt;
#pragma unroll 9
        for (int j = 0; j < 81; ++j) {
            const float wj = s_w1[j * 256 + u];
#pragma unroll
            for (int r = 0; r < BQ; ++r) acc[r] += wj * s_h[q + 4 * r][162 + j];
        }
        const float w2 = hw[UTTT_HEAD_VFC2_W + u];
#pragma unroll
        for (int r = 0; r < BQ; ++r) {
            float v = w2 * fmaxf(acc[r], 0.0f);
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
            if (lane == 0) s_v[q + 4 * r][u >> 6] = v;
        }
    }
    // policy FC (162 -> 81): thread t < 81 * HB = output t % 81 of board t / 81
    if (t < 81 * HB) {
        const int o = t % 81, bi = t / 81;
        float z = hw[UTTT_HEAD_PFC_B + o];
#pragma unroll 9
        for (int j = 0; j < 162; ++j) z += s_pw[j * 81 + o] * s_h[bi][j];
        s_z[bi][o] = z;
    }
    __syncthreads();
    if (t < nb) value[b0 + t] = tanhf(((s_v[t][0] + s_v[t][1]) + (s_v[t][2] + s_v[t][3])) + hw[UTTT_HEAD_VFC2_B]);
    // softmax over the 81 logits of a board: one wave per board, lanes hold z[lane], z[lane + 64]
    for (int bi = wv; bi < nb; bi += HT / 64) {
        float *po = policy + (size_t)(b0 + bi) * 81;
        const bool two = lane + 64 < 81;
        const float z0 = s_z[bi][lane], z1 = two ? s_z[bi][lane + 64] : -INFINITY;
        if (!softmax) {  // logits (tests compare them: the random-init net's softmax is saturated)
            po[lane] = z0;
            if (two) po[lane + 64] = z1;
            continue;
        }
        float m = fmaxf(z0, z1);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
        const float e0 = expf(z0 - m), e1 = two ? expf(z1 - m) : 0.0f;
        float sum = e0 + e1;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off);
        po[lane] = e0 / sum;
        if (two) po[lane + 64] = e1 / sum;
    }
}

}  // namespace nn
}  // namespace uttt

using namespace uttt;

extern "C" {

int uttt_nn_stem(uttt_engine_t *e, const float *w, const float *b, float *out) {
    const uttt_state_t *leaf;
    const int32_t *tree_of, *n_dev;
    int32_t n, max_n;
    hipStream_t st;
    int rc = engine_pending_view(e, &leaf, &tree_of, &n, &n_dev, &max_n, &st);
    if (rc) return rc;
    if (!w || !b || !out) {
        set_error("uttt_nn_stem: null pointer");
        return UTTT_ERR_ARG;
    }
    if (n_dev) n = max_n;  // count on the device: grid for every tree, the kernel reads the count
    if (n == 0) return UTTT_OK;
    hipLaunchKernelGGL(nn::k_stem, dim3((n + nn::SB - 1) / nn::SB), dim3(256), 0, st, leaf, tree_of, n, n_dev, w, b,
                       out);
    hipError_t r = hipGetLastError();
    if (r != hipSuccess) {
        set_error("k_stem launch: %s", hipGetErrorString(r));
        return UTTT_ERR_HIP;
    }
    return UTTT_OK;
}

int uttt_nn_stem_states(const uttt_state_t *states, int32_t n, const float *w, const float *b, float *out,
                        void *stream) {
    if (!states || !w || !b || !out || n < 0) {
        set_error("uttt_nn_stem_states: bad arguments");
        return UTTT_ERR_ARG;
    }
    if (n == 0) return UTTT_OK;
    hipLaunchKernelGGL(nn::k_stem, dim3((n + nn::SB - 1) / nn::SB), dim3(256), 0, (hipStream_t)stream, states, nullptr, n,
                       (const int32_t *)nullptr, w, b, out);
    hipError_t r = hipGetLastError();
    if (r != hipSuccess) {
        set_error("k_stem launch: %s", hipGetErrorString(r));
        return UTTT_ERR_HIP;
    }
    return UTTT_OK;
}

int uttt_nn_heads(const float *act, const float *head_weights, int32_t n, float *policy, float *value, int32_t softmax,
                  void *stream) {
    if (!act || !head_weights || !policy || !value || n < 0) {
        set_error("uttt_nn_heads: bad arguments");
        return UTTT_ERR_ARG;
    }
    if (n == 0) return UTTT_OK;
    hipLaunchKernelGGL(nn::k_heads, dim3((n + nn::HB - 1) / nn::HB), dim3(nn::HT), 0, (hipStream_t)stream, act, head_weights, n,
                       (const int32_t *)nullptr, policy, value, softmax ? 1 : 0);
    hipError_t r = hipGetLastError();
    if (r != hipSuccess) {
        set_error("k_heads launch: %s", hipGetErrorString(r));
        return UTTT_ERR_HIP;
    }
    return UTTT_OK;
}

int uttt_nn_heads_dev(const float *act, const float *head_weights, const int32_t *n_dev, int32_t max_n, float *policy,
                      float *value, int32_t softmax, void *stream) {
    if (!act || !head_weights || !n_dev || !policy || !value || max_n < 0) {
        set_error("uttt_nn_heads_dev: bad arguments");
        return UTTT_ERR_ARG;
    }
    if (max_n == 0) return UTTT_OK;
    hipLaunchKernelGGL(nn::k_heads, dim3((max_n + nn::HB - 1) / nn::HB), dim3(nn::HT), 0, (hipStream_t)stream, act,
                       head_weights, max_n, n_dev, policy, value, softmax ? 1 : 0);
    hipError_t r = hipGetLastError();
    if (r != hipSuccess) {
        set_error("k_heads launch: %s", hipGetErrorString(r));
        return UTTT_ERR_HIP;
    }
    return UTTT_OK;
}

}  // extern "C"
