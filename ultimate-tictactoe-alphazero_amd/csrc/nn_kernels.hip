// nn_kernels.hip — the DualNetwork leaf evaluator's non-GEMM parts on gfx950
// (dual_network.py:89-121 with BatchNorm folded into the convolutions; NHWC f32):
//
//   k_stem      leaf bitboards -> relu(conv3x3(3->128) + b), written NHWC. The input
//               planes (own, opponent, legal; uttt_game.cpp:244-280) are 0/1, so the
//               conv is a masked sum of 27 weight rows; no NCHW tensor is built.
//   k_epilogue  relu(conv + b [+ residual]) in one pass (MIOpen computes the bare conv).
//   k_heads     1x1 convs (128->2, 128->1) + ReLU, policy FC 162->81 + softmax,
//               value FC 81->256 + ReLU + FC 256->1 + tanh: one workgroup per position.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "uttt_bits.h"
#include "uttt_engine.h"
#include "uttt_nn.h"

namespace uttt {

void set_error(const char *fmt, ...);
int engine_pending_view(uttt_engine_t *e, const uttt_state_t **leaf, const int32_t **tree_of, int32_t *n,
                        hipStream_t *stream);

namespace nn {

constexpr int C = 128;  // DN_FILTERS

// out[s][pos][c] = relu(b[c] + sum_{ch,ky,kx} w[ch*9+ky*3+kx][c] * in_ch(R+ky-1, C+kx-1))
// One workgroup per leaf: the 27x128 weights and, per output position, the
// 27-bit mask of set input taps go to LDS; then each thread sums the weight
// rows of the set taps for (position, 4 channels) items and stores float4s.
__global__ __launch_bounds__(256) void k_stem(const uttt_state_t *__restrict__ leaf, const int32_t *__restrict__ tree_of,
                                              int n, const float *__restrict__ w, const float *__restrict__ b,
                                              float *__restrict__ out) {
    __shared__ float4 s_w[27 * (C / 4)];
    __shared__ uint32_t s_mask[81];
    const int slot = blockIdx.x;
    const int t = threadIdx.x;
    for (int i = t; i < 27 * (C / 4); i += 256) s_w[i] = reinterpret_cast<const float4 *>(w)[i];
    if (t < 81) {
        const uttt_state_t s = leaf[tree_of[slot]];
        uint32_t lm[3];
        legal_mask(s, lm);
        const int R = t / 9, Cc = t % 9;
        uint32_t m = 0u;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
                const int r = R + ky - 1, c = Cc + kx - 1;
                if (r < 0 || r > 8 || c < 0 || c > 8) continue;
                const int a = action_at(r * 9 + c), tap = ky * 3 + kx;
                m |= bit_of(s.own, a) << tap;
                m |= bit_of(s.opp, a) << (9 + tap);
                m |= bit_of(lm, a) << (18 + tap);
            }
        s_mask[t] = m;
    }
    __syncthreads();
    constexpr int CG = C / 4;
    float4 *o = reinterpret_cast<float4 *>(out) + (size_t)slot * 81 * CG;
    for (int i = t; i < 81 * CG; i += 256) {
        const int pos = i / CG, cg = i % CG;
        float4 acc = reinterpret_cast<const float4 *>(b)[cg];
        for (uint32_t m = s_mask[pos]; m; m &= m - 1u) {
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

// y = relu(x + bias[c] (+ r)), NHWC rows of C channels, float4 per thread, grid-stride.
__global__ __launch_bounds__(256) void k_epilogue(const float *__restrict__ x, const float *__restrict__ bias,
                                                  const float *__restrict__ r, float *__restrict__ y, int64_t n4) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        float4 v = reinterpret_cast<const float4 *>(x)[i];
        const float4 bb = reinterpret_cast<const float4 *>(bias)[i % (C / 4)];
        v.x += bb.x;
        v.y += bb.y;
        v.z += bb.z;
        v.w += bb.w;
        if (r) {
            const float4 rv = reinterpret_cast<const float4 *>(r)[i];
            v.x += rv.x;
            v.y += rv.y;
            v.z += rv.z;
            v.w += rv.w;
        }
        v.x = fmaxf(v.x, 0.0f);
        v.y = fmaxf(v.y, 0.0f);
        v.z = fmaxf(v.z, 0.0f);
        v.w = fmaxf(v.w, 0.0f);
        reinterpret_cast<float4 *>(y)[i] = v;
    }
}

// Head weight block (uttt_nn.h UTTT_HEAD_*): folded 1x1 convs then the FC layers.
__global__ __launch_bounds__(256) void k_heads(const float *__restrict__ act, const float *__restrict__ hw, int n,
                                               float *__restrict__ policy, float *__restrict__ value, int softmax) {
    __shared__ float s_act[81 * (C + 1)];  // +1 pad: column reads by position stride
    __shared__ float s_h[3 * 81];          // relu(1x1 conv): [p0 | p1 | v] x 81 (NCHW flatten order)
    __shared__ float s_u[256];
    __shared__ float s_red[256];
    const int row = blockIdx.x;
    if (row >= n) return;
    const int t = threadIdx.x;
    const float *a = act + (size_t)row * 81 * C;
    for (int i = t; i < 81 * C / 4; i += 256) {
        const float4 v = reinterpret_cast<const float4 *>(a)[i];
        const int pos = (i * 4) / C, c = (i * 4) % C;
        float *d = s_act + pos * (C + 1) + c;
        d[0] = v.x;
        d[1] = v.y;
        d[2] = v.z;
        d[3] = v.w;
    }
    __syncthreads();
    if (t < 243) {
        const int o = t / 81, pos = t % 81;  // o: 0,1 policy planes, 2 value plane
        const float *wv = hw + (o < 2 ? UTTT_HEAD_PCONV_W + o * C : UTTT_HEAD_VCONV_W);
        const float bo = hw[o < 2 ? UTTT_HEAD_PCONV_B + o : UTTT_HEAD_VCONV_B];
        const float *x = s_act + pos * (C + 1);
        float acc = 0.0f;
        for (int c = 0; c < C; ++c) acc += wv[c] * x[c];
        s_h[t] = fmaxf(acc + bo, 0.0f);
    }
    __syncthreads();
    // value FC1 (81 -> 256) + ReLU
    {
        const float *w1 = hw + UTTT_HEAD_VFC1_W + t * 81;
        float acc = hw[UTTT_HEAD_VFC1_B + t];
        for (int j = 0; j < 81; ++j) acc += w1[j] * s_h[162 + j];
        s_u[t] = fmaxf(acc, 0.0f);
    }
    // policy logits (162 -> 81)
    float z = -INFINITY;
    if (t < 81) {
        const float *wp = hw + UTTT_HEAD_PFC_W + t * 162;
        float acc = hw[UTTT_HEAD_PFC_B + t];
        for (int j = 0; j < 162; ++j) acc += wp[j] * s_h[j];
        z = acc;
    }
    __syncthreads();
    // value FC2 (256 -> 1) + tanh: block reduction
    s_red[t] = hw[UTTT_HEAD_VFC2_W + t] * s_u[t];
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (t < off) s_red[t] += s_red[t + off];
        __syncthreads();
    }
    if (t == 0) value[row] = tanhf(s_red[0] + hw[UTTT_HEAD_VFC2_B]);
    if (!softmax) {  // logits (tests compare them: the random-init net's softmax is saturated)
        if (t < 81) policy[(size_t)row * 81 + t] = z;
        return;
    }
    __syncthreads();
    // softmax over 81 logits (threads 0..80 hold z; the others -inf)
    s_red[t] = z;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (t < off) s_red[t] = fmaxf(s_red[t], s_red[t + off]);
        __syncthreads();
    }
    const float zmax = s_red[0];
    __syncthreads();
    const float e = t < 81 ? expf(z - zmax) : 0.0f;
    s_red[t] = e;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (t < off) s_red[t] += s_red[t + off];
        __syncthreads();
    }
    if (t < 81) policy[(size_t)row * 81 + t] = e / s_red[0];
}

}  // namespace nn
}  // namespace uttt

using namespace uttt;

extern "C" {

int uttt_nn_stem(uttt_engine_t *e, const float *w, const float *b, float *out) {
    const uttt_state_t *leaf;
    const int32_t *tree_of;
    int32_t n;
    hipStream_t st;
    int rc = engine_pending_view(e, &leaf, &tree_of, &n, &st);
    if (rc) return rc;
    if (!w || !b || !out) {
        set_error("uttt_nn_stem: null pointer");
        return UTTT_ERR_ARG;
    }
    if (n == 0) return UTTT_OK;
    hipLaunchKernelGGL(nn::k_stem, dim3(n), dim3(256), 0, st, leaf, tree_of, n, w, b, out);
    hipError_t r = hipGetLastError();
    if (r != hipSuccess) {
        set_error("k_stem launch: %s", hipGetErrorString(r));
        return UTTT_ERR_HIP;
    }
    return UTTT_OK;
}

int uttt_nn_epilogue(const float *x, const float *bias, const float *residual, float *y, int64_t rows,
                     int32_t channels, void *stream) {
    if (!x || !bias || !y || rows < 0 || channels != nn::C) {
        set_error("uttt_nn_epilogue: bad arguments (channels must be %d)", nn::C);
        return UTTT_ERR_ARG;
    }
    const int64_t n4 = rows * channels / 4;
    if (n4 == 0) return UTTT_OK;
    int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 256 * 16);
    hipLaunchKernelGGL(nn::k_epilogue, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, bias, residual, y, n4);
    hipError_t r = hipGetLastError();
    if (r != hipSuccess) {
        set_error("k_epilogue launch: %s", hipGetErrorString(r));
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
    hipLaunchKernelGGL(nn::k_heads, dim3(n), dim3(256), 0, (hipStream_t)stream, act, head_weights, n, policy, value,
                       softmax ? 1 : 0);
    hipError_t r = hipGetLastError();
    if (r != hipSuccess) {
        set_error("k_heads launch: %s", hipGetErrorString(r));
        return UTTT_ERR_HIP;
    }
    return UTTT_OK;
}

}  // extern "C"
