// wino_conv.hip — the residual tower's 3x3 convolution (dual_network.py:28-45,
// 128 -> 128 channels, stride 1, pad 1, on 9x9 boards) as one fused gfx950
// kernel: Winograd F(2x2, 3x3) with f32 MFMA, bias + residual + ReLU epilogue.
//
// Direct 3x3 conv costs 9 MACs per (output, ci, co); F(2x2,3x3) covers a 2x2
// output tile with 16 MACs per (ci, co). A 9x9 board takes 5x5 tiles (10x10
// outputs, 19 discarded), so per real output: 16*25/81 = 4.94 MACs vs 9 —
// 1.82x fewer MFMA cycles than the direct form, whose MIOpen implicit GEMM
// already runs at the f32 MFMA roof on this shape.
//
//   V = B^T d B     d: 4x4 input window of a tile, per input channel
//   M = V (.) U     per transform point xi (16): a [tiles x 128] x [128 x 128] GEMM
//   Y = A^T M A     2x2 outputs of the tile
// with U = G g G^T precomputed per weight (host, double precision).
// Arithmetic: adds/subtracts in the transforms, f32 MFMA (exact f32 fma chain)
// for the products, f32 accumulation; differs from the direct conv by
// rounding only (tests: tests/test_engine_gpu.py, vs torch fp32).
//
// Workgroup = 8 waves = 64 tiles (GEMM rows, ~2.6 boards) x 128 output
// channels; each wave owns 32 tiles x 32 channels. Per 16-channel chunk: the
// boards' inputs are staged in LDS, transformed to V in LDS (double buffered),
// then per xi: 8 k-steps of v_mfma_f32_32x32x2_f32 into M (A = V from LDS,
// B = U from L2 into registers, prefetched one xi ahead) and M is folded into
// the four output accumulators with the A^T (.) A signs. No intermediate
// leaves the CU; the output is written once with bias, residual and ReLU.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "uttt_nn.h"

namespace uttt {
void set_error(const char *fmt, ...);

namespace wino {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int C = 128;     // channels in and out
constexpr int WT = 64;     // tiles per workgroup
constexpr int KC = 16;     // input channels per chunk
constexpr int NB = 4;      // boards a 64-tile window can touch (tiles t0..t0+63, 25 per board)
constexpr int XS = NB * 81;

// A^T = [[1,1,1,0],[0,1,-1,-1]]: sign of M[u][v] in Y[a][b] is AT[a][u]*AT[b][v]
__host__ __device__ constexpr int at(int a, int u) { return a == 0 ? (u < 3 ? 1 : 0) : (u == 0 ? 0 : (u == 1 ? 1 : -1)); }

template <int S>
__device__ __forceinline__ void fold(floatx16 &y, const floatx16 &m) {
    if constexpr (S == 1) y += m;
    else if constexpr (S == -1) y -= m;
}

// Wave tile: 32 tiles x 32 output channels (one 32x32 MFMA accumulator per
// transform point). 8 waves = 2 tile halves x 4 channel quarters, 2 waves per
// SIMD: one wave's transform / fold VALU work issues beside the other's MFMAs.
constexpr int NT = 512;

// U is stored in the B-fragment order U[xi][chunk][co][h][s] (ci = chunk*KC + 2s + h),
// so a lane's 8 values of one point are 32 contiguous bytes: two buffer_load_b128
// with the lane part in voffset and the (xi, chunk) part in soffset.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr int UCHUNK = C * KC;  // floats per (xi, chunk)

__device__ __forceinline__ void load_b(float (&bn)[KC / 2], rsrc_t u, int xi, int chunk, int voff) {
    const int soff = (xi * (C / KC) + chunk) * UCHUNK * 4;
    typedef float f4 __attribute__((ext_vector_type(4)));
    const f4 lo = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(u, voff, soff, 0));
    const f4 hi = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(u, voff + 16, soff, 0));
    bn[0] = lo.x; bn[1] = lo.y; bn[2] = lo.z; bn[3] = lo.w;
    bn[4] = hi.x; bn[5] = hi.y; bn[6] = hi.z; bn[7] = hi.w;
}

template <int XI>
__device__ __forceinline__ void fold_xi(floatx16 (&Y)[4], const floatx16 &m) {
    constexpr int u = XI / 4, v = XI % 4;
    fold<at(0, u) * at(0, v)>(Y[0], m);
    fold<at(0, u) * at(1, v)>(Y[1], m);
    fold<at(1, u) * at(0, v)>(Y[2], m);
    fold<at(1, u) * at(1, v)>(Y[3], m);
}

// One chunk's 16 point GEMMs: M_xi = V_xi[32 tiles][KC] x U_xi[KC][32 co], folded into Y.
// B of the next point (or of the next chunk's first point) is prefetched one point ahead.
template <int XI, int MODE>
__device__ __forceinline__ void xi_loop(floatx16 (&Y)[4], const float *__restrict__ sv, rsrc_t u,
                                        float (&bc)[KC / 2], float (&bn)[KC / 2], int chunk, int voff) {
    if constexpr (XI < 16) {
        if constexpr (XI + 1 < 16) load_b(bn, u, XI + 1, chunk, voff);
        else if (chunk + 1 < C / KC) load_b(bn, u, 0, chunk + 1, voff);
        floatx16 m = {};
        const float *a = sv + XI * KC * WT;
#pragma unroll
        for (int s = 0; s < KC / 2; ++s)
            m = __builtin_amdgcn_mfma_f32_32x32x2f32(a[2 * s * WT], bc[s], m, 0, 0, 0);
        if constexpr (MODE == 3) Y[0] += m;
        else fold_xi<XI>(Y, m);
        // the fold must retire here: left alone, the compiler sinks all 16 folds
        // below the last point and keeps 16 live M accumulators (spills)
        asm volatile("" : "+v"(Y[0]), "+v"(Y[1]), "+v"(Y[2]), "+v"(Y[3]));
#pragma unroll
        for (int i = 0; i < KC / 2; ++i) bc[i] = bn[i];

        xi_loop<XI + 1, MODE>(Y, sv, u, bc, bn, chunk, voff);
    }
}

constexpr int XF4 = XS * (KC / 4);           // float4s staged per chunk (1296)
constexpr int XPT = (XF4 + NT - 1) / NT;     // per thread (3)

__device__ __forceinline__ void load_x(float4 (&xr)[XPT], const float *__restrict__ x, int b0, int n_boards, int c0,
                                       int tid) {
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
        const int i = tid + k * NT;
        xr[k] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (i < XF4) {
            const int q = i % (KC / 4), bp = i / (KC / 4);
            const int b = b0 + bp / 81;
            if (b < n_boards) xr[k] = reinterpret_cast<const float4 *>(x + ((size_t)b * 81 + bp % 81) * C + c0)[q];
        }
    }
}

__device__ __forceinline__ void store_x(float *__restrict__ sX, const float4 (&xr)[XPT], int tid) {
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
        const int i = tid + k * NT;
        if (i < XF4) {
            const int q = i % (KC / 4), bp = i / (KC / 4);
            sX[(4 * q + 0) * XS + bp] = xr[k].x;
            sX[(4 * q + 1) * XS + bp] = xr[k].y;
            sX[(4 * q + 2) * XS + bp] = xr[k].z;
            sX[(4 * q + 3) * XS + bp] = xr[k].w;
        }
    }
}

// V = B^T d B for this thread's (tile, ci) items; B^T = [[1,0,-1,0],[0,1,1,0],[0,-1,1,0],[0,1,0,-1]]
__device__ __forceinline__ void transform(float *__restrict__ sv, const float *__restrict__ sX, int t0, int b0,
                                          int ntiles, int tid) {
    for (int it = tid; it < WT * KC; it += NT) {
        const int tl = it % WT, ci = it / WT;
        const int T = t0 + tl;
        const int tt = T % 25, ty = tt / 5, tx = tt % 5;
        const float *xs = sX + ci * XS + (T / 25 - b0) * 81;
        float d[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int R = 2 * ty - 1 + i, Cc = 2 * tx - 1 + j;
                const bool ok = T < ntiles && R >= 0 && R <= 8 && Cc >= 0 && Cc <= 8;
                d[i][j] = ok ? xs[R * 9 + Cc] : 0.0f;
            }
        float t[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            t[0][j] = d[0][j] - d[2][j];
            t[1][j] = d[1][j] + d[2][j];
            t[2][j] = d[2][j] - d[1][j];
            t[3][j] = d[1][j] - d[3][j];
        }
        float *vs = sv + ci * WT + tl;
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            vs[(a * 4 + 0) * KC * WT] = t[a][0] - t[a][2];
            vs[(a * 4 + 1) * KC * WT] = t[a][1] + t[a][2];
            vs[(a * 4 + 2) * KC * WT] = t[a][2] - t[a][1];
            vs[(a * 4 + 3) * KC * WT] = t[a][1] - t[a][3];
        }
    }
}

// MODE (timing ablations only; 0 in the product): 1 skip the input transform,
// 2 skip the point GEMMs, 3 skip the output-transform fold.
//
// Pipeline per 16-channel chunk c (one phase between barriers): transform
// chunk c+1 (sX -> sV[(c+1)&1]) and the GEMMs of chunk c (sV[c&1]) run in the
// same phase on different waves' issue slots, while chunk c+2's inputs are in
// flight to registers; they land in sX after the phase's barrier.
template <bool RES, int MODE = 0>
__global__ __launch_bounds__(NT) void k_wino_conv(const float *__restrict__ x, const float *__restrict__ u,
                                                  const float *__restrict__ bias, const float *__restrict__ res,
                                                  float *__restrict__ y, int n_boards) {
    __shared__ float sX[KC * XS];          // [ci][board_local*81 + pos]
    __shared__ float sV[2][16 * KC * WT];  // [buf][xi][ci][tile]
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int ntiles = n_boards * 25;
    const int t0 = blockIdx.x * WT;
    const int b0 = t0 / 25;
    const int r = lane & 31, h = lane >> 5;
    const int trow = (wv & 1) * 32;        // this wave's tile half
    const int col = (wv >> 1) * 32 + r;    // this lane's output channel
    floatx16 Y[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) Y[i] = floatx16{};
    float bc[KC / 2], bn[KC / 2];
    float4 xr[XPT];
    const rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(u), 0, 16 * C * C * 4, 0x00020000);
    const int voff = (col * 2 + h) * (KC / 2) * 4;

    load_x(xr, x, b0, n_boards, 0, tid);
    store_x(sX, xr, tid);
    load_b(bc, ur, 0, 0, voff);
    __syncthreads();
    if (MODE != 1) transform(sV[0], sX, t0, b0, ntiles, tid);
    load_x(xr, x, b0, n_boards, KC, tid);
    __syncthreads();
    store_x(sX, xr, tid);
    __syncthreads();
    constexpr int NCH = C / KC;
#pragma unroll 1
    for (int c = 0; c < NCH; ++c) {
        const int c0 = c * KC;
        if (c + 2 < NCH) load_x(xr, x, b0, n_boards, c0 + 2 * KC, tid);
        // waves w and w+4 share a SIMD: one transforms while the other issues MFMAs
        const bool tr = MODE != 1 && c + 1 < NCH;
        if (tr && wv < 4) transform(sV[(c + 1) & 1], sX, t0, b0, ntiles, tid);
        if constexpr (MODE != 2) xi_loop<0, MODE>(Y, sV[c & 1] + h * WT + trow + r, ur, bc, bn, c, voff);
        if (tr && wv >= 4) transform(sV[(c + 1) & 1], sX, t0, b0, ntiles, tid);
        __syncthreads();
        if (c + 2 < NCH) store_x(sX, xr, tid);
        __syncthreads();
    }

    // epilogue: Y[a*2+b] = output (2ty+a, 2tx+b) of the tile; + bias, + residual, ReLU
    const float bb = bias[col];
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int T = t0 + trow + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        if (T >= ntiles) continue;
        const int board = T / 25, tt = T % 25, ty = tt / 5, tx = tt % 5;
#pragma unroll
        for (int ab = 0; ab < 4; ++ab) {
            const int oy = 2 * ty + (ab >> 1), ox = 2 * tx + (ab & 1);
            if (oy > 8 || ox > 8) continue;
            const size_t idx = ((size_t)board * 81 + oy * 9 + ox) * C + col;
            float v = Y[ab][reg] + bb;
            if (RES) v += res[idx];
            y[idx] = fmaxf(v, 0.0f);
        }
    }
}

}  // namespace wino
}  // namespace uttt

using namespace uttt;

extern "C" {

int uttt_nn_wino_weights(const float *w, float *u) {
    // U[xi=(p,q)][ci][co] = (G g G^T)[p][q], g = w[co][ci][3][3], G = [[1,0,0],[.5,.5,.5],[.5,-.5,.5],[0,0,1]],
    // stored as U[xi][ci/KC][co][ci%2][(ci%KC)/2] (the kernel's B-fragment order)
    if (!w || !u) {
        set_error("uttt_nn_wino_weights: null pointer");
        return UTTT_ERR_ARG;
    }
    static const double G[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
    for (int co = 0; co < wino::C; ++co)
        for (int ci = 0; ci < wino::C; ++ci) {
            const float *g = w + ((size_t)co * wino::C + ci) * 9;
            double tg[4][3];
            for (int p = 0; p < 4; ++p)
                for (int k = 0; k < 3; ++k)
                    tg[p][k] = G[p][0] * g[0 * 3 + k] + G[p][1] * g[1 * 3 + k] + G[p][2] * g[2 * 3 + k];
            for (int p = 0; p < 4; ++p)
                for (int q = 0; q < 4; ++q) {
                    const double v = tg[p][0] * G[q][0] + tg[p][1] * G[q][1] + tg[p][2] * G[q][2];
                    u[((((size_t)(p * 4 + q) * (wino::C / wino::KC) + ci / wino::KC) * wino::C + co) * 2 + (ci & 1)) *
                          (wino::KC / 2) + (ci % wino::KC) / 2] = (float)v;
                }
        }
    return UTTT_OK;
}

int uttt_nn_conv3x3_wino(const float *x, const float *u, const float *bias, const float *residual, float *y,
                         int32_t n_boards, void *stream) {
    if (!x || !u || !bias || !y || n_boards < 0 || x == y || (residual && residual == y)) {
        set_error("uttt_nn_conv3x3_wino: bad arguments (output must not alias the input or residual)");
        return UTTT_ERR_ARG;
    }
    if (n_boards == 0) return UTTT_OK;
    const int tiles = n_boards * 25;
    const dim3 grid((tiles + wino::WT - 1) / wino::WT);
    if (residual)
        hipLaunchKernelGGL(wino::k_wino_conv<true>, grid, dim3(wino::NT), 0, (hipStream_t)stream, x, u, bias, residual, y,
                           n_boards);
    else
        hipLaunchKernelGGL(wino::k_wino_conv<false>, grid, dim3(wino::NT), 0, (hipStream_t)stream, x, u, bias, nullptr, y,
                           n_boards);
    hipError_t r = hipGetLastError();
    if (r != hipSuccess) {
        set_error("k_wino_conv launch: %s", hipGetErrorString(r));
        return UTTT_ERR_HIP;
    }
    return UTTT_OK;
}

// Diagnostic (not declared in uttt_nn.h): the same launch with a timing ablation.
int uttt_diag_wino_ablation(const float *x, const float *u, const float *bias, float *y, int32_t n_boards, int32_t mode,
                            void *stream) {
    const dim3 grid((n_boards * 25 + wino::WT - 1) / wino::WT);
    hipStream_t st = (hipStream_t)stream;
    switch (mode) {
        case 1: hipLaunchKernelGGL((wino::k_wino_conv<false, 1>), grid, dim3(wino::NT), 0, st, x, u, bias, nullptr, y, n_boards); break;
        case 2: hipLaunchKernelGGL((wino::k_wino_conv<false, 2>), grid, dim3(wino::NT), 0, st, x, u, bias, nullptr, y, n_boards); break;
        case 3: hipLaunchKernelGGL((wino::k_wino_conv<false, 3>), grid, dim3(wino::NT), 0, st, x, u, bias, nullptr, y, n_boards); break;
        default: hipLaunchKernelGGL((wino::k_wino_conv<false, 0>), grid, dim3(wino::NT), 0, st, x, u, bias, nullptr, y, n_boards);
    }
    return hipGetLastError() == hipSuccess ? UTTT_OK : UTTT_ERR_HIP;
}

}  // extern "C"
