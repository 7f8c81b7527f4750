// wino3_conv.hip — the residual tower's 3x3 convolution (dual_network.py:28-45,
// 128 -> 128 channels, stride 1, pad 1, on 9x9 boards) as Winograd F(3x3, 3x3)
// with f32 MFMA, bias + residual + ReLU fused into the epilogue.
//
// A 9x9 board is exactly 3x3 tiles of 3x3 outputs (5x5 input windows), so no
// output is computed and thrown away: 9 tiles x 25 transform points = 225
// MACs per (board, ci, co) against 400 for F(2x2,3x3) (5x5 tiles of 2x2, 19
// outputs cropped) and 729 for the direct form.
//
//   V = B^T d B     d: 5x5 input window of a tile, per input channel
//   M = V (.) U     per transform point xi (25): a [tiles x 128] x [128 x 128] GEMM
//   Y = A^T M A     3x3 outputs of the tile
// Toom-Cook points {0, 1, -1, 2, inf} (fp32 error study:
// DESIGN.md §5); U = G g G^T precomputed per weight on the host in double.
// Every transform coefficient is a small integer (B^T, A^T) so V and the fold
// cost adds and exact power-of-two / small-integer scalings; products run on
// v_mfma_f32_16x16x4_f32 (exact f32 fma chain) with f32 accumulation.
//
// Workgroup = 8 waves = 32 tiles (~3.6 boards) x 128 output channels; wave w
// owns output channels 16w..16w+15 for all 32 tiles (two 16-row MFMA blocks
// sharing one B fragment). Per 16-channel chunk c (a phase between barriers):
// chunk c+1 is transformed into the other V buffer while chunk c's 25 point
// GEMMs run (the two waves of a SIMD take these in opposite order), and chunk
// c+2's inputs are in flight to registers. M of each point is folded (row
// half of A^T M A) into fifteen accumulators right after its MFMA chain; the
// column half runs once in the epilogue.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "uttt_nn.h"

namespace uttt {
void set_error(const char *fmt, ...);

namespace wino3 {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef float floatx8 __attribute__((ext_vector_type(8)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

constexpr int C = 128;           // channels in and out
constexpr int NP = 25;           // transform points
constexpr int WT = 32;           // tiles per workgroup
constexpr int KC = 16;           // input channels per chunk
constexpr int NCH = C / KC;      // chunks
constexpr int NB = 5;            // boards a 32-tile window can touch (9 tiles per board)
constexpr int PB = 121;          // a board staged zero-padded to 11x11: windows need no bounds masks
constexpr int XS = NB * PB;      // staged input floats per channel
constexpr int NT = 512;          // threads (8 waves)
constexpr int VB = NP * (KC / 4) * 64 * 2;  // floats per V buffer: [xi][ks][q][m][rt]

// Toom-Cook F(3,3) on {0, 1, -1, 2, inf}
__host__ __device__ constexpr int bt(int a, int i) {
    constexpr int m[5][5] = {{2, -1, -2, 1, 0}, {0, -2, -1, 1, 0}, {0, 2, -3, 1, 0}, {0, -1, 0, 1, 0}, {0, 2, -1, -2, 1}};
    return m[a][i];
}
__host__ __device__ constexpr int at(int a, int u) {
    constexpr int m[3][5] = {{1, 1, 1, 1, 0}, {0, 1, -1, 2, 0}, {0, 1, 1, 4, 1}};
    return m[a][u];
}

// The output transform is applied in two halves. Per point xi = (u, v) the
// MFMA result M (both 16-row blocks: 8 floats per lane, four register pairs)
// is folded into the row-transformed accumulators S[a][v] += A^T[a][u] * M;
// the column half Y[a][b] = sum_v S[a][v] A^T[b][v] runs once, in the
// epilogue. The fold is written as packed-f32 asm (v_pk_add_f32 /
// v_pk_fma_f32 on aligned pairs; hipcc lowers the vector form to scalar adds)
// and, being volatile, stays in program order right where it is issued.
struct Acc {
    floatx2 p[4];
};

template <int K>
__device__ __forceinline__ void fold(Acc &s, const floatx2 (&m)[4], floatx2 k2, floatx2 k4) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if constexpr (K == 1) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(s.p[i]) : "v"(m[i]));
        else if constexpr (K == -1) asm volatile("v_pk_add_f32 %0, %0, %1 neg_lo:[0,1] neg_hi:[0,1]" : "+v"(s.p[i]) : "v"(m[i]));
        else if constexpr (K == 2) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(s.p[i]) : "v"(m[i]), "v"(k2));
        else if constexpr (K == 4) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(s.p[i]) : "v"(m[i]), "v"(k4));
        else static_assert(K == 0, "A^T coefficients are 0, +-1, 2, 4");
    }
}

template <int XI>
__device__ __forceinline__ void fold_xi(Acc (&S)[15], const floatx2 (&m)[4], floatx2 k2, floatx2 k4) {
    constexpr int u = XI / 5, v = XI % 5;
    fold<at(0, u)>(S[0 * 5 + v], m, k2, k4);
    fold<at(1, u)>(S[1 * 5 + v], m, k2, k4);
    fold<at(2, u)>(S[2 * 5 + v], m, k2, k4);
}

// The fold of a point, as a list of single packed ops: op o = (a, pair j) over the
// rows a with A^T[a][u] != 0; spread over the next point's 8 MFMAs (an op or two
// after each) instead of issued in one burst.
__host__ __device__ constexpr int n_rows(int u) { return (at(0, u) != 0) + (at(1, u) != 0) + (at(2, u) != 0); }
__host__ __device__ constexpr int nth_row(int u, int i) {
    int a = 0;
    for (; a < 3; ++a)
        if (at(a, u) != 0 && i-- == 0) break;
    return a;
}

template <int P, int O>
__device__ __forceinline__ void fold_op(Acc (&S)[15], const floatx2 (&m)[4], floatx2 k2, floatx2 k4) {
    constexpr int u = P / 5, v = P % 5;
    if constexpr (O < 4 * n_rows(u)) {
        constexpr int a = nth_row(u, O / 4), j = O % 4, K = at(a, u);
        if constexpr (K == 1) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(S[a * 5 + v].p[j]) : "v"(m[j]));
        else if constexpr (K == -1)
            asm volatile("v_pk_add_f32 %0, %0, %1 neg_lo:[0,1] neg_hi:[0,1]" : "+v"(S[a * 5 + v].p[j]) : "v"(m[j]));
        else if constexpr (K == 2) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(S[a * 5 + v].p[j]) : "v"(m[j]), "v"(k2));
        else asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(S[a * 5 + v].p[j]) : "v"(m[j]), "v"(k4));
    }
}

// ops of point P that go after MFMA slot SL (0..7)
template <int P, int SL, int O = 0>
__device__ __forceinline__ void fold_slot(Acc (&S)[15], const floatx2 (&m)[4], floatx2 k2, floatx2 k4) {
    constexpr int nops = 4 * n_rows(P / 5);
    if constexpr (O < nops) {
        if constexpr (O * 8 / nops == SL) fold_op<P, O>(S, m, k2, k4);
        fold_slot<P, SL, O + 1>(S, m, k2, k4);
    }
}

// U stored in B-fragment order U[xi][chunk][co][q][ks] (ci = chunk*16 + 4ks + q):
// a lane's 4 values of one point are 16 contiguous bytes.
__device__ __forceinline__ floatx4 load_b(rsrc_t u, int xi, int chunk, int voff) {
    const int soff = (xi * NCH + chunk) * (C * KC) * 4;
    return __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(u, voff, soff, 0));
}

// A fragments of one point: av[ks] = (V[tile m][ci 4ks+q], V[tile 16+m][ci 4ks+q])
__device__ __forceinline__ void load_a(floatx2 (&av)[KC / 4], const floatx2 *__restrict__ sv, int xi) {
#pragma unroll
    for (int ks = 0; ks < KC / 4; ++ks) av[ks] = sv[(xi * (KC / 4) + ks) * 64];
}

// Point loop, software-pipelined: B (L2) three points ahead, A (LDS) two points ahead.
template <int XI>
__device__ __forceinline__ floatx4 load_b_ahead(rsrc_t u, int chunk, int voff) {
    if constexpr (XI < NP) return load_b(u, XI, chunk, voff);
    else return load_b(u, XI - NP, (chunk + 1) % NCH, voff);  // next chunk in this workgroup's order
}

// The fold of point XI-1 is issued after point XI's MFMAs, so it never waits
// on a just-issued chain and the next point's MFMAs follow without a bubble.
template <int XI, int MODE>
__device__ __forceinline__ void xi_loop(Acc (&S)[15], const floatx2 *__restrict__ sv, rsrc_t u, floatx4 &b0,
                                        floatx4 &b1, floatx4 &b2, floatx2 (&a0)[KC / 4], floatx2 (&a1)[KC / 4],
                                        floatx2 (&mprev)[4], floatx2 k2, floatx2 k4, int chunk, int voff) {
    if constexpr (XI <= NP) {
        floatx2 m[4];
        if constexpr (XI < NP) {
            floatx4 b3 = b0;
            floatx2 a2[KC / 4];
            if constexpr (MODE & 32) {
#pragma unroll
                for (int ks = 0; ks < KC / 4; ++ks) {
                    a2[ks] = a0[ks];
                    asm volatile("" : "+v"(a2[ks]));  // opaque copy: no CSE of the MFMAs
                }
                asm volatile("" : "+v"(b3));
            } else {
                b3 = load_b_ahead<XI + 3>(u, chunk, voff);
                if constexpr (XI + 2 < NP) load_a(a2, sv, XI + 2);
            }
            __builtin_amdgcn_sched_barrier(0);  // keep the prefetches at the top (the scheduler sinks them to their use)
            floatx4 m0 = {}, m1 = {};
            constexpr bool fold_here = XI > 0 && !(MODE & 64) && (MODE & 3) != 3;
#define UTTT_SLOT(ks)                                                                   \
    m0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[ks].x, b0[ks], m0, 0, 0, 0);           \
    if constexpr (fold_here) fold_slot<XI - 1, 2 * ks>(S, mprev, k2, k4);               \
    m1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[ks].y, b0[ks], m1, 0, 0, 0);           \
    if constexpr (fold_here) fold_slot<XI - 1, 2 * ks + 1>(S, mprev, k2, k4);
            UTTT_SLOT(0) UTTT_SLOT(1) UTTT_SLOT(2) UTTT_SLOT(3)
#undef UTTT_SLOT
            static_assert(KC / 4 == 4, "slot sequence written for four k-steps");
            // pin this point's MFMAs inside its own region (a use here), so the
            // previous point's fold issues among them instead of the MFMAs sinking
            // to just before their own fold and that fold waiting on the chain
            if constexpr (!(MODE & 512)) asm volatile("" : "+v"(m0), "+v"(m1));
            m[0] = __builtin_shufflevector(m0, m0, 0, 1);
            m[1] = __builtin_shufflevector(m0, m0, 2, 3);
            m[2] = __builtin_shufflevector(m1, m1, 0, 1);
            m[3] = __builtin_shufflevector(m1, m1, 2, 3);
            b0 = b1;
            b1 = b2;
            b2 = b3;
#pragma unroll
            for (int ks = 0; ks < KC / 4; ++ks) {
                a0[ks] = a1[ks];
                a1[ks] = a2[ks];
            }
        }
        if constexpr (XI > 0 && (MODE & 64)) {
            asm volatile("" : "+v"(mprev[0]), "+v"(mprev[1]), "+v"(mprev[2]), "+v"(mprev[3]));  // diagnostic: no fold
        } else if constexpr (XI > 0 && (MODE & 3) == 3) {
            fold<1>(S[0], mprev, k2, k4);
        } else if constexpr (XI == NP) {
            fold_xi<XI - 1>(S, mprev, k2, k4);  // the last point: no MFMAs left to spread it over
        }
        if constexpr (XI < NP) {
#pragma unroll
            for (int i = 0; i < 4; ++i) mprev[i] = m[i];
            xi_loop<XI + 1, MODE>(S, sv, u, b0, b1, b2, a0, a1, mprev, k2, k4, chunk, voff);
        }
    }
}

constexpr int XF4 = NB * 81 * (KC / 4);   // float4s staged per chunk (1620)
constexpr int XPT = (XF4 + NT - 1) / NT;  // per thread (4)

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
            const int pos = bp % 81, sp = (bp / 81) * PB + (pos / 9 + 1) * 11 + pos % 9 + 1;
            sX[(4 * q + 0) * XS + sp] = xr[k].x;
            sX[(4 * q + 1) * XS + sp] = xr[k].y;
            sX[(4 * q + 2) * XS + sp] = xr[k].z;
            sX[(4 * q + 3) * XS + sp] = xr[k].w;
        }
    }
}

// V = B^T d B for item pairs (tiles m and 16+m of one input channel ci), it =
// first .. WT/2*KC step `step`, in packed f32; V[xi][ks][q][m][rt] (ci = 4ks + q)
// takes each pair as one ds_write_b64, and one ds_read_b64 per lane then
// yields both 16-row A fragments of a k-step. Boards past n_boards are staged
// as zeros, so their (discarded) tiles need no mask.
// x -> B^T x for one 5-vector of tile pairs, common subexpressions shared:
// 9 packed ops (5 of them fma) instead of ~20 for the rows written out.
__device__ __forceinline__ void bt5(const floatx2 (&d)[5], floatx2 (&t)[5]) {
    const floatx2 two = {2.0f, 2.0f}, mtwo = {-2.0f, -2.0f};
    const floatx2 e = d[3] - d[2];
    const floatx2 f = d[1] - d[2];
    const floatx2 t3 = d[3] - d[1];
    const floatx2 g = d[0] - d[2];
    const floatx2 h = d[4] - d[2];
    t[0] = __builtin_elementwise_fma(two, g, t3);   //  2d0 - d1 - 2d2 + d3
    t[1] = __builtin_elementwise_fma(mtwo, d[1], e); // -2d1 - d2 + d3
    t[2] = __builtin_elementwise_fma(two, f, e);    //  2d1 - 3d2 + d3
    t[3] = t3;                                      //  -d1 + d3
    t[4] = __builtin_elementwise_fma(mtwo, t3, h);  //  2d1 - d2 - 2d3 + d4
}

__device__ __forceinline__ void transform(float *__restrict__ sv, const float *__restrict__ sX, int t0, int b0,
                                          int first, int step) {
    for (int it = first; it < (WT / 2) * KC; it += step) {
        const int m = it % (WT / 2), ci = it / (WT / 2);
        const float *xs[2];
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int T = t0 + 16 * r + m;
            const int tt = T % 9, ty = tt / 3, tx = tt % 3;
            xs[r] = sX + ci * XS + (T / 9 - b0) * PB + 3 * ty * 11 + 3 * tx;
        }
        floatx2 d[5][5];
#pragma unroll
        for (int i = 0; i < 5; ++i)
#pragma unroll
            for (int j = 0; j < 5; ++j) d[i][j] = floatx2{xs[0][i * 11 + j], xs[1][i * 11 + j]};
        floatx2 t[5][5];  // t = B^T d (t[a][j])
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const floatx2 col[5] = {d[0][j], d[1][j], d[2][j], d[3][j], d[4][j]};
            floatx2 o[5];
            bt5(col, o);
#pragma unroll
            for (int a = 0; a < 5; ++a) t[a][j] = o[a];
        }
        floatx2 *vs = reinterpret_cast<floatx2 *>(sv) + (ci >> 2) * 64 + (ci & 3) * 16 + m;
#pragma unroll
        for (int a = 0; a < 5; ++a) {  // V = t B
            floatx2 o[5];
            bt5(t[a], o);
#pragma unroll
            for (int b = 0; b < 5; ++b) vs[(a * 5 + b) * (KC / 4) * 64] = o[b];
        }
    }
}

// MODE (timing ablations only; 0 in the product): 1 skip the input transform,
// 2 skip the point GEMMs, 3 skip the output-transform fold; +4 adds clock
// stamps (s_memtime / s_memrealtime) into g_clk / g_phase; +8 raises waves 4-7
// to s_setprio 1; +16 swaps which half transforms the even chunks; +32 runs the
// point loop on registers only (no A / B operand loads); +64 skips the fold;
// +128 raises the transforming waves to s_setprio 3 for the transform.
__device__ unsigned long long g_clk[4096][2];
// MODE+4 phase stamps (core clocks) of workgroups 0..63, waves 0 and 4, first 8 chunks:
// [wg][w][0] prologue, per chunk c: [1+4c] transform, [2+4c] gemm(+epilogue), [3+4c] barrier A, [4+4c] barrier B
__device__ unsigned int g_phase[64][2][40];

// Persistent: one workgroup per CU walks tile sets blockIdx.x, +gridDim.x, ...
// The chunk pipeline (stage two chunks ahead, transform one ahead, GEMM) runs
// straight across set boundaries, so only the first set pays a prologue; a
// set's epilogue (output transform, bias, residual, ReLU, store) follows the
// GEMMs of its last chunk.
template <bool RES, int MODE = 0>
__global__ __launch_bounds__(NT) void k_wino3_conv(const float *__restrict__ x, const float *__restrict__ u,
                                                   const float *__restrict__ bias, const float *__restrict__ res,
                                                   float *__restrict__ y, int n_boards) {
    __shared__ float sX[KC * XS];               // [ci][board_local*121 + padded pos], border = 0
    __shared__ __attribute__((aligned(16))) float sV[2][VB];  // [buf][xi][ks][q][m][rt]
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int ntiles = n_boards * 9;
    const int nsets = (ntiles + WT - 1) / WT;
    if ((int)blockIdx.x >= nsets) return;
    const int my_sets = (nsets - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
    const int G = my_sets * NCH;  // chunks this workgroup runs
    auto set_t0 = [&](int g) { return ((int)blockIdx.x + (g / NCH) * (int)gridDim.x) * WT; };
    const int co = wv * 16 + (lane & 15);
    unsigned long long t_core = 0, t_real = 0;
    if ((MODE & 4) && tid == 0) {
        t_core = __builtin_amdgcn_s_memtime();
        t_real = __builtin_amdgcn_s_memrealtime();
    }
    Acc S[15];  // [a][v]: row-transformed accumulators; pairs 0-1 block rt=0, 2-3 rt=1
#pragma unroll
    for (int i = 0; i < 15; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) S[i].p[j] = floatx2{0.0f, 0.0f};
    const floatx2 k2 = {2.0f, 2.0f}, k4 = {4.0f, 4.0f};
    float4 xr[XPT];
    const rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(u), 0, NP * C * C * 4, 0x00020000);
    const int voff = (co * 4 + (lane >> 4)) * 16;
    // Every workgroup takes the chunks in the same order: the f32 accumulation order of a
    // board's results must not depend on which workgroup (= where in the batch) it lands.
    const int c_rot = 0;
    auto chunk_of = [&](int g) { return (g % NCH + c_rot) % NCH; };
    floatx4 b0v = load_b(ur, 0, c_rot, voff), b1v = load_b(ur, 1, c_rot, voff), b2v = load_b(ur, 2, c_rot, voff);
    const float bb = bias[co];

    for (int i = tid; i < KC * XS; i += NT) sX[i] = 0.0f;  // the padding border stays zero
    __syncthreads();
    load_x(xr, x, set_t0(0) / 9, n_boards, chunk_of(0) * KC, tid);
    store_x(sX, xr, tid);
    __syncthreads();
    if ((MODE & 3) != 1) transform(sV[0], sX, set_t0(0), set_t0(0) / 9, tid, NT);
    if (G > 1) load_x(xr, x, set_t0(1) / 9, n_boards, chunk_of(1) * KC, tid);
    __syncthreads();
    if (G > 1) store_x(sX, xr, tid);
    __syncthreads();
    // Waves w and w+4 share a SIMD. A chunk's transform is 256 tile-pair items,
    // one per lane of one wave per SIMD: one half of the workgroup transforms
    // (then joins the GEMMs) while the other half starts its MFMAs at once; the
    // halves alternate by chunk so both carry the same delay.
    const int tfirst = tid & 255;
    if ((MODE & 8) && wv >= 4) __builtin_amdgcn_s_setprio(1);
    const int my_half = (wv >= 4) ^ ((MODE & 16) ? 1 : 0);
    const bool stamp = (MODE & 4) && blockIdx.x < 64 && (tid == 0 || tid == 256);
    unsigned long long ts = stamp ? __builtin_amdgcn_s_memtime() : 0;
    int gs = 0;
    auto mark = [&](int k) {
        if (stamp && gs < NCH) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            g_phase[blockIdx.x][tid >> 8][k] = (unsigned int)(t - ts);
            ts = t;
        }
    };
    if (stamp) g_phase[blockIdx.x][tid >> 8][0] = (unsigned int)(ts - t_core);
#pragma unroll 1
    for (int g = 0; g < G; ++g) {
        gs = g;
        const int c = g % NCH, ch = chunk_of(g);
        if (g + 2 < G) load_x(xr, x, set_t0(g + 2) / 9, n_boards, chunk_of(g + 2) * KC, tid);
        const bool tr = (MODE & 3) != 1 && g + 1 < G && my_half == (g & 1 ? 0 : 1);
        if (tr) {
            if (MODE & 128) __builtin_amdgcn_s_setprio(3);
            transform(sV[(g + 1) & 1], sX, set_t0(g + 1), set_t0(g + 1) / 9, tfirst, 256);
            if (MODE & 128) __builtin_amdgcn_s_setprio(0);
        }
        mark(1 + 4 * c);
        if constexpr ((MODE & 3) != 2) {
            const floatx2 *sv = reinterpret_cast<const floatx2 *>(sV[g & 1]) + lane;
            floatx2 a0[KC / 4], a1[KC / 4];
            load_a(a0, sv, 0);
            load_a(a1, sv, 1);
            floatx2 mprev[4];
            xi_loop<0, MODE>(S, sv, ur, b0v, b1v, b2v, a0, a1, mprev, k2, k4, ch, voff);
        }
        if (c == NCH - 1) {
            // epilogue of this set: Y[a][b] = sum_v S[a][v] A^T[b][v]; element 4rt + r is
            // tile 16rt + 4(lane>>4) + r, output (3ty+a, 3tx+b); + bias, + residual, ReLU
            const int t0 = set_t0(g);
            floatx8 Y[9];
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int b = 0; b < 3; ++b) {
                    floatx8 acc = {};
#pragma unroll
                    for (int v = 0; v < 5; ++v) {
                        if (at(b, v) == 0) continue;
                        const Acc &q = S[a * 5 + v];
                        const floatx8 sv8 = {q.p[0].x, q.p[0].y, q.p[1].x, q.p[1].y,
                                             q.p[2].x, q.p[2].y, q.p[3].x, q.p[3].y};
                        acc = at(b, v) == 1 ? acc + sv8
                            : at(b, v) == -1 ? acc - sv8
                                             : __builtin_elementwise_fma(floatx8((float)at(b, v)), sv8, acc);
                    }
                    Y[a * 3 + b] = acc;
                }
#pragma unroll
            for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int T = t0 + 16 * rt + 4 * (lane >> 4) + r;
                    if (T >= ntiles) continue;
                    const int board = T / 9, tt = T % 9, ty = tt / 3, tx = tt % 3;
#pragma unroll
                    for (int ab = 0; ab < 9; ++ab) {
                        const size_t idx = ((size_t)board * 81 + (3 * ty + ab / 3) * 9 + 3 * tx + ab % 3) * C + co;
                        float v = Y[ab][4 * rt + r] + bb;
                        if (RES) v += res[idx];
                        y[idx] = fmaxf(v, 0.0f);
                    }
                }
#pragma unroll
            for (int i = 0; i < 15; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) S[i].p[j] = floatx2{0.0f, 0.0f};
        }
        mark(2 + 4 * c);
        __syncthreads();
        mark(3 + 4 * c);
        if (g + 2 < G) store_x(sX, xr, tid);
        __syncthreads();
        mark(4 + 4 * c);
    }
    if ((MODE & 4) && tid == 0 && blockIdx.x < 4096) {
        g_clk[blockIdx.x][0] = (__builtin_amdgcn_s_memtime() - t_core) / my_sets;
        g_clk[blockIdx.x][1] = (__builtin_amdgcn_s_memrealtime() - t_real) / my_sets;
    }
}

// One workgroup per CU (LDS and registers allow exactly one), never more than tile sets.
static int grid_size(int n_boards) {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            cus <= 0)
            cus = 256;
    }
    const int nsets = (n_boards * 9 + WT - 1) / WT;
    return nsets < cus ? nsets : cus;
}

}  // namespace wino3
}  // namespace uttt

using namespace uttt;

extern "C" {

int uttt_nn_wino3_weights(const float *w, float *u) {
    // U[xi=(p,q)][ci][co] = (G g G^T)[p][q], g = w[co][ci][3][3], G of F(3,3) on {0,1,-1,2,inf},
    // stored as U[xi][ci/16][co][ci%4][(ci%16)/4] (the kernel's B-fragment order)
    if (!w || !u) {
        set_error("uttt_nn_wino3_weights: null pointer");
        return UTTT_ERR_ARG;
    }
    static const double G[5][3] = {{0.5, 0, 0},
                                   {-0.5, -0.5, -0.5},
                                   {-1.0 / 6, 1.0 / 6, -1.0 / 6},
                                   {1.0 / 6, 1.0 / 3, 2.0 / 3},
                                   {0, 0, 1}};
    using namespace wino3;
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
                    u[((((size_t)(p * 5 + q) * NCH + ci / KC) * C + co) * 4 + (ci & 3)) * 4 + (ci % KC) / 4] = (float)v;
                }
        }
    return UTTT_OK;
}

int uttt_nn_conv3x3_wino3(const float *x, const float *u, const float *bias, const float *residual, float *y,
                          int32_t n_boards, void *stream) {
    if (!x || !u || !bias || !y || n_boards < 0 || x == y || (residual && residual == y)) {
        set_error("uttt_nn_conv3x3_wino3: bad arguments (output must not alias the input or residual)");
        return UTTT_ERR_ARG;
    }
    if (n_boards == 0) return UTTT_OK;
    const dim3 grid(wino3::grid_size(n_boards));
    if (residual)
        hipLaunchKernelGGL(wino3::k_wino3_conv<true>, grid, dim3(wino3::NT), 0, (hipStream_t)stream, x, u, bias, residual,
                           y, n_boards);
    else
        hipLaunchKernelGGL(wino3::k_wino3_conv<false>, grid, dim3(wino3::NT), 0, (hipStream_t)stream, x, u, bias, nullptr,
                           y, n_boards);
    hipError_t r = hipGetLastError();
    if (r != hipSuccess) {
        set_error("k_wino3_conv launch: %s", hipGetErrorString(r));
        return UTTT_ERR_HIP;
    }
    return UTTT_OK;
}

// Diagnostic (not declared in uttt_nn.h): the same launch with a timing ablation.
int uttt_diag_wino3_ablation(const float *x, const float *u, const float *bias, float *y, int32_t n_boards,
                             int32_t mode, void *stream) {
    const dim3 grid(wino3::grid_size(n_boards));
    hipStream_t st = (hipStream_t)stream;
    using namespace wino3;
    switch (mode) {
        case 1: hipLaunchKernelGGL((k_wino3_conv<false, 1>), grid, dim3(NT), 0, st, x, u, bias, nullptr, y, n_boards); break;
        case 2: hipLaunchKernelGGL((k_wino3_conv<false, 2>), grid, dim3(NT), 0, st, x, u, bias, nullptr, y, n_boards); break;
        case 3: hipLaunchKernelGGL((k_wino3_conv<false, 3>), grid, dim3(NT), 0, st, x, u, bias, nullptr, y, n_boards); break;
        case 4: hipLaunchKernelGGL((k_wino3_conv<false, 4>), grid, dim3(NT), 0, st, x, u, bias, nullptr, y, n_boards); break;
        case 5: hipLaunchKernelGGL((k_wino3_conv<false, 5>), grid, dim3(NT), 0, st, x, u, bias, nullptr, y, n_boards); break;
        case 7: hipLaunchKernelGGL((k_wino3_conv<false, 7>), grid, dim3(NT), 0, st, x, u, bias, nullptr, y, n_boards); break;
        case 8: hipLaunchKernelGGL((k_wino3_conv<false, 8>), grid, dim3(NT), 0, st, x, u, bias, nullptr, y, n_boards); break;
        case 16: hipLaunchKernelGGL((k_wino3_conv<false, 16>), grid, dim3(NT), 0, st, x, u, bias, nullptr, y, n_boards); break;
        case 24: hipLaunchKernelGGL((k_wino3_conv<false, 24>), grid, dim3(NT), 0, st, x, u, bias, nullptr, y, n_boards); break;
        case 33: hipLaunchKernelGGL((k_wino3_conv<false, 33>), grid, dim3(NT), 0, st, x, u, bias, nullptr, y, n_boards); break;
        case 35: hipLaunchKernelGGL((k_wino3_conv<false, 35>), grid, dim3(NT), 0, st, x, u, bias, nullptr, y, n_boards); break;
        case 128: hipLaunchKernelGGL((k_wino3_conv<false, 128>), grid, dim3(NT), 0, st, x, u, bias, nullptr, y, n_boards); break;
        case 144: hipLaunchKernelGGL((k_wino3_conv<false, 144>), grid, dim3(NT), 0, st, x, u, bias, nullptr, y, n_boards); break;
        case 6: hipLaunchKernelGGL((k_wino3_conv<false, 6>), grid, dim3(NT), 0, st, x, u, bias, nullptr, y, n_boards); break;
        case 512: hipLaunchKernelGGL((k_wino3_conv<false, 512>), grid, dim3(NT), 0, st, x, u, bias, nullptr, y, n_boards); break;
        case 69: hipLaunchKernelGGL((k_wino3_conv<false, 69>), grid, dim3(NT), 0, st, x, u, bias, nullptr, y, n_boards); break;
        case 97: hipLaunchKernelGGL((k_wino3_conv<false, 97>), grid, dim3(NT), 0, st, x, u, bias, nullptr, y, n_boards); break;
        case 65: hipLaunchKernelGGL((k_wino3_conv<false, 65>), grid, dim3(NT), 0, st, x, u, bias, nullptr, y, n_boards); break;
        default: hipLaunchKernelGGL((k_wino3_conv<false, 0>), grid, dim3(NT), 0, st, x, u, bias, nullptr, y, n_boards);
    }
    return hipGetLastError() == hipSuccess ? UTTT_OK : UTTT_ERR_HIP;
}

// Diagnostic: MODE-4 phase stamps, out[64][2][40] (see g_phase).
int uttt_diag_wino3_phases(unsigned int *out) {
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpyFromSymbol(out, HIP_SYMBOL(wino3::g_phase), sizeof(unsigned int) * 64 * 2 * 40) != hipSuccess)
        return UTTT_ERR_HIP;
    return UTTT_OK;
}

// Diagnostic: median shader clock (MHz) and median workgroup duration (us) of the last MODE-4 launch.
int uttt_diag_wino3_clock(double *mhz, double *wg_us) {
    static unsigned long long h[4096][2];
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpyFromSymbol(h, HIP_SYMBOL(wino3::g_clk), sizeof(h)) != hipSuccess)
        return UTTT_ERR_HIP;
    double r[4096], d[4096];
    int n = 0;
    for (int i = 0; i < 4096; ++i)
        if (h[i][1] > 0) {
            r[n] = 100.0 * (double)h[i][0] / (double)h[i][1];
            d[n++] = (double)h[i][1] / 100.0;
        }
    if (!n) return UTTT_ERR_ARG;
    auto med = [n](double *a) {
        for (int i = 1; i < n; ++i)
            for (int j = i; j > 0 && a[j - 1] > a[j]; --j) { double t = a[j]; a[j] = a[j - 1]; a[j - 1] = t; }
        return a[n / 2];
    };
    *mhz = med(r);
    *wg_us = med(d);
    return UTTT_OK;
}

}  // extern "C"
