// wino3p_impl.h — k_wino3p_conv: the split-f16 Winograd F(3x3,3x3) tower conv of wino3h_impl.h with
// its phases overlapped instead of taken in turn.
//
// k_wino3h_conv runs every chunk as [load inputs] [transform] [barrier, stage inputs] [25 point
// GEMMs] in lockstep over the workgroup's 8 waves: the matrix pipe and the L2 -> CU stream of U
// idle while the transform and staging run (about half of a launch). Here the
// point GEMMs of chunk g run in column-major point order (all u of v = 0, then v = 1, ...), so the
// 5 V slots of a column are free once every wave has passed that column; the transform of chunk
// g+1 is computed one column at a time (u_i[b] = (d_i B)[b] from the staged window, then
// V[.][b] = B^T u[.][b], split, stored into the freed slots) and its pieces are interleaved with
// the MFMAs of the next column. The inputs of chunk g+2 are staged straight into LDS by DMA
// (buffer_load ... lds, no registers, zeros past the batch) once the transform of g+1 has read
// the staged window; the per-board V scale is applied to V before the split (a power of two:
// the same bits as scaling the inputs, barring underflow).
//
// Same arithmetic as k_wino3h_conv: every S element receives its products and fold terms in the
// same order (points of one column v go to S[.][v] in u order either way), the row and column
// transforms are the same expressions (bt5), the epilogue is shared. Output bits equal the
// product kernel's (tools/diag/wino3h_variants.py checks it on every run).
#pragma once

#include "wino3h_impl.h"

namespace uttt {
namespace wino3h {

// column-major point order: P -> u = P % 5, v = P / 5, point XI = 5u + v
__host__ __device__ constexpr int xi_of(int P) { return (P % 5) * 5 + P / 5; }

template <int P>
__device__ __forceinline__ BFrag load_b_col(rsrc_t u, int chunk, int voff) {
    if constexpr (P < NP) return load_b(u, xi_of(P), chunk, voff);
    else return load_b(u, xi_of(P - NP), (chunk + 1) % NCH, voff);  // next chunk in this workgroup's order
}

// one transform item (tile slot, channel pair) of the next chunk
struct TItem {
    const float *xs;  // window origin (row -1, column -1) in sX, channel pair applied
    char *vw;         // V slot 0 of the item in sV (fragment swizzle applied)
    float sv;         // its board's V scale (power of two)
};
struct TCol {
    floatx2 u[5];  // u_i[b], rows 0..4 of the window, for the column being transformed
    floatx2 o[5];  // V[a][b], a = 0..4
};

__device__ __forceinline__ TItem t_item(const float *sX, char *sV, int it, int h, float sv) {
    const int p = it % (KC / 2), lt = it / (KC / 2);
    const int gt = min(32 * h + lt, GB * 9 - 1), gb = gt / 9, tt = gt - 9 * gb, ty = tt / 3, tx = tt % 3;
    const int rt = lt >> 4, m = lt & 15, kq = p >> 2, w = p & 3;
    TItem t;
    t.xs = sX + spos(gb - 3 * h, 3 * ty - 1, 3 * tx - 1) * KC + 2 * p;
    t.vw = sV + rt * 2 * VPLANE + kq * 256 + ((m ^ (2 * kq)) * 16) + 4 * w;
    t.sv = sv;
    return t;
}

// u_i[B] = (d_i B)[B] for window row i, as bt5 computes that output (same expression, same bits)
template <int B>
__device__ __forceinline__ floatx2 row_t(const float *__restrict__ xs, int i) {
    const float *r = xs + i * SR * KC;
    auto d = [&](int j) { return *reinterpret_cast<const floatx2 *>(r + j * KC); };
    const floatx2 two = {2.0f, 2.0f}, mtwo = {-2.0f, -2.0f};
    if constexpr (B == 0) return __builtin_elementwise_fma(two, d(0) - d(2), d(3) - d(1));
    else if constexpr (B == 1) return __builtin_elementwise_fma(mtwo, d(1), d(3) - d(2));
    else if constexpr (B == 2) return __builtin_elementwise_fma(two, d(1) - d(2), d(3) - d(2));
    else if constexpr (B == 3) return d(3) - d(1);
    else return __builtin_elementwise_fma(mtwo, d(3) - d(1), d(4) - d(2));
}

template <int B, int A, bool SCALE = true>
__device__ __forceinline__ void col_store(const TItem &ti, const TCol &tc) {
    const floatx2 s2 = {ti.sv, ti.sv};
    uint32_t hi, lo;
    if constexpr (SCALE) split(tc.o[A] * s2, hi, lo);
    else split(tc.o[A], hi, lo);
    char *q = ti.vw + (A * 5 + B) * 4 * VPLANE;
    *reinterpret_cast<uint32_t *>(q) = hi;
    *reinterpret_cast<uint32_t *>(q + VPLANE) = lo;
}

// piece K (0..4) of the transform of column B, spread over the 5 points of a GEMM column
template <int B, int K, bool SCALE = true>
__device__ __forceinline__ void col_piece(const TItem &ti, TCol &tc) {
    if constexpr (K == 0) {
        tc.u[0] = row_t<B>(ti.xs, 0);
        tc.u[1] = row_t<B>(ti.xs, 1);
    } else if constexpr (K == 1) {
        tc.u[2] = row_t<B>(ti.xs, 2);
        tc.u[3] = row_t<B>(ti.xs, 3);
    } else if constexpr (K == 2) {
        tc.u[4] = row_t<B>(ti.xs, 4);
        bt5(tc.u, tc.o);
    } else if constexpr (K == 3) {
        col_store<B, 0, SCALE>(ti, tc);
        col_store<B, 1, SCALE>(ti, tc);
        col_store<B, 2, SCALE>(ti, tc);
    } else {
        col_store<B, 3, SCALE>(ti, tc);
        col_store<B, 4, SCALE>(ti, tc);
    }
}

template <int B, bool SCALE = true>
__device__ __forceinline__ void col_all(const TItem &ti) {
    TCol tc;
    col_piece<B, 0, SCALE>(ti, tc);
    col_piece<B, 1, SCALE>(ti, tc);
    col_piece<B, 2, SCALE>(ti, tc);
    col_piece<B, 3, SCALE>(ti, tc);
    col_piece<B, 4, SCALE>(ti, tc);
}

// the whole transform of one chunk (prologue only)
__device__ __forceinline__ void transform_cols_all(const TItem &ti) {
    col_all<0>(ti);
    col_all<1>(ti);
    col_all<2>(ti);
    col_all<3>(ti);
    col_all<4>(ti);
}

// Inputs of chunk `chunk` of the set whose staged boards start at b0 -> sX by LDS-DMA: 4 boards x 9
// rows, each row two DMA instructions (cells 0-7 by all 64 lanes, cell 8 by 8 lanes), 72 per chunk
// dealt over the 8 waves. A buffer resource whose range ends at the batch's last board returns
// zeros past it. No VGPRs hold the data; the issuing wave's vmcnt covers it.
__device__ __forceinline__ void dma_x(float *sX, const float *__restrict__ x, int b0, int n_boards, int chunk, int wv,
                                      int lane) {
    const int rows = min((n_boards - b0) * 81, SB * 81);
    const rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(x + (size_t)b0 * 81 * C), 0,
                                                        rows > 0 ? rows * C * 4 : 0, 0x00020000);
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const int j = wv + 8 * k;  // 0..71
        const int pair = j >> 1, kb = pair / 9, r = pair - 9 * kb;
        if (j & 1) {  // cell 8: lanes 0..7
            if (lane < 8) {
                const int voff = ((kb * 81 + r * 9 + 8) * C + chunk * KC) * 4 + lane * 16;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    xr, (__attribute__((address_space(3))) void *)(sX + spos(kb, r, 8) * KC), 16, voff, 0, 0, 2);
            }
        } else {  // cells 0..7: lane = 8 * cell + quad
            const int voff = ((kb * 81 + r * 9 + (lane >> 3)) * C + chunk * KC) * 4 + (lane & 7) * 16;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                xr, (__attribute__((address_space(3))) void *)(sX + spos(kb, r, 0) * KC), 16, voff, 0, 0, 2);
        }
    }
}

// Fold of point P's M into S (as fold_slot), without row SKIP (-1: none). In column-major order the
// point after (3, v) is (4, v), whose MFMAs accumulate straight onto S[2][v]: the fold of (3, v) into
// that row must land first, so it is applied before those MFMAs (fold_row_now) and skipped here.
template <int P, int O, int SKIP>
__device__ __forceinline__ void fold_op_x(Acc (&S)[15], const floatx2 (&m)[4], floatx2 k2, floatx2 k4) {
    constexpr int u = P / 5, a = nth_row(u, O / 4);
    if constexpr (a != SKIP) fold_op<P, O, 0>(S, m, k2, k4);
}
template <int P, int SL, int SKIP, int O = 0>
__device__ __forceinline__ void fold_slot_x(Acc (&S)[15], const floatx2 (&m)[4], floatx2 k2, floatx2 k4) {
    constexpr int nops = 4 * n_rows(P / 5);
    if constexpr (O < nops && !acc_direct<P, 0>()) {
        if constexpr (O * NSLOT / nops == SL) fold_op_x<P, O, SKIP>(S, m, k2, k4);
        fold_slot_x<P, SL, SKIP, O + 1>(S, m, k2, k4);
    }
}
// S[2][v] += A^T[2][u] M of point P = (u, v) now, with compiler-visible packed ops (the compiler pads
// the MFMA-result read hazard): same operations, same bits as the inline-asm fold
template <int P>
__device__ __forceinline__ void fold_row_now(Acc (&S)[15], const floatx2 (&m)[4], floatx2 k2, floatx2 k4) {
    constexpr int u = P / 5, v = P % 5, K = at(2, u);
    static_assert(K == 4 || K == 1, "row 2 coefficient");
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if constexpr (K == 1) S[10 + v].p[j] = S[10 + v].p[j] + m[j];
        else S[10 + v].p[j] = __builtin_elementwise_fma(m[j], k4, S[10 + v].p[j]);
    }
    (void)k2;
}

// Point loop of one chunk in column-major order, U PF points ahead from L2, V (A operand) one point
// ahead from LDS when ALA. The fold of the previous point is issued among this point's MFMAs
// (as xi_loop). During column v >= 1 the transform of the next chunk's column v - 1 is computed
// piece by piece; a workgroup barrier opens every column (its V slots, and the previous column's,
// are then read by no wave: the previous column's slots may be rewritten).
template <int P, int PF, bool ALA>
__device__ __forceinline__ void col_loop(Acc (&S)[15], const char *__restrict__ sv, rsrc_t u, BFrag (&bq)[PF],
                                         AFrag &a0, floatx2 (&mprev)[4], floatx2 k2, floatx2 k4, int chunk, int voff,
                                         const TItem &ti, TCol &tc, bool tr) {
    if constexpr (P <= NP) {
        constexpr int XI = P < NP ? xi_of(P) : 0;
        constexpr int XP_ = P > 0 ? xi_of(P - 1) : 0;  // previous point (its fold runs here)
        floatx2 m[4];
        if constexpr (P < NP) {
            if constexpr (P % 5 == 0 && P > 0) {
                // column P/5 opens: the DMA'd inputs of the next chunk must have landed before the
                // first transform piece reads them (column 1): this wave's DMA is older than the
                // 10 U loads column 0 issued
                if constexpr (P == 5) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
                lds_barrier();
            }
            const BFrag b2 = load_b_col<P + PF>(u, chunk, voff);
            const BFrag b0 = bq[0];
            if constexpr (!ALA) a0 = load_a(sv, XI);
            AFrag a1;
            if constexpr (ALA && P + 1 < NP) a1 = load_a(sv, xi_of(P + 1));
            // (4, v) after (3, v): the previous fold's row-2 part before this point's MFMAs read S[2][v]
            constexpr int SKIP = (P > 0 && P % 5 == 4) ? 2 : -1;
            if constexpr (SKIP == 2) fold_row_now<XP_>(S, mprev, k2, k4);
            __builtin_amdgcn_sched_barrier(0);
            floatx4 m0 = {}, m1 = {};
            constexpr int srow = nth_row(XI / 5, 0) * 5 + XI % 5;
            if constexpr (acc_direct<XI, 0>()) {
                m0 = floatx4{S[srow].p[0].x, S[srow].p[0].y, S[srow].p[1].x, S[srow].p[1].y};
                m1 = floatx4{S[srow].p[2].x, S[srow].p[2].y, S[srow].p[3].x, S[srow].p[3].y};
            }
            constexpr bool fold_here = P > 0;
            m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.l, a0.h0, m0, 0, 0, 0);
            if constexpr (fold_here) fold_slot_x<XP_, 0, SKIP>(S, mprev, k2, k4);
            m1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.l, a0.h1, m1, 0, 0, 0);
            if constexpr (fold_here) fold_slot_x<XP_, 1, SKIP>(S, mprev, k2, k4);
            m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.h, a0.l0, m0, 0, 0, 0);
            if constexpr (fold_here) fold_slot_x<XP_, 2, SKIP>(S, mprev, k2, k4);
            m1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.h, a0.l1, m1, 0, 0, 0);
            if constexpr (fold_here) fold_slot_x<XP_, 3, SKIP>(S, mprev, k2, k4);
            m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.h, a0.h0, m0, 0, 0, 0);
            if constexpr (fold_here) fold_slot_x<XP_, 4, SKIP>(S, mprev, k2, k4);
            m1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.h, a0.h1, m1, 0, 0, 0);
            if constexpr (fold_here) fold_slot_x<XP_, 5, SKIP>(S, mprev, k2, k4);
            asm volatile("" : "+v"(m0), "+v"(m1));  // keep this point's MFMAs in its own region
            if constexpr (acc_direct<XI, 0>()) {
                S[srow].p[0] = __builtin_shufflevector(m0, m0, 0, 1);
                S[srow].p[1] = __builtin_shufflevector(m0, m0, 2, 3);
                S[srow].p[2] = __builtin_shufflevector(m1, m1, 0, 1);
                S[srow].p[3] = __builtin_shufflevector(m1, m1, 2, 3);
            }
            m[0] = __builtin_shufflevector(m0, m0, 0, 1);
            m[1] = __builtin_shufflevector(m0, m0, 2, 3);
            m[2] = __builtin_shufflevector(m1, m1, 0, 1);
            m[3] = __builtin_shufflevector(m1, m1, 2, 3);
            // the next chunk's transform, column P/5 - 1, piece P % 5
            if constexpr (P >= 5) {
                if (tr) col_piece<P / 5 - 1, P % 5>(ti, tc);
            }
#pragma unroll
            for (int i = 0; i + 1 < PF; ++i) bq[i] = bq[i + 1];
            bq[PF - 1] = b2;
            if constexpr (ALA && P + 1 < NP) a0 = a1;
        }
        if constexpr (P == NP) fold_all<XP_, 0>(S, mprev, k2, k4);  // nothing left to spread it over
        if constexpr (P < NP) {
#pragma unroll
            for (int i = 0; i < 4; ++i) mprev[i] = m[i];
            col_loop<P + 1, PF, ALA>(S, sv, u, bq, a0, mprev, k2, k4, chunk, voff, ti, tc, tr);
        }
    }
}

template <bool RES, int PF = 3, bool ALA = true>
__global__ __launch_bounds__(NT) void k_wino3p_conv(const float *__restrict__ x, const uint16_t *__restrict__ u,
                                                    float u_scale, const float *__restrict__ bias,
                                                    const float *__restrict__ res, float *__restrict__ y,
                                                    const uint32_t *__restrict__ x_amax, int x_amax_per_board,
                                                    uint32_t *__restrict__ y_amax, uint32_t *__restrict__ amax_clear,
                                                    int clear_count, int n_boards) {
    __shared__ __attribute__((aligned(16))) char smem[XP * KC * 4 + VB];
    float *const sX = reinterpret_cast<float *>(smem);
    char *const sV = smem + XP * KC * 4;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = (int)blockIdx.x * NT + tid; i < clear_count; i += (int)gridDim.x * NT) amax_clear[i] = 0u;
    const int nsets = n_sets(n_boards);
    if ((int)blockIdx.x >= nsets) return;
    const int my_sets = (nsets - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
    const int G = my_sets * NCH;
    auto set_of = [&](int g) { return (int)blockIdx.x + (g / NCH) * (int)gridDim.x; };
    auto set_b0 = [&](int g) { const int st = set_of(g); return GB * (st >> 1) + 3 * (st & 1); };
    const int co4 = wv * 16 + 4 * (lane >> 4);
    const floatx4 bb4 = *reinterpret_cast<const floatx4 *>(bias + co4);

    Acc S[15];
#pragma unroll
    for (int i = 0; i < 15; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) S[i].p[j] = floatx2{0.0f, 0.0f};
    const floatx2 k2 = {2.0f, 2.0f}, k4 = {4.0f, 4.0f};
    const rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(u), 0, NP * C * C * 4, 0x00020000);
    const int kq = lane >> 4;
    const int voff = wv * 1024 + lane * 16;
    const char *sv_lane = sV + kq * 256 + (((lane & 15) ^ (2 * kq)) * 16);

    for (int i = fresh(tid); i < NPAD * (KC / 4); i += NT) {
        const int j = i / (KC / 4), q = i % (KC / 4);
        const int pos = j < 50 ? (j / 10) * 10 * SR + j % 10
                      : (j < 86 ? (((j - 50) / 9) * 10 + (j - 50) % 9 + 1) * SR : XP - 1);
        reinterpret_cast<float4 *>(sX + pos * KC)[q] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    // the transform item of this thread in chunk g (its set's scales sc)
    auto item_for = [&](int g, const SetScale &scg) {
        const int h = set_of(g) & 1, it = fresh(tid);
        const int gt = min(32 * h + it / (KC / 2), GB * 9 - 1);
        return t_item(sX, sV, it, h, scg.of(gt / 9 - 3 * h));
    };
    // prologue: chunk 0 staged, transformed whole; chunk 1 staged behind it
    dma_x(sX, x, set_b0(0), n_boards, 0, wv, lane);
    SetScale sc = set_scale(x_amax, x_amax_per_board, set_b0(0), n_boards);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    transform_cols_all(item_for(0, sc));
    __syncthreads();
    if (G > 1) dma_x(sX, x, set_b0(1), n_boards, 1 % NCH, wv, lane);
    BFrag bq[PF];
#pragma unroll
    for (int i = 0; i < PF; ++i) bq[i] = load_b(ur, xi_of(i), 0, voff);

#pragma unroll 1
    for (int g = 0; g < G; ++g) {
        const int c = g % NCH;
        const bool tr = g + 1 < G;
        // the next chunk's item and V scale (its set's scales: this set's, or the next set's)
        SetScale sc_next = sc;
        if (c == NCH - 1 && tr) sc_next = set_scale(x_amax, x_amax_per_board, set_b0(g + 1), n_boards);
        const TItem ti = item_for(g + 1, sc_next);
        TCol tc;
        {
            AFrag a0;
            if constexpr (ALA) a0 = load_a(sv_lane, 0);
            floatx2 mprev[4];
            col_loop<0, PF, ALA>(S, sv_lane, ur, bq, a0, mprev, k2, k4, c, voff, ti, tc, tr);
        }
        // the set's results leave before the next chunk's inputs are requested: the DMA below is
        // then the youngest op the next chunk's column-1 vmcnt wait must cover
        if (c == NCH - 1) set_epilogue<RES, kFoldAT>(S, set_of(g), sc, u_scale, bb4, res, y, y_amax, n_boards, tid, lane);
        lds_barrier();  // column 4 of this chunk read by every wave: its slots take the next chunk's
        if (tr) col_all<4>(ti);
        lds_barrier();  // the next chunk's V complete; its staged inputs no longer read
        if (g + 2 < G) dma_x(sX, x, set_b0(g + 2), n_boards, (g + 2) % NCH, wv, lane);
        sc = sc_next;
    }
}

}  // namespace wino3h
}  // namespace uttt
