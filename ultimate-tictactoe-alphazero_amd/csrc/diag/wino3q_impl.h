// wino3q_impl.h — k_wino3q_conv: k_wino3h_conv's algorithm and arithmetic (same output bits) with
// 16 waves per workgroup instead of 8: wave w owns output channels 16 (w mod 8) .. +15 of ONE
// 16-tile MFMA block (w / 8) instead of both blocks, so its fold accumulators are half as many
// (60 VGPRs instead of 120), the kernel fits 128 VGPRs and every SIMD holds 4 waves instead of 2.
//
// Why (round 3, tools/pmc_sq.sh on the product kernel, 16,384 boards): per wave, 33% of the cycles
// wait on s_waitcnt / barriers and 36% on issue stalls, with the matrix pipe busy 22% of the time
// and VALU issue about a third: at 2 waves per SIMD nothing covers the latencies. Same LDS layout,
// same U stream (the two waves of a channel group read the same U lines, close together in time:
// L1), same transform (by the first 8 waves), same per-block MFMA chain order, same fold, same
// epilogue per block.
#pragma once

#include "wino3h_impl.h"
#include "wino3p_impl.h"

namespace uttt {
namespace wino3h {

constexpr int NTQ = 1024;                       // threads (16 waves)
constexpr int XPTQ = (XF4 + NTQ - 1) / NTQ;     // staged float4s per thread (3)

struct Acc1 {
    floatx2 p[2];  // one tile block: the MFMA result's 4 floats
};

// fold of point P into S for one block: ops O = (row a, pair j), 2 * n_rows(u) of them, issued
// after this point's 2nd and 3rd MFMA (>= 2 MFMAs after the previous point's last MFMA wrote m)
template <int P, int O>
__device__ __forceinline__ void fold_op1(Acc1 (&S)[15], const floatx2 (&m)[2], floatx2 k2, floatx2 k4) {
    constexpr int u = P / 5, v = P % 5;
    if constexpr (O < 2 * n_rows(u) && !acc_direct<P, 0>()) {
        constexpr int a = nth_row(u, O / 2), j = O % 2, K = at(a, u);
        if constexpr (K == 1) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(S[a * 5 + v].p[j]) : "v"(m[j]));
        else if constexpr (K == -1)
            asm volatile("v_pk_add_f32 %0, %0, %1 neg_lo:[0,1] neg_hi:[0,1]" : "+v"(S[a * 5 + v].p[j]) : "v"(m[j]));
        else if constexpr (K == 2) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(S[a * 5 + v].p[j]) : "v"(m[j]), "v"(k2));
        else asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(S[a * 5 + v].p[j]) : "v"(m[j]), "v"(k4));
    }
}
template <int P, int SL, int O = 0>
__device__ __forceinline__ void fold_slot1(Acc1 (&S)[15], const floatx2 (&m)[2], floatx2 k2, floatx2 k4) {
    constexpr int nops = 2 * n_rows(P / 5);
    if constexpr (O < nops) {
        if constexpr (O * 2 / nops == SL) fold_op1<P, O>(S, m, k2, k4);
        fold_slot1<P, SL, O + 1>(S, m, k2, k4);
    }
}

struct AFrag1 {
    halfx8 h, l;
};
__device__ __forceinline__ AFrag1 load_a1(const char *__restrict__ sv, int xi) {
    // sv points at this lane's 16-byte slot of this wave's block
    const char *p = sv + xi * 4 * VPLANE;
    AFrag1 a;
    a.h = *reinterpret_cast<const halfx8 *>(p);
    a.l = *reinterpret_cast<const halfx8 *>(p + VPLANE);
    return a;
}

// point loop (as xi_loop, one block): U PF points ahead from L2, V one point ahead from LDS
template <int XI, int PF>
__device__ __forceinline__ void xi_loop1(Acc1 (&S)[15], const char *__restrict__ sv, rsrc_t u, BFrag (&bq)[PF],
                                         AFrag1 &a0, floatx2 (&mprev)[2], floatx2 k2, floatx2 k4, int chunk,
                                         int voff) {
    if constexpr (XI <= NP) {
        floatx2 m[2];
        if constexpr (XI < NP) {
            // U for point XI + PF of this chunk (none past the chunk: the next chunk's first points are
            // requested after its transform, so no U registers are live across the transform)
            BFrag b2;
            if constexpr (XI + PF < NP) b2 = load_b(u, XI + PF, chunk, voff);
            const BFrag b0 = bq[0];
            AFrag1 a1;
            if constexpr (XI + 1 < NP) a1 = load_a1(sv, XI + 1);
            __builtin_amdgcn_sched_barrier(0);
            floatx4 m0 = {};
            constexpr int srow = nth_row(XI / 5, 0) * 5 + XI % 5;
            if constexpr (acc_direct<XI, 0>()) m0 = floatx4{S[srow].p[0].x, S[srow].p[0].y, S[srow].p[1].x, S[srow].p[1].y};
            constexpr bool fold_here = XI > 0;
            m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.l, a0.h, m0, 0, 0, 0);
            m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.h, a0.l, m0, 0, 0, 0);
            if constexpr (fold_here) fold_slot1<XI - 1, 0>(S, mprev, k2, k4);
            m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.h, a0.h, m0, 0, 0, 0);
            if constexpr (fold_here) fold_slot1<XI - 1, 1>(S, mprev, k2, k4);
            asm volatile("" : "+v"(m0));  // keep this point's MFMAs in its own region
            if constexpr (acc_direct<XI, 0>()) {
                S[srow].p[0] = __builtin_shufflevector(m0, m0, 0, 1);
                S[srow].p[1] = __builtin_shufflevector(m0, m0, 2, 3);
            }
            m[0] = __builtin_shufflevector(m0, m0, 0, 1);
            m[1] = __builtin_shufflevector(m0, m0, 2, 3);
#pragma unroll
            for (int i = 0; i + 1 < PF; ++i) bq[i] = bq[i + 1];
            if constexpr (XI + PF < NP) bq[PF - 1] = b2;
            if constexpr (XI + 1 < NP) a0 = a1;
        }
        if constexpr (XI == NP) {
            fold_slot1<XI - 1, 0>(S, mprev, k2, k4);
            fold_slot1<XI - 1, 1>(S, mprev, k2, k4);
        }
        if constexpr (XI < NP) {
            mprev[0] = m[0];
            mprev[1] = m[1];
            xi_loop1<XI + 1, PF>(S, sv, u, bq, a0, mprev, k2, k4, chunk, voff);
        }
    }
}

// inputs of a chunk -> registers (1024 threads; nontemporal, zeros past the batch)
__device__ __forceinline__ void load_xq(float4 (&xr)[XPTQ], const float *__restrict__ x, int b0, int n_boards,
                                        int chunk, int tid) {
    const int rows = (n_boards - b0) * 81;
#pragma unroll
    for (int k = 0; k < XPTQ; ++k) {
        const int i = tid + k * NTQ;
        xr[k] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (i < XF4) {
            const int q = i % (KC / 4), bp = i / (KC / 4);
            if (bp < rows) {
                const floatx4 t = __builtin_nontemporal_load(
                    reinterpret_cast<const floatx4 *>(x + ((size_t)b0 * 81 + bp) * C + chunk * KC) + q);
                xr[k] = make_float4(t.x, t.y, t.z, t.w);
            }
        }
    }
}

__device__ __forceinline__ void store_xq(float *__restrict__ sX, const float4 (&xr)[XPTQ], const SetScale &sc, int tid) {
#pragma unroll
    for (int k = 0; k < XPTQ; ++k) {
        const int i = tid + k * NTQ;
        if (i < XF4) {
            const int q = i % (KC / 4), bp = i / (KC / 4);
            const int kb = bp / 81, pos = bp - 81 * kb, sp = spos(kb, pos / 9, pos % 9);
            const float sv = sc.of(kb);
            float4 v = xr[k];
            v.x *= sv;
            v.y *= sv;
            v.z *= sv;
            v.w *= sv;
            reinterpret_cast<float4 *>(sX + sp * KC)[q] = v;
        }
    }
}

// set_epilogue for the wave's block tb
template <bool RES>
__device__ __forceinline__ void set_epilogue1(Acc1 (&S)[15], int st, int tb, const SetScale &sc, float u_scale,
                                              floatx4 bb4, const float *__restrict__ res, float *__restrict__ y,
                                              uint32_t *__restrict__ y_amax, int n_boards, int tid, int lane) {
    const int grp = st >> 1, h = st & 1;
    const int el = fresh(lane);
    const int gt = 32 * h + 16 * tb + (el & 15), gb = gt / 9, tt = gt - 9 * gb;
    const int board = GB * grp + gb;
    const bool live = gt < GB * 9 && board < n_boards;
    const int co4e = ((fresh(tid) >> 6) & 7) * 16 + 4 * (el >> 4);
    const size_t off = ((size_t)board * 81 + (tt / 3) * 27 + (tt % 3) * 3) * C + co4e;
    const float inv = 1.0f / (sc.of(gb - 3 * h) * u_scale);
    float vmax = 0.0f;
    floatx4 rv[9];
    if constexpr (RES) {
#pragma unroll
        for (int ab = 0; ab < 9; ++ab) {
            rv[ab] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
            if (live) rv[ab] = *reinterpret_cast<const floatx4 *>(res + off + ((ab / 3) * 9 + ab % 3) * C);
        }
    }
    floatx4 Y[9];
#pragma unroll
    for (int ab = 0; ab < 9; ++ab) {
        const int a = ab / 3, b = ab % 3;
        floatx4 acc = {};
#pragma unroll
        for (int v = 0; v < 5; ++v) {
            if (at(b, v) == 0) continue;
            const Acc1 &q = S[a * 5 + v];
            const floatx4 s4 = {q.p[0].x, q.p[0].y, q.p[1].x, q.p[1].y};
            acc = at(b, v) == 1 ? acc + s4
                : at(b, v) == -1 ? acc - s4
                                 : __builtin_elementwise_fma(floatx4((float)at(b, v)), s4, acc);
        }
        Y[ab] = acc;
    }
#pragma unroll
    for (int i = 0; i < 15; ++i) {
        S[i].p[0] = floatx2{0.0f, 0.0f};
        S[i].p[1] = floatx2{0.0f, 0.0f};
    }
#pragma unroll
    for (int ab = 0; ab < 9 && live; ++ab) {
        floatx4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = __builtin_fmaf(Y[ab][r], inv, bb4[r]);
        if constexpr (RES) v += rv[ab];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.0f);
        *reinterpret_cast<floatx4 *>(y + off + ((ab / 3) * 9 + ab % 3) * C) = v;
        vmax = fmaxf(vmax, fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])));
    }
    if (y_amax) {
        vmax = fmaxf(vmax, __shfl_xor(vmax, 16));
        vmax = fmaxf(vmax, __shfl_xor(vmax, 32));
        if (el < 16 && live) atomicMax(y_amax + board, __builtin_bit_cast(uint32_t, vmax));
    }
}

template <bool RES, int PF = 3>
__global__ __launch_bounds__(NTQ) void k_wino3q_conv(const float *__restrict__ x, const uint16_t *__restrict__ u,
                                                     float u_scale, const float *__restrict__ bias,
                                                     const float *__restrict__ res, float *__restrict__ y,
                                                     const uint32_t *__restrict__ x_amax, int x_amax_per_board,
                                                     uint32_t *__restrict__ y_amax, uint32_t *__restrict__ amax_clear,
                                                     int clear_count, int n_boards) {
    __shared__ __attribute__((aligned(16))) char smem[XP * KC * 4 + VB];
    float *const sX = reinterpret_cast<float *>(smem);
    char *const sV = smem + XP * KC * 4;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wc = wv & 7, tb = wv >> 3;
    for (int i = (int)blockIdx.x * NTQ + tid; i < clear_count; i += (int)gridDim.x * NTQ) amax_clear[i] = 0u;
    const int nsets = n_sets(n_boards);
    if ((int)blockIdx.x >= nsets) return;
    const int my_sets = (nsets - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
    const int G = my_sets * NCH;
    auto set_of = [&](int g) { return (int)blockIdx.x + (g / NCH) * (int)gridDim.x; };
    auto set_b0 = [&](int g) { const int st = set_of(g); return GB * (st >> 1) + 3 * (st & 1); };
    const int co4 = wc * 16 + 4 * (lane >> 4);
    const floatx4 bb4 = *reinterpret_cast<const floatx4 *>(bias + co4);

    Acc1 S[15];
#pragma unroll
    for (int i = 0; i < 15; ++i) {
        S[i].p[0] = floatx2{0.0f, 0.0f};
        S[i].p[1] = floatx2{0.0f, 0.0f};
    }
    const floatx2 k2 = {2.0f, 2.0f}, k4 = {4.0f, 4.0f};
    float4 xr[XPTQ];
    const rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(u), 0, NP * C * C * 4, 0x00020000);
    const int kq = lane >> 4;
    const int voff = wc * 1024 + lane * 16;
    const char *sv_lane = sV + tb * 2 * VPLANE + kq * 256 + (((lane & 15) ^ (2 * kq)) * 16);

    for (int i = fresh(tid); i < NPAD * (KC / 4); i += NTQ) {
        const int j = i / (KC / 4), q = i % (KC / 4);
        const int pos = j < 50 ? (j / 10) * 10 * SR + j % 10
                      : (j < 86 ? (((j - 50) / 9) * 10 + (j - 50) % 9 + 1) * SR : XP - 1);
        reinterpret_cast<float4 *>(sX + pos * KC)[q] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    __syncthreads();
    SetScale sc = set_scale(x_amax, x_amax_per_board, set_b0(0), n_boards);
    load_xq(xr, x, set_b0(0), n_boards, 0, tid);
    store_xq(sX, xr, sc, tid);
    __syncthreads();
#pragma unroll 1
    for (int g = 0; g < G; ++g) {
        const int c = g % NCH;
        if (g + 1 < G) load_xq(xr, x, set_b0(g + 1), n_boards, (g + 1) % NCH, fresh(tid));
        SetScale sc_next = sc;
        if (c == NCH - 1 && g + 1 < G) sc_next = set_scale(x_amax, x_amax_per_board, set_b0(g + 1), n_boards);
        if (wv < NITEM / 64) {  // waves 0-7: one item per thread, column by column (inputs already scaled)
            const TItem ti = t_item(sX, sV, fresh(tid), set_of(g) & 1, 1.0f);
            col_all<0, false>(ti);
            col_all<1, false>(ti);
            col_all<2, false>(ti);
            col_all<3, false>(ti);
            col_all<4, false>(ti);
        }
        BFrag bq[PF];  // this chunk's first U fragments
#pragma unroll
        for (int i = 0; i < PF; ++i) bq[i] = load_b(ur, i, c, voff);
        lds_barrier();
        if (g + 1 < G) store_xq(sX, xr, sc_next, fresh(tid));
        {
            AFrag1 a0 = load_a1(sv_lane, 0);
            floatx2 mprev[2];
            xi_loop1<0, PF>(S, sv_lane, ur, bq, a0, mprev, k2, k4, c, voff);
        }
        if (c == NCH - 1) set_epilogue1<RES>(S, set_of(g), tb, sc, u_scale, bb4, res, y, y_amax, n_boards, tid, lane);
        sc = sc_next;
        lds_barrier();
    }
}

}  // namespace wino3h
}  // namespace uttt
