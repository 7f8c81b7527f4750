// wino3h_impl.h — k_wino3h_conv, the split-f16 Winograd F(3x3,3x3) tower conv, as a template
// shared by the product library (csrc/wino3h_conv.hip: MODE 0 only) and the diagnostics library
// (csrc/diag/wino3h_diag.hip: timing ablations, phase stamps, prefetch variants). MODE bits are
// `if constexpr` branches: MODE 0 compiles none of them. Algorithm and layout: wino3h_conv.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdint>

#include "uttt_nn.h"

namespace uttt {

namespace wino3h {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef float floatx8 __attribute__((ext_vector_type(8)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));

constexpr int C = 128;        // channels in and out
constexpr int NP = 25;        // transform points
constexpr int KC = 32;        // input channels per chunk (one K=32 MFMA step)
constexpr int NCH = C / KC;   // chunks per set
constexpr int GB = 7;         // boards per group: its 63 tiles are two sets of 32 tile slots
constexpr int TS = 32;        // tile slots per set (two 16-tile MFMA blocks; the group's 64th is empty)
constexpr int SB = 4;         // boards a set's tiles touch: boards 0-3 or 3-6 of its group
constexpr int SR = 10;        // staged row stride: one zero column (shared by neighbouring rows) + 9 cells
constexpr int XP = (SB * 10 + 1) * SR + 1;  // staged positions (411): boards stacked under shared zero rows
constexpr int NT = 512;       // threads (8 waves)
constexpr int NITEM = TS * (KC / 2);             // transform items per chunk (tile slot, channel pair): 512
constexpr int VPLANE = 1024;                     // bytes of one (xi, rt, hi|lo) A plane: 4 kq x 16 rows x 16 B
constexpr int VB = NP * 4 * VPLANE;              // V bytes: [xi][rt][h][kq][row^2kq][8 f16]
constexpr int XF4 = SB * 81 * (KC / 4);          // float4s staged per chunk (2592)
constexpr int XPT = (XF4 + NT - 1) / NT;         // per thread (6)
static_assert(NITEM == NT, "one transform item per thread");
constexpr int NPAD = XP - SB * 81;  // zero positions of the staged layout (87)
static_assert(NPAD == 5 * 10 + 4 * 9 + 1, "pad positions: shared zero rows, zero column, last position");
static_assert(XP * KC * 4 + VB <= 160 * 1024, "LDS");

// Sets of n boards: two per full group of 7, one or two for a partial last group
// (the first set of a group covers boards 0-2 and 5 tiles of board 3).
__host__ __device__ constexpr int n_sets(int n) { return 2 * (n / GB) + (n % GB == 0 ? 0 : (n % GB <= 3 ? 1 : 2)); }
// Staged position of cell (r, c) of staged board k; r or c = -1 / 9 land on zero pads.
__host__ __device__ constexpr int spos(int k, int r, int c) { return (10 * k + r + 1) * SR + c + 1; }

// Toom-Cook F(3,3) on {0, 1, -1, 2, inf} (as wino3_conv.hip)
__host__ __device__ constexpr int at(int a, int u) {
    constexpr int m[3][5] = {{1, 1, 1, 1, 0}, {0, 1, -1, 2, 0}, {0, 1, 1, 4, 1}};
    return m[a][u];
}

// Variant bits (diagnostic builds; the product is MODE 0)
constexpr int kNoALookahead = 1 << 21;  // V fragments read at their own point (frees 16 VGPRs for U prefetch)
constexpr int kBufferX = 1 << 22;       // input loads as buffer loads, zero beyond the batch: no branches
constexpr int kFoldBuiltin = 1 << 23;   // fold as compiler-visible ops (hazards padded by the compiler)
constexpr int kFoldScalar = 1 << 24;    // ... as scalar v_add_f32 / v_fma_f32 pairs (TU built with -fno-slp-vectorize)
constexpr int kALook2 = 1 << 25;        // V fragments two points ahead (LDS latency) instead of one
constexpr int kSerialPrologue = 1 << 26;  // sX pads zeroed and fenced before the first loads are issued
constexpr int kSplitCvt = 1 << 27;        // f16 lo of the split by convert back, subtract, convert (round 2)
constexpr int kF16 = (int)(1u << 31);     // f16 mode (not f32-level): M = Vhi Uhi only, U's hi plane only (uttt_nn_*_f16)
constexpr int kL2Prefetch = 1 << 28;      // the inputs two chunks ahead touched into L2 (one dword per 128-B row)
constexpr int kFoldAT = 1 << 18;          // the fold along u by A^T itself (rounds 1-3) instead of Z A^T
constexpr int kEpiBarrier = 1 << 7;       // a set's epilogue starts after every wave's last point GEMMs (a barrier):
                                          // the earlier waves' epilogue VALU no longer takes the issue slots of
                                          // their SIMD partners' last point GEMMs
constexpr int kEpiOrder = 1 << 12;        // epilogue by branch-free buffer loads / stores, tile block 1's residual requested
                                           // before block 0's stores (round 5: same bits, 1-5% slower than the product)
constexpr int kEpiLoad = 1 << 14;
constexpr int kEpiNT = 1 << 15;            // kEpiOrder with nontemporal output stores          // the next set's second chunk's inputs requested before the epilogue's stores
constexpr int kResEarly = 1 << 11;        // residual form: both tile blocks' residual loads issued at the epilogue's start
constexpr int kEpiPrio = 1 << 10;         // ... instead: waves 4-7 run a set's last point loop at s_setprio 1
constexpr int kEarlyLoad = 1 << 19;       // the chunk-after-next's inputs requested at the end of this chunk's
                                          // point GEMMs (before the barrier the earlier waves wait at), except
                                          // after a set's last chunk (its epilogue needs the registers)
constexpr int kStagger = 1 << 30;         // waves 4-7 walk the 25 points from kStaggerRot on (their SIMD partners
                                          // from 0), so the partners' fold-free and fold-heavy points interleave
constexpr int kStaggerRot = 12;
constexpr int kHandoff = 1 << 20;         // k_wino3t_tower: every load of an activation, residual or per-board max
                                          // another workgroup of the launch wrote, and every such store, is sc1
                                          // (write-through, L1 bypassed): the hand-off needs no fence
                                          // (MI355X_MICROARCH.md, inter-workgroup visibility, table row 1)
constexpr int kFoldPacked = 1 << 29;      // fold as inline-asm packed v_pk_add_f32 / v_pk_fma_f32 (rounds 1-3)

struct Acc {
    floatx2 p[4];  // pairs 0-1: rows block 0 (4 tiles), 2-3: block 1
};

// fold of point P, as single packed ops o = (row a with A^T[a][u] != 0, pair j),
// spread over the next point's six MFMA slots
__host__ __device__ constexpr int n_rows(int u) { return (at(0, u) != 0) + (at(1, u) != 0) + (at(2, u) != 0); }
__host__ __device__ constexpr int nth_row(int u, int i) {
    int a = 0;
    for (; a < 3; ++a)
        if (at(a, u) != 0 && i-- == 0) break;
    return a;
}

// The fold's transform along u (round 4). Rounds 1-3 accumulated S = A^T M. Any invertible Z gives
// the same output through S' = (Z A^T) M, Y = (Z^-1 S') A, and Z = [c0 c1 c4]^-1 (ci the columns of
// A^T) makes three of Z A^T's five columns unit vectors: points u = 0, 1, 4 (15 of 25) accumulate
// straight into their S' row as the MFMA's C operand, and only u = 2, 3 are folded, with integer
// coefficients (2, -1: exact scalings). Fold ops per chunk: 15 -> 10 folded points, 360 -> 240 f32 adds
// per wave. Z^-1 = [[1,1,0],[0,1,0],[0,1,1]]: the epilogue restores S[0] = S'[0] + S'[1], S[2] = S'[2] + S'[1].
__host__ __device__ constexpr int zat(int a, int u) {
    constexpr int m[3][5] = {{1, 0, 2, -1, 0}, {0, 1, -1, 2, 0}, {0, 0, 2, 2, 1}};
    return m[a][u];
}
template <int MODE>
__host__ __device__ constexpr int fat(int a, int u) { return (MODE & kFoldAT) ? at(a, u) : zat(a, u); }
template <int MODE>
__host__ __device__ constexpr int f_rows(int u) { return (fat<MODE>(0, u) != 0) + (fat<MODE>(1, u) != 0) + (fat<MODE>(2, u) != 0); }
template <int MODE>
__host__ __device__ constexpr int f_nth(int u, int i) {
    int a = 0;
    for (; a < 3; ++a)
        if (fat<MODE>(a, u) != 0 && i-- == 0) break;
    return a;
}

// Points whose fold column has one nonzero (coefficient 1) accumulate straight into their S row as
// the MFMA's C operand (round 2: u = 0 / 4 under A^T; round 4: u = 0 / 1 / 4 under Z A^T)
template <int P, int MODE>
__host__ __device__ constexpr bool acc_direct() { return f_rows<MODE>(P / 5) == 1; }

template <int P, int O, int MODE>
__device__ __forceinline__ void fold_op(Acc (&S)[15], const floatx2 (&m)[4], floatx2 k2, floatx2 k4) {
    constexpr int u = P / 5, v = P % 5;
    if constexpr (O < 4 * f_rows<MODE>(u) && !acc_direct<P, MODE>()) {
        constexpr int a = f_nth<MODE>(u, O / 4), j = O % 4, K = fat<MODE>(a, u);
        // Inline asm is outside the compiler's hazard recognizer, so nothing pads these reads of
        // the previous point's MFMA results; the schedule keeps >= 6 instructions, one of them an
        // MFMA, between producer and reader, and the output bits equal those of a compiler-visible
        // fold (builtin packed ops, hazard-padded; 7% slower from spills) on the same inputs
        // (round 2, tools/diag/wino3h_modes.py).
        if constexpr (MODE & kFoldScalar) {
            floatx2 &t = S[a * 5 + v].p[j];
            if constexpr (K == 1) {
                t.x = t.x + m[j].x;
                t.y = t.y + m[j].y;
            } else if constexpr (K == -1) {
                t.x = t.x - m[j].x;
                t.y = t.y - m[j].y;
            } else {
                t.x = __builtin_fmaf(m[j].x, (float)K, t.x);
                t.y = __builtin_fmaf(m[j].y, (float)K, t.y);
            }
        } else if constexpr (MODE & kFoldBuiltin) {
            if constexpr (K == 1) S[a * 5 + v].p[j] = S[a * 5 + v].p[j] + m[j];
            else if constexpr (K == -1) S[a * 5 + v].p[j] = S[a * 5 + v].p[j] - m[j];
            else S[a * 5 + v].p[j] = __builtin_elementwise_fma(m[j], K == 2 ? k2 : k4, S[a * 5 + v].p[j]);
        } else if constexpr (!(MODE & kFoldPacked)) {
            // product: two scalar ops per pair. A packed f32 op beside MFMAs costs several times its
            // issue slot (MI355X_MICROARCH.md, price of one filler: 2 v_pk_add_f32 +26 cycles against 2
            // v_fma_f32); the scalar pair gives the same bits (round 4, tools/diag/wino3h_variants.py:
            // 1,344 boards 71.7-73.3 -> 67.2-67.6 us, 16,384 boards 722-737 -> 689-694 us)
            floatx2 &t = S[a * 5 + v].p[j];
            if constexpr (K == 1) {
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(t.x) : "v"(m[j].x));
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(t.y) : "v"(m[j].y));
            } else if constexpr (K == -1) {
                asm volatile("v_sub_f32 %0, %0, %1" : "+v"(t.x) : "v"(m[j].x));
                asm volatile("v_sub_f32 %0, %0, %1" : "+v"(t.y) : "v"(m[j].y));
            } else if constexpr (K == 2) {
                asm volatile("v_fma_f32 %0, %1, 2.0, %0" : "+v"(t.x) : "v"(m[j].x));
                asm volatile("v_fma_f32 %0, %1, 2.0, %0" : "+v"(t.y) : "v"(m[j].y));
            } else {
                asm volatile("v_fma_f32 %0, %1, 4.0, %0" : "+v"(t.x) : "v"(m[j].x));
                asm volatile("v_fma_f32 %0, %1, 4.0, %0" : "+v"(t.y) : "v"(m[j].y));
            }
        } else if constexpr (K == 1) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(S[a * 5 + v].p[j]) : "v"(m[j]));
        else if constexpr (K == -1)
            asm volatile("v_pk_add_f32 %0, %0, %1 neg_lo:[0,1] neg_hi:[0,1]" : "+v"(S[a * 5 + v].p[j]) : "v"(m[j]));
        else if constexpr (K == 2) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(S[a * 5 + v].p[j]) : "v"(m[j]), "v"(k2));
        else asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(S[a * 5 + v].p[j]) : "v"(m[j]), "v"(k4));
    }
}

constexpr int NSLOT = 6;  // MFMAs per point
template <int P, int SL, int MODE, int O = 0>
__device__ __forceinline__ void fold_slot(Acc (&S)[15], const floatx2 (&m)[4], floatx2 k2, floatx2 k4) {
    constexpr int nops = 4 * f_rows<MODE>(P / 5);
    if constexpr (O < nops) {
        if constexpr (O * NSLOT / nops == SL) fold_op<P, O, MODE>(S, m, k2, k4);
        fold_slot<P, SL, MODE, O + 1>(S, m, k2, k4);
    }
}

template <int P, int MODE>
__device__ __forceinline__ void fold_all(Acc (&S)[15], const floatx2 (&m)[4], floatx2 k2, floatx2 k4) {
    fold_slot<P, 0, MODE>(S, m, k2, k4);
    fold_slot<P, 1, MODE>(S, m, k2, k4);
    fold_slot<P, 2, MODE>(S, m, k2, k4);
    fold_slot<P, 3, MODE>(S, m, k2, k4);
    fold_slot<P, 4, MODE>(S, m, k2, k4);
    fold_slot<P, 5, MODE>(S, m, k2, k4);
}

// U fragments (hi, lo) of one point: U[xi][chunk][h][co/16][kq][co%16][8 f16]; each of the
// two loads reads 1 KB contiguous and lane-linear per wave (hi and lo planes 8 KB apart)
struct BFrag {
    halfx8 h, l;
};
constexpr int UPLANE = C * 4 * 16;  // bytes of one (xi, chunk, hi|lo) plane
template <bool HI = false>  // HI: the hi plane only (kF16)
__device__ __forceinline__ BFrag load_b(rsrc_t u, int xi, int chunk, int voff) {
    const int soff = (xi * NCH + chunk) * 2 * UPLANE;
    BFrag b;
    b.h = __builtin_bit_cast(halfx8, __builtin_amdgcn_raw_buffer_load_b128(u, voff, soff, 0));
    if constexpr (HI) b.l = b.h;
    else b.l = __builtin_bit_cast(halfx8, __builtin_amdgcn_raw_buffer_load_b128(u, voff + UPLANE, soff, 0));
    return b;
}
// the XI-th point a wave visits: the points in order from ROT (0 in the product)
template <int XI, int ROT>
__host__ __device__ constexpr int pt() { return (XI + ROT) % NP; }
// un: the weights of the workgroup's next chunk when it is another conv's (k_wino3t_tower: a set's last
// chunk prefetches the next work item's U), else u
template <int XI, int ROT = 0, bool HI = false>
__device__ __forceinline__ BFrag load_b_ahead(rsrc_t u, int chunk, int voff, rsrc_t un) {
    if constexpr (XI < NP) return load_b<HI>(u, pt<XI, ROT>(), chunk, voff);
    else return load_b<HI>(un, pt<XI - NP, ROT>(), (chunk + 1) % NCH, voff);  // next chunk in this workgroup's order
}

// A fragments (V hi / lo of both row blocks) of one point
struct AFrag {
    halfx8 h0, l0, h1, l1;
};
template <bool HI = false>  // HI: the hi planes only (kF16)
__device__ __forceinline__ AFrag load_a(const char *__restrict__ sv, int xi) {
    // sv already points at this lane's 16-byte slot within a plane
    const char *p = sv + xi * 4 * VPLANE;
    AFrag a;
    a.h0 = *reinterpret_cast<const halfx8 *>(p);
    a.h1 = *reinterpret_cast<const halfx8 *>(p + 2 * VPLANE);
    if constexpr (HI) {
        a.l0 = a.h0;
        a.l1 = a.h1;
    } else {
        a.l0 = *reinterpret_cast<const halfx8 *>(p + VPLANE);
        a.l1 = *reinterpret_cast<const halfx8 *>(p + 3 * VPLANE);
    }
    return a;
}

// Point loop, software-pipelined: B PF points ahead (L2), A one point ahead (LDS).
// The fold of point XI-1 is issued among point XI's MFMAs.
template <int XI, int MODE, int PF, int ROT = 0>
__device__ __forceinline__ void xi_loop(Acc (&S)[15], const char *__restrict__ sv, rsrc_t u, BFrag (&bq)[PF],
                                        AFrag &a0, floatx2 (&mprev)[4], floatx2 k2, floatx2 k4, int chunk, int voff,
                                        AFrag *a_next, rsrc_t un) {
    if constexpr (XI <= NP) {
        floatx2 m[4];
        if constexpr (XI < NP) {
            BFrag b2;
            if constexpr (MODE & 32) {  // diagnostic: no B loads (operands reused, laundered)
                b2 = bq[0];
                asm volatile("" : "+v"(b2.h), "+v"(b2.l));
            } else {
                b2 = load_b_ahead<XI + PF, ROT, (MODE & kF16) != 0>(u, chunk, voff, un);
            }
            const BFrag b0 = bq[0];
            if constexpr (MODE & kNoALookahead) a0 = load_a<(MODE & kF16) != 0>(sv, pt<XI, ROT>());  // this point's V, waited for here
            AFrag a1, a2;
            if constexpr (MODE & kALook2) {  // a_next holds point XI+1 (loaded a point ago); load XI+2
                if constexpr (XI + 1 < NP) a1 = *a_next;
                if constexpr (XI + 2 < NP) a2 = load_a<(MODE & kF16) != 0>(sv, pt<XI + 2, ROT>());
            } else if constexpr (XI + 1 < NP && !(MODE & kNoALookahead)) {
                if constexpr (MODE & 16) {  // diagnostic: no A loads
                    a1 = a0;
                    asm volatile("" : "+v"(a1.h0), "+v"(a1.l0), "+v"(a1.h1), "+v"(a1.l1));
                } else {
                    a1 = load_a<(MODE & kF16) != 0>(sv, pt<XI + 1, ROT>());
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            floatx4 m0 = {}, m1 = {};
            constexpr int P = pt<XI, ROT>();
            constexpr int srow = f_nth<MODE>(P / 5, 0) * 5 + P % 5;  // the S row of a direct point
            if constexpr (acc_direct<P, MODE>()) {
                m0 = floatx4{S[srow].p[0].x, S[srow].p[0].y, S[srow].p[1].x, S[srow].p[1].y};
                m1 = floatx4{S[srow].p[2].x, S[srow].p[2].y, S[srow].p[3].x, S[srow].p[3].y};
            }
            constexpr bool fold_here = XI > 0 && !(MODE & 64);
            if constexpr (MODE & kF16) {  // the hi x hi product alone, the fold spread over its two MFMAs
                m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.h, a0.h0, m0, 0, 0, 0);
                if constexpr (fold_here) {
                    fold_slot<pt<XI - 1, ROT>(), 0, MODE>(S, mprev, k2, k4);
                    fold_slot<pt<XI - 1, ROT>(), 1, MODE>(S, mprev, k2, k4);
                    fold_slot<pt<XI - 1, ROT>(), 2, MODE>(S, mprev, k2, k4);
                }
                m1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.h, a0.h1, m1, 0, 0, 0);
                if constexpr (fold_here) {
                    fold_slot<pt<XI - 1, ROT>(), 3, MODE>(S, mprev, k2, k4);
                    fold_slot<pt<XI - 1, ROT>(), 4, MODE>(S, mprev, k2, k4);
                    fold_slot<pt<XI - 1, ROT>(), 5, MODE>(S, mprev, k2, k4);
                }
            } else {
                // small terms first, then the hi x hi product
                m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.l, a0.h0, m0, 0, 0, 0);
                if constexpr (fold_here) fold_slot<pt<XI - 1, ROT>(), 0, MODE>(S, mprev, k2, k4);
                m1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.l, a0.h1, m1, 0, 0, 0);
                if constexpr (fold_here) fold_slot<pt<XI - 1, ROT>(), 1, MODE>(S, mprev, k2, k4);
                m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.h, a0.l0, m0, 0, 0, 0);
                if constexpr (fold_here) fold_slot<pt<XI - 1, ROT>(), 2, MODE>(S, mprev, k2, k4);
                m1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.h, a0.l1, m1, 0, 0, 0);
                if constexpr (fold_here) fold_slot<pt<XI - 1, ROT>(), 3, MODE>(S, mprev, k2, k4);
                m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.h, a0.h0, m0, 0, 0, 0);
                if constexpr (fold_here) fold_slot<pt<XI - 1, ROT>(), 4, MODE>(S, mprev, k2, k4);
                m1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.h, a0.h1, m1, 0, 0, 0);
                if constexpr (fold_here) fold_slot<pt<XI - 1, ROT>(), 5, MODE>(S, mprev, k2, k4);
            }
            asm volatile("" : "+v"(m0), "+v"(m1));  // keep this point's MFMAs in its own region
            if constexpr (acc_direct<P, MODE>()) {
                S[srow].p[0] = __builtin_shufflevector(m0, m0, 0, 1);
                S[srow].p[1] = __builtin_shufflevector(m0, m0, 2, 3);
                S[srow].p[2] = __builtin_shufflevector(m1, m1, 0, 1);
                S[srow].p[3] = __builtin_shufflevector(m1, m1, 2, 3);
            }
            m[0] = __builtin_shufflevector(m0, m0, 0, 1);
            m[1] = __builtin_shufflevector(m0, m0, 2, 3);
            m[2] = __builtin_shufflevector(m1, m1, 0, 1);
            m[3] = __builtin_shufflevector(m1, m1, 2, 3);
#pragma unroll
            for (int i = 0; i + 1 < PF; ++i) bq[i] = bq[i + 1];
            bq[PF - 1] = b2;
            if constexpr (XI + 1 < NP && !(MODE & kNoALookahead)) a0 = a1;
            if constexpr ((MODE & kALook2) && XI + 2 < NP) *a_next = a2;
        }
        if constexpr (XI == NP && !(MODE & 64)) fold_all<pt<XI - 1, ROT>(), MODE>(S, mprev, k2, k4);  // nothing left to spread it over
        if constexpr (XI < NP) {
#pragma unroll
            for (int i = 0; i < 4; ++i) mprev[i] = m[i];
            xi_loop<XI + 1, MODE, PF, ROT>(S, sv, u, bq, a0, mprev, k2, k4, chunk, voff, a_next, un);
        }
    }
}

// inputs of chunk `chunk` of the set starting at board b0 -> registers
template <int MODE>
__device__ __forceinline__ void load_x(float4 (&xr)[XPT], const float *__restrict__ x, int b0, int n_boards, int chunk,
                                       int tid) {
    // the staged boards are consecutive: their positions are one run of rows of x
    const int rows = (n_boards - b0) * 81;
    if constexpr (MODE & (kBufferX | kHandoff)) {
        // one resource per set whose range ends at the batch's last board: loads past it return 0,
        // so no lane branches and the compiler counts the loads exactly (precise vmcnt waits)
        const int nb = min(rows, SB * 81);
        const rsrc_t xr_ = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(x + (size_t)b0 * 81 * C), 0,
                                                             nb * C * 4, 0x00020000);
#pragma unroll
        for (int k = 0; k < XPT; ++k) {
            const int i = tid + k * NT;
            const int q = i % (KC / 4), bp = i / (KC / 4);
            const int off = i < XF4 ? (bp * C + chunk * KC + 4 * q) * 4 : 0x7ffffff0;
            const floatx4 t = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr_, off, 0,
                                                                                               (MODE & kHandoff) ? 16 : 2));
            xr[k] = make_float4(t.x, t.y, t.z, t.w);
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
        const int i = tid + k * NT;
        xr[k] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (i < XF4) {
            const int q = i % (KC / 4), bp = i / (KC / 4);
            if (bp < rows) {
                const float4 *src = reinterpret_cast<const float4 *>(x + ((size_t)b0 * 81 + bp) * C + chunk * KC) + q;
                if constexpr (!(MODE & 512)) {
                    const floatx4 t = __builtin_nontemporal_load(reinterpret_cast<const floatx4 *>(src));
                    xr[k] = make_float4(t.x, t.y, t.z, t.w);
                }
                else xr[k] = *src;
            }
        }
    }
}

// Per-board V scales of the SB staged boards of a set (powers of two, uniform over the workgroup)
struct SetScale {
    static_assert(SB == 4, "of() selects among exactly four staged boards");
    float s[SB];
    __device__ __forceinline__ float of(int kb) const {
        // a select chain, not a dynamically indexed array (that would live in scratch)
        return kb == 0 ? s[0] : (kb == 1 ? s[1] : (kb == 2 ? s[2] : s[3]));
    }
};

// registers -> sX[padded position][32 channels], scaled by its board's sv (a power of two: exact)
__device__ __forceinline__ void store_x(float *__restrict__ sX, const float4 (&xr)[XPT], const SetScale &sc, int tid) {
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
        const int i = tid + k * NT;
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

// x -> B^T x for one 5-vector (channel pairs), common subexpressions shared
__device__ __forceinline__ void bt5(const floatx2 (&d)[5], floatx2 (&t)[5]) {
    const floatx2 two = {2.0f, 2.0f}, mtwo = {-2.0f, -2.0f};
    const floatx2 e = d[3] - d[2];
    const floatx2 f = d[1] - d[2];
    const floatx2 t3 = d[3] - d[1];
    const floatx2 g = d[0] - d[2];
    const floatx2 h = d[4] - d[2];
    t[0] = __builtin_elementwise_fma(two, g, t3);
    t[1] = __builtin_elementwise_fma(mtwo, d[1], e);
    t[2] = __builtin_elementwise_fma(two, f, e);
    t[3] = t3;
    t[4] = __builtin_elementwise_fma(mtwo, t3, h);
}

// (v0, v1) -> packed f16 hi (round to nearest: |v - hi| <= 2^-11 |v|, exact in f32) and
// f16 lo = the remainder rounded to nearest. hi is one v_cvt_pk_f16_f32. lo is one
// v_fma_mixlo_f16 + one v_fma_mixhi_f16 (-hi * 1 + v from the f16 half of hi, rounded to
// f16): v - hi is exact in f32 (Sterbenz), so this equals converting hi back, subtracting and
// converting (5 instructions and a hazard nop; MIX = false, diagnostics) bit for bit.
// The compiler folds an fma on a converted half back into that sequence, hence the asm.
typedef _Float16 halfx2 __attribute__((ext_vector_type(2)));
template <bool MIX = true>
__device__ __forceinline__ void split(floatx2 v, uint32_t &hi, uint32_t &lo) {
    const halfx2 h = __builtin_convertvector(v, halfx2);
    hi = __builtin_bit_cast(uint32_t, h);
    if constexpr (MIX) {
        uint32_t l;
        asm volatile("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(l) : "v"(hi), "v"(v.x));
        asm volatile("v_fma_mixhi_f16 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(l) : "v"(hi), "v"(v.y));
        lo = l;
    } else {
        const floatx2 r = v - __builtin_convertvector(h, floatx2);
        lo = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, halfx2));
    }
}

// V = B^T d B for item it = (tile slot lt, channel pair p) of a set that is half h of its
// group -> split -> sV in fragment order, in two halves: transform_rows (u = d B; reads sX
// only) and transform_cols (V = B^T u, split, LDS stores into sV). Slot 31 of the second half has no tile: it repeats tile 62, whose
// results the epilogue drops.
__device__ __forceinline__ void transform_rows(floatx2 (&uu)[5][5], const float *__restrict__ sX, int it, int h) {
    const int p = it % (KC / 2), lt = it / (KC / 2);
    const int gt = min(32 * h + lt, GB * 9 - 1), gb = gt / 9, tt = gt - 9 * gb, ty = tt / 3, tx = tt % 3;
    const float *xs = sX + spos(gb - 3 * h, 3 * ty - 1, 3 * tx - 1) * KC + 2 * p;
    // one row of d live at a time (loads one row ahead; fenced so the scheduler does not
    // hoist all 25 of them next to the fifteen live accumulators)
    floatx2 d[2][5];
#pragma unroll
    for (int j = 0; j < 5; ++j) d[0][j] = *reinterpret_cast<const floatx2 *>(xs + j * KC);
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        if (i < 4) {
#pragma unroll
            for (int j = 0; j < 5; ++j) d[(i + 1) & 1][j] = *reinterpret_cast<const floatx2 *>(xs + ((i + 1) * SR + j) * KC);
        }
        __builtin_amdgcn_sched_barrier(0);
        bt5(d[i & 1], uu[i]);
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <bool MIX = true, bool HI = false>
__device__ __forceinline__ void transform_cols(char *__restrict__ sv, const floatx2 (&uu)[5][5], int it) {
    const int p = it % (KC / 2), lt = it / (KC / 2);
    // A fragment: lane (row m, kq) holds k = 8kq..8kq+7; channel pair p is k = 2p, 2p+1
    const int rt = lt >> 4, m = lt & 15, kq = p >> 2, w = p & 3;
    char *base = sv + rt * 2 * VPLANE + kq * 256 + ((m ^ (2 * kq)) * 16) + 4 * w;
#pragma unroll
    for (int b = 0; b < 5; ++b) {
        const floatx2 col[5] = {uu[0][b], uu[1][b], uu[2][b], uu[3][b], uu[4][b]};
        floatx2 o[5];
        bt5(col, o);
#pragma unroll
        for (int a = 0; a < 5; ++a) {
            uint32_t hi, lo;
            split<MIX>(o[a], hi, lo);
            char *q = base + (a * 5 + b) * 4 * VPLANE;
            *reinterpret_cast<uint32_t *>(q) = hi;
            if constexpr (!HI) *reinterpret_cast<uint32_t *>(q + VPLANE) = lo;  // kF16 never reads lo
        }
    }
}

template <bool MIX = true, bool HI = false>
__device__ __forceinline__ void transform(char *__restrict__ sv, const float *__restrict__ sX, int it, int h) {
    floatx2 uu[5][5];
    transform_rows(uu, sX, it, h);
    transform_cols<MIX, HI>(sv, uu, it);
}

// An opaque copy: index math derived from it is recomputed where it is used
// instead of being hoisted out of the chunk loop into (spilled) registers.
__device__ __forceinline__ int fresh(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

// Workgroup barrier for the LDS hand-offs only: unlike __syncthreads() it does not wait
// for outstanding global loads (the next chunk's inputs) or stores (the epilogue).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ float pow2_scale(float amax) {
    // largest power of two s with 36 * amax * s <= 2^15 (1 for 0 / non-finite)
    const float b = 36.0f * amax;
    if (!(b > 0.0f) || !(b < 3.0e38f)) return 1.0f;
    int e;
    frexpf(b, &e);  // 2^(e-1) <= b < 2^e
    e = 15 - e;
    e = e > 100 ? 100 : (e < -100 ? -100 : e);
    return ldexpf(1.0f, e);
}

// V scales of the staged boards b0 .. b0+SB-1 (boards past the end: 1). x_amax holds one
// max per board (per_board) or one bound for every board.
template <bool SC1 = false>  // SC1: the maxima were written by other workgroups of this launch (k_wino3t_tower)
__device__ __forceinline__ SetScale set_scale(const uint32_t *__restrict__ x_amax, int per_board, int b0, int n_boards) {
    SetScale sc;
#pragma unroll
    for (int k = 0; k < SB; ++k) {
        const int b = b0 + k;
        uint32_t bits;
        if constexpr (SC1)
            // (made wave-uniform again: the vector sc1 load would otherwise keep the scales in VGPRs)
            bits = per_board ? (b < n_boards ? (uint32_t)__builtin_amdgcn_readfirstlane((int)__hip_atomic_load(
                                                   const_cast<uint32_t *>(x_amax) + b, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT))
                                             : 0u)
                             : x_amax[0];
        else bits = per_board ? (b < n_boards ? x_amax[b] : 0u) : x_amax[0];
        sc.s[k] = pow2_scale(__builtin_bit_cast(float, bits));
    }
    return sc;
}

// After a set's last chunk: Y[a][b] = sum_v S[a][v] A^T[b][v], scale, bias, residual, ReLU, one 16-byte
// store per output position straight from registers, per-board output max; S is zeroed for the next set.
template <bool RES, int MODE>
__device__ __forceinline__ void set_epilogue(Acc (&S)[15], int st, const SetScale &sc, float u_scale, floatx4 bb4,
                                             const float *__restrict__ res, float *__restrict__ y,
                                             uint32_t *__restrict__ y_amax, int n_boards, int tid, int lane,
                                             int wave_base = 0, uint32_t *s_bmax = nullptr) {
    // Y[a][b] = sum_v S[a][v] A^T[b][v]; element 4rt + r is channel 16wv + 4(lane>>4) + r
    // of tile slot 16rt + (lane & 15)
    const int grp = st >> 1, h = st & 1;
    const int el = fresh(lane);
    // Straight from registers: the MFMA output puts 4 consecutive channels of one tile
    // in a lane (U is the A operand), so every output position is one 16-byte store
    // (+ one 16-byte residual load, issued before Y is formed); no LDS round trip and
    // no barrier.
    size_t off[2];
    bool live[2];
    int board_of[2];
    float inv[2];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
        const int gt = 32 * h + 16 * rt + (el & 15), gb = gt / 9, tt = gt - 9 * gb;
        const int board = GB * grp + gb;
        live[rt] = gt < GB * 9 && board < n_boards;  // not the empty slot or a board past the end
        // this lane's 4 output channels, recomputed here rather than kept live (spilled) over the loop
        const int co4e = (wave_base + (fresh(tid) >> 6)) * 16 + 4 * (el >> 4);
        off[rt] = ((size_t)board * 81 + (tt / 3) * 27 + (tt % 3) * 3) * C + co4e;
        board_of[rt] = board;
        // this tile's board's V scale times su: both powers of two, so 1/x is exact
        inv[rt] = 1.0f / (sc.of(gb - 3 * h) * u_scale);
    }
    // kHandoff: residual loads and output stores through buffer resources with sc1 (same offsets and values)
    // (k_wino3t_tower runs every conv through the RES form: res == nullptr makes the residual loads read
    // nothing (an empty range) and skips the add, so a plain conv's bits are the plain kernel's)
    [[maybe_unused]] rsrc_t yr_h, rr_h;
    [[maybe_unused]] const bool has_res = res != nullptr;
    if constexpr (MODE & kHandoff) {
        const int nbytes = n_boards * 81 * C * 4;
        yr_h = __builtin_amdgcn_make_buffer_rsrc(y, 0, nbytes, 0x00020000);
        rr_h = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(has_res ? res : y), 0, has_res ? nbytes : 0,
                                                 0x00020000);
    }
    // kResEarly (diagnostic): every residual load of the set's epilogue in flight before Y is formed
    floatx4 rve[2][9];
    if constexpr (RES && (MODE & kResEarly)) {
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int ab = 0; ab < 9; ++ab) {
                rve[rt][ab] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
                if (live[rt]) rve[rt][ab] = *reinterpret_cast<const floatx4 *>(res + off[rt] + ((ab / 3) * 9 + ab % 3) * C);
            }
    }
    if constexpr (!(MODE & kFoldAT)) {  // S = Z^-1 S': rows 0 and 2 get row 1 added (both tile blocks)
#pragma unroll
        for (int v = 0; v < 5; ++v)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                S[v].p[j] = S[v].p[j] + S[5 + v].p[j];
                S[10 + v].p[j] = S[10 + v].p[j] + S[5 + v].p[j];
            }
    }
    if constexpr (MODE & (kEpiOrder | kEpiNT)) {
        // Diagnostic (round 5): branch-free buffer loads and stores, a dead tile's (the empty slot, a board
        // past the end) at an offset past the buffer (loads return 0, stores are dropped), so the compiler
        // counts them exactly, and tile block 1's residual requested before block 0's stores, so its wait
        // does not include them (vmcnt counts loads and stores in one counter). Same bits as the product;
        // interleaved A/B 1-5% slower, so the product keeps the form below.
        // dead offset 0xFFF00000: plus the largest position offset (20 x 512 B) it stays past the range
        const uint32_t nbytes = (uint32_t)min((size_t)n_boards * 81 * C * 4, (size_t)0xFFE00000u);
        const rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(y, 0, (int)nbytes, 0x00020000);
        const rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(res ? res : y), 0, (int)nbytes, 0x00020000);
        uint32_t vo[2];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) vo[rt] = live[rt] ? (uint32_t)(off[rt] * 4) : 0xFFF00000u;
        auto rload = [&](int rt, floatx4 (&rv)[9]) {
#pragma unroll
            for (int ab = 0; ab < 9; ++ab)
                rv[ab] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(
                                                         rr, vo[rt] + ((ab / 3) * 9 + ab % 3) * C * 4, 0, 0));
        };
        floatx4 rv[9];
        if constexpr (RES) rload(0, rv);
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
            floatx4 out[9];
            float vmax = 0.0f;
#pragma unroll
            for (int ab = 0; ab < 9; ++ab) {
                const int a = ab / 3, b = ab % 3;
                floatx4 acc = {};
#pragma unroll
                for (int v = 0; v < 5; ++v) {
                    if (at(b, v) == 0) continue;
                    const Acc &q = S[a * 5 + v];
                    const floatx4 s4 = {q.p[2 * rt].x, q.p[2 * rt].y, q.p[2 * rt + 1].x, q.p[2 * rt + 1].y};
                    acc = at(b, v) == 1 ? acc + s4
                        : at(b, v) == -1 ? acc - s4
                                         : __builtin_elementwise_fma(floatx4((float)at(b, v)), s4, acc);
                }
                floatx4 o;
#pragma unroll
                for (int r = 0; r < 4; ++r) o[r] = __builtin_fmaf(acc[r], inv[rt], bb4[r]);
                if constexpr (RES) o += rv[ab];
#pragma unroll
                for (int r = 0; r < 4; ++r) o[r] = fmaxf(o[r], 0.0f);
                out[ab] = o;
                vmax = fmaxf(vmax, fmaxf(fmaxf(o[0], o[1]), fmaxf(o[2], o[3])));
            }
#pragma unroll
            for (int i = 0; i < 15; ++i) {
                S[i].p[2 * rt] = floatx2{0.0f, 0.0f};
                S[i].p[2 * rt + 1] = floatx2{0.0f, 0.0f};
            }
            if constexpr (RES)
                if (rt == 0) rload(1, rv);  // in flight under block 0's stores
#pragma unroll
            for (int ab = 0; ab < 9; ++ab)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, out[ab]), yr,
                                                       vo[rt] + ((ab / 3) * 9 + ab % 3) * C * 4, 0,
                                                       (MODE & kEpiNT) ? 2 : 0);
            if (y_amax) {
                vmax = live[rt] ? vmax : 0.0f;
                vmax = fmaxf(vmax, __shfl_xor(vmax, 16));
                vmax = fmaxf(vmax, __shfl_xor(vmax, 32));
                if (el < 16 && live[rt]) {
                    if (s_bmax) atomicMax(s_bmax + (board_of[rt] - (GB * (grp) + 3 * h)), __builtin_bit_cast(uint32_t, vmax));
                    else atomicMax(y_amax + board_of[rt], __builtin_bit_cast(uint32_t, vmax));
                }
            }
        }
        return;
    }
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
        float vmax = 0.0f;
        // tile block rt: residual loads first (in flight while Y is formed)
        floatx4 rv[9];
        if constexpr (RES && (MODE & kResEarly)) {
#pragma unroll
            for (int ab = 0; ab < 9; ++ab) rv[ab] = rve[rt][ab];
        } else if constexpr (RES) {
#pragma unroll
            for (int ab = 0; ab < 9; ++ab) {
                rv[ab] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
                if (live[rt]) {
                    if constexpr (MODE & kHandoff) {
                        rv[ab] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                 rr_h, (int)((off[rt] + ((ab / 3) * 9 + ab % 3) * C) * 4), 0, 16));
                    } else {
                        const floatx4 *src = reinterpret_cast<const floatx4 *>(res + off[rt] + ((ab / 3) * 9 + ab % 3) * C);
                        rv[ab] = (MODE & 65536) ? __builtin_nontemporal_load(src) : *src;
                    }
                }
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
                const Acc &q = S[a * 5 + v];
                const floatx4 s4 = {q.p[2 * rt].x, q.p[2 * rt].y, q.p[2 * rt + 1].x, q.p[2 * rt + 1].y};
                acc = at(b, v) == 1 ? acc + s4
                    : at(b, v) == -1 ? acc - s4
                                     : __builtin_elementwise_fma(floatx4((float)at(b, v)), s4, acc);
            }
            Y[ab] = acc;
        }
#pragma unroll
        for (int i = 0; i < 15; ++i) {
            S[i].p[2 * rt] = floatx2{0.0f, 0.0f};
            S[i].p[2 * rt + 1] = floatx2{0.0f, 0.0f};
        }
#pragma unroll
        for (int ab = 0; ab < 9 && live[rt]; ++ab) {
            floatx4 v;
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = __builtin_fmaf(Y[ab][r], inv[rt], bb4[r]);
            if constexpr (RES && (MODE & kHandoff)) {
                if (has_res) v += rv[ab];
            } else if constexpr (RES) {
                v += rv[ab];
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.0f);
            floatx4 *dst = reinterpret_cast<floatx4 *>(y + off[rt] + ((ab / 3) * 9 + ab % 3) * C);
            if constexpr (MODE & 8) {  // diagnostic: no output stores (kept live)
                asm volatile("" ::"v"(v));
            } else if constexpr (MODE & kHandoff) {
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, v), yr_h,
                                                       (int)((off[rt] + ((ab / 3) * 9 + ab % 3) * C) * 4), 0, 16);
            } else if constexpr (MODE & 131072) {
                __builtin_nontemporal_store(v, dst);
            } else {
                *dst = v;
            }
            vmax = fmaxf(vmax, fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])));
        }
        if (y_amax) {
            // the 4 lanes of a tile (lane bits 4-5: channel quads) -> one max per tile,
            // then one atomic per (tile, wave) into its board's slot
            vmax = fmaxf(vmax, __shfl_xor(vmax, 16));
            vmax = fmaxf(vmax, __shfl_xor(vmax, 32));
            if (el < 16 && live[rt]) {  // v >= 0: u32 bit order = value order
                // s_bmax: the workgroup's maxima of its staged boards in LDS, flushed to y_amax by one
                // thread per board after the next barrier (flush_bmax); else straight to y_amax
                if (s_bmax) atomicMax(s_bmax + (board_of[rt] - (GB * (grp) + 3 * h)), __builtin_bit_cast(uint32_t, vmax));
                else atomicMax(y_amax + board_of[rt], __builtin_bit_cast(uint32_t, vmax));
            }
        }
    }
}

// After the barrier that follows a set's epilogue: one global atomic per staged board with tiles in the
// set instead of one per (tile, wave) (72 per board; same-address global atomics serialize: round 3,
// the engine's striped counters), and the LDS row is cleared for the next set (>= 3 barriers later).
__device__ __forceinline__ void flush_bmax(uint32_t *s_bmax, uint32_t *__restrict__ y_amax, int b0, int n_boards,
                                           int tid) {
    if (tid < SB) {
        const uint32_t m = s_bmax[tid];
        if (m && b0 + tid < n_boards) atomicMax(y_amax + b0 + tid, m);
        s_bmax[tid] = 0u;
    }
}

// MODE+4 phase stamps (core clocks, s_memtime) of workgroups 0..63, waves 0 and 4, first 8
// chunks: per chunk [after load_x issue, after transform, after barrier+store_x, after GEMMs,
// after epilogue, after closing barrier] relative to the chunk's start.
#ifdef UTTT_DIAG_BUILD
__device__ unsigned int g_stamp[64][2][8][6];
#define UTTT_WINO3H_STAMP(b, w, g, k, v) (g_stamp[b][w][g][k] = (v))
#else
#define UTTT_WINO3H_STAMP(b, w, g, k, v) ((void)0)
#endif

// MODE (timing ablations only; 0 in the product): 1 skip the transform, 2 skip the
// point GEMMs, 64 skip the fold, 512 plain (L2-allocating) input loads, 65536 nontemporal
// residual loads, 131072 nontemporal output stores.
// The product streams the conv input with nontemporal loads: 8 lanes read one whole 128-B
// line, each line once per launch, and L2-allocating them would evict U (1.6 MB, re-read
// per set) from the XCD's L2 (-4..6% at bench batch sizes). The epilogue's residual loads
// and output stores are plain: one wave covers 64 B (16 channels) of a position's 512-B
// row, so the two waves that share a 128-B line meet in L2 instead of each moving the line
// to or from HBM (residual conv 106.7 -> 91.0 us at 1,344 boards, round 2,
// tools/diag/wino3h_modes.py).
template <bool RES, int MODE = 0, int PF = 3>
__global__ __launch_bounds__(NT) void k_wino3h_conv(const float *__restrict__ x, const uint16_t *__restrict__ u,
                                                    float u_scale, const float *__restrict__ bias,
                                                    const float *__restrict__ res, float *__restrict__ y,
                                                    const uint32_t *__restrict__ x_amax, int x_amax_per_board,
                                                    uint32_t *__restrict__ y_amax, uint32_t *__restrict__ amax_clear,
                                                    int clear_count, int n_boards, const int32_t *__restrict__ n_dev) {
    // sX [padded position][channel] (border = 0) then sV
    __shared__ __attribute__((aligned(16))) char smem[XP * KC * 4 + VB];
    __shared__ uint32_t s_bmax[SB];
    float *const sX = reinterpret_cast<float *>(smem);
    char *const sV = smem + XP * KC * 4;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid < SB) s_bmax[tid] = 0u;  // ordered before the first epilogue by the prologue's barrier
    // zero the per-board max row a later conv of this forward accumulates into
    for (int i = (int)blockIdx.x * NT + tid; i < clear_count; i += (int)gridDim.x * NT) amax_clear[i] = 0u;
    // a device-resident board count (the engine's pending count): the grid was sized for n_boards
    if (n_dev) n_boards = min(n_boards, *n_dev);
    const int nsets = n_sets(n_boards);
    if ((int)blockIdx.x >= nsets) return;
    const int my_sets = (nsets - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
    const int G = my_sets * NCH;
    auto set_of = [&](int g) { return (int)blockIdx.x + (g / NCH) * (int)gridDim.x; };
    auto set_b0 = [&](int g) { const int st = set_of(g); return GB * (st >> 1) + 3 * (st & 1); };  // first staged board
    const int co4 = wv * 16 + 4 * (lane >> 4);  // the 4 output channels of this lane's MFMA results
    const floatx4 bb4 = *reinterpret_cast<const floatx4 *>(bias + co4);

    Acc S[15];
#pragma unroll
    for (int i = 0; i < 15; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) S[i].p[j] = floatx2{0.0f, 0.0f};
    const floatx2 k2 = {2.0f, 2.0f}, k4 = {4.0f, 4.0f};
    float4 xr[XPT];
    // MODE 256 (diagnostic): u holds 8 replicas, workgroup b reads replica b % 8
    // MODE 8192 (diagnostic): replica (b / 8) % 8, i.e. the workgroups of one XCD spread over 8 copies
    const uint16_t *ub = (MODE & 256)    ? u + (size_t)(blockIdx.x % 8) * (NP * C * C * 2)
                         : (MODE & 8192) ? u + (size_t)((blockIdx.x >> 3) & 7) * (NP * C * C * 2)
                                         : u;
    const rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(ub), 0, NP * C * C * 4, 0x00020000);
    const int kq = lane >> 4;
    const int voff = wv * 1024 + lane * 16;  // U fragment of lane (co, kq): lane-linear (uttt_nn_wino3h_weights)
    // Every workgroup takes the chunks in the same order: the f32 accumulation order of a
    // board's results must not depend on which workgroup (= where in the batch) it lands.
    const int c_rot = 0;
    auto chunk_of = [&](int g) { return (g % NCH + c_rot) % NCH; };
    // 16-byte slot m ^ 2kq: conflict-free for both the transform's ds_write_b32 (32-lane groups,
    // 32 banks) and the point loop's ds_read_b128 (lane groups {0-3,12-15,20-27}, ... of
    // MI355X_MICROARCH.md §LDS); m ^ 4kq made the reads 2-way
    const char *sv_lane = sV + kq * 256 + (((lane & 15) ^ (2 * kq)) * 16);

    // the first chunk's inputs, scales and U fragments are requested before anything else, and the
    // pads of sX (never written after this; the staged cells are rewritten every chunk) are zeroed
    // while they are in flight: the 5 shared zero rows (10 positions each), the zero column of the
    // 36 board rows, the last position. Pads and staged cells are disjoint: one barrier covers both.
    auto zero_pads = [&]() {
        for (int i = fresh(tid); i < NPAD * (KC / 4); i += NT) {
            const int j = i / (KC / 4), q = i % (KC / 4);
            const int pos = j < 50 ? (j / 10) * 10 * SR + j % 10
                          : (j < 86 ? (((j - 50) / 9) * 10 + (j - 50) % 9 + 1) * SR : XP - 1);
            reinterpret_cast<float4 *>(sX + pos * KC)[q] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        }
    };
    if constexpr (MODE & kSerialPrologue) {  // diagnostic: the round-2 order (pads, barrier, then loads)
        zero_pads();
        __syncthreads();
    }
    load_x<MODE>(xr, x, set_b0(0), n_boards, chunk_of(0), tid);
    SetScale sc = set_scale(x_amax, x_amax_per_board, set_b0(0), n_boards);  // V scales of the current set
    // kStagger (diagnostic): waves 4-7 start their point walk at kStaggerRot
    const int rot = ((MODE & kStagger) && wv >= 4) ? kStaggerRot : 0;
    BFrag bq[PF];
#pragma unroll
    for (int i = 0; i < PF; ++i) bq[i] = load_b<(MODE & kF16) != 0>(ur, (i + rot) % NP, c_rot, voff);
    if constexpr (!(MODE & kSerialPrologue)) zero_pads();
    store_x(sX, xr, sc, tid);
    __syncthreads();
    const bool stamp = (MODE & 4) && blockIdx.x < 64 && (tid == 0 || tid == 256);
    auto mark = [&](int g, int k, unsigned long long t0) {
        if (stamp && g < 8) UTTT_WINO3H_STAMP(blockIdx.x, tid >> 8, g, k, (unsigned int)(__builtin_amdgcn_s_memtime() - t0));
    };
    uint32_t pf_sink = 0u;
#pragma unroll 1
    for (int g = 0; g < G; ++g) {
        const int c = g % NCH, ch = chunk_of(g);
        const unsigned long long t0 = (MODE & 4) ? __builtin_amdgcn_s_memtime() : 0ull;
        if constexpr (MODE & kL2Prefetch) {
            // diagnostic: the previous touch is consumed here, a chunk after it was issued; then the rows
            // of chunk g + 2 are touched with plain (L2-allocating) loads, so its nontemporal loads hit L2
            asm volatile("" ::"v"(pf_sink));
            if (g + 2 < G) {
                const int b0n = set_b0(g + 2), rows = min((n_boards - b0n) * 81, SB * 81);
                const int bp = fresh(tid);
                if (bp < rows) pf_sink = *reinterpret_cast<const uint32_t *>(x + ((size_t)b0n * 81 + bp) * C + chunk_of(g + 2) * KC);
            }
        }
        // the next chunk's inputs load during this chunk's transform (registers are
        // free then; the point loop needs nearly all of them)
        if (!(MODE & kEarlyLoad) || g == 0 || c == 0)
            if (!((MODE & kEpiLoad) && c == 0 && g > 0))  // kEpiLoad: requested before the last epilogue
                if (g + 1 < G) load_x<MODE>(xr, x, set_b0(g + 1), n_boards, chunk_of(g + 1), fresh(tid));
        // the next chunk's V scales: this set's, or the next set's after its last chunk
        SetScale sc_next = sc;
        if (c == NCH - 1 && g + 1 < G) sc_next = set_scale(x_amax, x_amax_per_board, set_b0(g + 1), n_boards);
        mark(g, 0, t0);
        if constexpr ((MODE & 3) != 1) transform<!(MODE & kSplitCvt), (MODE & kF16) != 0>(sV, sX, fresh(tid), set_of(g) & 1);
        mark(g, 1, t0);
        lds_barrier();
        if (g + 1 < G) store_x(sX, xr, sc_next, fresh(tid));
        mark(g, 2, t0);
        if constexpr (MODE & kEpiPrio)
            if (c == NCH - 1 && wv >= 4) __builtin_amdgcn_s_setprio(1);
        if constexpr ((MODE & 3) != 2) {
            AFrag a0, an;
            if constexpr (!(MODE & kNoALookahead)) a0 = load_a<(MODE & kF16) != 0>(sv_lane, rot);
            if constexpr (MODE & kALook2) an = load_a<(MODE & kF16) != 0>(sv_lane, (1 + rot) % NP);
            floatx2 mprev[4];
            if ((MODE & kStagger) && rot) xi_loop<0, MODE, PF, kStaggerRot>(S, sv_lane, ur, bq, a0, mprev, k2, k4, ch, voff, &an, ur);
            else xi_loop<0, MODE, PF>(S, sv_lane, ur, bq, a0, mprev, k2, k4, ch, voff, &an, ur);
        }
        if constexpr (MODE & kEpiPrio)
            if (c == NCH - 1 && wv >= 4) __builtin_amdgcn_s_setprio(0);
        if constexpr (MODE & kEpiBarrier)
            if (c == NCH - 1) __builtin_amdgcn_s_barrier();
        mark(g, 3, t0);
        if constexpr (MODE & kEarlyLoad)
            if (c != NCH - 1 && g + 2 < G) load_x<MODE>(xr, x, set_b0(g + 2), n_boards, chunk_of(g + 2), fresh(tid));
        if constexpr (MODE & kEpiLoad)
            if (c == NCH - 1 && g + 2 < G) load_x<MODE>(xr, x, set_b0(g + 2), n_boards, chunk_of(g + 2), fresh(tid));
        if (c == NCH - 1)
            set_epilogue<RES, MODE>(S, set_of(g), sc, u_scale, bb4, res, y, y_amax, n_boards, tid, lane, 0, s_bmax);
        sc = sc_next;
        mark(g, 4, t0);
        lds_barrier();
        if (c == NCH - 1 && y_amax) flush_bmax(s_bmax, y_amax, set_b0(g), n_boards, tid);
        mark(g, 5, t0);
    }
}

// ----------------------------------------------------------------------------------------------------
// k_wino3t_tower: the whole residual tower (n_layers convs, dual_network.py:28-45 x 16 blocks) as ONE
// persistent dataflow launch over work items (layer l, set st) instead of one launch per conv (round 6,
// VERDICT r5 item 1). A board's layer-l+1 inputs are its own layer-l outputs, and a 7-board group's
// two sets read and write only that group's boards, so layer l+1 of group g may start as soon as both
// of its layer-l sets are done, whatever the other groups do. Items are handed out by a ticket counter in
// layer-major order; an item waits (one lane polling done[g] with sc1 loads) only for the layer before it
// of its own group, whose tickets are smaller and were taken by running workgroups: the smallest unfinished
// ticket can always proceed, so the launch cannot deadlock whatever the residency. What this buys: no
// launch boundary between convs, and no chip-wide phase lock (every workgroup of a per-conv launch reaches
// its epilogue's HBM burst at the same moment, 13-18% of a launch); the second, half
// empty round of sets of each per-conv launch disappears into the stream of items.
//
// Each item runs the product's set pipeline unchanged (the same chunk order, point order, fold and
// epilogue arithmetic), so every output bit equals the per-conv kernels' and a board's outputs still
// depend on that board alone. Hand-offs between workgroups (activations, residuals, per-board maxima)
// are sc1 stores and sc1 loads (kHandoff); a producer signals done[g] with one agent-scope atomic add
// after every wave's vmcnt(0) and a barrier (MI355X_MICROARCH.md, inter-workgroup visibility, row 1).
//
// Buffers: block b's input X_b is x0 (b even) or x1 (b odd); conv 2b: X_b -> t; conv 2b+1: t (+ X_b) ->
// X_{b+1}. Per-board maxima: conv l reads row (l-1)%4 (the stem's one bound for l = 0), maxes into row
// l%4 and clears its sets' boards in row (l+1)%4 for conv l+1; max row 0 is cleared at the launch's end.
constexpr int kTowerCtlDone = 64;
__device__ __forceinline__ uint32_t ld_sc1(const uint32_t *p) {
    return __hip_atomic_load(const_cast<uint32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Workgroups are persistent for at most `max_items` items (round 6, measured against one persistent
// workgroup per CU): a per-conv launch's short-lived workgroups let the other lane's kernels onto the CUs
// every ~70 us, and a tower whose 256 workgroups held every CU for the whole forward locked the other lane
// out (lanes then ran their towers one after another: 6.94M against 7.03M sims/s, configs[1] 17.0M against
// 25.2M). A workgroup that has run max_items items exits, so CUs free up continuously and out of phase;
// the grid covers max_items x workgroups >= every item; a workgroup that finds every ticket taken (one sc1
// load of the ticket, no atomic) exits at once.
// Counters: two blocks of kTowerCtlWords words used by alternate launches (`parity`), so a late
// workgroup of this launch that still reads this block's ticket never sees it reset: the workgroup that
// finishes the launch's last item (items-done counter, [32]) resets the OTHER block (ticket [0], items
// [32], done[g] [64 + g]) for the next launch and clears max row 0.
template <int MODE = kHandoff, int PF = 3>
__global__ __launch_bounds__(NT) void k_wino3t_tower(float *act, int64_t act_stride, const uint16_t *__restrict__ u_all,
                                                     const float *__restrict__ u_scale_all,
                                                     const float *__restrict__ bias_all, int n_layers,
                                                     const uint32_t *__restrict__ stem_amax, uint32_t *rows,
                                                     int row_stride, uint32_t *ctl_base, int ctl_words, int parity,
                                                     int max_items, int max_boards, const int32_t *__restrict__ n_dev) {
    static_assert(MODE & kHandoff, "the tower's hand-offs need the sc1 forms");
    __shared__ __attribute__((aligned(16))) char smem[XP * KC * 4 + VB];
    __shared__ uint32_t s_bmax[SB];
    __shared__ int s_next[2];  // the next ticket, whether its dependency was seen met
    float *const sX = reinterpret_cast<float *>(smem);
    char *const sV = smem + XP * KC * 4;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    uint32_t *const ctl = ctl_base + (size_t)(parity & 1) * ctl_words;
    uint32_t *const done = ctl + kTowerCtlDone;
    int n_boards = max_boards;
    if (n_dev) n_boards = min(n_boards, *n_dev);
    const int nsets = n_sets(n_boards), total = n_layers * nsets;
    if (total == 0) {  // no item, so no last item: workgroup 0 resets the other block for the next launch
        if (blockIdx.x == 0) {
            uint32_t *const other = ctl_base + (size_t)((parity + 1) & 1) * ctl_words;
            for (int w = tid; w < ctl_words; w += NT) other[w] = 0u;
        }
        return;
    }
    constexpr int UL = NP * C * C * 2;  // u16 per layer
    const int kq = lane >> 4;
    const int voff = wv * 1024 + lane * 16;
    const char *sv_lane = sV + kq * 256 + (((lane & 15) ^ (2 * kq)) * 16);
    const int co4 = wv * 16 + 4 * (lane >> 4);
    const floatx2 k2 = {2.0f, 2.0f}, k4 = {4.0f, 4.0f};
    // item -> (layer, set); the layer's input, residual, output, maxima rows and weights
    // buffers act + k * act_stride: k = 0 X_even, 1 t, 2 X_odd (offsets, not a select of pointers, which
    // the compiler turns into a table in scratch)
    auto buf = [&](int k) -> float * { return act + (size_t)k * act_stride; };
    auto in_of = [&](int l) { return buf((l & 1) ? 1 : 2 * ((l >> 1) & 1)); };
    auto res_of = [&](int l) -> float * { return (l & 1) ? buf(2 * ((l >> 1) & 1)) : nullptr; };
    auto out_of = [&](int l) { return buf((l & 1) ? 2 - 2 * ((l >> 1) & 1) : 1); };
    auto urs = [&](int l) {
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(u_all + (size_t)l * UL), 0, NP * C * C * 4,
                                                 0x00020000);
    };
    auto scale_of = [&](int l, int b0) {
        return l == 0 ? set_scale<true>(stem_amax, 0, b0, n_boards)
                      : set_scale<true>(rows + (size_t)((l - 1) & 3) * row_stride, 1, b0, n_boards);
    };
    // the sets of group g (2, or 1 for a last group of <= 3 boards)
    auto sets_in = [&](int g) { return min(2, nsets - 2 * g); };

    // a ticket, or `total` once they are all taken (a workgroup that finds none takes nothing)
    if (tid == 0) s_next[0] = ld_sc1(ctl) >= (uint32_t)total ? total : (int)atomicAdd(ctl, 1u);
    if (tid < SB) s_bmax[tid] = 0u;
    for (int i = fresh(tid); i < NPAD * (KC / 4); i += NT) {  // the staged layout's zero pads (never rewritten)
        const int j = i / (KC / 4), q = i % (KC / 4);
        const int pos = j < 50 ? (j / 10) * 10 * SR + j % 10
                      : (j < 86 ? (((j - 50) / 9) * 10 + (j - 50) % 9 + 1) * SR : XP - 1);
        reinterpret_cast<float4 *>(sX + pos * KC)[q] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    Acc S[15];
#pragma unroll
    for (int i = 0; i < 15; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) S[i].p[j] = floatx2{0.0f, 0.0f};
    float4 xr[XPT];
    BFrag bq[PF];
    __syncthreads();
    int cur = uni(s_next[0]);
    bool staged = false;  // the current item's first chunk is already staged in sX (and bq holds its U)
    SetScale sc;
    uint32_t nxt_raw = 0u;  // lane 0: the next ticket
    int items = 0;
    bool last = false;  // this workgroup finished the launch's last item
#pragma unroll 1
    while (cur < total) {
        const int l = cur / nsets, st = cur - l * nsets, grp = st >> 1, h = st & 1, b0 = GB * grp + 3 * h;
        const rsrc_t ur = urs(l);
        ++items;
        // the next ticket (returns during this item), unless this is the workgroup's last item
        if (tid == 0) nxt_raw = items < max_items ? atomicAdd(ctl, 1u) : (uint32_t)total;
        if (!staged) {
            // wait for layer l-1 of this group (one lane polls; the rest join at the barrier), then stage
            if (tid == 0 && l > 0) {
                const uint32_t need = (uint32_t)(l * sets_in(grp));
                while (ld_sc1(done + grp) < need) __builtin_amdgcn_s_sleep(2);
            }
            __syncthreads();
            sc = scale_of(l, b0);
            load_x<MODE>(xr, in_of(l), b0, n_boards, 0, fresh(tid));
#pragma unroll
            for (int i = 0; i < PF; ++i) bq[i] = load_b(ur, i, 0, voff);
            store_x(sX, xr, sc, fresh(tid));
            __syncthreads();
        }
        // conv l+1's max row starts from zero on this set's boards (conv l+1 runs after both sets signal)
        if (tid < SB && b0 + tid < n_boards && l + 1 < n_layers)
            st_sc1(rows + (size_t)((l + 1) & 3) * row_stride + b0 + tid, 0u);
        const floatx4 bb4 = *reinterpret_cast<const floatx4 *>(bias_all + (size_t)l * C + co4);
        const float u_scale = u_scale_all[l];
        const float *const xin = in_of(l);
        int nxt = total, nl = l, nb0 = 0;
        bool nready = false;
#pragma unroll 1
        for (int c = 0; c < NCH; ++c) {
            if (c == NCH - 1) {  // the next item, as lane 0 polled it during chunk NCH-2 (uniform via LDS)
                nxt = uni(s_next[0]);
                nready = uni(s_next[1]) != 0;
                if (nxt < total) {
                    nl = nxt / nsets;
                    const int nst = nxt - nl * nsets;
                    nb0 = GB * (nst >> 1) + 3 * (nst & 1);
                }
            }
            if (c + 1 < NCH) load_x<MODE>(xr, xin, b0, n_boards, c + 1, fresh(tid));
            else if (nready) load_x<MODE>(xr, in_of(nl), nb0, n_boards, 0, fresh(tid));
            SetScale sc_next = sc;
            if (c == NCH - 1 && nready) sc_next = scale_of(nl, nb0);
            if (c == NCH - 2 && tid == 0) {
                const int t = (int)nxt_raw;
                int ready = 0;
                if (t < total) {
                    const int tl = t / nsets, tg = (t - tl * nsets) >> 1;
                    ready = tl == 0 || ld_sc1(done + tg) >= (uint32_t)(tl * sets_in(tg));
                }
                s_next[0] = t < total ? t : total;
                s_next[1] = ready;
            }
            transform<true, false>(sV, sX, fresh(tid), h);
            lds_barrier();
            if (c + 1 < NCH || nready) store_x(sX, xr, sc_next, fresh(tid));
            {
                AFrag a0 = load_a(sv_lane, 0), an;
                floatx2 mprev[4];
                const rsrc_t un = (c == NCH - 1 && nxt < total) ? urs(nl) : ur;
                xi_loop<0, MODE, PF>(S, sv_lane, ur, bq, a0, mprev, k2, k4, c, voff, &an, un);
            }
            if (c == NCH - 1) {
                // one epilogue instantiation for both forms (two inlined side by side spill ~84 VGPRs)
                set_epilogue<true, MODE>(S, st, sc, u_scale, bb4, res_of(l), out_of(l), rows + (size_t)(l & 3) * row_stride,
                                         n_boards, tid, lane, 0, s_bmax);
            }
            sc = sc_next;
            lds_barrier();
        }
        flush_bmax(s_bmax, rows + (size_t)(l & 3) * row_stride, b0, n_boards, tid);
        // publish: every wave's stores (outputs, maxima, the cleared row) complete, then one agent-scope add
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            __hip_atomic_fetch_add(done + grp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // the launch's last item: every other item has published (its add came first)
            s_next[1] = __hip_atomic_fetch_add(ctl + 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                        (uint32_t)(total - 1);
        }
        __syncthreads();
        last = uni(s_next[1]) != 0;  // (then no ticket is left, so this is also the workgroup's last item)
        cur = nxt;
        staged = nready && nxt < total;
    }
    if (last) {
        // reset the other block for the next launch (its launch, the previous one, is complete) and clear max
        // row 0 (written by conv 28, read by conv 29: both done) for the next forward's conv 0
        uint32_t *const other = ctl_base + (size_t)((parity + 1) & 1) * ctl_words;
        for (int w = tid; w < ctl_words; w += NT) other[w] = 0u;
        for (int b = tid; b < row_stride; b += NT) rows[b] = 0u;
    }
}

// Small batches: k_wino3s_conv<RES, SPLIT>. A set's 128 output channels are split over SPLIT
// workgroups of NW = 8 / SPLIT waves, each wave in the product's role (16 channels x 32 tile slots,
// the same U fragments, V fragments, MFMA order, fold and epilogue), so every output element is
// computed by the same instruction sequence as in k_wino3h_conv: the same bits, and a board's outputs
// still depend on that board alone. One set per SPLIT workgroups (no persistent loop): a batch of s
// sets runs on s x SPLIT CUs instead of s, and each CU streams 1 / SPLIT of U per chunk. Staging is
// synchronous and covers the boards in the batch only; the transform covers only the tile slots
// that hold a tile of such a board (the others' V columns are stale, their MFMA columns independent,
// their results dropped by the epilogue).
template <bool RES, int SPLIT, int PF = 3, int MODE = 0>
__global__ __launch_bounds__(64 * (8 / SPLIT)) void k_wino3s_conv(const float *__restrict__ x,
                                                                 const uint16_t *__restrict__ u, float u_scale,
                                                                 const float *__restrict__ bias,
                                                                 const float *__restrict__ res, float *__restrict__ y,
                                                                 const uint32_t *__restrict__ x_amax,
                                                                 int x_amax_per_board, uint32_t *__restrict__ y_amax,
                                                                 uint32_t *__restrict__ amax_clear, int clear_count,
                                                                 int n_boards, const int32_t *__restrict__ n_dev) {
    static_assert(SPLIT == 2 || SPLIT == 4 || SPLIT == 8, "split of the 8 channel waves");
    constexpr int NW = 8 / SPLIT, NTS = 64 * NW;
    __shared__ __attribute__((aligned(16))) char smem[XP * KC * 4 + VB];
    __shared__ uint32_t s_bmax[SB];
    float *const sX = reinterpret_cast<float *>(smem);
    char *const sV = smem + XP * KC * 4;
    const int tid = threadIdx.x, lane = tid & 63;
    if (tid < SB) s_bmax[tid] = 0u;
    const int part = (int)blockIdx.x % SPLIT, st = (int)blockIdx.x / SPLIT;
    const int wave_base = part * NW, wv = wave_base + (tid >> 6);  // the product's wave role
    for (int i = (int)blockIdx.x * NTS + tid; i < clear_count; i += (int)gridDim.x * NTS) amax_clear[i] = 0u;
    if (n_dev) n_boards = min(n_boards, *n_dev);
    if (st >= n_sets(n_boards)) return;
    const int h = st & 1, b0 = GB * (st >> 1) + 3 * h;  // first staged board
    // tile slots holding a tile of a board in the batch (slots are tiles 32h .. 32h + 31 of the group)
    const int group_tiles = 9 * min(n_boards - GB * (st >> 1), GB);
    const int live_slots = min(TS, group_tiles - 32 * h);
    const int staged = min(n_boards - b0, SB) * 81;  // staged positions of boards in the batch
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
    BFrag bq[PF];
#pragma unroll
    for (int i = 0; i < PF; ++i) bq[i] = load_b<(MODE & kF16) != 0>(ur, i, 0, voff);
    const SetScale sc = set_scale(x_amax, x_amax_per_board, b0, n_boards);
    for (int i = tid; i < NPAD * (KC / 4); i += NTS) {  // the zero pads of the staged layout (as the product)
        const int j = i / (KC / 4), q = i % (KC / 4);
        const int pos = j < 50 ? (j / 10) * 10 * SR + j % 10
                      : (j < 86 ? (((j - 50) / 9) * 10 + (j - 50) % 9 + 1) * SR : XP - 1);
        reinterpret_cast<float4 *>(sX + pos * KC)[q] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
#pragma unroll 1
    for (int ch = 0; ch < NCH; ++ch) {
        // stage this chunk's inputs of the boards in the batch, scaled by their board's sv (as store_x)
        for (int i = tid; i < staged * (KC / 4); i += NTS) {
            const int q = i % (KC / 4), bp = i / (KC / 4);
            const floatx4 t = __builtin_nontemporal_load(
                reinterpret_cast<const floatx4 *>(x + ((size_t)b0 * 81 + bp) * C + ch * KC) + q);
            const int kb = bp / 81, pos = bp - 81 * kb, sp = spos(kb, pos / 9, pos % 9);
            const float sv = sc.of(kb);
            reinterpret_cast<float4 *>(sX + sp * KC)[q] = make_float4(t.x * sv, t.y * sv, t.z * sv, t.w * sv);
        }
        lds_barrier();
        for (int it = tid; it < live_slots * (KC / 2); it += NTS) transform<true, (MODE & kF16) != 0>(sV, sX, it, h);
        lds_barrier();
        AFrag a0 = load_a<(MODE & kF16) != 0>(sv_lane, 0), an;
        floatx2 mprev[4];
        xi_loop<0, MODE, PF>(S, sv_lane, ur, bq, a0, mprev, k2, k4, ch, voff, &an, ur);
        lds_barrier();  // sX and sV are rewritten by the next chunk
    }
    set_epilogue<RES, 0>(S, st, sc, u_scale, bb4, res, y, y_amax, n_boards, tid, lane, wave_base, s_bmax);
    if (y_amax) {
        lds_barrier();
        flush_bmax(s_bmax, y_amax, b0, n_boards, tid);
    }
}

// Channel split for a batch of n boards: -1 (default) automatic, else forced (uttt_nn_wino3h_set_split;
// 0 or 1: the persistent kernel, 2: k_wino3s_conv<2>). Automatic: split 2 up to 28 boards (four groups
// of 7). Round 3, isolated, same box (tools/diag/conv_split_time.py, profiles/r3/conv_split.log, plain /
// residual us): 1 board 30.5 / 30.6 -> 22.4 / 22.5, 4-16 boards 33.4 / 36.1 -> 31.6 / 32.8, 25 boards
// 33.8 / 36.7 -> 32.0 / 33.2, but 50 boards 33.4 / 35.8 -> 39.1 / 40.6. Splits 4 and 8 are slower at
// every size, and a deeper U prefetch (6 to 12 points) changes nothing (tools/diag/conv_small_pf.py,
// profiles/r3/conv_small_pf.log): a set's four chunks are a serial chain of staging, transform and
// point GEMMs whose latency, not the U stream, sets a small launch's time.
inline int g_split = -1;
constexpr int kSplitMaxBoards = 28;
static int split_for(int n_boards) {
    if (g_split >= 0) return g_split <= 1 ? 1 : g_split;
    return n_boards <= kSplitMaxBoards ? 2 : 1;
}

// Workgroups per launch: at most cap, cap = CUs x UTTT_WINO3H_GRID (a real number, default 1:
// persistent, a workgroup loops over sets b, b + grid, ...; 0 = one workgroup per set, so the
// dispatcher hands sets of concurrent launches to whichever CU frees first)
static int grid_size(int n_boards) {
    static int cap = -1;
    if (cap < 0) {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            cus <= 0)
            cus = 256;
        const char *e = getenv("UTTT_WINO3H_GRID");
        const double k = e && *e ? atof(e) : 1.0;
        cap = k <= 0.0 ? (1 << 30) : (int)(k * cus + 0.5) > 0 ? (int)(k * cus + 0.5) : 1;
    }
    const int nsets = n_sets(n_boards);
    return nsets < cap ? nsets : cap;
}

}  // namespace wino3h
}  // namespace uttt
