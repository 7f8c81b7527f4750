// wino3h_diag.hip — diagnostics-only instantiations of k_wino3h_conv (timing ablations, phase
// stamps, prefetch-distance variants) in their own library, libuttt_diag.so (Makefile target
// `diag`, used by tools/diag/*.py). Nothing in the product library or its tests loads it.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "uttt_nn.h"
#include "wino3h_impl.h"
#include "wino3p_impl.h"
#include "wino3q_impl.h"

using namespace uttt;

// diagnostic: the residual form of an ablation launch (residual = g_diag_res if set, else x)
static const float *g_diag_res = nullptr;
template <int MODE>
static void ablation_res(const float *x, const uint16_t *u, float u_scale, const float *bias, float *y,
                         const uint32_t *x_amax, int32_t n_boards, hipStream_t st) {
    using namespace wino3h;
    hipLaunchKernelGGL((k_wino3h_conv<true, MODE>), dim3(grid_size(n_boards)), dim3(NT), 0, st, x, u, u_scale, bias,
                       g_diag_res ? g_diag_res : x, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr);
}

extern "C" {

int uttt_diag_wino3h_scalar(const float *x, const uint16_t *u, float u_scale, const float *bias, const float *res,
                            float *y, const uint32_t *x_amax, int32_t n_boards, void *stream);

// Diagnostic: the residual tensor of the ablation's residual form (null: x itself)
void uttt_diag_wino3h_set_residual(const float *res) { g_diag_res = res; }

// Diagnostic (not declared in uttt_nn.h): the same launch with a timing ablation.
int uttt_diag_wino3h_ablation(const float *x, const uint16_t *u, float u_scale, const float *bias, float *y,
                              const uint32_t *x_amax, int32_t n_boards, int32_t mode, void *stream) {
    const dim3 grid(wino3h::grid_size(n_boards));
    hipStream_t st = (hipStream_t)stream;
    using namespace wino3h;
    if (mode & (1 << 20)) {  // the residual form (residual = x)
        switch (mode & ~(1 << 20)) {
            case 65536: ablation_res<65536>(x, u, u_scale, bias, y, x_amax, n_boards, st); break;
            case 131072: ablation_res<131072>(x, u, u_scale, bias, y, x_amax, n_boards, st); break;
            case 196608: ablation_res<196608>(x, u, u_scale, bias, y, x_amax, n_boards, st); break;
            case 8: ablation_res<8>(x, u, u_scale, bias, y, x_amax, n_boards, st); break;
            case kResEarly: ablation_res<kResEarly>(x, u, u_scale, bias, y, x_amax, n_boards, st); break;
            case kEpiOrder: ablation_res<kEpiOrder>(x, u, u_scale, bias, y, x_amax, n_boards, st); break;
            case kEpiLoad: ablation_res<kEpiLoad>(x, u, u_scale, bias, y, x_amax, n_boards, st); break;
            case kEpiNT: ablation_res<kEpiNT>(x, u, u_scale, bias, y, x_amax, n_boards, st); break;
            case kEpiOrder | kEpiLoad: ablation_res<kEpiOrder | kEpiLoad>(x, u, u_scale, bias, y, x_amax, n_boards, st); break;
            default: ablation_res<0>(x, u, u_scale, bias, y, x_amax, n_boards, st);
        }
        return hipGetLastError() == hipSuccess ? UTTT_OK : UTTT_ERR_HIP;
    }
    switch (mode) {
        case 131072: hipLaunchKernelGGL((k_wino3h_conv<false, 131072>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 1: hipLaunchKernelGGL((k_wino3h_conv<false, 1>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 2: hipLaunchKernelGGL((k_wino3h_conv<false, 2>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 64: hipLaunchKernelGGL((k_wino3h_conv<false, 64>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 16: hipLaunchKernelGGL((k_wino3h_conv<false, 16>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 32: hipLaunchKernelGGL((k_wino3h_conv<false, 32>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 48: hipLaunchKernelGGL((k_wino3h_conv<false, 48>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 49: hipLaunchKernelGGL((k_wino3h_conv<false, 49>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 112: hipLaunchKernelGGL((k_wino3h_conv<false, 112>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 256: hipLaunchKernelGGL((k_wino3h_conv<false, 256>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case kEpiOrder: hipLaunchKernelGGL((k_wino3h_conv<false, kEpiOrder>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case kEpiLoad: hipLaunchKernelGGL((k_wino3h_conv<false, kEpiLoad>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case kEpiNT: hipLaunchKernelGGL((k_wino3h_conv<false, kEpiNT>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case kEpiOrder | kEpiLoad: hipLaunchKernelGGL((k_wino3h_conv<false, kEpiOrder | kEpiLoad>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 8: hipLaunchKernelGGL((k_wino3h_conv<false, 8>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 4: hipLaunchKernelGGL((k_wino3h_conv<false, 4>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 12: hipLaunchKernelGGL((k_wino3h_conv<false, 12>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 36: hipLaunchKernelGGL((k_wino3h_conv<false, 36>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 68: hipLaunchKernelGGL((k_wino3h_conv<false, 68>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 116: hipLaunchKernelGGL((k_wino3h_conv<false, 116>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 20: hipLaunchKernelGGL((k_wino3h_conv<false, 20>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 512: hipLaunchKernelGGL((k_wino3h_conv<false, 512>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 8192: hipLaunchKernelGGL((k_wino3h_conv<false, 8192>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 8196: hipLaunchKernelGGL((k_wino3h_conv<false, 8196>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 260: hipLaunchKernelGGL((k_wino3h_conv<false, 260>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 65: hipLaunchKernelGGL((k_wino3h_conv<false, 65>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        default: hipLaunchKernelGGL((k_wino3h_conv<false, 0>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr);
    }
    return hipGetLastError() == hipSuccess ? UTTT_OK : UTTT_ERR_HIP;
}

// Diagnostic: MODE-4 phase stamps, out[64][2][8][6] (see g_stamp).
int uttt_diag_wino3h_stamps(unsigned int *out) {
    if (!out || hipMemcpyFromSymbol(out, HIP_SYMBOL(wino3h::g_stamp), sizeof(unsigned int) * 64 * 2 * 8 * 6) != hipSuccess)
        return UTTT_ERR_HIP;
    return UTTT_OK;
}

// Diagnostic: pipeline variants, product arithmetic (same output bits as the product launch):
// variant 0 product, 1 buffer-loaded inputs, 2 no V lookahead + U PF 4, 3 no V lookahead + PF 5,
// 4 = 1 + 2, 5 = 1 + 3; residual form when res is non-null.
int uttt_diag_wino3h_variant(const float *x, const uint16_t *u, float u_scale, const float *bias, const float *res,
                             float *y, const uint32_t *x_amax, int32_t n_boards, int32_t variant, void *stream) {
    const dim3 grid(wino3h::grid_size(n_boards));
    hipStream_t st = (hipStream_t)stream;
    using namespace wino3h;
#define UTTT_V(M, P)                                                                                                  \
    do {                                                                                                              \
        if (res)                                                                                                      \
            hipLaunchKernelGGL((k_wino3h_conv<true, M, P>), grid, dim3(NT), 0, st, x, u, u_scale, bias, res, y, x_amax, \
                               1, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr);                                                    \
        else                                                                                                          \
            hipLaunchKernelGGL((k_wino3h_conv<false, M, P>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y,   \
                               x_amax, 1, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr);                                            \
    } while (0)
#define UTTT_Q(PF_)                                                                                                    \
    do {                                                                                                              \
        if (res)                                                                                                      \
            hipLaunchKernelGGL((k_wino3q_conv<true, PF_>), grid, dim3(NTQ), 0, st, x, u, u_scale, bias, res, y, x_amax, \
                               1, nullptr, nullptr, 0, n_boards);                                                    \
        else                                                                                                          \
            hipLaunchKernelGGL((k_wino3q_conv<false, PF_>), grid, dim3(NTQ), 0, st, x, u, u_scale, bias, nullptr, y,   \
                               x_amax, 1, nullptr, nullptr, 0, n_boards);                                            \
    } while (0)
#define UTTT_P(PF_, ALA_)                                                                                              \
    do {                                                                                                              \
        if (res)                                                                                                      \
            hipLaunchKernelGGL((k_wino3p_conv<true, PF_, ALA_>), grid, dim3(NT), 0, st, x, u, u_scale, bias, res, y,   \
                               x_amax, 1, nullptr, nullptr, 0, n_boards);                                            \
        else                                                                                                          \
            hipLaunchKernelGGL((k_wino3p_conv<false, PF_, ALA_>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, \
                               y, x_amax, 1, nullptr, nullptr, 0, n_boards);                                         \
    } while (0)
    switch (variant) {
        case 1: UTTT_V(kBufferX, 3); break;
        case 2: UTTT_V(kNoALookahead, 4); break;
        case 3: UTTT_V(kNoALookahead, 5); break;
        case 4: UTTT_V(kBufferX | kNoALookahead, 4); break;
        case 5: UTTT_V(kBufferX | kNoALookahead, 5); break;
        case 6: UTTT_V(kNoALookahead, 3); break;
        case 20: UTTT_V(kFoldBuiltin, 3); break;
        case 70: UTTT_V(kFoldPacked | kFoldAT, 3); break;  // the round-3 product (packed fold along A^T)
        case 75: UTTT_V(kFoldAT, 3); break;                // scalar fold along A^T (round-4 first step)
        case 76: UTTT_V(kEarlyLoad, 3); break;
        case 77: UTTT_V(kEarlyLoad | kBufferX, 3); break;
        case 78: UTTT_V(kEpiBarrier, 3); break;
        case 81: UTTT_V(kEpiOrder, 3); break;  // the branch-free ordered epilogue (round 5 A/B)
        case 82: UTTT_V(kEpiNT, 3); break;
        case 83: UTTT_V(kEpiLoad, 3); break;
        case 79: UTTT_V(kEpiPrio, 3); break;
        case 80: UTTT_V(kEpiBarrier | kEarlyLoad, 3); break;
        case 71: UTTT_V(kBufferX, 3); break;
        case 72: UTTT_V(kBufferX, 4); break;
        case 73: UTTT_V(kStagger | kFoldPacked, 3); break;
        case 74: UTTT_V(kStagger, 3); break;
        case 40: UTTT_V(kALook2, 2); break;
        case 41: UTTT_V(kALook2, 3); break;
        case 42: UTTT_V(kALook2 | kBufferX, 3); break;
        case 50: UTTT_V(kSerialPrologue, 3); break;
        case 51: UTTT_V(kSplitCvt, 3); break;
        case 52: UTTT_V(kSplitCvt | kSerialPrologue, 3); break;
        case 60: UTTT_V(kL2Prefetch, 3); break;
        case 30: UTTT_Q(3); break;
        case 31: UTTT_Q(2); break;
        case 32: UTTT_Q(4); break;
        case 22: return uttt_diag_wino3h_scalar(x, u, u_scale, bias, res, y, x_amax, n_boards, stream);
        case 10: UTTT_P(3, true); break;
        case 11: UTTT_P(3, false); break;
        case 12: UTTT_P(2, true); break;
        case 13: UTTT_P(4, false); break;
        default: UTTT_V(0, 3);
    }
#undef UTTT_V
#undef UTTT_P
#undef UTTT_Q
    return hipGetLastError() == hipSuccess ? UTTT_OK : UTTT_ERR_HIP;
}

int uttt_diag_wino3h_pf(const float *x, const uint16_t *u, float u_scale, const float *bias, float *y,
                        const uint32_t *x_amax, int32_t n_boards, int32_t pf, void *stream) {
    const dim3 grid(wino3h::grid_size(n_boards));
    hipStream_t st = (hipStream_t)stream;
    using namespace wino3h;
    switch (pf) {
        case 3: hipLaunchKernelGGL((k_wino3h_conv<false, 0, 3>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 4: hipLaunchKernelGGL((k_wino3h_conv<false, 0, 4>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 6: hipLaunchKernelGGL((k_wino3h_conv<false, 0, 6>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        case 8: hipLaunchKernelGGL((k_wino3h_conv<false, 0, 8>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); break;
        default: hipLaunchKernelGGL((k_wino3h_conv<false, 0, 2>), grid, dim3(NT), 0, st, x, u, u_scale, bias, nullptr, y, x_amax, 0, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr);
    }
    return hipGetLastError() == hipSuccess ? UTTT_OK : UTTT_ERR_HIP;
}

// k_wino3s_conv (the small-batch channel split) at other prefetch distances: split 2 or 4, PF 3 / 6 / 9 / 12
int uttt_diag_wino3s(const float *x, const uint16_t *u, float u_scale, const float *bias, const float *res, float *y,
                     const uint32_t *x_amax, int32_t n_boards, int32_t split, int32_t pf, void *stream) {
    using namespace wino3h;
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid((unsigned)(n_sets(n_boards) * split));
#define UTTT_S(SP, PFV)                                                                                             \
    do {                                                                                                            \
        if (res)                                                                                                    \
            hipLaunchKernelGGL((k_wino3s_conv<true, SP, PFV>), grid, dim3(64 * (8 / SP)), 0, st, x, u, u_scale, bias, \
                               res, y, x_amax, 1, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr);         \
        else                                                                                                        \
            hipLaunchKernelGGL((k_wino3s_conv<false, SP, PFV>), grid, dim3(64 * (8 / SP)), 0, st, x, u, u_scale,    \
                               bias, nullptr, y, x_amax, 1, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr); \
    } while (0)
    if (split == 2) {
        if (pf == 6) UTTT_S(2, 6);
        else if (pf == 9) UTTT_S(2, 9);
        else if (pf == 12) UTTT_S(2, 12);
        else UTTT_S(2, 3);
    } else {
        if (pf == 6) UTTT_S(4, 6);
        else if (pf == 9) UTTT_S(4, 9);
        else if (pf == 12) UTTT_S(4, 12);
        else UTTT_S(4, 3);
    }
#undef UTTT_S
    return hipGetLastError() == hipSuccess ? UTTT_OK : UTTT_ERR_HIP;
}

}  // extern "C"
