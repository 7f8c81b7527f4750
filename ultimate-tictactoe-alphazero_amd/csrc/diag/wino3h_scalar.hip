// wino3h_scalar.hip — diagnostics: k_wino3h_conv with its fold as scalar v_add_f32 / v_fma_f32 pairs
// (compiler-visible, hazards padded by the compiler; this TU is built with -fno-slp-vectorize so the
// pairs are not re-packed). MI355X_MICROARCH.md prices a v_pk_fma_f32 beside MFMAs above two
// v_fma_f32. The transform keeps its packed floatx2 math. Part of libuttt_diag.so only.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "uttt_nn.h"
#include "wino3h_impl.h"

using namespace uttt;

extern "C" int uttt_diag_wino3h_scalar(const float *x, const uint16_t *u, float u_scale, const float *bias,
                                       const float *res, float *y, const uint32_t *x_amax, int32_t n_boards,
                                       void *stream) {
    using namespace wino3h;
    const dim3 grid(grid_size(n_boards));
    hipStream_t st = (hipStream_t)stream;
    if (res)
        hipLaunchKernelGGL((k_wino3h_conv<true, kFoldScalar, 3>), grid, dim3(NT), 0, st, x, u, u_scale, bias, res, y,
                           x_amax, 1, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr);
    else
        hipLaunchKernelGGL((k_wino3h_conv<false, kFoldScalar, 3>), grid, dim3(NT), 0, st, x, u, u_scale, bias,
                           nullptr, y, x_amax, 1, nullptr, nullptr, 0, n_boards, (const int32_t *)nullptr);
    return hipGetLastError() == hipSuccess ? UTTT_OK : UTTT_ERR_HIP;
}
