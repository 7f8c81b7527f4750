// MFMA issue-rate microbenchmark (diagnostic): cycles per instruction for the
// f32 / f16 16x16 forms, one and two waves per SIMD, every CU busy.
// hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_rate tools/diag/mfma_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

template <int KIND>
__global__ void k(float *out, int iters, unsigned long long *cyc) {
    f4 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    float a = threadIdx.x * 1e-3f;
    h4 x4 = {(_Float16)a, (_Float16)1, (_Float16)2, (_Float16)3};
    h8 x8 = {(_Float16)a, (_Float16)1, (_Float16)2, (_Float16)3, (_Float16)a, (_Float16)1, (_Float16)2, (_Float16)3};
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if constexpr (KIND == 0) {
                c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c1, 0, 0, 0);
            } else if constexpr (KIND == 1) {
                c0 = __builtin_amdgcn_mfma_f32_16x16x16f16(x4, x4, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x16f16(x4, x4, c1, 0, 0, 0);
            } else if constexpr (KIND == 2) {
                c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(x8, x8, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(x8, x8, c1, 0, 0, 0);
            } else {  // f16 16x16x16 with 4 scalar f32 adds between MFMA pairs
                c0 = __builtin_amdgcn_mfma_f32_16x16x16f16(x4, x4, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x16f16(x4, x4, c1, 0, 0, 0);
                asm volatile("v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1" : "+v"(c2.x) : "v"(a));
            }
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
    out[blockIdx.x * blockDim.x + threadIdx.x] = c0.x + c1.y + c2.x + c3.x;
}

template <int KIND>
void run(const char *name, int wpsimd) {
    float *out;
    unsigned long long *cyc, h;
    const int blocks = 256, threads = 256 * wpsimd, iters = 2000;
    hipMalloc(&out, blocks * threads * 4);
    hipMalloc(&cyc, 8);
    k<KIND><<<blocks, threads>>>(out, 10, cyc);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    k<KIND><<<blocks, threads>>>(out, iters, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
    const double n = (double)iters * 16 * wpsimd;  // MFMAs per SIMD
    printf("%-28s waves/SIMD %d: %.2f cyc/MFMA per SIMD (s_memtime), %.3f ms\n", name, wpsimd, (double)h / (iters * 16.0),
           ms);
    (void)n;
    hipFree(out);
    hipFree(cyc);
}

int main() {
    for (int w = 1; w <= 2; ++w) {
        run<0>("mfma_f32_16x16x4f32", w);
        run<1>("mfma_f32_16x16x16f16", w);
        run<2>("mfma_f32_16x16x32_f16", w);
        run<3>("16x16x16f16 + 2 v_add/MFMA", w);
    }
    return 0;
}
