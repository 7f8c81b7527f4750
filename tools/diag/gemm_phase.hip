// Point-GEMM phase of k_wino3h_conv in isolation, register U path, by wave shape and U prefetch depth
// (diagnostic, round 5): is the phase's U stream bound by bytes in flight (a deeper prefetch or a wave
// with more registers would help) or by the per-CU vector-memory rate (nothing would)?
//
// A workgroup per CU loops over 32-channel chunks of one 32-tile set. Per point and wave: COB U
// fragment pairs (16 output channels each, hi and lo, 1 KB lane-linear per 16-B load, from the
// product's 1.6 MB layout in L2), the 4 V fragments of the set's two 16-tile blocks from LDS (one point
// ahead), 6 * COB v_mfma_f32_16x16x32_f16 and the product's fold after the u = 2, 3 points (24 scalar
// adds per co-block). Shapes: WAVES = 8, COB = 1 (the product: 2 waves per SIMD, each 16 co) and
// WAVES = 4, COB = 2 (one wave per SIMD with the whole 512-register file, each 32 co: the same U bytes
// per CU, half the V reads). PF = U points in flight. Prints us per chunk from events (the slowest
// wave sets it) and the U rate per CU.
//   hipcc --offload-arch=gfx950 -O3 -o tools/diag/gemm_phase tools/diag/gemm_phase.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

constexpr int NP = 25, NCH = 4, C = 128;
constexpr int VPLANE = 1024, VB = NP * 4 * VPLANE;  // 102,400 B
constexpr int XB = 411 * 32 * 4;                    // 52,608 B (the staged input, unused here)
constexpr int UPLANE = C * 4 * 16;                  // 8 KB

struct U2 {
    halfx8 h, l;
};
struct A4 {
    halfx8 h0, l0, h1, l1;
};

template <int COB>
struct UF {
    U2 c[COB];
};

template <int COB>
__device__ __forceinline__ UF<COB> load_u(rsrc_t u, int xi, int ch, int voff) {
    const int soff = (xi * NCH + ch) * 2 * UPLANE;
    UF<COB> f;
#pragma unroll
    for (int k = 0; k < COB; ++k) {
        f.c[k].h = __builtin_bit_cast(halfx8, __builtin_amdgcn_raw_buffer_load_b128(u, voff + k * 1024, soff, 0));
        f.c[k].l = __builtin_bit_cast(halfx8, __builtin_amdgcn_raw_buffer_load_b128(u, voff + k * 1024 + UPLANE, soff, 0));
    }
    return f;
}

__device__ __forceinline__ A4 load_a(const char *sv, int xi) {
    const char *p = sv + xi * 4 * VPLANE;
    A4 a;
    a.h0 = *reinterpret_cast<const halfx8 *>(p);
    a.l0 = *reinterpret_cast<const halfx8 *>(p + VPLANE);
    a.h1 = *reinterpret_cast<const halfx8 *>(p + 2 * VPLANE);
    a.l1 = *reinterpret_cast<const halfx8 *>(p + 3 * VPLANE);
    return a;
}

template <int WAVES, int COB, int PF>
__global__ __launch_bounds__(64 * WAVES) void k_gemm(const uint16_t *__restrict__ u, int chunks, float *sink) {
    __shared__ __attribute__((aligned(16))) char smem[XB + VB];
    const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < (XB + VB) / 4; i += 64 * WAVES)
        reinterpret_cast<uint32_t *>(smem)[i] = 0x3c003c00u ^ (i * 2654435761u & 0x03ff03ffu);
    __syncthreads();
    const char *sV = smem + XB;
    const int kq = lane >> 4;
    const char *sv_lane = sV + kq * 256 + (((lane & 15) ^ (2 * kq)) * 16);
    const rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(u), 0, NP * C * C * 4, 0x00020000);
    const int voff = wv * COB * 1024 + lane * 16;  // this wave's COB x 16 output channels
    floatx4 S[COB][6];
#pragma unroll
    for (int k = 0; k < COB; ++k)
#pragma unroll
        for (int i = 0; i < 6; ++i) S[k][i] = floatx4{0, 0, 0, 0};
    UF<COB> bq[PF];
#pragma unroll
    for (int i = 0; i < PF; ++i) bq[i] = load_u<COB>(ur, i, 0, voff);
#pragma unroll 1
    for (int g = 0; g < chunks; ++g) {
        const int ch = g % NCH;
        A4 a0 = load_a(sv_lane, 0);
#pragma unroll
        for (int xi = 0; xi < NP; ++xi) {
            const int nx = xi + PF < NP ? xi + PF : xi + PF - NP;
            const int nch = xi + PF < NP ? ch : (ch + 1) % NCH;
            const UF<COB> b2 = load_u<COB>(ur, nx, nch, voff);
            const UF<COB> b0 = bq[0];
            A4 a1 = a0;
            if (xi + 1 < NP) a1 = load_a(sv_lane, xi + 1);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = 0; k < COB; ++k) {
                floatx4 m0 = {}, m1 = {};
                m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.c[k].l, a0.h0, m0, 0, 0, 0);
                m1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.c[k].l, a0.h1, m1, 0, 0, 0);
                m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.c[k].h, a0.l0, m0, 0, 0, 0);
                m1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.c[k].h, a0.l1, m1, 0, 0, 0);
                m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.c[k].h, a0.h0, m0, 0, 0, 0);
                m1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.c[k].h, a0.h1, m1, 0, 0, 0);
                if (xi / 5 == 2 || xi / 5 == 3) {
#pragma unroll
                    for (int r = 0; r < 3; ++r)
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            asm volatile("v_add_f32 %0, %0, %1" : "+v"(S[k][2 * r][i]) : "v"(m0[i]));
                            asm volatile("v_add_f32 %0, %0, %1" : "+v"(S[k][2 * r + 1][i]) : "v"(m1[i]));
                        }
                } else {
                    S[k][0] += m0;
                    S[k][1] += m1;
                }
            }
#pragma unroll
            for (int i = 0; i + 1 < PF; ++i) bq[i] = bq[i + 1];
            bq[PF - 1] = b2;
            a0 = a1;
        }
    }
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < COB; ++k)
#pragma unroll
        for (int i = 0; i < 6; ++i) acc += S[k][i][0] + S[k][i][1] + S[k][i][2] + S[k][i][3];
    if (acc == 1.2345f) sink[blockIdx.x * 512 + tid] = acc;
}

template <int WAVES, int COB, int PF>
static void run(const uint16_t *u, int chunks, float *sink, int cus, bool &first) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL((k_gemm<WAVES, COB, PF>), dim3(cus), dim3(64 * WAVES), 0, 0, u, chunks, sink);
        CK(hipGetLastError());
        CK(hipEventRecord(e1, 0));
        CK(hipDeviceSynchronize());
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep && ms < best) best = ms;
    }
    const double us_chunk = best * 1e3 / chunks;
    const double ub = (double)NP * C * C * 4 / NCH;  // U bytes per chunk per CU
    printf("%s{\"waves\": %d, \"co_blocks_per_wave\": %d, \"u_prefetch_points\": %d, \"us_per_chunk\": %.3f, "
           "\"u_GBps_per_cu\": %.1f, \"u_TBps\": %.2f}",
           first ? "" : ", ", WAVES, COB, PF, us_chunk, ub / (us_chunk * 1e-6) / 1e9, ub * cus / (us_chunk * 1e-6) / 1e12);
    first = false;
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

int main(int argc, char **argv) {
    const int chunks = argc > 1 ? atoi(argv[1]) : 64;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const size_t ubytes = (size_t)NP * C * C * 4;
    uint16_t *u = nullptr;
    float *sink = nullptr;
    CK(hipMalloc(&u, ubytes));
    CK(hipMalloc(&sink, (size_t)cus * 512 * 4));
    std::vector<uint16_t> h(ubytes / 2);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (uint16_t)(0x3800u | ((i * 2654435761u) >> 22 & 0x3ffu));
    CK(hipMemcpy(u, h.data(), ubytes, hipMemcpyHostToDevice));
    printf("{\"chunks\": %d, \"workgroups\": %d, \"mfma_floor_note\": \"per SIMD and chunk 300 MFMAs x 16 cycles = 4.8k "
           "cycles in every shape\", \"results\": [",
           chunks, cus);
    bool first = true;
    for (int r = 0; r < 2; ++r) {
        run<8, 1, 2>(u, chunks, sink, cus, first);
        run<8, 1, 3>(u, chunks, sink, cus, first);
        run<8, 1, 4>(u, chunks, sink, cus, first);
        run<8, 1, 6>(u, chunks, sink, cus, first);
        run<4, 2, 2>(u, chunks, sink, cus, first);
        run<4, 2, 3>(u, chunks, sink, cus, first);
        run<4, 2, 5>(u, chunks, sink, cus, first);
        run<4, 2, 8>(u, chunks, sink, cus, first);
    }
    printf("]}\n");
    return 0;
}
