// GEMM-phase microbenchmark for k_wino3h_conv's U stream (diagnostic; VERDICT r4 "Next round" 2a):
// does streaming the transformed weights U through LDS-DMA make the point GEMMs faster than the
// product's vector loads into registers?
//
// One workgroup per CU, 8 waves, the product's LDS image sizes (V 100 KB + a 52.6 KB region that
// holds the staged input in the product). Each wave runs the product's point loop on one chunk
// after another: per point 4 V fragments from LDS (ds_read_b128, one point ahead), 2 U fragments
// (hi, lo; 1 KB lane-linear each per wave), 6 v_mfma_f32_16x16x32_f16, and the product's fold
// (24 scalar f32 adds after each of the 10 points with u = 2, 3). No transform, staging or
// epilogue: the loop is the GEMM phase alone. U comes from the product's 1.6 MB layout in L2:
//   MODE 0: buffer_load_dwordx4 into registers, 3 points ahead (the product);
//   MODE 1: per-wave LDS-DMA ring (buffer_load_dwordx4 ... lds) of 3 points in the 52.6 KB region,
//           each wave reading back only what it loaded (no barrier), ds_read_b128 one point ahead;
//   MODE 2: as 1 with a 4-point ring ahead... capped by the region: 3 points x 2 KB x 8 waves = 48 KB.
// Prints cycles per chunk (median workgroup, s_memtime) and the chip's U and V byte rates.
//   hipcc --offload-arch=gfx950 -O3 -o tools/diag/lds_ring tools/diag/lds_ring.hip
#include <hip/hip_runtime.h>

#include <algorithm>
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
constexpr int XB = 411 * 32 * 4;                    // 52,608 B
constexpr int UPLANE = C * 4 * 16;                  // 8 KB: one (xi, chunk, hi|lo) plane
constexpr int RING = 3;                             // points in flight per wave (MODE 1)

struct U2 {
    halfx8 h, l;
};
struct A4 {
    halfx8 h0, l0, h1, l1;
};

__device__ __forceinline__ U2 load_u_reg(rsrc_t u, int xi, int ch, int voff) {
    const int soff = (xi * NCH + ch) * 2 * UPLANE;
    U2 b;
    b.h = __builtin_bit_cast(halfx8, __builtin_amdgcn_raw_buffer_load_b128(u, voff, soff, 0));
    b.l = __builtin_bit_cast(halfx8, __builtin_amdgcn_raw_buffer_load_b128(u, voff + UPLANE, soff, 0));
    return b;
}

// LDS-DMA of one point's U (hi then lo, 1 KB each) into this wave's ring slot: M0 = the slot's LDS
// byte address, each lane's 16 B land at M0 + 16 lane. Hidden from the compiler's vmcnt bookkeeping:
// the caller waits with its own counted s_waitcnt (2 instructions per point).
__device__ __forceinline__ void dma_u(rsrc_t u, int xi, int ch, int voff, uint32_t lds_slot) {
    const int soff = (xi * NCH + ch) * 2 * UPLANE;
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, %4 offen lds\n\t"
        "s_mov_b32 m0, %5\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, %6 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(u), "s"(lds_slot), "s"(soff), "s"(lds_slot + 1024u), "s"(soff + UPLANE)
        : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
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

__device__ __forceinline__ void fold24(floatx4 (&S)[6], const floatx4 &m0, const floatx4 &m1) {
    // the product's fold of one u = 2 / 3 point: 3 rows x 2 blocks x 4 lanes-values, scalar adds
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(S[2 * r][i]) : "v"(m0[i]));
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(S[2 * r + 1][i]) : "v"(m1[i]));
        }
}

template <int MODE>
__global__ __launch_bounds__(512) void k_ring(const uint16_t *__restrict__ u, int chunks, float *sink,
                                              unsigned long long *cyc) {
    __shared__ __attribute__((aligned(16))) char smem[XB + VB];
    const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    // V: arbitrary non-zero f16 (random-ish operands keep the clock honest)
    for (int i = tid; i < (XB + VB) / 4; i += 512) reinterpret_cast<uint32_t *>(smem)[i] = 0x3c003c00u ^ (i * 2654435761u & 0x03ff03ffu);
    __syncthreads();
    const char *sV = smem + XB;
    const int kq = lane >> 4;
    const char *sv_lane = sV + kq * 256 + (((lane & 15) ^ (2 * kq)) * 16);
    const rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(u), 0, NP * C * C * 4, 0x00020000);
    const int voff = wv * 1024 + lane * 16;
    // this wave's ring: RING slots of 2 KB (hi, lo) in the X region
    const uint32_t ring0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char *)(smem) + wv * (RING * 2048);
    const char *ring_lane = smem + wv * (RING * 2048) + lane * 16;
    floatx4 S[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) S[i] = floatx4{0, 0, 0, 0};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if constexpr (MODE == 0) {
        U2 bq[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) bq[i] = load_u_reg(ur, i, 0, voff);
#pragma unroll 1
        for (int g = 0; g < chunks; ++g) {
            const int ch = g % NCH;
            A4 a0 = load_a(sv_lane, 0);
#pragma unroll
            for (int xi = 0; xi < NP; ++xi) {
                const int nx = xi + 3 < NP ? xi + 3 : xi + 3 - NP;
                const int nch = xi + 3 < NP ? ch : (ch + 1) % NCH;
                const U2 b2 = load_u_reg(ur, nx, nch, voff);
                const U2 b0 = bq[0];
                A4 a1 = a0;
                if (xi + 1 < NP) a1 = load_a(sv_lane, xi + 1);
                __builtin_amdgcn_sched_barrier(0);
                floatx4 m0 = {}, m1 = {};
                m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.l, a0.h0, m0, 0, 0, 0);
                m1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.l, a0.h1, m1, 0, 0, 0);
                m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.h, a0.l0, m0, 0, 0, 0);
                m1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.h, a0.l1, m1, 0, 0, 0);
                m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.h, a0.h0, m0, 0, 0, 0);
                m1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.h, a0.h1, m1, 0, 0, 0);
                if (xi / 5 == 2 || xi / 5 == 3) fold24(S, m0, m1);
                else {
                    S[0] += m0;
                    S[1] += m1;
                }
                bq[0] = bq[1];
                bq[1] = bq[2];
                bq[2] = b2;
                a0 = a1;
            }
        }
    } else {
        // prologue: points 0..RING-1 of chunk 0 into the ring
#pragma unroll
        for (int i = 0; i < RING; ++i) dma_u(ur, i, 0, voff, ring0 + i * 2048);
#pragma unroll 1
        for (int g = 0; g < chunks; ++g) {
            const int ch = g % NCH;
            A4 a0 = load_a(sv_lane, 0);
            // U of point 0 from its slot (its DMA is the oldest of the RING in flight)
            wait_vm<2 * (RING - 1)>();
            U2 b0;
            b0.h = *reinterpret_cast<const halfx8 *>(ring_lane);
            b0.l = *reinterpret_cast<const halfx8 *>(ring_lane + 1024);
#pragma unroll
            for (int xi = 0; xi < NP; ++xi) {
                const int slot = xi % RING;
                A4 a1 = a0;
                if (xi + 1 < NP) a1 = load_a(sv_lane, xi + 1);
                __builtin_amdgcn_sched_barrier(0);
                floatx4 m0 = {}, m1 = {};
                m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.l, a0.h0, m0, 0, 0, 0);
                m1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.l, a0.h1, m1, 0, 0, 0);
                m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.h, a0.l0, m0, 0, 0, 0);
                m1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.h, a0.l1, m1, 0, 0, 0);
                m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.h, a0.h0, m0, 0, 0, 0);
                m1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(b0.h, a0.h1, m1, 0, 0, 0);
                // the slot of point xi is free once its fragments are in registers (the MFMAs above
                // consumed them): refill it with point xi + RING (next chunk's first points at the end)
                {
                    const int nx = xi + RING < NP ? xi + RING : xi + RING - NP;
                    const int nch = xi + RING < NP ? ch : (ch + 1) % NCH;
                    asm volatile("" ::"v"(b0.h), "v"(b0.l));  // after the reads of this slot completed
                    dma_u(ur, nx, nch, voff, ring0 + slot * 2048);
                }
                // the next point's U: its DMA is now the oldest but RING - 1 ... wait for it, read it
                if (xi + 1 < NP) {
                    wait_vm<2 * (RING - 1)>();
                    const char *q = ring_lane + ((xi + 1) % RING) * 2048;
                    b0.h = *reinterpret_cast<const halfx8 *>(q);
                    b0.l = *reinterpret_cast<const halfx8 *>(q + 1024);
                }
                if (xi / 5 == 2 || xi / 5 == 3) fold24(S, m0, m1);
                else {
                    S[0] += m0;
                    S[1] += m1;
                }
                a0 = a1;
            }
        }
        wait_vm<0>();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float acc = 0.0f;
#pragma unroll
    for (int i = 0; i < 6; ++i) acc += S[i][0] + S[i][1] + S[i][2] + S[i][3];
    if (acc == 1.2345f) sink[blockIdx.x * 512 + tid] = acc;
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

int main(int argc, char **argv) {
    const int chunks = argc > 1 ? atoi(argv[1]) : 64;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const size_t ubytes = (size_t)NP * C * C * 4;
    uint16_t *u = nullptr;
    float *sink = nullptr;
    unsigned long long *cyc = nullptr;
    CK(hipMalloc(&u, ubytes));
    CK(hipMalloc(&sink, (size_t)cus * 512 * 4));
    CK(hipMalloc(&cyc, cus * 8));
    std::vector<uint16_t> h(ubytes / 2);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (uint16_t)(0x3800u | ((i * 2654435761u) >> 22 & 0x3ffu));
    CK(hipMemcpy(u, h.data(), ubytes, hipMemcpyHostToDevice));
    printf("{\"chunks\": %d, \"workgroups\": %d, \"results\": [", chunks, cus);
    for (int rep = 0; rep < 3; ++rep)
        for (int mode = 0; mode < 2; ++mode) {
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0));
            CK(hipEventCreate(&e1));
            for (int warm = 0; warm < 2; ++warm) {
                CK(hipEventRecord(e0, 0));
                if (mode == 0) hipLaunchKernelGGL(k_ring<0>, dim3(cus), dim3(512), 0, 0, u, chunks, sink, cyc);
                else hipLaunchKernelGGL(k_ring<1>, dim3(cus), dim3(512), 0, 0, u, chunks, sink, cyc);
                CK(hipGetLastError());
                CK(hipEventRecord(e1, 0));
                CK(hipDeviceSynchronize());
            }
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            std::vector<unsigned long long> c(cus);
            CK(hipMemcpy(c.data(), cyc, cus * 8, hipMemcpyDeviceToHost));
            std::sort(c.begin(), c.end());
            const double med = (double)c[cus / 2] / chunks;
            const double ubytes_per_chunk = (double)ubytes / NCH;  // per workgroup
            const double us = ms * 1e3;
            printf("%s{\"mode\": %d, \"rep\": %d, \"cycles_per_chunk_median\": %.0f, \"cycles_per_chunk_max\": %.0f, "
                   "\"us\": %.1f, \"u_TBps\": %.2f, \"u_B_per_clk_per_cu\": %.1f}",
                   (rep || mode) ? ", " : "", mode, rep, med, (double)c[cus - 1] / chunks, us,
                   ubytes_per_chunk * chunks * cus / (us * 1e-6) / 1e12, ubytes_per_chunk / med);
            CK(hipEventDestroy(e0));
            CK(hipEventDestroy(e1));
        }
    printf("]}\n");
    return 0;
}
