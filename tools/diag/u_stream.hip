// U-stream microbenchmark (diagnostic): every workgroup (8 waves, one per CU) reads the
// split-f16 conv's U (25 points x 4 chunks x hi/lo planes, 1.6 MB) with the conv's
// per-wave access pattern (two 16-byte buffer loads per lane per point, PF points in
// flight) and nothing else, SETS times. Prints the per-CU rate and the cycles per
// 32-channel chunk that the U stream alone needs.
// hipcc --offload-arch=gfx950 -O3 -o /tmp/u_stream tools/diag/u_stream.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef unsigned int u4 __attribute__((ext_vector_type(4)));
constexpr int C = 128, NP = 25, NCH = 4, UPLANE = C * 4 * 16;

// PAT 0: the conv's lane order (lane (co, kq) at co*64 + kq*16: a wave's 1 KB, lanes permuted);
// PAT 1: the same 1 KB lane-linear; PAT 2: lane-linear LDS-DMA (global_load_lds_dwordx4) into
// a ring in LDS (never read back)
template <int PF, int PAT>
__global__ __launch_bounds__(512) void k_stream(const unsigned short *u, int sets, unsigned *out,
                                                unsigned long long *cyc) {
    __shared__ __attribute__((aligned(16))) char ring[8][2][PF][1024];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int co = wv * 16 + (lane & 15), kq = lane >> 4;
    const int voff = PAT == 0 ? (co * 4 + kq) * 16 : wv * 1024 + lane * 16;
    const rsrc_t ur = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short *>(u), 0, NP * C * C * 4, 0x00020000);
    u4 acc = {0, 0, 0, 0};
    u4 q[PF][2];
    const int total = sets * NCH * NP;
    auto ld = [&](int i, u4 (&d)[2]) {
        const int xi = i % NP, ch = (i / NP) % NCH;
        const int soff = (xi * NCH + ch) * 2 * UPLANE;
        if constexpr (PAT == 2) {
#if defined(__HIP_DEVICE_COMPILE__)  // the builtin exists in the device pass only
            const char *g = reinterpret_cast<const char *>(u) + soff + voff;
            __builtin_amdgcn_global_load_lds(g, &ring[wv][0][i % PF][0], 16, 0, 0);
            __builtin_amdgcn_global_load_lds(g + UPLANE, &ring[wv][1][i % PF][0], 16, 0, 0);
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PF) : "memory");
#endif
        } else {
            d[0] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(ur, voff, soff, 0));
            d[1] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(ur, voff + UPLANE, soff, 0));
        }
    };
#pragma unroll
    for (int i = 0; i < PF; ++i) ld(i, q[i]);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < total; i += PF) {
#pragma unroll
        for (int j = 0; j < PF; ++j) {
            acc ^= q[j][0] ^ q[j][1];
            if (i + j + PF < total) ld(i + j + PF, q[j]);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
    out[blockIdx.x * 512 + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

template <int PF, int PAT>
void run(const unsigned short *u, unsigned *out, unsigned long long *cyc, int blocks, int sets) {
    k_stream<PF, PAT><<<blocks, 512>>>(u, 1, out, cyc);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    k_stream<PF, PAT><<<blocks, 512>>>(u, sets, out, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h;
    hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
    const double bytes_cu = (double)sets * NCH * NP * 8 * 2 * 1024;
    printf("{\"pat\": %d, \"pf\": %d, \"blocks\": %d, \"sets\": %d, \"ms\": %.3f, \"GBps_per_cu\": %.1f, \"TBps_chip\": %.2f, "
           "\"cycles_per_chunk_wg0\": %.0f, \"B_per_clk_wg0\": %.1f}\n",
           PAT, PF, blocks, sets, ms, bytes_cu / (ms * 1e6), bytes_cu * blocks / (ms * 1e9), (double)h / (sets * NCH),
           bytes_cu / (double)h);
}

int main() {
    unsigned short *u;
    unsigned *out;
    unsigned long long *cyc;
    hipMalloc(&u, (size_t)NP * C * C * 4);
    hipMemset(u, 1, (size_t)NP * C * C * 4);
    hipMalloc(&out, 1024 * 512 * 4);
    hipMalloc(&cyc, 8);
    for (int blocks : {256, 32}) {
        run<3, 0>(u, out, cyc, blocks, 16);
        run<8, 0>(u, out, cyc, blocks, 16);
        run<3, 1>(u, out, cyc, blocks, 16);
        run<8, 1>(u, out, cyc, blocks, 16);
        run<3, 2>(u, out, cyc, blocks, 16);
        run<8, 2>(u, out, cyc, blocks, 16);
    }
    return 0;
}
