// Dependent-load latency microbenchmark (diagnostic): the unit of k_select's latency model.
// Every wave walks its own chain of STEPS dependent loads; each step is one wave-wide load of
// 64 consecutive int32 (256 B, one child-scan iteration of k_select) whose lane-0 value is the
// next position. Chains are random over a buffer of SPAN bytes: 1 GiB (every step misses the
// XCD's L2) or 2 MiB (L2-resident after the first pass). Loads are plain or agent-scope
// (`sc1`, what the evaluation-cache probes use). Waves launch as k_select's do: 4 per
// workgroup, one wave per tree. Prints one JSON object: per configuration the mean and the
// slowest wave's time per dependent step, from the constant 100 MHz clock (s_memrealtime).
// hipcc --offload-arch=gfx950 -O3 -o tools/diag/chase tools/diag/chase.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

template <bool SC1>
__global__ __launch_bounds__(256) void k_chase(const int *__restrict__ next, int n_nodes, int steps,
                                               unsigned long long *ticks, int *sink) {
    const int lane = threadIdx.x & 63;
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
    int node = (int)(((unsigned long long)w * 2654435761ull) % (unsigned long long)n_nodes);
    int acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int s = 0; s < steps; ++s) {
        const int *p = next + (size_t)node * 64 + lane;
        const int v = SC1 ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *p;
        acc += v;
        node = __builtin_amdgcn_readfirstlane(v);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        ticks[w] = t1 - t0;
        sink[w] = acc;
    }
}

int main(int argc, char **argv) {
    const int steps = argc > 1 ? atoi(argv[1]) : 200;
    const size_t big = 1ull << 30;
    int *d_next = nullptr, *d_sink = nullptr;
    unsigned long long *d_ticks = nullptr;
    CK(hipMalloc(&d_next, big));
    CK(hipMalloc(&d_sink, 4096 * sizeof(int)));
    CK(hipMalloc(&d_ticks, 4096 * sizeof(unsigned long long)));
    std::mt19937_64 rng(12345);
    printf("{\"unit\": \"us per dependent 256-B wave load\", \"steps\": %d, \"configs\": [", steps);
    bool first = true;
    for (size_t span : {big, (size_t)2 << 20}) {
        const int n_nodes = (int)(span / 256);
        // a random cyclic permutation of the nodes: every chain step lands on a new 256-B node
        std::vector<int> perm(n_nodes);
        for (int i = 0; i < n_nodes; ++i) perm[i] = i;
        for (int i = n_nodes - 1; i > 0; --i) std::swap(perm[i], perm[rng() % (unsigned)(i + 1)]);
        std::vector<int> host((size_t)n_nodes * 64);
        for (int i = 0; i < n_nodes; ++i) {
            const int nx = perm[(i + 1) % n_nodes];
            for (int l = 0; l < 64; ++l) host[(size_t)perm[i] * 64 + l] = nx;
        }
        CK(hipMemcpy(d_next, host.data(), host.size() * sizeof(int), hipMemcpyHostToDevice));
        for (int sc1 = 0; sc1 < 2; ++sc1) {
            for (int waves : {2048, 64}) {
                const int blocks = waves / 4;
                hipEvent_t e0, e1;
                CK(hipEventCreate(&e0));
                CK(hipEventCreate(&e1));
                float ms = 0.0f;
                for (int rep = 0; rep < 2; ++rep) {  // the first pass warms the small span into L2
                    CK(hipEventRecord(e0, 0));
                    if (sc1) hipLaunchKernelGGL(k_chase<true>, dim3(blocks), dim3(256), 0, 0, d_next, n_nodes, steps, d_ticks, d_sink);
                    else hipLaunchKernelGGL(k_chase<false>, dim3(blocks), dim3(256), 0, 0, d_next, n_nodes, steps, d_ticks, d_sink);
                    CK(hipGetLastError());
                    CK(hipEventRecord(e1, 0));
                    CK(hipDeviceSynchronize());
                    CK(hipEventElapsedTime(&ms, e0, e1));
                }
                std::vector<unsigned long long> t(waves);
                CK(hipMemcpy(t.data(), d_ticks, waves * sizeof(unsigned long long), hipMemcpyDeviceToHost));
                double sum = 0, mx = 0;
                for (auto v : t) {
                    sum += (double)v;
                    mx = mx > (double)v ? mx : (double)v;
                }
                const double us_mean = sum / waves / steps * 0.01, us_max = mx / steps * 0.01;  // 100 MHz ticks
                printf("%s{\"span_bytes\": %zu, \"loads\": \"%s\", \"waves\": %d, \"us_mean\": %.3f, \"us_max\": %.3f, "
                       "\"us_per_step_events\": %.3f}",
                       first ? "" : ", ", span, sc1 ? "sc1 (agent)" : "plain", waves, us_mean, us_max, ms * 1e3 / steps);
                first = false;
            }
        }
    }
    printf("]}\n");
    CK(hipFree(d_next));
    CK(hipFree(d_sink));
    CK(hipFree(d_ticks));
    return 0;
}
