// Probe: cost of a grid-wide barrier inside one persistent kernel vs a kernel boundary, on gfx950.
// Decides whether a persistent decode-step kernel (phases separated by grid barriers, the next phase's weights
// requested before the barrier) can beat one launch per phase (~4.5 us floor per decoder launch, r03k trace).
// Every spin is bounded: a barrier that does not complete within the limit sets an error flag and the kernel
// exits, so the grid always drains.
// build: hipcc -O3 --offload-arch=gfx950 -o tools/barrier_probe tools/barrier_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

constexpr unsigned SPIN_LIMIT = 1u << 22;

__device__ __forceinline__ bool grid_barrier(unsigned* count, unsigned* gen, unsigned nblocks, unsigned& my_gen,
                                             int* err) {
    __shared__ int ok;
    __syncthreads();
    if (threadIdx.x == 0) {
        ok = 1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const unsigned g = my_gen;
        const unsigned arrived = __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (arrived == nblocks - 1) {
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            unsigned spins = 0;
            while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
                if (++spins > SPIN_LIMIT || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        my_gen = g + 1;
    }
    __syncthreads();
    return ok;
}

// rounds of: read `bytes_per_block` of a weight stream (16 B per lane per request), write one float per block,
// barrier; a block then reads the value another block wrote (checks visibility across XCDs)
__global__ __launch_bounds__(256) void persist_kernel(const u32x4* w, size_t w_per_block, float* act, unsigned* count,
                                                      unsigned* gen, int* err, int rounds, float* sink) {
    unsigned my_gen = 0;
    const unsigned nb = gridDim.x;
    float acc = 0.f;
    for (int r = 0; r < rounds; ++r) {
        const u32x4* wb = w + ((size_t)blockIdx.x + (size_t)r * nb) % (nb * 4) * w_per_block;
        for (size_t i = threadIdx.x; i < w_per_block; i += 256) {
            const u32x4 v = __builtin_nontemporal_load(wb + i);
            acc += __uint_as_float(v.x ^ v.y ^ v.z ^ v.w);
        }
        if (threadIdx.x == 0) act[(size_t)r * nb + blockIdx.x] = (float)(r + blockIdx.x);
        if (!grid_barrier(count, gen, nb, my_gen, err)) break;
        if (threadIdx.x == 0) {
            const unsigned other = (blockIdx.x + 97) % nb;
            if (act[(size_t)r * nb + other] != (float)(r + other)) __hip_atomic_store(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (acc == 12345.f) sink[blockIdx.x] = acc;
}

__global__ __launch_bounds__(256) void phase_kernel(const u32x4* w, size_t w_per_block, float* act, int r, float* sink) {
    const unsigned nb = gridDim.x;
    float acc = 0.f;
    const u32x4* wb = w + ((size_t)blockIdx.x + (size_t)r * nb) % (nb * 4) * w_per_block;
    for (size_t i = threadIdx.x; i < w_per_block; i += 256) {
        const u32x4 v = __builtin_nontemporal_load(wb + i);
        acc += __uint_as_float(v.x ^ v.y ^ v.z ^ v.w);
    }
    if (threadIdx.x == 0) act[(size_t)r * nb + blockIdx.x] = (float)(r + blockIdx.x);
    if (acc == 12345.f) sink[blockIdx.x] = acc;
}

int main(int argc, char** argv) {
    const int nb = argc > 1 ? atoi(argv[1]) : 256;
    const int rounds = argc > 2 ? atoi(argv[2]) : 288;
    const size_t kb = argc > 3 ? atoi(argv[3]) : 0;   // KB of weights per block per round
    const size_t wpb = kb * 1024 / 16;
    u32x4* w;
    float *act, *sink;
    unsigned* sync;
    int* err;
    CK(hipMalloc(&w, (wpb ? wpb : 1) * nb * 4 * 16));
    CK(hipMemset(w, 1, (wpb ? wpb : 1) * nb * 4 * 16));
    CK(hipMalloc(&act, (size_t)rounds * nb * 4));
    CK(hipMalloc(&sink, nb * 4));
    CK(hipMalloc(&sync, 64));
    CK(hipMalloc(&err, 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best_p = 1e30f, best_k = 1e30f;
    for (int it = 0; it < 5; ++it) {
        CK(hipMemset(sync, 0, 64));
        CK(hipMemset(err, 0, 4));
        unsigned* count = sync;
        unsigned* gen = sync + 8;
        void* args[] = {&w, (void*)&wpb, &act, &count, &gen, &err, (void*)&rounds, &sink};
        CK(hipEventRecord(e0));
        CK(hipLaunchCooperativeKernel((const void*)persist_kernel, dim3(nb), dim3(256), args, 0, 0));
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        int herr;
        CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
        if (herr) {
            printf("persistent kernel error flag %d\n", herr);
            return 2;
        }
        best_p = ms < best_p ? ms : best_p;
        CK(hipEventRecord(e0));
        for (int r = 0; r < rounds; ++r) hipLaunchKernelGGL(phase_kernel, dim3(nb), dim3(256), 0, 0, w, wpb, act, r, sink);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        best_k = ms < best_k ? ms : best_k;
    }
    printf("blocks %d rounds %d KB/block/round %zu: persistent %.2f us/round, kernel-per-round %.2f us/round\n", nb,
           rounds, kb, best_p * 1e3 / rounds, best_k * 1e3 / rounds);
    return 0;
}
