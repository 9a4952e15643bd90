// stage_bench.hip -- microbenchmarks of single pipeline kernels on synthetic sorted keys, with
// the kernels' ablation switches, plus calibration kernels (copy, single-word dequeue).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/stage_bench tools/stage_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../projects2014-metagenome_amd/csrc/boss_pipeline.hip"

using namespace mtg;

__device__ __forceinline__ uint64_t splitmix(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

// strictly increasing keys: i * S + jitter < (i + 1) * S
__global__ void gen_sorted(Key<1> *keys, uint64_t n, uint64_t S) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        keys[i].w[0] = i * S + splitmix(i) % S;
}

__global__ void copy_kernel(const uint4 *__restrict__ a, uint4 *__restrict__ b, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

__global__ void dequeue_kernel(uint32_t *counter, uint32_t *sink) {
    __shared__ uint32_t s_tile;
    const uint32_t t = take_tile(counter, &s_tile);
    if (t == 0xFFFFFFFFu) sink[0] = t;
}

__global__ void atomic64_kernel(unsigned long long *tot) {
    if (threadIdx.x == 0) {
        atomicAdd(&tot[0], 1ull);
        atomicAdd(&tot[1], 2ull);
    }
}

template <typename F>
static float time_ms(hipStream_t s, int reps, F f) {
    hipEvent_t a, b;
    HIP_CHECK(hipEventCreate(&a));
    HIP_CHECK(hipEventCreate(&b));
    f();
    HIP_CHECK(hipStreamSynchronize(s));
    HIP_CHECK(hipEventRecord(a, s));
    for (int i = 0; i < reps; ++i) f();
    HIP_CHECK(hipEventRecord(b, s));
    HIP_CHECK(hipEventSynchronize(b));
    float ms;
    HIP_CHECK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char **argv) {
    const uint64_t R = argc > 1 ? strtoull(argv[1], nullptr, 10) : 373000000ull;
    const unsigned K = 31;
    hipStream_t s;
    HIP_CHECK(hipStreamCreate(&s));
    Key<1> *keys, *tmp;
    HIP_CHECK(hipMalloc(&keys, R * 8 + 64));
    HIP_CHECK(hipMalloc(&tmp, R * 8 + 64));
    gen_sorted<<<4096, 256, 0, s>>>(keys, R, (1ull << (2 * K)) / R);
    const unsigned B = bucket_bits<1>(R, 2 * K);
    const unsigned bshift = 2 * K - B;
    const uint64_t nb = 1ull << B;
    uint64_t *bstart;
    HIP_CHECK(hipMalloc(&bstart, (nb + 2) * 8));
    uint8_t *flags;
    HIP_CHECK(hipMalloc(&flags, R + 64));
    unsigned long long *tot;
    HIP_CHECK(hipMalloc(&tot, 64));
    uint32_t *counter;
    HIP_CHECK(hipMalloc(&counter, 64));

    float t = time_ms(s, 3, [&] {
        bucket_index_kernel<1><<<8192, 256, 0, s>>>(keys, R, bshift, nb, bstart);
    });
    printf("bucket_index B=%u: %.3f ms\n", B, t);
    t = time_ms(s, 3, [&] {
        copy_kernel<<<8192, 256, 0, s>>>((const uint4 *)keys, (uint4 *)tmp, R / 2);
    });
    printf("copy %.2f GB: %.3f ms = %.0f GB/s\n", R * 16 / 1e9, t, R * 16 / 1e9 / (t * 1e-3));
    const uint64_t tiles = ceil_div(R, DummyTraits<1>::TILE);
    for (uint32_t nbk : {65536u, 262144u, (uint32_t)tiles}) {
        t = time_ms(s, 3, [&] {
            HIP_CHECK(hipMemsetAsync(counter, 0, 4, s));
            dequeue_kernel<<<nbk, 256, 0, s>>>(counter, counter + 8);
        });
        printf("dequeue %u blocks: %.3f ms (%.1f ns/block)\n", nbk, t, t * 1e6 / nbk);
        t = time_ms(s, 3, [&] { atomic64_kernel<<<nbk, 256, 0, s>>>(tot); });
        printf("2x atomic64 %u blocks: %.3f ms\n", nbk, t);
    }
    const uint64_t stiles = ceil_div(R, DummyTraits<1>::TILE);
    const uint64_t wtiles = ceil_div(R, DummyTraits<1>::WTILE);
    uint8_t *in_flag;
    HIP_CHECK(hipMalloc(&in_flag, R + 64));
    uint32_t *tcnt;
    HIP_CHECK(hipMalloc(&tcnt, wtiles * 4 + 64));
    t = time_ms(s, 3, [&] {
        HIP_CHECK(hipMemsetAsync(in_flag, 0, R, s));
        dummy_sink_kernel<1><<<dim3((unsigned)stiles), dim3(256), 0, s>>>(keys, R, K, bstart, bshift,
                                                                         flags, in_flag);
    });
    printf("memset + dummy_sink: %.3f ms\n", t);
    t = time_ms(s, 3, [&] {
        dummy_count_kernel<<<dim3((unsigned)wtiles), dim3(256), 0, s>>>(flags, in_flag, R, K - 1, tcnt);
    });
    std::vector<uint32_t> h(wtiles);
    HIP_CHECK(hipMemcpy(h.data(), tcnt, wtiles * 4, hipMemcpyDeviceToHost));
    uint64_t sum = 0;
    for (auto v : h) sum += v;
    printf("dummy_count: %.3f ms  dummies=%lu\n", t, (unsigned long)sum);
    return 0;
}
