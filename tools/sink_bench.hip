// sink_bench.hip -- the dummy-sink join (boss_kernels.hpp: dummy_sink_kernel) on the edges of a
// random genome (every edge but the last has a successor, as in a covered genome), with the
// kernel's timing ablations: what bounds it (stores, staging, search).
// Build: make -C tools sink_bench    Run: tools/sink_bench [genome_chars]
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../projects2014-metagenome_amd/csrc/boss_pipeline.hip"

using namespace mtg;

__device__ __forceinline__ uint64_t gmix64(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

__global__ void gen_genome(uint8_t *g, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        g[i] = (uint8_t)(gmix64(i / 32) >> (2 * (i % 32))) & 3;
}

// edge i over chars g[i .. i + 31]: label g[i + 31] in the low 2 bits, node chars above it with the
// most recent char on top (the layout the sink probe's to_next assumes)
__global__ void gen_edges(const uint8_t *g, uint64_t ne, uint64_t *out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ne; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t x = g[i + 31];
        for (int j = 0; j < 31; ++j) x |= (uint64_t)g[i + j] << (2 + 2 * j);
        out[i] = x;
    }
}

template <typename F>
static float time_ms(hipStream_t s, int reps, F f) {
    hipEvent_t a, b;
    HIP_CHECK(hipEventCreate(&a));
    HIP_CHECK(hipEventCreate(&b));
    f();
    HIP_CHECK(hipEventRecord(a, s));
    for (int r = 0; r < reps; ++r) f();
    HIP_CHECK(hipEventRecord(b, s));
    HIP_CHECK(hipEventSynchronize(b));
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char **argv) {
    const uint64_t G = argc > 1 ? strtoull(argv[1], nullptr, 10) : 373000000ull;
    const unsigned K = 32;  // BOSS k + 1 = 32 chars per edge (k = 31 DBG)
    hipStream_t s;
    HIP_CHECK(hipStreamCreate(&s));
    uint8_t *g;
    HIP_CHECK(hipMalloc(&g, G + 64));
    gen_genome<<<8192, 256, 0, s>>>(g, G);
    const uint64_t ne = G - 31;
    uint64_t *ka, *kb;
    HIP_CHECK(hipMalloc(&ka, ne * 8 + 64));
    HIP_CHECK(hipMalloc(&kb, ne * 8 + 64));
    gen_edges<<<8192, 256, 0, s>>>(g, ne, ka);
    size_t tb = 0;
    HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, tb, ka, kb, (int)ne, 0, 64, s));
    void *tmp;
    HIP_CHECK(hipMalloc(&tmp, tb));
    HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(tmp, tb, ka, kb, (int)ne, 0, 64, s));
    int *nsel;
    HIP_CHECK(hipMalloc(&nsel, 8));
    size_t tu = 0;
    HIP_CHECK(hipcub::DeviceSelect::Unique(nullptr, tu, kb, ka, nsel, (int)ne, s));
    void *tmp2;
    HIP_CHECK(hipMalloc(&tmp2, tu));
    HIP_CHECK(hipcub::DeviceSelect::Unique(tmp2, tu, kb, ka, nsel, (int)ne, s));
    int R32 = 0;
    HIP_CHECK(hipMemcpy(&R32, nsel, 4, hipMemcpyDeviceToHost));
    const uint64_t R = (uint64_t)R32;
    const Key<1> *keys = (const Key<1> *)ka;
    const unsigned B = bucket_bits<1>(R, 2 * K);
    const unsigned bshift = 2 * K - B;
    const uint64_t nb = 1ull << B;
    uint64_t *bstart;
    HIP_CHECK(hipMalloc(&bstart, (nb + 2) * 8));
    bucket_index_kernel<1><<<8192, 256, 0, s>>>(keys, R, bshift, nb, bstart);
    uint8_t *flags, *in_flag;
    HIP_CHECK(hipMalloc(&flags, R + 64));
    HIP_CHECK(hipMalloc(&in_flag, R + 64));
    const uint64_t stiles = ceil_div(R, DummyTraits<1>::TILE);
    HIP_CHECK(hipMemsetAsync(in_flag, 0, R, s));
    dummy_sink_kernel<1><<<dim3((unsigned)stiles), dim3(256), 0, s>>>(keys, R, K, bstart, bshift, flags, in_flag);
    HIP_CHECK(hipStreamSynchronize(s));
    {
        std::vector<uint8_t> f(R), in(R);
        HIP_CHECK(hipMemcpy(f.data(), flags, R, hipMemcpyDeviceToHost));
        HIP_CHECK(hipMemcpy(in.data(), in_flag, R, hipMemcpyDeviceToHost));
        uint64_t sinks = 0, firsts = 0, marked = 0;
        for (uint64_t i = 0; i < R; ++i) sinks += f[i] & 1, firsts += (f[i] >> 1) & 1, marked += in[i];
        printf("edges %lu (of %lu windows), bucket bits %u: sinks %lu, nodes %lu, marked in %lu\n", (unsigned long)R,
               (unsigned long)ne, B, (unsigned long)sinks, (unsigned long)firsts, (unsigned long)marked);
    }
    auto run = [&](const char *what, auto kern) {
        const float t = time_ms(s, 5, [&] {
            kern<<<dim3((unsigned)stiles), dim3(256), 0, s>>>(keys, R, K, bstart, bshift, flags, in_flag);
        });
        printf("%-44s %.3f ms  (%.1f GB/s of 19 B/edge)\n", what, t, R * 19.0 / 1e9 / (t * 1e-3));
    };
    const float tm = time_ms(s, 5, [&] { HIP_CHECK(hipMemsetAsync(in_flag, 0, R, s)); });
    printf("%-44s %.3f ms\n", "memset in_flag", tm);
    run("dummy_sink (product)", dummy_sink_kernel<1, 0>);
    run("no in_flag stores", dummy_sink_kernel<1, 1>);
    run("no flags stores", dummy_sink_kernel<1, 2>);
    run("no stores", dummy_sink_kernel<1, 3>);
    run("staging, no search", dummy_sink_kernel<1, 8>);
    run("no staging, no search (tile loads + flags)", dummy_sink_kernel<1, 4>);
    const float tc = time_ms(s, 5, [&] {
        HIP_CHECK(hipMemcpyAsync(kb, ka, R * 8, hipMemcpyDeviceToDevice, s));
    });
    printf("%-44s %.3f ms (%.0f GB/s read+write)\n", "D2D copy of the keys", tc, R * 16 / 1e9 / (tc * 1e-3));
    return 0;
}
