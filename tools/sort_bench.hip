// sort_bench.hip -- microbenchmark of the K2 radix pass on N random 62-bit keys:
//   copy   : 8 B/lane streaming read + write of the same bytes (achievable pass floor)
//   mtg    : the pipeline's onesweep radix sort (all passes), per-pass times
//   rocprim: hipcub::DeviceRadixSort::SortKeys over bits [0, 62) (known-good reference)
// Usage: sort_bench [n_keys]
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <chrono>
#include <cstdio>
#include <vector>

#include "../projects2014-metagenome_amd/csrc/boss_pipeline.hip"

using namespace mtg;

__global__ void fill_kernel(Key<1> *k, uint64_t n, uint64_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = (i + seed) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        k[i].w[0] = (z ^ (z >> 31)) >> 2;
    }
}

// keys[i] = keys[hash(i) % (n / dupf)]: every distinct key about dupf times, shuffled
__global__ void dup_kernel(Key<1> *k, uint64_t n, int dupf) {
    const uint64_t m = n / dupf;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = i * 0xD6E8FEB86659FD93ull;
        z ^= z >> 32;
        uint64_t j = z % m;
        uint64_t y = (j + 7) * 0x9E3779B97F4A7C15ull;
        y = (y ^ (y >> 30)) * 0xBF58476D1CE4E5B9ull;
        y = (y ^ (y >> 27)) * 0x94D049BB133111EBull;
        k[i].w[0] = (y ^ (y >> 31)) >> 2;
    }
}

template <int ITEMS>
__global__ __launch_bounds__(512) void copy_kernel(const uint64_t *__restrict__ in,
                                                   uint64_t *__restrict__ out, uint64_t n) {
    const uint64_t base = (uint64_t)blockIdx.x * 512 * ITEMS;
    uint64_t v[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        uint64_t i = base + j * 512 + threadIdx.x;
        v[j] = i < n ? in[i] : 0;
    }
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        uint64_t i = base + j * 512 + threadIdx.x;
        if (i < n) out[i] = v[j];
    }
}

static double now_ms() {
    return std::chrono::duration<double, std::milli>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1200000000ull;
    Ctx c;
    HIP_CHECK(hipStreamCreate(&c.stream));
    HIP_CHECK(hipMalloc(&c.small, sizeof(Small)));
    Key<1> *a, *b;
    HIP_CHECK(hipMalloc(&a, n * 8));
    HIP_CHECK(hipMalloc(&b, n * 8));
    hipEvent_t e0, e1;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    float ms;
    const double gb = 2.0 * n * 8 / 1e9;

    for (int rep = 0; rep < 3; ++rep) {
        HIP_CHECK(hipEventRecord(e0, c.stream));
        copy_kernel<16><<<dim3((unsigned)ceil_div(n, 512 * 16)), dim3(512), 0, c.stream>>>(
            (const uint64_t *)a, (uint64_t *)b, n);
        HIP_CHECK(hipEventRecord(e1, c.stream));
        HIP_CHECK(hipEventSynchronize(e1));
        HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        printf("copy   : %.3f ms  %.0f GB/s\n", ms, gb / ms * 1e3);
    }

    for (int rep = 0; rep < 3; ++rep) {
        fill_kernel<<<4096, 256, 0, c.stream>>>(a, n, rep);
        HIP_CHECK(hipStreamSynchronize(c.stream));
        Key<1> *ka = a, *kb = b;
        uint32_t *nv = nullptr;
        c.radix_ms = 0;
        c.radix_launches = 0;
        c.radix_bytes = 0;
        double t0 = now_ms();
        radix_sort<1, false>(c, &ka, &kb, &nv, &nv, n, 62, true);
        HIP_CHECK(hipStreamSynchronize(c.stream));
        double t1 = now_ms();
        printf("mtg    : total %.3f ms, %lu passes, avg pass %.3f ms = %.0f GB/s\n", t1 - t0,
               (unsigned long)c.radix_launches, c.radix_ms / c.radix_launches,
               gb / (c.radix_ms / c.radix_launches) * 1e3);
        std::vector<uint64_t> h(1 << 20);
        HIP_CHECK(hipMemcpy(h.data(), ka, h.size() * 8, hipMemcpyDeviceToHost));
        bool ok = true;
        for (size_t i = 1; i < h.size(); ++i) ok &= h[i - 1] <= h[i];
        printf("         sorted prefix ok=%d\n", ok);
        if (ka != a) std::swap(a, b);
    }

    // MSD sort + unique on keys with `dupf` copies of each distinct key (shuffled)
    for (int dupf : {1, 8}) {
        for (int rep = 0; rep < 2; ++rep) {
            fill_kernel<<<4096, 256, 0, c.stream>>>(a, n, 100 + rep);
            if (dupf > 1) dup_kernel<<<4096, 256, 0, c.stream>>>(a, n, dupf);
            HIP_CHECK(hipStreamSynchronize(c.stream));
            Key<1> *ka = a, *kb = b;
            uint32_t *nv = nullptr;
            c.radix_ms = 0;
            c.radix_launches = 0;
            c.radix_bytes = 0;
            c.track_partition = true;
            double t0 = now_ms();
            uint64_t u = msd_sort_unique<1, false>(c, &ka, &kb, &nv, &nv, n, 62, 0, dupf);
            HIP_CHECK(hipStreamSynchronize(c.stream));
            double t1 = now_ms();
            c.track_partition = false;
            printf("msd dup=%d: total %.3f ms, unique %lu, %lu partition passes avg %.3f ms = %.0f GB/s\n",
                   dupf, t1 - t0, (unsigned long)u, (unsigned long)c.radix_launches,
                   c.radix_ms / std::max<uint64_t>(1, c.radix_launches),
                   c.radix_launches ? c.radix_bytes / c.radix_ms / 1e6 : 0.0);
            std::vector<uint64_t> h(1 << 20);
            HIP_CHECK(hipMemcpy(h.data(), ka, h.size() * 8, hipMemcpyDeviceToHost));
            bool ok = true;
            for (size_t i = 1; i < h.size(); ++i) ok &= h[i - 1] < h[i];
            printf("         strictly increasing prefix ok=%d\n", ok);
            if (ka != a) std::swap(a, b);
        }
    }

    // ablations of one pass (shift 0): timing only, outputs are not a sort
    {
        constexpr int TILE = SortTraits<1>::TILE;
        const uint64_t tiles = ceil_div(n, TILE);
        std::vector<uint64_t> starts(256);
        for (int d = 0; d < 256; ++d) starts[d] = (n / 256) * d;
        uint64_t *dstart;
        HIP_CHECK(hipMalloc(&dstart, 256 * 8));
        HIP_CHECK(hipMemcpy(dstart, starts.data(), 256 * 8, hipMemcpyHostToDevice));
        uint32_t ep;
        auto run = [&](auto kern, const char *name) {
            for (int rep = 0; rep < 2; ++rep) {
                uint64_t *desc = acquire_desc(c, tiles * 256, &ep);
                if (rep == 0) HIP_CHECK(hipMemsetAsync(desc, 0, tiles * 256 * 8, c.stream));
                HIP_CHECK(hipMemsetAsync(&c.small->counter, 0, 4, c.stream));
                HIP_CHECK(hipMemsetAsync(desc, 0, 256 * 8, c.stream));
                HIP_CHECK(hipEventRecord(e0, c.stream));
                kern<<<dim3((unsigned)tiles), dim3(512), 0, c.stream>>>(a, b, nullptr, nullptr, n, 0u,
                                                                      dstart, desc, ep, &c.small->counter,
                                                                      &c.small->error);
                HIP_CHECK(hipEventRecord(e1, c.stream));
                HIP_CHECK(hipEventSynchronize(e1));
                HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
                printf("abl %-28s: %.3f ms  %.0f GB/s\n", name, ms, gb / ms * 1e3);
            }
        };
        fill_kernel<<<4096, 256, 0, c.stream>>>(a, n, 7);
        run(onesweep_kernel<1, false, 0>, "full pass");
        run(onesweep_kernel<1, false, 1>, "atomic cursor (no lookback)");
        run(onesweep_kernel<1, false, 2>, "no scatter");
        run(onesweep_kernel<1, false, 3>, "no lookback, no scatter");
        run(onesweep_kernel<1, false, 4>, "no ranking");
        run(onesweep_kernel<1, false, 5>, "no ranking, no lookback");
        run(onesweep_kernel<1, false, 7>, "no ranking/lookback/scatter");
    }

    {
        size_t temp = 0;
        uint64_t *ka = (uint64_t *)a, *kb = (uint64_t *)b;
        HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, temp, ka, kb, (int)std::min<uint64_t>(n, 2000000000ull), 0, 62, c.stream));
        void *dtemp;
        HIP_CHECK(hipMalloc(&dtemp, temp));
        for (int rep = 0; rep < 3; ++rep) {
            fill_kernel<<<4096, 256, 0, c.stream>>>(a, n, rep);
            HIP_CHECK(hipEventRecord(e0, c.stream));
            HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(dtemp, temp, ka, kb, (int)n, 0, 62, c.stream));
            HIP_CHECK(hipEventRecord(e1, c.stream));
            HIP_CHECK(hipEventSynchronize(e1));
            HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
            printf("rocprim: total %.3f ms (= %.3f ms per 8-bit pass equivalent, %.0f GB/s)\n", ms,
                   ms / 8, gb / (ms / 8) * 1e3);
        }
    }
    return 0;
}
