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

namespace mtg {
// the round-4 kernel (per-probe byte stores), for the A/B below
template <int L, int ABL = 0>
__global__ __launch_bounds__(256) void dummy_sink_kernel_r4(
    const Key<L> *__restrict__ keys, uint64_t n, unsigned K, const uint64_t *__restrict__ start,
    unsigned bshift, uint8_t *__restrict__ flags, uint8_t *__restrict__ in_flag,
    const Key<L> *__restrict__ q = nullptr, uint64_t nq = 0) {
    using T = DummyTraits<L>;
    const Key<L> *__restrict__ look = q ? q : keys;
    const uint64_t nl = q ? nq : n;
    constexpr int PER = T::PER;
    __shared__ Key<L> s_r[T::CAP];
    __shared__ uint64_t s_lo[4];
    __shared__ uint32_t s_cnt[4], s_off[4];
    const uint32_t tid = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * T::TILE;
    const uint32_t tn = (uint32_t)min((uint64_t)T::TILE, n - base);
    const Key<L> m3 = Key<L>::from(3);

    if (tid < 4) {
        // key range of the sink probes of label c = tid, read off the bucket index
        const Key<L> c = shl(Key<L>::from(tid), 2 * (K - 1));
        const Key<L> lo = (shr(keys[base], 2) | c) & ~m3;
        const Key<L> hi = shr(keys[base + tn - 1], 2) | c | m3;
        const uint64_t blo = bits_at(shr(lo, bshift), 0, 32), bhi = bits_at(shr(hi, bshift), 0, 32);
        const uint64_t a = start[blo], b = start[bhi + 1];
        s_lo[tid] = a;
        s_cnt[tid] = (uint32_t)min(b - a, (uint64_t)0xFFFFFFFFu);
    }
    const uint32_t j0 = tid * PER;
    Key<L> x[PER];
    uint32_t first = 0;
    {
        Key<L> prev = base + j0 > 0 && j0 < tn ? keys[base + j0 - 1] : Key<L>::zero();
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            x[q] = Key<L>::zero();
            if (j0 + q < tn) {
                x[q] = keys[base + j0 + q];
                if (base + j0 + q == 0 || shr(prev, 2) != shr(x[q], 2)) first |= 1u << q;
                prev = x[q];
            }
        }
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t cum = 0;
        for (int c = 0; c < 4; ++c) {
            s_off[c] = ~0u;  // ~0 = global fallback
            if ((uint64_t)cum + s_cnt[c] <= (uint64_t)T::CAP) {
                s_off[c] = cum;
                cum += s_cnt[c];
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        if (ABL & 4) break;
        if (s_off[c] == ~0u) continue;
        const uint64_t a = s_lo[c];
        const uint32_t off = s_off[c];
        for (uint32_t j = tid; j < s_cnt[c]; j += 256) s_r[off + j] = look[a + j];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        if (j0 + q >= tn) continue;
        if (ABL & 12) {
            if (!(ABL & 2)) flags[base + j0 + q] = (uint8_t)(1u | (((first >> q) & 1u) << 1)) ^ (uint8_t)s_r[q & 7].w[0];
            continue;
        }
        const uint32_t c = (uint32_t)(x[q].w[0] & 3);
        // to_next(x, K, 0): node a_2..a_K, label 0 (kmer_boss.hpp:147-169)
        const Key<L> p = (shr(x[q], 2) | shl(Key<L>::from(c), 2 * (K - 1))) & ~m3;
        uint64_t hit = ~0ull;
        const uint32_t off = s_off[c];
        if (off != ~0u) {
            const uint32_t cnt = s_cnt[c];
            uint32_t lo = 0, hi = cnt;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_r[off + mid] < p) lo = mid + 1; else hi = mid;
            }
            if (lo < cnt && shr(s_r[off + lo], 2) == shr(p, 2)) hit = s_lo[c] + lo;
        } else {
            const uint64_t i = lower_bound_bucketed(look, start, bshift, p);
            if (i < nl && shr(look[i], 2) == shr(p, 2)) hit = i;
        }
        if (!(ABL & 1) && hit != ~0ull) in_flag[hit] = 1;
        if (!(ABL & 2)) flags[base + j0 + q] = (uint8_t)((hit == ~0ull ? 1u : 0u) | (((first >> q) & 1u) << 1));
        else if (hit == 12345) flags[0] = 1;  // keep the search
    }
}

}  // namespace mtg

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
    {
        // the round-5 kernel against the round-4 one: byte-identical flags and in-edge marks
        uint8_t *f2, *in2;
        HIP_CHECK(hipMalloc(&f2, R + 64));
        HIP_CHECK(hipMalloc(&in2, R + 64));
        HIP_CHECK(hipMemsetAsync(in2, 0, R, s));
        dummy_sink_kernel_r4<1><<<dim3((unsigned)stiles), dim3(256), 0, s>>>(keys, R, K, bstart, bshift, f2, in2);
        HIP_CHECK(hipStreamSynchronize(s));
        std::vector<uint8_t> a(R), b(R), c(R), d(R);
        HIP_CHECK(hipMemcpy(a.data(), flags, R, hipMemcpyDeviceToHost));
        HIP_CHECK(hipMemcpy(b.data(), f2, R, hipMemcpyDeviceToHost));
        HIP_CHECK(hipMemcpy(c.data(), in_flag, R, hipMemcpyDeviceToHost));
        HIP_CHECK(hipMemcpy(d.data(), in2, R, hipMemcpyDeviceToHost));
        printf("round-5 vs round-4 kernel: flags %s, in-edge marks %s\n", a == b ? "equal" : "DIFFER",
               c == d ? "equal" : "DIFFER");
        if (a != b || c != d) return 1;
    }
    auto run = [&](const char *what, auto kern) {
        const float t = time_ms(s, 5, [&] {
            kern<<<dim3((unsigned)stiles), dim3(256), 0, s>>>(keys, R, K, bstart, bshift, flags, in_flag, nullptr, 0);
        });
        printf("%-44s %.3f ms  (%.1f GB/s of 19 B/edge)\n", what, t, R * 19.0 / 1e9 / (t * 1e-3));
    };
    const float tm = time_ms(s, 5, [&] { HIP_CHECK(hipMemsetAsync(in_flag, 0, R, s)); });
    printf("%-44s %.3f ms\n", "memset in_flag", tm);
    run("dummy_sink round 4 (per-probe stores)", dummy_sink_kernel_r4<1, 0>);
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
