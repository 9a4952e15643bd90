// stage_bench.hip -- microbenchmarks of single pipeline kernels on synthetic sorted keys, with
// the kernels' ablation switches, plus calibration kernels (copy, single-word dequeue).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/stage_bench tools/stage_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
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

// 8-byte-per-lane copy: the access width of the partition pass, for FETCH_SIZE/WRITE_SIZE calibration
__global__ void copy8_kernel(const uint64_t *__restrict__ a, uint64_t *__restrict__ b, uint64_t n) {
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

// mode 0: uniform; 1: min of two (canonical-like skew); 2: like 1 with every key ~6x
__global__ void gen_random(Key<1> *keys, uint64_t n, unsigned bits, int mode) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t j = mode == 2 ? splitmix(i) % (n / 6) : i;
        uint64_t a = splitmix(j * 7919 + 13) >> (64 - bits);
        if (mode) a = min(a, splitmix(j * 104729 + 7) >> (64 - bits));
        keys[i].w[0] = a;
    }
}

// histogram variants over the top 8 of 62 bits: mode 0 read only, 1 block-shared LDS atomics,
// 2 per-wave LDS copies, 3 per-wave copies of 16-bit packed pairs
template <int MODE>
__global__ __launch_bounds__(512) void hist_variant(const Key<1> *__restrict__ keys, uint64_t n,
                                                    uint32_t *__restrict__ out) {
    __shared__ uint32_t s_h[8 * 256];
    for (int i = threadIdx.x; i < 8 * 256; i += 512) s_h[i] = 0;
    __syncthreads();
    const uint32_t w = threadIdx.x / 64;
    uint32_t acc = 0;
    const uint64_t base = (uint64_t)blockIdx.x * 8192;
    const uint64_t end = min(n, base + 8192);
    for (uint64_t i = base + 2 * threadIdx.x; i < end; i += 1024) {
        const ulonglong2 v = *(const ulonglong2 *)(keys + i);
        const uint32_t b0 = (uint32_t)(v.x >> 54), b1 = (uint32_t)(v.y >> 54);
        if (MODE == 0) acc += b0 + b1;
        if (MODE == 1) { atomicAdd(&s_h[b0], 1u); atomicAdd(&s_h[b1], 1u); }
        if (MODE == 2) { atomicAdd(&s_h[w * 256 + b0], 1u); atomicAdd(&s_h[w * 256 + b1], 1u); }
        if (MODE == 3) {
            atomicAdd(&s_h[w * 128 + (b0 >> 1)], 1u << (16 * (b0 & 1)));
            atomicAdd(&s_h[w * 128 + (b1 >> 1)], 1u << (16 * (b1 & 1)));
        }
    }
    __syncthreads();
    if (MODE == 0) { if (acc == 0xFFFFFFFF) out[0] = acc; return; }
    if (threadIdx.x < 256) {
        uint32_t c = 0;
        if (MODE == 1) c = s_h[threadIdx.x];
        if (MODE == 2) for (int q = 0; q < 8; ++q) c += s_h[q * 256 + threadIdx.x];
        if (MODE == 3) for (int q = 0; q < 8; ++q) c += (s_h[q * 128 + threadIdx.x / 2] >> (16 * (threadIdx.x & 1))) & 0xFFFF;
        out[(uint64_t)blockIdx.x * 256 + threadIdx.x] = c;
    }
}

/*
 * EXPERIMENT (measured, not used by the library): persistent form of the partition pass: gridDim.x workgroups (one per CU) walk the tiles
 * tile = blockIdx.x, blockIdx.x + gridDim.x, ... and keep the NEXT tile's keys in flight in
 * registers while the current one is ranked, reserved (one cursor atomic per (tile, bucket)),
 * reordered in LDS and written.  The reservation atomics are issued before the prefetch, so
 * waiting for them does not wait for the prefetch; the LDS tile (16 K keys at 1024 threads)
 * allows one workgroup per CU, whose phases would otherwise never overlap.
 */
template <int L, bool HAS_VAL, int BLOCK>
__global__ __launch_bounds__(BLOCK) void msd_partition_pipe_kernel(
    const Key<L> *__restrict__ kin, Key<L> *__restrict__ kout, const uint32_t *__restrict__ vin,
    uint32_t *__restrict__ vout, uint64_t n, unsigned nbits, unsigned b, unsigned bp,
    unsigned long long *__restrict__ cursor, uint64_t ntiles,
    const unsigned long long *__restrict__ fake_start = nullptr) {
    // fake_start (microbenchmark only): no reservation atomics, runs land at a tile-dependent
    // place inside their bucket -- the same write pattern without the atomics' cost
    constexpr int ITEMS = MsdTraits<L>::ITEMS;
    constexpr int TILE = ITEMS * BLOCK;
    constexpr int WMAX = MSD_WIN << 8;
    constexpr int PER = WMAX / BLOCK > 0 ? WMAX / BLOCK : 1;
    __shared__ Key<L> s_keys[TILE];
    __shared__ uint32_t s_vals[HAS_VAL ? TILE : 1];
    __shared__ uint32_t s_cnt[WMAX];
    __shared__ uint32_t s_loff[WMAX];
    __shared__ unsigned long long s_gbase[WMAX];
    __shared__ uint32_t s_scan[BLOCK / 64 + 1];
    __shared__ uint32_t s_wbase;

    const uint32_t tid = threadIdx.x;
    const unsigned sub = b - bp;
    const uint32_t wsize = min((uint32_t)WMAX, (uint32_t)MSD_WIN << sub);
    uint64_t tile = blockIdx.x;
    if (tile >= ntiles) return;

    Key<L> k[ITEMS];
    uint32_t v[ITEMS];
    auto load = [&](uint64_t t, Key<L> (&kk)[ITEMS], uint32_t (&vv)[ITEMS]) {
        const uint64_t base = t * TILE;
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint64_t i = base + (uint64_t)j * BLOCK + tid;
            kk[j] = i < n ? kin[i] : Key<L>::zero();
            if (HAS_VAL) vv[j] = i < n ? vin[i] : 0;
        }
    };
    load(tile, k, v);
    for (; tile < ntiles; tile += gridDim.x) {
        const uint64_t base = tile * TILE;
        for (uint32_t i = tid; i < wsize; i += BLOCK) s_cnt[i] = 0;
        if (tid == 0) s_wbase = key_prefix(k[0], nbits, bp) << sub;
        __syncthreads();
        const uint32_t wbase = s_wbase;
        uint32_t r[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            r[j] = 0xFFFFFFFFu;
            if (base + (uint64_t)j * BLOCK + tid < n) {
                const uint32_t lb = key_prefix(k[j], nbits, b) - wbase;
                if (lb < wsize) {
                    r[j] = atomicAdd(&s_cnt[lb], 1u);
                } else {
                    const unsigned long long o = atomicAdd(&cursor[lb + wbase], 1ull);
                    kout[o] = k[j];
                    if (HAS_VAL) vout[o] = v[j];
                }
            }
        }
        __syncthreads();
        uint32_t c[PER];
        uint32_t sum = 0;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const uint32_t i = tid * PER + q;
            c[q] = i < wsize ? s_cnt[i] : 0;
            sum += c[q];
        }
        uint32_t total;
        uint32_t off = block_exclusive_sum<BLOCK>(sum, s_scan, &total);
        unsigned long long g[PER];
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const uint32_t i = tid * PER + q;
            g[q] = 0;
            if (i < wsize) {
                s_loff[i] = off;
                if (c[q]) {
                    if (fake_start) {
                        const unsigned long long bs = fake_start[wbase + i], be = fake_start[wbase + i + 1];
                        const unsigned long long room = be - bs > c[q] ? be - bs - c[q] : 0;
                        g[q] = bs + (room ? (tile * c[q]) % room : 0);
                    } else {
                        g[q] = atomicAdd(&cursor[wbase + i], (unsigned long long)c[q]);
                    }
                }
            }
            off += c[q];
        }
        // the next tile's keys travel while this one is reordered and written
        Key<L> kn[ITEMS];
        uint32_t vn[ITEMS];
        const uint64_t next = tile + gridDim.x;
        if (next < ntiles) load(next, kn, vn);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            if (r[j] != 0xFFFFFFFFu) {
                const uint32_t lb = key_prefix(k[j], nbits, b) - wbase;
                const uint32_t pos = s_loff[lb] + r[j];
                s_keys[pos] = k[j];
                if (HAS_VAL) s_vals[pos] = v[j];
            }
        }
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const uint32_t i = tid * PER + q;
            if (i < wsize) s_gbase[i] = g[q];
        }
        __syncthreads();
        for (uint32_t p = tid; p < total; p += BLOCK) {
            const Key<L> key = s_keys[p];
            const uint32_t lb = key_prefix(key, nbits, b) - wbase;
            const uint64_t o = s_gbase[lb] + (p - s_loff[lb]);
            kout[o] = key;
            if (HAS_VAL) vout[o] = s_vals[p];
        }
        __syncthreads();
        if (next < ntiles) {
#pragma unroll
            for (int j = 0; j < ITEMS; ++j) {
                k[j] = kn[j];
                if (HAS_VAL) v[j] = vn[j];
            }
        }
    }
}
// Result on MI355X: no faster than msd_partition_kernel (bits 6/8/9: 4.29/5.01/5.32 ms vs
// 3.89/4.81/5.27 ms); without the reservation atomics (fake_start) it is slower still.

// level-1 MSD partition of n random keys: histogram, host scan, partition with cursor strides
static void partition_bench(hipStream_t s, uint64_t n) {
    Key<1> *a, *b;
    HIP_CHECK(hipMalloc(&a, n * 8 + 64));
    HIP_CHECK(hipMalloc(&b, n * 8 + 64));
    uint32_t *cnt;
    unsigned long long *cur;
    HIP_CHECK(hipMalloc(&cnt, 256 * 4));
    HIP_CHECK(hipMalloc(&cur, 256 * 8));
    const uint64_t tiles = ceil_div(n, MsdTraits<1>::TILE);
    for (int mode = 1; mode < 2; ++mode) {
        gen_random<<<8192, 256, 0, s>>>(a, n, 62, mode);
        {
            uint32_t *rows;
            HIP_CHECK(hipMalloc(&rows, tiles * 256 * 4));
            float th[4];
            th[0] = time_ms(s, 3, [&] { hist_variant<0><<<dim3((unsigned)tiles), dim3(512), 0, s>>>(a, n, rows); });
            th[1] = time_ms(s, 3, [&] { hist_variant<1><<<dim3((unsigned)tiles), dim3(512), 0, s>>>(a, n, rows); });
            th[2] = time_ms(s, 3, [&] { hist_variant<2><<<dim3((unsigned)tiles), dim3(512), 0, s>>>(a, n, rows); });
            th[3] = time_ms(s, 3, [&] { hist_variant<3><<<dim3((unsigned)tiles), dim3(512), 0, s>>>(a, n, rows); });
            printf("hist variants (read-only, shared, per-wave, per-wave packed): %.3f %.3f %.3f %.3f ms\n",
                   th[0], th[1], th[2], th[3]);
            HIP_CHECK(hipFree(rows));
        }
        float t = time_ms(s, 3, [&] {
            HIP_CHECK(hipMemsetAsync(cnt, 0, 256 * 4, s));
            msd_hist_kernel<1><<<dim3((unsigned)tiles), dim3(MSD_BLOCK), 0, s>>>(a, n, 62, 8, 0, cnt);
        });
        printf("mode %d msd_hist level1 n=%lu: %.3f ms = %.0f GB/s\n", mode, (unsigned long)n, t,
               n * 8 / 1e9 / (t * 1e-3));
        std::vector<uint32_t> h(256);
        HIP_CHECK(hipMemcpy(h.data(), cnt, 256 * 4, hipMemcpyDeviceToHost));
        std::vector<unsigned long long> st(256);
        unsigned long long acc = 0;
        for (int i = 0; i < 256; ++i) { st[i] = acc; acc += h[i]; }
        for (unsigned bits : {6u, 8u, 9u}) {
            std::vector<uint32_t> hh(1u << bits, 0);
            {   // bucket starts for this digit width, from a host pass over a key sample is not
                // exact: recount on the device
                uint32_t *c2;
                HIP_CHECK(hipMalloc(&c2, (1u << bits) * 4));
                HIP_CHECK(hipMemset(c2, 0, (1u << bits) * 4));
                msd_hist_kernel<1><<<dim3((unsigned)tiles), dim3(MSD_BLOCK), 0, s>>>(a, n, 62, bits, 0, c2);
                HIP_CHECK(hipMemcpy(hh.data(), c2, (1u << bits) * 4, hipMemcpyDeviceToHost));
                HIP_CHECK(hipFree(c2));
            }
            std::vector<unsigned long long> st2(1u << bits);
            unsigned long long acc2 = 0;
            for (uint32_t i = 0; i < (1u << bits); ++i) { st2[i] = acc2; acc2 += hh[i]; }
            unsigned long long *cur2;
            HIP_CHECK(hipMalloc(&cur2, (1u << bits) * 8));
            for (int blk : {512, 1024}) {
                const uint64_t ptiles = ceil_div(n, (uint64_t)MsdTraits<1>::ITEMS * blk);
                t = time_ms(s, 3, [&] {
                    HIP_CHECK(hipMemcpyAsync(cur2, st2.data(), (1u << bits) * 8, hipMemcpyHostToDevice, s));
                    if (blk == 512)
                        msd_partition_kernel<1, false, 512><<<dim3((unsigned)xcd_grid(ptiles)), dim3(512), 0, s>>>(
                            a, b, nullptr, nullptr, n, 62, bits, 0, cur2);
                    else
                        msd_partition_kernel<1, false, 1024><<<dim3((unsigned)xcd_grid(ptiles)), dim3(1024), 0, s>>>(
                            a, b, nullptr, nullptr, n, 62, bits, 0, cur2);
                });
                printf("mode %d partition bits=%u block=%d: %.3f ms = %.0f GB/s\n", mode, bits, blk, t,
                       2.0 * n * 8 / 1e9 / (t * 1e-3));
            }
            int ncu = 0;
            HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
            for (int blk : {512, 1024}) {
                for (int per_cu : {1, 2, 4}) {
                    if (blk == 1024 && per_cu > 1) continue;
                    const uint64_t ptiles = ceil_div(n, (uint64_t)MsdTraits<1>::ITEMS * blk);
                    const unsigned grid = (unsigned)std::min<uint64_t>(ptiles, (uint64_t)ncu * per_cu);
                    t = time_ms(s, 3, [&] {
                        HIP_CHECK(hipMemcpyAsync(cur2, st2.data(), (1u << bits) * 8, hipMemcpyHostToDevice, s));
                        if (blk == 512)
                            msd_partition_pipe_kernel<1, false, 512><<<dim3(grid), dim3(512), 0, s>>>(
                                a, b, nullptr, nullptr, n, 62, bits, 0, cur2, ptiles);
                        else
                            msd_partition_pipe_kernel<1, false, 1024><<<dim3(grid), dim3(1024), 0, s>>>(
                                a, b, nullptr, nullptr, n, 62, bits, 0, cur2, ptiles);
                    });
                    printf("mode %d pipe partition bits=%u block=%d grid=%u: %.3f ms = %.0f GB/s\n", mode, bits, blk,
                           grid, t, 2.0 * n * 8 / 1e9 / (t * 1e-3));
                }
            }
            {   // the same write pattern without the reservation atomics
                unsigned long long *fs;
                std::vector<unsigned long long> st3(st2);
                st3.push_back(n);
                HIP_CHECK(hipMalloc(&fs, st3.size() * 8));
                HIP_CHECK(hipMemcpy(fs, st3.data(), st3.size() * 8, hipMemcpyHostToDevice));
                const uint64_t ptiles = ceil_div(n, (uint64_t)MsdTraits<1>::ITEMS * 1024);
                t = time_ms(s, 3, [&] {
                    msd_partition_pipe_kernel<1, false, 1024><<<dim3((unsigned)ncu), dim3(1024), 0, s>>>(
                        a, b, nullptr, nullptr, n, 62, bits, 0, cur2, ptiles, fs);
                });
                printf("mode %d pipe partition bits=%u block=1024 NO ATOMICS: %.3f ms = %.0f GB/s\n", mode, bits, t,
                       2.0 * n * 8 / 1e9 / (t * 1e-3));
                HIP_CHECK(hipFree(fs));
                HIP_CHECK(hipMemcpyAsync(cur2, st2.data(), (1u << bits) * 8, hipMemcpyHostToDevice, s));
                msd_partition_pipe_kernel<1, false, 1024><<<dim3((unsigned)ncu), dim3(1024), 0, s>>>(
                    a, b, nullptr, nullptr, n, 62, bits, 0, cur2, ptiles);
                HIP_CHECK(hipStreamSynchronize(s));
            }
            {   // check the pipe kernel's output is a partition of the input (bucket counts + sum)
                std::vector<unsigned long long> cend(1u << bits);
                HIP_CHECK(hipMemcpy(cend.data(), cur2, (1u << bits) * 8, hipMemcpyDeviceToHost));
                bool ok = true;
                for (uint32_t i = 0; i < (1u << bits); ++i) ok &= cend[i] == st2[i] + hh[i];
                std::vector<uint64_t> ho(n);
                HIP_CHECK(hipMemcpy(ho.data(), b, n * 8, hipMemcpyDeviceToHost));
                uint64_t badb = 0;
                for (uint32_t i = 0; i < (1u << bits); ++i)
                    for (uint64_t q = st2[i]; q < st2[i] + hh[i]; ++q) badb += (ho[q] >> (62 - bits)) != i;
                printf("pipe partition bits=%u check: cursors %s, %lu keys in a wrong bucket\n", bits,
                       ok ? "ok" : "BAD", (unsigned long)badb);
            }
            HIP_CHECK(hipFree(cur2));
        }
    }
    HIP_CHECK(hipFree(a));
    HIP_CHECK(hipFree(b));
}

// reads of 150 random ACGT + '$' (151-byte stride)
__global__ void gen_reads(uint8_t *seq, uint64_t len) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < len;
         i += (uint64_t)gridDim.x * blockDim.x)
        seq[i] = i % 151 == 150 ? '$' : "ACGT"[splitmix(i) & 3];
}

static void extract_bench(hipStream_t s, uint64_t reads) {
    const uint64_t len = reads * 151;
    const unsigned K = 31;
    uint8_t *seq;
    HIP_CHECK(hipMalloc(&seq, len + 64));
    gen_reads<<<8192, 256, 0, s>>>(seq, len);
    const uint64_t npos = len - K + 1;
    constexpr int TILE = ExtractTraits<1>::TILE;
    const uint64_t tiles = ceil_div(npos, TILE);
    uint32_t *tcnt, *hist, *rows;
    uint64_t *toff;
    Key<1> *out;
    HIP_CHECK(hipMalloc(&tcnt, tiles * 4));
    HIP_CHECK(hipMalloc(&toff, (tiles + 1) * 8));
    HIP_CHECK(hipMalloc(&hist, 512 * 4));
    HIP_CHECK(hipMalloc(&rows, tiles * 256 * 4));
    HIP_CHECK(hipMalloc(&out, npos * 8));
    float t = time_ms(s, 3, [&] {
        extract_kernel<1, false, true><<<dim3((unsigned)tiles), dim3(256), 0, s>>>(
            seq, len, K, 1, nullptr, nullptr, 0, nullptr, 255, nullptr, nullptr, tcnt, nullptr, nullptr, 0);
    });
    printf("extract count: %.3f ms\n", t);
    std::vector<uint32_t> h(tiles);
    HIP_CHECK(hipMemcpy(h.data(), tcnt, tiles * 4, hipMemcpyDeviceToHost));
    std::vector<uint64_t> o(tiles + 1, 0);
    for (uint64_t i = 0; i < tiles; ++i) o[i + 1] = o[i] + h[i];
    HIP_CHECK(hipMemcpy(toff, o.data(), (tiles + 1) * 8, hipMemcpyHostToDevice));
    const double bytes = len + o[tiles] * 8.0;
    t = time_ms(s, 3, [&] {
        extract_kernel<1, false, false><<<dim3((unsigned)tiles), dim3(256), 0, s>>>(
            seq, len, K, 1, nullptr, nullptr, 0, nullptr, 255, out, nullptr, nullptr, toff, nullptr, 0);
    });
    printf("extract write: %.3f ms = %.0f GB/s (%lu k-mers)\n", t, bytes / 1e9 / (t * 1e-3),
           (unsigned long)o[tiles]);
    HIP_CHECK(hipFree(seq));
    HIP_CHECK(hipFree(out));
    HIP_CHECK(hipFree(rows));
}

int main(int argc, char **argv) {
    if (argc > 1 && std::string(argv[1]) == "calib") {
        // one 8-byte-lane copy of 1.2e9 words (9.6 GB read + 9.6 GB written)
        const uint64_t n = 1200000000ull;
        uint64_t *a, *b;
        HIP_CHECK(hipMalloc(&a, n * 8));
        HIP_CHECK(hipMalloc(&b, n * 8));
        HIP_CHECK(hipMemset(a, 1, n * 8));
        copy8_kernel<<<16384, 256>>>(a, b, n);
        HIP_CHECK(hipDeviceSynchronize());
        printf("copy8 bytes read %lu written %lu\n", (unsigned long)(n * 8), (unsigned long)(n * 8));
        return 0;
    }
    const uint64_t R = argc > 1 ? strtoull(argv[1], nullptr, 10) : 373000000ull;
    const unsigned K = 31;
    hipStream_t s;
    HIP_CHECK(hipStreamCreate(&s));
    extract_bench(s, 10000000ull);
    partition_bench(s, 1200000000ull);
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
