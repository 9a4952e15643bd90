// part_bench.hip -- microbenchmark of the K2 level-2 partition pass (the bench's headline pass):
// N 62-bit keys already grouped by their top 9 bits (as the fused K1 leaves them), partitioned by
// the next 9 bits.  Variants: the product kernel (1024- and 512-thread tiles, nontemporal or not),
// a persistent kernel that loads the next tile into registers while writing the current one
// from LDS, and a one-shot copy of the same bytes (the achievable floor).  Every variant's output
// is checked: bucket prefixes nondecreasing and the key sum unchanged.
// Usage: part_bench [n_keys] [reps]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../projects2014-metagenome_amd/csrc/boss_pipeline.hip"

using namespace mtg;

__device__ __forceinline__ uint64_t pb_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// key i: top 9 of 62 bits = i * 512 / n (grouped), the rest random
__global__ void fill_grouped_kernel(Key<1> *k, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t seg = (uint64_t)((unsigned __int128)i * 512 / n);
        k[i].w[0] = (seg << 53) | (pb_mix64(i * 0x9E3779B97F4A7C15ull + 1) >> 11);
    }
}

__global__ void check_kernel(const Key<1> *k, uint64_t n, unsigned shift, unsigned long long *sum, uint32_t *bad) {
    unsigned long long s = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        s += k[i].w[0];
        if (i && (k[i - 1].w[0] >> shift) > (k[i].w[0] >> shift)) atomicOr(bad, 1u);
    }
    atomicAdd(sum, s);
}

__global__ __launch_bounds__(256) void copy_nt_kernel(const ulonglong2 *__restrict__ in, ulonglong2 *__restrict__ out,
                                                      uint64_t n16) {
    const uint64_t base = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    ulonglong2 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint64_t i = base + j * 256;
        if (i < n16) {
            v[j].x = __builtin_nontemporal_load(&in[i].x);
            v[j].y = __builtin_nontemporal_load(&in[i].y);
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint64_t i = base + j * 256;
        if (i < n16) {
            __builtin_nontemporal_store(v[j].x, &out[i].x);
            __builtin_nontemporal_store(v[j].y, &out[i].y);
        }
    }
}

// persistent variant: after a tile is staged in LDS its registers are free, so the next tile's
// loads are issued before the current tile's runs are written
template <bool NT, bool CONTIG = false>
__global__ __launch_bounds__(1024) void part_persist_kernel(const Key<1> *__restrict__ kin, Key<1> *__restrict__ kout,
                                                            uint64_t n, unsigned nbits, unsigned b, unsigned bp,
                                                            unsigned long long *__restrict__ cursor, uint64_t ntiles) {
    constexpr int ITEMS = 16, BLOCK = 1024, TILE = ITEMS * BLOCK, W = 512;
    __shared__ Key<1> s_keys[TILE];
    __shared__ uint32_t s_cnt[W];
    __shared__ uint32_t s_loff[W];
    __shared__ unsigned long long s_gbase[W];
    __shared__ uint32_t s_scan[BLOCK / 64 + 1];
    __shared__ uint32_t s_wb;
    const uint32_t tid = threadIdx.x;
    const unsigned sub = b - bp;
    const uint32_t wsize = min((uint32_t)W, 1u << sub);
    Key<1> k[ITEMS];
    // CONTIG: each workgroup walks its own contiguous slice of tiles (else tiles blockIdx + i * grid)
    const uint64_t per = (ntiles + gridDim.x - 1) / gridDim.x;
    uint64_t t = CONTIG ? blockIdx.x * per : blockIdx.x;
    const uint64_t tend = CONTIG ? min(ntiles, t + per) : ntiles;
    const uint64_t step = CONTIG ? 1 : gridDim.x;
    auto load = [&](uint64_t tile) {
        const uint64_t base = tile * TILE;
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint64_t i = base + (uint64_t)j * BLOCK + tid;
            if (i < n) k[j] = load_key(kin + i, NT);
        }
    };
    if (t < tend) load(t);
    for (; t < tend; t += step) {
        const uint64_t base = t * TILE;
        for (uint32_t i = tid; i < wsize; i += BLOCK) s_cnt[i] = 0;
        if (tid == 0) s_wb = key_prefix(k[0], nbits, bp);
        __syncthreads();
        const uint32_t wbase = s_wb << sub;
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
                }
            }
        }
        __syncthreads();
        const uint32_t cnt = tid < wsize ? s_cnt[tid] : 0;
        uint32_t total;
        const uint32_t off = block_exclusive_sum<BLOCK>(cnt, s_scan, &total);
        if (tid < wsize) {
            s_loff[tid] = off;
            s_gbase[tid] = cnt ? atomicAdd(&cursor[wbase + tid], (unsigned long long)cnt) : 0;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            if (r[j] != 0xFFFFFFFFu) {
                const uint32_t lb = key_prefix(k[j], nbits, b) - wbase;
                s_keys[s_loff[lb] + r[j]] = k[j];
            }
        }
        __syncthreads();
        if (t + step < tend) load(t + step);
        for (uint32_t p = tid; p < total; p += BLOCK) {
            const Key<1> key = s_keys[p];
            const uint32_t lb = key_prefix(key, nbits, b) - wbase;
            store_key(kout + s_gbase[lb] + (p - s_loff[lb]), key, NT);
        }
        __syncthreads();
    }
}

typedef uint64_t u64x2a8 __attribute__((ext_vector_type(2), aligned(8)));

// the product kernel with 16-byte loads (VLD: two adjacent keys per lane) and 16-byte stores
// (VST: a lane writes two consecutive staged keys with one 8-byte-aligned dwordx4 when both are
// in one bucket)
template <bool NT, bool VLD, bool VST>
__global__ __launch_bounds__(1024) void part_vec_kernel(const Key<1> *__restrict__ kin, Key<1> *__restrict__ kout,
                                                        uint64_t n, unsigned nbits, unsigned b, unsigned bp,
                                                        unsigned long long *__restrict__ cursor) {
    constexpr int ITEMS = 16, BLOCK = 1024, TILE = ITEMS * BLOCK, W = 512;
    __shared__ __attribute__((aligned(16))) Key<1> s_keys[TILE];
    __shared__ uint32_t s_cnt[W];
    __shared__ uint32_t s_loff[W];
    __shared__ unsigned long long s_gbase[W];
    __shared__ uint32_t s_scan[BLOCK / 64 + 1];
    const uint32_t tid = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * TILE;
    const unsigned sub = b - bp;
    const uint32_t wsize = min((uint32_t)W, 1u << sub);
    for (uint32_t i = tid; i < wsize; i += BLOCK) s_cnt[i] = 0;
    const uint32_t wbase = key_prefix(kin[base], nbits, bp) << sub;
    __syncthreads();
    Key<1> k[ITEMS];
    bool have[ITEMS];
    if constexpr (VLD) {
#pragma unroll
        for (int j = 0; j < ITEMS / 2; ++j) {
            const uint64_t i = base + 2 * ((uint64_t)j * BLOCK + tid);
            have[2 * j] = i < n;
            have[2 * j + 1] = i + 1 < n;
            if (i + 1 < n) {
                const ulonglong2 *p = (const ulonglong2 *)(kin + i);
                if (NT) {
                    k[2 * j].w[0] = __builtin_nontemporal_load(&p->x);
                    k[2 * j + 1].w[0] = __builtin_nontemporal_load(&p->y);
                } else {
                    const ulonglong2 v = *p;
                    k[2 * j].w[0] = v.x;
                    k[2 * j + 1].w[0] = v.y;
                }
            } else if (i < n) {
                k[2 * j] = kin[i];
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const uint64_t i = base + (uint64_t)j * BLOCK + tid;
            have[j] = i < n;
            if (i < n) k[j] = load_key(kin + i, NT);
        }
    }
    uint32_t r[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        r[j] = 0xFFFFFFFFu;
        if (have[j]) {
            const uint32_t lb = key_prefix(k[j], nbits, b) - wbase;
            if (lb < wsize) {
                r[j] = atomicAdd(&s_cnt[lb], 1u);
            } else {
                const unsigned long long o = atomicAdd(&cursor[lb + wbase], 1ull);
                kout[o] = k[j];
            }
        }
    }
    __syncthreads();
    const uint32_t cnt = tid < wsize ? s_cnt[tid] : 0;
    uint32_t total;
    const uint32_t off = block_exclusive_sum<BLOCK>(cnt, s_scan, &total);
    if (tid < wsize) {
        s_loff[tid] = off;
        s_gbase[tid] = cnt ? atomicAdd(&cursor[wbase + tid], (unsigned long long)cnt) : 0;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        if (r[j] != 0xFFFFFFFFu) {
            const uint32_t lb = key_prefix(k[j], nbits, b) - wbase;
            s_keys[s_loff[lb] + r[j]] = k[j];
        }
    }
    __syncthreads();
    if constexpr (VST) {
        for (uint32_t p = 2 * tid; p < total; p += 2 * BLOCK) {
            if (p + 1 < total) {
                const ulonglong2 v = *(const ulonglong2 *)&s_keys[p];
                const uint32_t l0 = key_prefix(Key<1>::from(v.x), nbits, b) - wbase;
                const uint32_t l1 = key_prefix(Key<1>::from(v.y), nbits, b) - wbase;
                const uint64_t o0 = s_gbase[l0] + (p - s_loff[l0]);
                if (l0 == l1) {
                    u64x2a8 w;
                    w.x = v.x;
                    w.y = v.y;
                    if (NT) __builtin_nontemporal_store(w, (u64x2a8 *)(kout + o0));
                    else *(u64x2a8 *)(kout + o0) = w;
                } else {
                    const uint64_t o1 = s_gbase[l1] + (p + 1 - s_loff[l1]);
                    store_key(kout + o0, Key<1>::from(v.x), NT);
                    store_key(kout + o1, Key<1>::from(v.y), NT);
                }
            } else {
                const Key<1> key = s_keys[p];
                const uint32_t lb = key_prefix(key, nbits, b) - wbase;
                store_key(kout + s_gbase[lb] + (p - s_loff[lb]), key, NT);
            }
        }
    } else {
        for (uint32_t p = tid; p < total; p += BLOCK) {
            const Key<1> key = s_keys[p];
            const uint32_t lb = key_prefix(key, nbits, b) - wbase;
            store_key(kout + s_gbase[lb] + (p - s_loff[lb]), key, NT);
        }
    }
}

// the product kernel staging its tile through LDS in ROUNDS slices of TILE / ROUNDS positions (the
// tile's bucket-ordered positions, so every run except the ones crossing a slice edge is written in
// one piece): 16K-key tiles in 128 / ROUNDS KiB of LDS, two workgroups per CU at ROUNDS >= 2
// XCD: workgroup b runs tile (b % 8) * per + b / 8, so each XCD (dispatch round-robin over 8)
// walks its own contiguous eighth of the tiles and its L2 sees neighbouring runs of a bucket
// XCD 2: chunks of G consecutive tiles dealt round-robin to the XCDs (all XCDs stay in one region)
template <int ROUNDS, int XCD = 0, int G = 32>
__global__ __launch_bounds__(1024) void part_rounds_kernel(const Key<1> *__restrict__ kin, Key<1> *__restrict__ kout,
                                                           uint64_t n, unsigned nbits, unsigned b, unsigned bp,
                                                           unsigned long long *__restrict__ cursor) {
    constexpr int ITEMS = 16, BLOCK = 1024, TILE = ITEMS * BLOCK, W = 512, SLICE = TILE / ROUNDS;
    const uint64_t ntiles = (n + TILE - 1) / TILE;
    const uint64_t per = (ntiles + 7) / 8;
    const uint64_t slot = blockIdx.x / 8, xcd = blockIdx.x % 8;
    const uint64_t tile = XCD == 1 ? xcd * per + slot : XCD == 2 ? ((slot / G) * 8 + xcd) * G + slot % G : blockIdx.x;
    if (tile >= ntiles) return;
    __shared__ Key<1> s_keys[SLICE];
    __shared__ uint32_t s_cnt[W];
    __shared__ uint32_t s_loff[W];
    __shared__ unsigned long long s_gbase[W];
    __shared__ uint32_t s_scan[BLOCK / 64 + 1];
    const uint32_t tid = threadIdx.x;
    const uint64_t base = tile * TILE;
    const unsigned sub = b - bp;
    const uint32_t wsize = min((uint32_t)W, 1u << sub);
    if (tid < wsize) s_cnt[tid] = 0;
    const uint32_t wbase = key_prefix(kin[base], nbits, bp) << sub;
    __syncthreads();
    Key<1> k[ITEMS];
    uint32_t r[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint64_t i = base + (uint64_t)j * BLOCK + tid;
        if (i < n) k[j] = load_key(kin + i, true);
    }
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
            }
        }
    }
    __syncthreads();
    const uint32_t cnt = tid < wsize ? s_cnt[tid] : 0;
    uint32_t total;
    const uint32_t off = block_exclusive_sum<BLOCK>(cnt, s_scan, &total);
    if (tid < wsize) {
        s_loff[tid] = off;
        s_gbase[tid] = cnt ? atomicAdd(&cursor[wbase + tid], (unsigned long long)cnt) : 0;
    }
    __syncthreads();
    // positions become tile-order positions; r[j] = that position (or ~0)
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
        if (r[j] != 0xFFFFFFFFu) r[j] += s_loff[key_prefix(k[j], nbits, b) - wbase];
#pragma unroll
    for (int q = 0; q < ROUNDS; ++q) {
        const uint32_t lo = q * SLICE;
#pragma unroll
        for (int j = 0; j < ITEMS; ++j)
            if (r[j] - lo < (uint32_t)SLICE) s_keys[r[j] - lo] = k[j];
        __syncthreads();
        const uint32_t hi = min(total, lo + SLICE);
        for (uint32_t p = lo + tid; p < hi; p += BLOCK) {
            const Key<1> key = s_keys[p - lo];
            const uint32_t lb = key_prefix(key, nbits, b) - wbase;
            store_key(kout + s_gbase[lb] + (p - s_loff[lb]), key, true);
        }
        if (q + 1 < ROUNDS) __syncthreads();
    }
}

// ---- atomic-free reservation: per-tile counts of the tile's window (the level-1 segment of its
// first key), a column scan per segment, and the partition pass reading its row of offsets
constexpr int PT_TILE = 16384, PT_W = 512;

__global__ __launch_bounds__(512) void tile_hist_kernel(const Key<1> *__restrict__ keys, uint64_t n, unsigned nbits,
                                                        unsigned b, unsigned bp, uint32_t *__restrict__ rows,
                                                        uint32_t *__restrict__ extra, uint32_t *__restrict__ tseg) {
    __shared__ uint32_t s_cnt[PT_W];
    const uint64_t base = (uint64_t)blockIdx.x * PT_TILE;
    const unsigned sub = b - bp;
    s_cnt[threadIdx.x] = 0;
    const uint32_t seg = key_prefix(keys[base], nbits, bp);
    const uint32_t wbase = seg << sub;
    __syncthreads();
    const uint64_t end = min(n, base + PT_TILE);
    auto add = [&](uint64_t x) {
        const uint32_t lb = key_prefix(Key<1>::from(x), nbits, b) - wbase;
        if (lb < PT_W) atomicAdd(&s_cnt[lb], 1u);
        else atomicAdd(&extra[lb + wbase], 1u);
    };
    for (uint64_t i = base + 2 * threadIdx.x; i < end; i += 1024) {
        if (i + 1 < end) {
            const ulonglong2 v = *(const ulonglong2 *)(keys + i);
            add(v.x);
            add(v.y);
        } else {
            add(keys[i].w[0]);
        }
    }
    __syncthreads();
    rows[(uint64_t)blockIdx.x * PT_W + threadIdx.x] = s_cnt[threadIdx.x];
    if (threadIdx.x == 0) tseg[blockIdx.x] = seg;
}

// segment s's tiles are [tfirst[s], tfirst[s + 1]) (tiles are grouped by the segment of their
// first key); thread (s, col): rows[t][col] -> exclusive offset within bucket s*512+col;
// extra[bucket] (out-of-window keys) reserve after the in-window runs: cursor = start + in-window
__global__ __launch_bounds__(512) void tile_scan_kernel(uint32_t *__restrict__ rows, const uint32_t *__restrict__ tseg,
                                                        uint64_t ntiles, unsigned nseg,
                                                        const unsigned long long *__restrict__ bstart,
                                                        unsigned long long *__restrict__ cursor) {
    const uint32_t s = blockIdx.x, col = threadIdx.x;
    // first tile of segment s by binary search over tseg (nondecreasing)
    auto lower = [&](uint32_t v) {
        uint64_t lo = 0, hi = ntiles;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) / 2;
            if (tseg[mid] < v) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    };
    const uint64_t t0 = lower(s), t1 = lower(s + 1);
    uint32_t acc = 0;
    for (uint64_t t = t0; t < t1; ++t) {
        const uint32_t c = rows[t * PT_W + col];
        rows[t * PT_W + col] = acc;
        acc += c;
    }
    const uint64_t g = (uint64_t)s * PT_W + col;
    cursor[g] = bstart[g] + acc;
}

__global__ __launch_bounds__(1024) void part_pre_kernel(const Key<1> *__restrict__ kin, Key<1> *__restrict__ kout,
                                                        uint64_t n, unsigned nbits, unsigned b, unsigned bp,
                                                        const uint32_t *__restrict__ rows,
                                                        const unsigned long long *__restrict__ bstart,
                                                        unsigned long long *__restrict__ cursor) {
    constexpr int ITEMS = 16, BLOCK = 1024, TILE = ITEMS * BLOCK, W = PT_W;
    __shared__ Key<1> s_keys[TILE];
    __shared__ uint32_t s_cnt[W];
    __shared__ uint32_t s_loff[W];
    __shared__ unsigned long long s_gbase[W];
    __shared__ uint32_t s_scan[BLOCK / 64 + 1];
    const uint32_t tid = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * TILE;
    const unsigned sub = b - bp;
    if (tid < W) s_cnt[tid] = 0;
    const uint32_t wbase = key_prefix(kin[base], nbits, bp) << sub;
    // the tile's reserved offsets: no atomics
    unsigned long long gb = 0;
    if (tid < W) gb = bstart[wbase + tid] + rows[(uint64_t)blockIdx.x * W + tid];
    __syncthreads();
    Key<1> k[ITEMS];
    uint32_t r[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const uint64_t i = base + (uint64_t)j * BLOCK + tid;
        if (i < n) k[j] = load_key(kin + i, true);
    }
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        r[j] = 0xFFFFFFFFu;
        if (base + (uint64_t)j * BLOCK + tid < n) {
            const uint32_t lb = key_prefix(k[j], nbits, b) - wbase;
            if (lb < W) {
                r[j] = atomicAdd(&s_cnt[lb], 1u);
            } else {
                const unsigned long long o = atomicAdd(&cursor[lb + wbase], 1ull);
                kout[o] = k[j];
            }
        }
    }
    __syncthreads();
    const uint32_t cnt = tid < W ? s_cnt[tid] : 0;
    uint32_t total;
    const uint32_t off = block_exclusive_sum<BLOCK>(cnt, s_scan, &total);
    if (tid < W) {
        s_loff[tid] = off;
        s_gbase[tid] = gb;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        if (r[j] != 0xFFFFFFFFu) {
            const uint32_t lb = key_prefix(k[j], nbits, b) - wbase;
            s_keys[s_loff[lb] + r[j]] = k[j];
        }
    }
    __syncthreads();
    for (uint32_t p = tid; p < total; p += BLOCK) {
        const Key<1> key = s_keys[p];
        const uint32_t lb = key_prefix(key, nbits, b) - wbase;
        store_key(kout + s_gbase[lb] + (p - s_loff[lb]), key, true);
    }
}

// exclusive scan of h[b0 .. b0 + nb) plus base into cur[b0 ..) (one workgroup of 1024)
__global__ __launch_bounds__(1024) void chunk_scan_kernel(const uint32_t *__restrict__ h, uint32_t b0, uint32_t nb,
                                                          unsigned long long base, unsigned long long *__restrict__ cur) {
    __shared__ unsigned long long s[1024];
    const uint32_t per = (nb + 1023) / 1024, i0 = threadIdx.x * per;
    unsigned long long t = 0;
    for (uint32_t j = 0; j < per && i0 + j < nb; ++j) t += h[b0 + i0 + j];
    s[threadIdx.x] = t;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        const unsigned long long v = threadIdx.x >= off ? s[threadIdx.x - off] : 0;
        __syncthreads();
        s[threadIdx.x] += v;
        __syncthreads();
    }
    unsigned long long acc = base + s[threadIdx.x] - t;
    for (uint32_t j = 0; j < per && i0 + j < nb; ++j) {
        cur[b0 + i0 + j] = acc;
        acc += h[b0 + i0 + j];
    }
}

// level-2 histogram by one global atomic per key (the cost of counting inside K1 pass B)
__global__ __launch_bounds__(256) void atomic_hist_kernel(const Key<1> *__restrict__ k, uint64_t n, uint32_t *__restrict__ h) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 4;
    for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
        const ulonglong2 a = *(const ulonglong2 *)(k + i), b = *(const ulonglong2 *)(k + i + 2);
        atomicAdd(&h[a.x >> 44], 1u);
        atomicAdd(&h[a.y >> 44], 1u);
        atomicAdd(&h[b.x >> 44], 1u);
        atomicAdd(&h[b.y >> 44], 1u);
    }
}

int main(int argc, char **argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1200000000ull;
    const int reps = argc > 2 ? atoi(argv[2]) : 3;
    hipStream_t s;
    HIP_CHECK(hipStreamCreate(&s));
    Key<1> *a, *o;
    HIP_CHECK(hipMalloc(&a, n * 8));
    HIP_CHECK(hipMalloc(&o, n * 8));
    const unsigned nbits = 62, bp = 9;
    uint32_t *h;
    unsigned long long *cur, *sum;
    uint32_t *bad;
    HIP_CHECK(hipMalloc(&h, (1u << 18) * 4));
    HIP_CHECK(hipMalloc(&cur, (1u << 18) * 8));
    HIP_CHECK(hipMalloc(&sum, 8));
    HIP_CHECK(hipMalloc(&bad, 4));
    fill_grouped_kernel<<<8192, 256, 0, s>>>(a, n);
    HIP_CHECK(hipMemsetAsync(sum, 0, 8, s));
    check_kernel<<<8192, 256, 0, s>>>(a, n, 62, sum, bad);
    unsigned long long want = 0;
    HIP_CHECK(hipMemcpyAsync(&want, sum, 8, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    hipEvent_t e0, e1;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    const double gb = 2.0 * n * 8 / 1e9;
    int cus = 0;
    HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));

    // cursors of the level-2 buckets (b bits) from a histogram + host scan
    auto set_cursors = [&](unsigned b) {
        const uint64_t nb = 1ull << b;
        HIP_CHECK(hipMemsetAsync(h, 0, nb * 4, s));
        msd_hist_kernel<1><<<dim3((unsigned)ceil_div(n, MsdTraits<1>::TILE)), dim3(MSD_BLOCK), 0, s>>>(a, n, nbits, b, bp, h);
        std::vector<uint32_t> hh(nb);
        std::vector<unsigned long long> cc(nb);
        HIP_CHECK(hipMemcpyAsync(hh.data(), h, nb * 4, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        unsigned long long acc = 0;
        for (uint64_t i = 0; i < nb; ++i) {
            cc[i] = acc;
            acc += hh[i];
        }
        HIP_CHECK(hipMemcpyAsync(cur, cc.data(), nb * 8, hipMemcpyHostToDevice, s));
    };
    auto run = [&](const char *name, unsigned b, auto launch) {
        double best = 1e30, tot = 0;
        for (int r = 0; r < reps; ++r) {
            if (b) set_cursors(b);
            HIP_CHECK(hipEventRecord(e0, s));
            launch();
            HIP_CHECK(hipGetLastError());
            HIP_CHECK(hipEventRecord(e1, s));
            HIP_CHECK(hipEventSynchronize(e1));
            float ms;
            HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
            best = std::min(best, (double)ms);
            tot += ms;
        }
        uint32_t bd = 0;
        unsigned long long got = 0;
        HIP_CHECK(hipMemsetAsync(sum, 0, 8, s));
        HIP_CHECK(hipMemsetAsync(bad, 0, 4, s));
        check_kernel<<<8192, 256, 0, s>>>(o, n, b ? nbits - b : 62, sum, bad);
        HIP_CHECK(hipMemcpyAsync(&got, sum, 8, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipMemcpyAsync(&bd, bad, 4, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        printf("%-34s best %.3f ms avg %.3f ms  %5.0f GB/s  %s\n", name, best, tot / reps, gb / best * 1e3,
               (got == want && !bd) ? "ok" : "WRONG");
        fflush(stdout);
    };

    run("copy (one-shot nt 16B)", 0, [&] {
        copy_nt_kernel<<<dim3((unsigned)ceil_div(n / 2, 1024)), dim3(256), 0, s>>>((const ulonglong2 *)a, (ulonglong2 *)o, n / 2);
    });
    if (argc > 4) run("product 1024 nt (9-bit)", 18, [&] {
        msd_partition_kernel<1, false, 1024, true><<<dim3((unsigned)xcd_grid(ceil_div(n, 16384))), dim3(1024), 0, s>>>(
            a, o, nullptr, nullptr, n, nbits, 18, bp, cur);
    });
    run("product 1024 (9-bit)", 18, [&] {
        msd_partition_kernel<1, false, 1024, false><<<dim3((unsigned)xcd_grid(ceil_div(n, 16384))), dim3(1024), 0, s>>>(
            a, o, nullptr, nullptr, n, nbits, 18, bp, cur);
    });
    run("product 512 nt (9-bit, 8K tiles)", 18, [&] {
        msd_partition_kernel<1, false, 512, true><<<dim3((unsigned)xcd_grid(ceil_div(n, 8192))), dim3(512), 0, s>>>(
            a, o, nullptr, nullptr, n, nbits, 18, bp, cur);
    });
    run("product 1024 nt (8-bit)", 17, [&] {
        msd_partition_kernel<1, false, 1024, true><<<dim3((unsigned)xcd_grid(ceil_div(n, 16384))), dim3(1024), 0, s>>>(
            a, o, nullptr, nullptr, n, nbits, 17, bp, cur);
    });
    const unsigned g16 = (unsigned)ceil_div(n, 16384);
    run("product 256 nt (9-bit, 4K tiles)", 18, [&] {
        msd_partition_kernel<1, false, 256, true><<<dim3((unsigned)xcd_grid(ceil_div(n, 4096))), dim3(256), 0, s>>>(
            a, o, nullptr, nullptr, n, nbits, 18, bp, cur);
    });
    run("product 512 (9-bit, 8K tiles, no nt)", 18, [&] {
        msd_partition_kernel<1, false, 512, false><<<dim3((unsigned)xcd_grid(ceil_div(n, 8192))), dim3(512), 0, s>>>(
            a, o, nullptr, nullptr, n, nbits, 18, bp, cur);
    });
    run("atomic level-2 hist (1 atomic/key)", 0, [&] {
        HIP_CHECK(hipMemsetAsync(h, 0, (1u << 18) * 4, s));
        atomic_hist_kernel<<<dim3(8192), dim3(256), 0, s>>>(a, n, h);
        copy_nt_kernel<<<1, 256, 0, s>>>((const ulonglong2 *)a, (ulonglong2 *)o, 0);
    });
    run("msd_hist level 2 (product)", 0, [&] {
        HIP_CHECK(hipMemsetAsync(h, 0, (1u << 18) * 4, s));
        msd_hist_kernel<1><<<dim3((unsigned)ceil_div(n, MsdTraits<1>::TILE)), dim3(MSD_BLOCK), 0, s>>>(a, n, nbits, 18, bp, h);
    });
    if (argc > 4)
    // level 2 chunk by chunk (C level-1 buckets each): histogram, scan, partition of the same
    // chunk back to back, so the partition re-reads the chunk from the MALL instead of HBM
    for (unsigned C : {2u, 4u, 8u, 16u, 64u}) {
        char nm[64];
        snprintf(nm, sizeof nm, "chunked hist+part C=%u", C);
        run(nm, 0, [&] {
            HIP_CHECK(hipMemsetAsync(h, 0, (1u << 18) * 4, s));
            for (unsigned b = 0; b < 512; b += C) {
                const uint64_t lo = (uint64_t)(((unsigned __int128)b * n + 511) / 512);
                const uint64_t hi = std::min<uint64_t>(n, (uint64_t)(((unsigned __int128)(b + C) * n + 511) / 512));
                const uint64_t m = hi - lo;
                msd_hist_kernel<1><<<dim3((unsigned)ceil_div(m, MsdTraits<1>::TILE)), dim3(MSD_BLOCK), 0, s>>>(a + lo, m, nbits, 18, bp, h);
                chunk_scan_kernel<<<1, 1024, 0, s>>>(h, b << 9, C << 9, lo, cur);
                msd_partition_kernel<1, false, 512, false><<<dim3((unsigned)xcd_grid(ceil_div(m, 8192))), dim3(512), 0, s>>>(
                    a + lo, o, nullptr, nullptr, m, nbits, 18, bp, cur);
            }
        });
        // check with the 18-bit prefix order
        uint32_t bd = 0;
        HIP_CHECK(hipMemsetAsync(bad, 0, 4, s));
        HIP_CHECK(hipMemsetAsync(sum, 0, 8, s));
        check_kernel<<<8192, 256, 0, s>>>(o, n, nbits - 18, sum, bad);
        HIP_CHECK(hipMemcpyAsync(&bd, bad, 4, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        printf("   18-bit order: %s\n", bd ? "WRONG" : "ok");
    }
    run("global hist + part 512 (product)", 0, [&] {
        HIP_CHECK(hipMemsetAsync(h, 0, (1u << 18) * 4, s));
        msd_hist_kernel<1><<<dim3((unsigned)ceil_div(n, MsdTraits<1>::TILE)), dim3(MSD_BLOCK), 0, s>>>(a, n, nbits, 18, bp, h);
        chunk_scan_kernel<<<1, 1024, 0, s>>>(h, 0, 1u << 18, 0, cur);
        msd_partition_kernel<1, false, 512, false><<<dim3((unsigned)xcd_grid(ceil_div(n, 8192))), dim3(512), 0, s>>>(
            a, o, nullptr, nullptr, n, nbits, 18, bp, cur);
    });
    if (argc > 3) {
    {  // atomic-free reservation
        const uint64_t nt = ceil_div(n, PT_TILE);
        uint32_t *rows, *tseg, *extra;
        unsigned long long *bst;
        HIP_CHECK(hipMalloc(&rows, nt * PT_W * 4));
        HIP_CHECK(hipMalloc(&tseg, nt * 4));
        HIP_CHECK(hipMalloc(&extra, (1u << 18) * 4));
        HIP_CHECK(hipMalloc(&bst, (1u << 18) * 8));
        set_cursors(18);
        HIP_CHECK(hipMemcpyAsync(bst, cur, (1u << 18) * 8, hipMemcpyDeviceToDevice, s));
        hipEvent_t e2, e3;
        HIP_CHECK(hipEventCreate(&e2));
        HIP_CHECK(hipEventCreate(&e3));
        for (int r = 0; r < reps; ++r) {
            HIP_CHECK(hipEventRecord(e0, s));
            tile_hist_kernel<<<dim3((unsigned)nt), dim3(512), 0, s>>>(a, n, nbits, 18, bp, rows, extra, tseg);
            HIP_CHECK(hipEventRecord(e2, s));
            tile_scan_kernel<<<dim3(512), dim3(PT_W), 0, s>>>(rows, tseg, nt, 512, bst, cur);
            HIP_CHECK(hipEventRecord(e3, s));
            part_pre_kernel<<<dim3((unsigned)nt), dim3(1024), 0, s>>>(a, o, n, nbits, 18, bp, rows, bst, cur);
            HIP_CHECK(hipEventRecord(e1, s));
            HIP_CHECK(hipEventSynchronize(e1));
            float m0, m1, m2;
            HIP_CHECK(hipEventElapsedTime(&m0, e0, e2));
            HIP_CHECK(hipEventElapsedTime(&m1, e2, e3));
            HIP_CHECK(hipEventElapsedTime(&m2, e3, e1));
            printf("pre-reserved: tile hist %.3f  scan %.3f  partition %.3f ms (%5.0f GB/s)\n", m0, m1, m2,
                   gb / m2 * 1e3);
        }
        uint32_t bd = 0;
        unsigned long long got = 0;
        HIP_CHECK(hipMemsetAsync(sum, 0, 8, s));
        HIP_CHECK(hipMemsetAsync(bad, 0, 4, s));
        check_kernel<<<8192, 256, 0, s>>>(o, n, nbits - 18, sum, bad);
        HIP_CHECK(hipMemcpyAsync(&got, sum, 8, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipMemcpyAsync(&bd, bad, 4, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        printf("pre-reserved: %s\n", (got == want && !bd) ? "ok" : "WRONG");
        // the product's histogram pass for comparison
        HIP_CHECK(hipEventRecord(e0, s));
        msd_hist_kernel<1><<<dim3((unsigned)ceil_div(n, MsdTraits<1>::TILE)), dim3(MSD_BLOCK), 0, s>>>(a, n, nbits, 18, bp, h);
        HIP_CHECK(hipEventRecord(e1, s));
        HIP_CHECK(hipEventSynchronize(e1));
        float mh;
        HIP_CHECK(hipEventElapsedTime(&mh, e0, e1));
        printf("product msd_hist level 2: %.3f ms\n", mh);
        fflush(stdout);
    }
    for (int per : {1, 2}) {
        char nm[64];
        snprintf(nm, sizeof nm, "persistent nt grid=%d*CUs", per);
        run(nm, 18, [&] {
            part_persist_kernel<true><<<dim3(per * cus), dim3(1024), 0, s>>>(a, o, n, nbits, 18, bp, cur,
                                                                             ceil_div(n, 16384));
        });
    }
    run("persistent contiguous grid=CUs nt", 18, [&] {
        part_persist_kernel<true, true><<<dim3(cus), dim3(1024), 0, s>>>(a, o, n, nbits, 18, bp, cur, ceil_div(n, 16384));
    });
    run("persistent grid=CUs (no nt)", 18, [&] {
        part_persist_kernel<false><<<dim3(cus), dim3(1024), 0, s>>>(a, o, n, nbits, 18, bp, cur, ceil_div(n, 16384));
    });
    }
    return 0;
}
