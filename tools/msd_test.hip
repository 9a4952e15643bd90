// msd_test.hip -- randomized check of msd_sort_unique / radix_sort against std::sort + unique
// on the host, over small and medium sizes, several significant-bit widths and dup factors.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#include "../projects2014-metagenome_amd/csrc/boss_pipeline.hip"

using namespace mtg;

template <int L, bool COUNTED>
static int check(Ctx &c, uint64_t n, unsigned nbits, int dupf, uint32_t seed, bool skew,
                 double hint_mult = 1.0, bool distinct = false) {
    std::mt19937_64 rng(seed);
    const uint64_t m = std::max<uint64_t>(1, n / dupf);
    std::vector<Key<L>> base(m);
    for (auto &k : base) {
        k = Key<L>::zero();
        for (int i = 0; i < L; ++i) k.w[i] = rng();
        k = k & Key<L>::lowmask(nbits);
        if (skew) {  // canonical-like: min of two random words -> denser low prefixes
            Key<L> k2 = Key<L>::zero();
            for (int i = 0; i < L; ++i) k2.w[i] = rng();
            k2 = k2 & Key<L>::lowmask(nbits);
            if (k2 < k) k = k2;
        }
    }
    std::vector<Key<L>> h(n);
    std::vector<uint32_t> hv(n);
    if (distinct) {  // a shuffled duplicate-free input (the rc sort's contract)
        std::sort(base.begin(), base.end(), [](auto &x, auto &y) { return x < y; });
        base.erase(std::unique(base.begin(), base.end(), [](auto &x, auto &y) { return x == y; }),
                   base.end());
        std::shuffle(base.begin(), base.end(), rng);
        n = base.size();
        h.assign(base.begin(), base.end());
        hv.resize(n);
        for (uint64_t i = 0; i < n; ++i) hv[i] = (uint32_t)(rng() % 300);
    } else {
        for (uint64_t i = 0; i < n; ++i) {
            h[i] = base[rng() % m];
            hv[i] = (uint32_t)(rng() % 300);
        }
    }
    // expected
    std::vector<std::pair<Key<L>, uint64_t>> e;
    for (uint64_t i = 0; i < n; ++i) e.push_back({h[i], hv[i]});
    std::sort(e.begin(), e.end(), [](auto &a, auto &b) { return a.first < b.first; });
    std::vector<Key<L>> ek;
    std::vector<uint32_t> ec;
    const uint32_t cmax = 65535;
    for (auto &p : e) {
        if (!ek.empty() && ek.back() == p.first) {
            uint64_t s = (uint64_t)ec.back() + p.second;
            ec.back() = (uint32_t)std::min<uint64_t>(s, cmax);
        } else {
            ek.push_back(p.first);
            ec.push_back((uint32_t)std::min<uint64_t>(p.second, cmax));
        }
    }
    Key<L> *a, *b;
    uint32_t *va, *vb;
    HIP_CHECK(hipMalloc(&a, n * sizeof(Key<L>) + 64));
    HIP_CHECK(hipMalloc(&b, n * sizeof(Key<L>) + 64));
    HIP_CHECK(hipMalloc(&va, n * 4 + 64));
    HIP_CHECK(hipMalloc(&vb, n * 4 + 64));
    HIP_CHECK(hipMemcpy(a, h.data(), n * sizeof(Key<L>), hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(va, hv.data(), n * 4, hipMemcpyHostToDevice));
    Key<L> *ka = a, *kb = b;
    uint32_t *pa = va, *pb = vb;
    uint64_t u = msd_sort_unique<L, COUNTED>(c, &ka, &kb, &pa, &pb, n, nbits, cmax, dupf * hint_mult,
                                             nullptr, distinct);
    std::vector<Key<L>> got(u);
    std::vector<uint32_t> gc(u);
    HIP_CHECK(hipMemcpy(got.data(), ka, u * sizeof(Key<L>), hipMemcpyDeviceToHost));
    if (COUNTED) HIP_CHECK(hipMemcpy(gc.data(), pa, u * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    if (u != ek.size()) bad = 1;
    for (uint64_t i = 0; !bad && i < u; ++i) {
        if (got[i] != ek[i]) bad = 2;
        if (COUNTED && gc[i] != ec[i]) bad = 3;
    }
    if (bad) {
        printf("FAIL L=%d counted=%d n=%lu nbits=%u dup=%d seed=%u: code %d (u=%lu want %zu)\n", L,
               COUNTED, (unsigned long)n, nbits, dupf, seed, bad, (unsigned long)u, ek.size());
        for (uint64_t i = 0; i < std::min<uint64_t>(u, 12); ++i)
            printf("   %lu: got %016lx want %016lx\n", (unsigned long)i, (unsigned long)got[i].w[0],
                   (unsigned long)(i < ek.size() ? ek[i].w[0] : 0));
    }
    hipFree(a); hipFree(b); hipFree(va); hipFree(vb);
    return bad ? 1 : 0;
}

int main() {
    Ctx c;
    HIP_CHECK(hipStreamCreate(&c.stream));
    HIP_CHECK(hipMalloc(&c.small, sizeof(Small)));
    int fails = 0, runs = 0;
    for (uint64_t n : {1ull, 2ull, 5ull, 20ull, 100ull, 1000ull, 5000ull, 20000ull, 300000ull, 3000000ull})
        for (unsigned nbits : {4u, 8u, 12u, 20u, 40u, 62u})
            for (int dupf : {1, 3, 20}) {
                fails += check<1, false>(c, n, nbits, dupf, 1 + runs, false); ++runs;
                fails += check<1, true>(c, n, nbits, dupf, 1 + runs, false); ++runs;
            }
    for (uint64_t n : {1ull, 7ull, 1000ull, 50000ull, 1000000ull})
        for (unsigned nbits : {66u, 93u, 126u})
            for (int dupf : {1, 5}) {
                fails += check<2, false>(c, n, nbits, dupf, 1 + runs, false); ++runs;
                fails += check<2, true>(c, n, nbits, dupf, 1 + runs, false); ++runs;
            }
    for (uint64_t n : {3ull, 1000ull, 200000ull})
        for (unsigned nbits : {130u, 189u, 255u}) {
            fails += check<4, false>(c, n, nbits, 2, 1 + runs, false); ++runs;
        }
    // wrong (too optimistic) duplication hints on skewed keys: overflow -> slices / fallback
    for (uint64_t n : {200000ull, 3000000ull, 20000000ull})
        for (double hint : {4.0, 16.0, 64.0}) {
            fails += check<1, false>(c, n, 62, 1, 1 + runs, true, hint); ++runs;
            fails += check<1, true>(c, n, 62, 2, 1 + runs, true, hint); ++runs;
            fails += check<2, false>(c, n / 4, 93, 1, 1 + runs, true, hint); ++runs;
        }
    // duplicate-free inputs through the local pass without hash tables (rc sort), incl. skew
    for (uint64_t n : {1ull, 50ull, 5000ull, 300000ull, 3000000ull, 20000000ull})
        for (unsigned nbits : {20u, 40u, 62u}) {
            fails += check<1, false>(c, n, nbits, 1, 1 + runs, runs & 1, 1.0, true); ++runs;
            fails += check<1, true>(c, n, nbits, 1, 1 + runs, runs & 1, 1.0, true); ++runs;
        }
    for (uint64_t n : {1000ull, 1000000ull})
        for (unsigned nbits : {66u, 126u}) {
            fails += check<2, false>(c, n, nbits, 1, 1 + runs, false, 1.0, true); ++runs;
        }
    printf("msd_test: %d / %d failed\n", fails, runs);
    return fails ? 1 : 0;
}
