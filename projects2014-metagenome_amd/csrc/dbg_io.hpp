// dbg_io.hpp -- the graph files `metagraph build` writes after construction (host code):
//   <base>.dbg          DBGSuccinct::serialize (dbg_succinct.cpp:754-770): BOSS::serialize
//                       (boss.cpp:245-262: F, k, state, W, last), the graph mode, the suffix-range
//                       index (boss.cpp:330-337, built as index_suffix_ranges, :3091-3161);
//   <base>.edgemask     the valid-edge mask of --mask-dummy (dbg_succinct.cpp:839-870:
//                       mark_all_dummy_edges flipped, boss.cpp:1681-1691);
//   <base>.dbg.weights  the chunk's weight vector (node_weights.cpp:55-68 renames the chunk's
//                       weights buffer), written by chunk_io.py in the int_vector layout.
// The BOSS navigation the index and the mask need (rank_W, rank_last, select_last, fwd,
// tighten_range: boss.hpp:655-666, boss.cpp:381-385, 521-536, 586-597) runs on the chunk arrays.
//
// Byte layout.  The reference's own framing: numbers are serialize_number (8-byte big-endian,
// common/serialization.cpp:38-46), F is serialize_number_vector_raw (count + values, :84-90), the
// suffix index is a raw native-endian pair<u64,u64> array.  The sdsl-lite containers (wt_huff<> for
// W, bit_vector_stat for last, bit_vector_small for the mask, int_vector<> for the weights) are
// written field by field as sdsl-lite 2.x serializes them (sdsl_io.hpp).  sdsl-lite is an empty
// submodule of the reference snapshot and no .dbg file exists in its tests, so the bytes are a
// restatement of the library's published layout, unpinned by a golden file; read_dbg parses the
// same layout back and checks the rank supports it can recompute.
#pragma once

#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <fstream>
#include <queue>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "sdsl_io.hpp"

namespace mtg {
namespace dbgio {

// ---------------------------------------------------------------------------------- framing

using sdslio::get_be;
using sdslio::get_raw;
using sdslio::put_be;
using sdslio::put_raw;
using sdslio::bit;

// ----------------------------------------------------------------------- BOSS navigation

struct BossNav {
    const uint8_t *W;
    const uint64_t *last;
    uint64_t n;  // rows incl. row 0
    uint64_t F[5];
    uint64_t k;
    uint64_t NF[5];
    std::vector<uint64_t> last_rank;     // ones in last before word w
    std::vector<uint64_t> wrank[5];      // W == c (exact, no minus) before each 64-row block

    BossNav(const uint8_t *W_, const uint64_t *last_, uint64_t n_, const uint64_t *F_, uint64_t k_)
        : W(W_), last(last_), n(n_), k(k_) {
        for (int c = 0; c < 5; ++c) F[c] = F_[c];
        const uint64_t nw = (n + 63) / 64;
        last_rank.assign(nw + 1, 0);
        for (uint64_t i = 0; i < nw; ++i) last_rank[i + 1] = last_rank[i] + __builtin_popcountll(last[i]);
        for (int c = 0; c < 5; ++c) wrank[c].assign(nw + 1, 0);
        for (uint64_t b = 0; b < nw; ++b) {
            uint64_t cnt[5] = {0, 0, 0, 0, 0};
            for (uint64_t i = 64 * b; i < std::min(n, 64 * b + 64); ++i)
                if (W[i] < 5) ++cnt[W[i]];
            for (int c = 0; c < 5; ++c) wrank[c][b + 1] = wrank[c][b] + cnt[c];
        }
        for (int c = 0; c < 5; ++c) NF[c] = rank_last(F[c]);  // recompute_NF
    }
    // #{p in [1, i] : last[p]} (boss.cpp:521-525; last[0] = 0)
    uint64_t rank_last(uint64_t i) const {
        if (i == 0) return 0;
        const uint64_t e = i + 1, w = e >> 6, b = e & 63;
        return last_rank[w] + (b ? __builtin_popcountll(last[w] & ((1ull << b) - 1)) : 0);
    }
    // position of the j-th set bit of last (boss.cpp:532-536)
    uint64_t select_last(uint64_t j) const {
        if (j == 0) return 0;
        uint64_t lo = 0, hi = last_rank.size() - 1;  // last word with last_rank[w] < j
        while (hi - lo > 1) {
            const uint64_t mid = (lo + hi) / 2;
            if (last_rank[mid] < j) lo = mid; else hi = mid;
        }
        uint64_t x = last[lo], r = j - last_rank[lo];
        for (uint64_t q = 1; q < r; ++q) x &= x - 1;
        return 64 * lo + __builtin_ctzll(x);
    }
    // #{p in [1, i] : W[p] == c} (boss.cpp:381-385)
    uint64_t rank_W(uint64_t i, uint8_t c) const {
        if (i == 0) return 0;
        const uint64_t e = i + 1, b = e >> 6;
        uint64_t r = wrank[c][b];
        for (uint64_t p = 64 * b; p < e; ++p) r += W[p] == c;
        return r - (c == 0 ? 1 : 0);
    }
    // boss.hpp:655-666
    bool tighten_range(uint64_t *rl, uint64_t *ru, uint8_t s) const {
        const uint64_t rk_rl = rank_W(*rl - 1, s) + 1;
        const uint64_t rk_ru = rank_W(*ru, s);
        if (rk_rl > rk_ru) return false;
        *rl = select_last(NF[s] + rk_rl - 1) + 1;
        *ru = select_last(NF[s] + rk_ru);
        return true;
    }
    // boss.cpp:586-597
    uint64_t fwd(uint64_t i, uint8_t c) const { return select_last(NF[c] + rank_W(i, c)); }
};

// BOSS::index_suffix_ranges (boss.cpp:3091-3161)
inline std::vector<std::pair<uint64_t, uint64_t>> index_suffix_ranges(const BossNav &b, uint64_t L) {
    std::vector<std::pair<uint64_t, uint64_t>> out;
    if (L == 0) return out;
    struct R {
        uint64_t idx, rl, ru;
    };
    std::vector<R> ranges{{0, 1, b.n - 1}};
    uint64_t num = 1;
    for (uint64_t len = 1; len < L; ++len) {
        std::vector<R> nx;
        nx.reserve(ranges.size() * 4);
        for (const R &r : ranges)
            for (uint8_t c = 1; c < 5; ++c) {
                uint64_t rl = r.rl, ru = r.ru;
                if (!b.tighten_range(&rl, &ru, c)) continue;
                nx.push_back({num * (c - 1) + r.idx, rl, ru});
            }
        ranges.swap(nx);
        num *= 4;
    }
    out.assign(num * 4, {b.n, 0});
    for (const R &r : ranges)
        for (uint8_t c = 1; c < 5; ++c) {
            uint64_t rl = r.rl, ru = r.ru;
            if (!b.tighten_range(&rl, &ru, c)) continue;
            out[num * (c - 1) + r.idx] = {rl, ru};
        }
    for (size_t i = 1; i < out.size(); ++i)
        if (!out[i].second) {
            out[i].second = out[i - 1].second;
            out[i].first = out[i - 1].second + 1;
        }
    return out;
}

// mark_all_dummy_edges (boss.cpp:1681-1691): the source-dummy tree from the main dummy node down to
// depth k - 1 (every node there starts with $), the sink dummies (W == $, from row 2), row 0.
// Returns the mask of VALID edges (the flipped mask DBGSuccinct keeps, dbg_succinct.cpp:839-870).
inline std::vector<uint64_t> valid_edges(const BossNav &b) {
    const uint64_t nw = (b.n + 63) / 64;
    std::vector<uint64_t> dummy(nw, 0);
    auto set = [&](uint64_t i) { dummy[i >> 6] |= 1ull << (i & 63); };
    set(0);
    if (b.n > 1) {
        std::vector<uint64_t> level{b.select_last(1)};  // last edge of the main dummy node
        for (uint64_t depth = 0; depth < b.k && !level.empty(); ++depth) {
            std::vector<uint64_t> next;
            for (uint64_t last_edge : level) {
                const uint64_t node = b.rank_last(last_edge);
                const uint64_t first = b.select_last(node - 1) + 1;
                for (uint64_t i = first; i <= last_edge; ++i) {
                    set(i);
                    const uint8_t c = b.W[i];
                    if (c >= 1 && c <= 4 && depth + 1 < b.k) next.push_back(b.fwd(i, c));
                }
            }
            level.swap(next);
        }
    }
    for (uint64_t i = 2; i < b.n; ++i)  // mark_sink_dummy_edges (boss.cpp:1659-1679)
        if (b.W[i] == 0) set(i);
    for (uint64_t w = 0; w < nw; ++w) dummy[w] = ~dummy[w];
    if (b.n % 64) dummy[nw - 1] &= (1ull << (b.n % 64)) - 1;
    return dummy;
}

// `concatenate --clear-dummy` (cli/build.cpp:400-405): DBGSuccinct::mask_dummy_kmers(with_pruning)
// (dbg_succinct.cpp:839-870) = BOSS::prune_and_mark_all_dummy_edges (boss.cpp:1693-1703):
//   erase_redundant_dummy_edges (:1609-1650) -- traverse the source-dummy tree (traverse_dummy_edges,
//     :1443-1597; the parallel split at depth min(6, k/2) visits the same tree) and mark a dummy edge
//     redundant when no path below it reaches a depth-k edge that is the single incoming edge of its
//     (real) target node (is_single_incoming, :725-738); erase those edges (erase_edges, :1342-1403:
//     `last` moves to the previous kept edge of the node, a "minus" W whose first occurrence was
//     erased loses its minus, F counts the kept rows);
//   then the mask of the remaining source dummies plus the sinks (W == $) and row 0, flipped.
struct Pruned {
    std::vector<uint8_t> W;
    std::vector<uint64_t> last;   // packed
    uint64_t n = 0;
    uint64_t F[5] = {0, 0, 0, 0, 0};
    std::vector<uint64_t> valid;  // packed, over the pruned rows
    uint64_t n_erased = 0;
};

inline Pruned prune_dummy_edges(const BossNav &b) {
    const uint64_t n = b.n, nw = (n + 63) / 64;
    std::vector<uint64_t> redundant(nw, 0), source(nw, 0);
    auto setb = [](std::vector<uint64_t> &v, uint64_t i) { v[i >> 6] |= 1ull << (i & 63); };
    auto getb = [](const std::vector<uint64_t> &v, uint64_t i) { return (v[i >> 6] >> (i & 63)) & 1; };
    if (n > 1) setb(source, 1);
    if (n > 2 && !bit(b.last, 1)) {
        // single[i]: edge i is the only edge into its target -- the next W in {c, c + 5} after i
        // is not the minus c + 5 (is_single_incoming via succ_W, boss.cpp:725-738)
        std::vector<uint64_t> single(nw, 0);
        uint8_t next_kind[5] = {0, 0, 0, 0, 0};  // 0 none, 1 plain, 2 minus
        for (uint64_t i = n; i-- > 1;) {
            const uint8_t w = b.W[i];
            const uint8_t c = w % 5;
            if (w >= 1 && w <= 4 && next_kind[c] != 2) setb(single, i);
            if (c) next_kind[c] = w > 5 ? 2 : 1;
        }
        const uint64_t K = b.k;  // check depth: the depth-k edges enter real nodes
        // depth-first over the tree; returns whether the edge is needed (not redundant)
        struct Frame {
            uint64_t first, cur;  // children rows [first, last] of the current node, cur = next child
            uint64_t last;
            bool any;
        };
        auto visit = [&](uint64_t root) {
            // iterative DFS so deep trees (k up to 84) and wide ones need no recursion limits
            std::vector<std::pair<uint64_t, Frame>> st;  // (edge, its children frame)
            auto open = [&](uint64_t e, uint64_t depth) -> int {
                // returns 1 / 0 when e is an end edge (needed / redundant), -1 when it has children
                setb(source, e);
                const uint8_t c = b.W[e] % 5;
                if (depth == K || c == 0) return (c == 0 || getb(single, e)) ? 1 : 0;
                const uint64_t le = b.fwd(e, c);
                const uint64_t node = b.rank_last(le);
                const uint64_t fe = b.select_last(node - 1) + 1;
                st.push_back({e, Frame{fe, fe, le, false}});
                return -1;
            };
            int r = open(root, 1);
            if (r >= 0) {
                if (!r) setb(redundant, root);
                return;
            }
            while (!st.empty()) {
                const size_t top = st.size() - 1;  // st[0] holds the root, at depth 1
                if (st[top].second.cur <= st[top].second.last) {
                    const uint64_t child = st[top].second.cur++;
                    const int rc = open(child, top + 2);  // may push the child's frame
                    if (rc == 1) st[top].second.any = true;
                    else if (rc == 0) setb(redundant, child);
                    continue;
                }
                const uint64_t e = st[top].first;
                const bool needed = st[top].second.any;
                st.pop_back();
                if (!needed) setb(redundant, e);
                else if (!st.empty()) st.back().second.any = true;
            }
        };
        for (uint64_t root = 2; root < n; ++root) {
            visit(root);
            if (bit(b.last, root)) break;
        }
    }
    Pruned out;
    uint64_t erased = 0;
    for (uint64_t w = 0; w < nw; ++w) erased += __builtin_popcountll(redundant[w]);
    out.n_erased = erased;
    const uint64_t m = n - erased, mw = (m + 63) / 64;
    out.n = m;
    out.W.resize(m);
    out.last.assign(std::max<uint64_t>(mw, 1), 0);
    std::vector<uint64_t> src(std::max<uint64_t>(mw, 1), 0);
    bool first_removed[5] = {false, false, false, false, false};
    uint64_t o = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t c = b.W[i];
        const bool li = bit(b.last, i);
        if (getb(redundant, i)) {
            if (c < 5) first_removed[c] = true;
            if (li && o > 1 && !((out.last[(o - 1) >> 6] >> ((o - 1) & 63)) & 1))
                out.last[(o - 1) >> 6] |= 1ull << ((o - 1) & 63);
            continue;
        }
        out.W[o] = (c > 5 && first_removed[c % 5]) ? (uint8_t)(c % 5) : c;
        first_removed[c % 5] = false;
        if (li) out.last[o >> 6] |= 1ull << (o & 63);
        if (getb(source, i)) src[o >> 6] |= 1ull << (o & 63);
        ++o;
    }
    // F: the kept rows up to each old boundary
    uint64_t F[5];
    for (int c = 0; c < 5; ++c) F[c] = b.F[c];
    {
        int c = 0;
        uint64_t count = 0;
        for (uint64_t i = 1; i <= F[4]; ++i) {
            while (c < 5 && i > F[c]) F[c++] = count;
            if (!getb(redundant, i)) ++count;
        }
        while (c < 5) F[c++] = count;
    }
    for (int c = 0; c < 5; ++c) out.F[c] = F[c];
    // mark_sink_dummy_edges on the pruned graph, row 0, flip
    out.valid.assign(std::max<uint64_t>(mw, 1), 0);
    for (uint64_t i = 0; i < m; ++i) {
        const bool dummy = i == 0 || ((src[i >> 6] >> (i & 63)) & 1) || (i >= 2 && out.W[i] == 0);
        if (!dummy) out.valid[i >> 6] |= 1ull << (i & 63);
    }
    return out;
}

// ------------------------------------------------------------------------ the graph files

constexpr uint64_t kStateStat = 3;  // BOSS::State::STAT (boss.hpp:325), the build's default state

struct DbgFile {
    uint64_t k = 0, n = 0, F[5] = {0, 0, 0, 0, 0}, state = 0, mode = 0, suffix_length = 0;
    std::vector<uint8_t> W;
    std::vector<uint64_t> last, valid;
    std::vector<std::pair<uint64_t, uint64_t>> ranges;
    bool has_mask = false;
};

inline uint64_t write_dbg_arrays(const std::string &base, const uint8_t *W, const uint64_t *last, uint64_t n,
                                 const uint64_t *F, uint64_t k, uint64_t mode, const std::vector<uint64_t> *valid,
                                 int64_t suffix_length, const uint32_t *weights, unsigned bits_per_count);

// `metagraph build` after construction (cli/build.cpp:323-352): optional --mask-dummy, the suffix
// index of length min(node_suffix_length, k) (default 20 / log2(4) = 10, config.cpp:22-23), then
// DBGSuccinct::serialize.  suffix_length < 0 selects that default.  Returns the valid edges
// (`nodes (k)` of `metagraph stats`, stats.cpp:72-76) when masking, else n - 1.
inline uint64_t write_dbg(const std::string &base, const uint8_t *W, const uint64_t *last, uint64_t n,
                          const uint64_t *F, uint64_t k, uint64_t mode, int mask_dummy, int64_t suffix_length,
                          const uint32_t *weights, unsigned bits_per_count) {
    if (mask_dummy == 2) {  // concatenate --clear-dummy: prune, then write the pruned graph and its mask
        BossNav full(W, last, n, F, k);
        Pruned p = prune_dummy_edges(full);
        return write_dbg_arrays(base, p.W.data(), p.last.data(), p.n, p.F, k, mode, &p.valid, suffix_length,
                                nullptr, 0);
    }
    std::vector<uint64_t> valid;
    if (mask_dummy) {
        BossNav nav(W, last, n, F, k);
        valid = valid_edges(nav);
    }
    return write_dbg_arrays(base, W, last, n, F, k, mode, mask_dummy ? &valid : nullptr, suffix_length, weights,
                            bits_per_count);
}

// the files of one BOSS table (+ its valid-edge mask when `valid`)
inline uint64_t write_dbg_arrays(const std::string &base, const uint8_t *W, const uint64_t *last, uint64_t n,
                                 const uint64_t *F, uint64_t k, uint64_t mode, const std::vector<uint64_t> *valid,
                                 int64_t suffix_length, const uint32_t *weights, unsigned bits_per_count) {
    BossNav nav(W, last, n, F, k);
    uint64_t L = suffix_length < 0 ? std::min<uint64_t>(10, k) : std::min<uint64_t>((uint64_t)suffix_length, k);
    if (L * 2 > 63) L = 0;  // "Node ranges for k-mer suffixes longer than ... cannot be indexed"
    uint64_t n_valid = n ? n - 1 : 0;
    {
        std::ofstream o(base + ".dbg", std::ios::binary);
        if (!o.good()) throw std::runtime_error("Can't write to file " + base + ".dbg");
        put_be(o, 5);
        for (int c = 0; c < 5; ++c) put_be(o, F[c]);
        put_be(o, k);
        put_be(o, kStateStat);
        sdslio::put_wt_huff(o, W, n);
        put_be(o, 4);  // logsigma of W: bits_per_char_W_
        sdslio::put_bit_vector_stat(o, last, n);
        put_be(o, mode);
        const auto ranges = index_suffix_ranges(nav, L);
        put_be(o, L);
        for (const auto &r : ranges) {
            put_raw<uint64_t>(o, r.first);
            put_raw<uint64_t>(o, r.second);
        }
        if (!o.good()) throw std::runtime_error("Can't write to file " + base + ".dbg");
    }
    if (valid) {
        n_valid = 0;
        for (uint64_t x : *valid) n_valid += __builtin_popcountll(x);
        std::ofstream o(base + ".edgemask", std::ios::binary);
        sdslio::put_bit_vector_small(o, valid->data(), n);
        if (!o.good()) throw std::runtime_error("Can't write to file " + base + ".edgemask");
    }
    if (weights && bits_per_count) {  // the chunk's weights buffer renamed (node_weights.cpp:62-68)
        const unsigned w = bits_per_count;
        std::vector<uint64_t> words((n * w + 63) / 64, 0);
        for (uint64_t i = 0; i < n; ++i) {
            const uint64_t v = (uint64_t)weights[i] & ((w >= 64) ? ~0ull : ((1ull << w) - 1));
            const uint64_t pos = i * w, q = pos >> 6, b = pos & 63;
            words[q] |= v << b;
            if (b + w > 64) words[q + 1] |= v >> (64 - b);
        }
        std::ofstream o(base + ".dbg.weights", std::ios::binary);
        sdslio::put_int_vector(o, words.data(), n * w, (uint8_t)w, false);
        if (!o.good()) throw std::runtime_error("Can't write to file " + base + ".dbg.weights");
    }
    return n_valid;
}

inline DbgFile read_dbg(const std::string &base) {
    DbgFile f;
    std::ifstream in(base + ".dbg", std::ios::binary);
    if (!in.good()) throw std::runtime_error("Can't read file " + base + ".dbg");
    if (get_be(in) != 5) throw std::runtime_error("ERROR: failed to load F vector, incompatible size");
    for (int c = 0; c < 5; ++c) f.F[c] = get_be(in);
    f.k = get_be(in);
    f.state = get_be(in);
    if (f.state != kStateStat) throw std::runtime_error("only the STAT representation is written here");
    f.W = sdslio::get_wt_huff(in);
    if (get_be(in) != 4) throw std::runtime_error("ERROR: failed to load W vector");
    uint64_t nb;
    f.last = sdslio::get_bit_vector_stat(in, &nb);
    if (nb != f.W.size()) throw std::runtime_error("ERROR: failed to load L vector");
    f.n = nb;
    f.mode = get_be(in);
    f.suffix_length = get_be(in);
    if (f.suffix_length) {
        uint64_t cnt = 1;
        for (uint64_t i = 0; i < f.suffix_length; ++i) cnt *= 4;
        f.ranges.resize(cnt);
        for (auto &r : f.ranges) {
            r.first = get_raw<uint64_t>(in);
            r.second = get_raw<uint64_t>(in);
        }
    }
    std::ifstream m(base + ".edgemask", std::ios::binary);
    if (m.good()) {
        uint64_t mb;
        f.valid = sdslio::get_bit_vector_small(m, &mb);
        if (mb != f.n) throw std::runtime_error("edgemask size differs from the graph");
        f.has_mask = true;
    }
    return f;
}

}  // namespace dbgio
}  // namespace mtg
