// sdsl_io.hpp -- the sdsl-lite containers of the graph files, written field by field as sdsl-lite 2.x
// serializes them (host code).  sdsl-lite is an empty submodule of the reference snapshot
// (hmusta/sdsl-lite, a fork of simongog/sdsl-lite 2.x: .gitmodules), so this restates the library's
// published serialization; no golden file pins the bytes.  Which container the
// reference instantiates where:
//   W of a STAT BOSS       wavelet_tree_stat = wavelet_tree_sdsl<sdsl::wt_huff<>>
//                          (common/vectors/wavelet_tree.hpp:221, serialize wavelet_tree.cpp:364-368)
//   last of a STAT BOSS    bit_vector_stat = bit_vector_sdsl<sdsl::bit_vector, rank_support_v5<1>,
//                          select_support_mcl<1>, select_support_scan<0>> (bit_vector_sdsl.hpp:451-455,
//                          serialize :267-281)
//   .edgemask              bit_vector_small = bit_vector_adaptive_stat<smallest_representation>: an
//                          sd_vector (bit_vector_sd.hpp) or an rrr_vector<63> (bit_vector_rrr<>),
//                          whichever predict_size says is smaller (bit_vector_adaptive.hpp:309-319),
//                          behind its BE type tag (:125-128)
//   .dbg.weights           sdsl::int_vector<> of width bits_per_count (node_weights.cpp:62-68)
//
// sdsl framing (int_vector.hpp, write_header / serialize): an int_vector<0> writes its size in bits
// (u64) and its width (u8); a fixed-width int_vector<w> (bit_vector = int_vector<1>, int_vector<64>)
// only the size in bits; then capacity() / 64 = ceil(bits / 64) u64 words, bits past the size zero.
// write_member of a fundamental type writes its bytes (little-endian here).
#pragma once

#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <istream>
#include <ostream>
#include <stdexcept>
#include <string>
#include <vector>

namespace mtg {
namespace sdslio {

template <typename T>
inline void put_raw(std::ostream &o, const T &v) { o.write((const char *)&v, sizeof(T)); }
template <typename T>
inline T get_raw(std::istream &in) {
    T v;
    if (!in.read((char *)&v, sizeof(T))) throw std::runtime_error("truncated sdsl container");
    return v;
}
inline void put_be(std::ostream &o, uint64_t v) {  // metagraph serialize_number (serialization.cpp:38-50)
    uint8_t b[8];
    for (int i = 0; i < 8; ++i) b[i] = (uint8_t)(v >> (56 - 8 * i));
    o.write((const char *)b, 8);
}
inline uint64_t get_be(std::istream &in) {
    uint8_t b[8];
    if (!in.read((char *)b, 8)) throw std::runtime_error("truncated file");
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v = v << 8 | b[i];
    return v;
}

// sdsl bits::hi(x) + 1 as the uint8 the containers pass as a width: 0 for x = 0 (hi(0) = -1)
inline uint8_t hi1(uint64_t x) { return x ? (uint8_t)(64 - __builtin_clzll(x)) : 0; }
// int_vector<0>::width(w): 1..64 kept, anything else becomes 64 (int_vector_trait<0>::set_width)
inline uint8_t set_width(uint8_t w) { return (w >= 1 && w <= 64) ? w : 64; }
inline bool bit(const uint64_t *w, uint64_t i) { return (w[i >> 6] >> (i & 63)) & 1; }
inline uint64_t popc(uint64_t x) { return (uint64_t)__builtin_popcountll(x); }

// an sdsl int_vector: n elements of `width` bits packed LSB first
struct IntVec {
    std::vector<uint64_t> words;
    uint64_t n = 0;
    uint8_t width = 64;
    IntVec() = default;
    IntVec(uint64_t n_, uint8_t w) : words((n_ * set_width(w) + 63) / 64, 0), n(n_), width(set_width(w)) {}
    void set(uint64_t i, uint64_t v) {
        if (width < 64) v &= (1ull << width) - 1;  // int_vector truncates
        const uint64_t pos = i * width, q = pos >> 6, b = pos & 63;
        words[q] &= ~(width == 64 ? ~0ull : (((1ull << width) - 1) << b));
        words[q] |= v << b;
        if (b + width > 64) {
            const uint64_t hi = b + width - 64;
            words[q + 1] &= ~((1ull << hi) - 1);
            words[q + 1] |= v >> (64 - b);
        }
    }
    uint64_t get(uint64_t i) const {
        const uint64_t pos = i * width, q = pos >> 6, b = pos & 63;
        uint64_t v = words[q] >> b;
        if (b + width > 64) v |= words[q + 1] << (64 - b);
        return width == 64 ? v : v & ((1ull << width) - 1);
    }
};

// fixed: an int_vector<w> with w > 0 (no width byte)
inline void put_int_vector(std::ostream &o, const uint64_t *words, uint64_t nbits, uint8_t width, bool fixed) {
    put_raw<uint64_t>(o, nbits);
    if (!fixed) put_raw<uint8_t>(o, width);
    o.write((const char *)words, (std::streamsize)(((nbits + 63) / 64) * 8));
}
inline void put_int_vector(std::ostream &o, const IntVec &v) { put_int_vector(o, v.words.data(), v.n * v.width, v.width, false); }
inline void put_bit_vector(std::ostream &o, const uint64_t *words, uint64_t nbits) { put_int_vector(o, words, nbits, 1, true); }
inline void put_u64_vector(std::ostream &o, const std::vector<uint64_t> &v) {  // int_vector<64>
    put_int_vector(o, v.data(), 64 * (uint64_t)v.size(), 64, true);
}
// reads an int_vector; fixed_width > 0 for int_vector<w>
inline IntVec get_int_vector(std::istream &in, uint8_t fixed_width) {
    IntVec v;
    const uint64_t nbits = get_raw<uint64_t>(in);
    v.width = fixed_width ? fixed_width : set_width(get_raw<uint8_t>(in));
    if (nbits % v.width) throw std::runtime_error("sdsl int_vector: size not a multiple of the width");
    if (nbits > (1ull << 46)) throw std::runtime_error("sdsl int_vector: implausible size");
    v.n = nbits / v.width;
    v.words.assign((nbits + 63) / 64, 0);
    if (!v.words.empty() && !in.read((char *)v.words.data(), (std::streamsize)(v.words.size() * 8)))
        throw std::runtime_error("truncated sdsl int_vector");
    return v;
}

// ------------------------------------------------------------------- rank_support_v<1> / v5<1>

// rank_support_v<1> (rank_support_v.hpp, constructor): per 512-bit block two words, the ones before
// the block, and the ones before each of its words 1..7 in 9-bit fields at bits 54, 45, .., 0;
// ((capacity >> 9) + 1) * 2 words; an empty vector gets int_vector<64>(2, 0)
inline std::vector<uint64_t> rank_v_words(const uint64_t *data, uint64_t nbits) {
    if (nbits == 0) return std::vector<uint64_t>(2, 0);
    const uint64_t nw = (nbits + 63) / 64;
    std::vector<uint64_t> bb(((64 * nw >> 9) + 1) << 1, 0);
    uint64_t sum = popc(data[0]), second = 0, j = 0, i;
    for (i = 1; i < nw; ++i) {
        if (!(i & 7)) {
            j += 2;
            bb[j - 1] = second;
            bb[j] = bb[j - 2] + sum;
            second = sum = 0;
        } else {
            second |= sum << (63 - 9 * (i & 7));
        }
        sum += popc(data[i]);
    }
    if (i & 7) {
        second |= sum << (63 - 9 * (i & 7));
        bb[j + 1] = second;
    } else {
        j += 2;
        bb[j - 1] = second;
        bb[j] = bb[j - 2] + sum;
        bb[j + 1] = 0;
    }
    return bb;
}

// rank_support_v5<1> (rank_support_v5.hpp, constructor): per 2048-bit superblock two words, the ones
// before it, and the ones before each of its 384-bit blocks 1..5 in 12-bit fields at bits 48, 36,
// 24, 12, 0; ((capacity >> 11) + 1) * 2 words
inline std::vector<uint64_t> rank_v5_words(const uint64_t *data, uint64_t nbits) {
    if (nbits == 0) return std::vector<uint64_t>(2, 0);
    const uint64_t nw = (nbits + 63) / 64;
    std::vector<uint64_t> bb(((64 * nw >> 11) + 1) << 1, 0);
    uint64_t sum = popc(data[0]), second = 0, j = 0, cnt = 1;
    for (uint64_t i = 1; i < nw; ++i, ++cnt) {
        if (cnt == 32) {
            j += 2;
            bb[j - 1] = second;
            bb[j] = bb[j - 2] + sum;
            second = sum = cnt = 0;
        } else if (cnt % 6 == 0) {
            second |= sum << (60 - 12 * (cnt / 6));
        }
        sum += popc(data[i]);
    }
    if (cnt % 6 == 0) second |= sum << (60 - 12 * (cnt / 6));
    if (cnt == 32) {
        j += 2;
        bb[j - 1] = second;
        bb[j] = bb[j - 2] + sum;
        bb[j + 1] = 0;
    } else {
        bb[j + 1] = second;
    }
    return bb;
}

// ------------------------------------------------------------------------ select_support_mcl<b>

// select_support_mcl<b, 1> (select_support_mcl.hpp: init_fast + serialize): u64 number of args (ones
// for b = 1, zeros for b = 0); when there are any: the superblock starts (int_vector<0> of width
// hi(size) + 1: the position of every 4096-th arg), the mini-or-long flags (a bit_vector over the
// superblocks, empty when no superblock is long), then per superblock either its long form
// (int_vector<0> of 4096 absolute positions, width hi(last position) + 1) or its mini form
// (int_vector<0> of 64 offsets -- every 64-th arg relative to the superblock's first -- of width
// hi(span) + 1).  A superblock is long when its span exceeds (hi(size) + 1)^4.
inline void put_select_mcl(std::ostream &o, const uint64_t *data, uint64_t nbits, bool b) {
    uint64_t args = 0;
    const uint64_t nw = (nbits + 63) / 64;
    for (uint64_t q = 0; q < nw; ++q) {
        uint64_t w = b ? data[q] : ~data[q];
        if (q == nw - 1 && (nbits & 63)) w &= (1ull << (nbits & 63)) - 1;
        args += popc(w);
    }
    put_raw<uint64_t>(o, args);
    if (!args) return;
    const uint8_t logn = hi1(nbits ? nbits : 1);
    const uint64_t logn2 = (uint64_t)logn * logn, logn4 = logn2 * logn2;
    constexpr uint64_t SB = 4096;
    const uint64_t sb = (args + SB - 1) / SB;
    IntVec super(sb, logn);
    std::vector<IntVec> mini(sb), lng(sb);
    std::vector<bool> is_long(sb, false);
    bool any_long = false;
    std::vector<uint64_t> pos(SB);
    uint64_t cnt = 0, sbc = 0;
    for (uint64_t q = 0; q < nw; ++q) {
        uint64_t w = b ? data[q] : ~data[q];
        if (q == nw - 1 && (nbits & 63)) w &= (1ull << (nbits & 63)) - 1;
        while (w) {
            const uint64_t i = 64 * q + (uint64_t)__builtin_ctzll(w);
            w &= w - 1;
            pos[cnt % SB] = i;
            ++cnt;
            if (cnt % SB == 0 || cnt == args) {
                const uint64_t last = (cnt - 1) % SB;
                super.set(sbc, pos[0]);
                const uint64_t diff = pos[last] - pos[0];
                if (diff > logn4) {
                    any_long = true;
                    is_long[sbc] = true;
                    lng[sbc] = IntVec(SB, hi1(pos[last]));
                    for (uint64_t j = 0; j <= last; ++j) lng[sbc].set(j, pos[j]);
                } else {
                    mini[sbc] = IntVec(64, hi1(diff));
                    for (uint64_t j = 0; j <= last; j += 64) mini[sbc].set(j / 64, pos[j] - pos[0]);
                }
                ++sbc;
            }
        }
    }
    put_int_vector(o, super);
    std::vector<uint64_t> flags(any_long ? (sb + 63) / 64 : 0, 0);
    if (any_long)
        for (uint64_t s = 0; s < sb; ++s)
            if (!is_long[s]) flags[s >> 6] |= 1ull << (s & 63);  // mini_or_long[i] = !miniblock[i].empty()
    put_bit_vector(o, flags.data(), any_long ? sb : 0);
    for (uint64_t s = 0; s < sb; ++s) put_int_vector(o, is_long[s] ? lng[s] : mini[s]);
}
inline void skip_select_mcl(std::istream &in) {
    const uint64_t args = get_raw<uint64_t>(in);
    if (!args) return;
    const uint64_t sb = (args + 4095) / 4096;
    const IntVec super = get_int_vector(in, 0);
    if (super.n != sb) throw std::runtime_error("select_support_mcl: superblock count mismatch");
    const IntVec flags = get_int_vector(in, 1);
    if (flags.n && flags.n != sb) throw std::runtime_error("select_support_mcl: flag count mismatch");
    for (uint64_t s = 0; s < sb; ++s) {
        const IntVec blk = get_int_vector(in, 0);
        const bool mini = !flags.n || bit(flags.words.data(), s);
        if (blk.n != (mini ? 64u : 4096u)) throw std::runtime_error("select_support_mcl: block size mismatch");
    }
}

// ------------------------------------------------------------------------------ bit_vector_stat

// bit_vector_stat::serialize (bit_vector_sdsl.hpp:267-281): the bit_vector, serialize_number(ones),
// rank_support_v5<1>, select_support_mcl<1>, select_support_scan<0> (which writes nothing)
inline void put_bit_vector_stat(std::ostream &o, const uint64_t *w, uint64_t nbits) {
    put_bit_vector(o, w, nbits);
    uint64_t ones = 0;
    for (uint64_t q = 0; q < (nbits + 63) / 64; ++q) ones += popc(w[q]);
    put_be(o, ones);
    put_u64_vector(o, rank_v5_words(w, nbits));
    put_select_mcl(o, w, nbits, true);
}
inline std::vector<uint64_t> get_bit_vector_stat(std::istream &in, uint64_t *nbits) {
    IntVec v = get_int_vector(in, 1);
    *nbits = v.n;
    const uint64_t ones = get_be(in);
    uint64_t c = 0;
    for (uint64_t x : v.words) c += popc(x);
    if (c != ones) throw std::runtime_error("bit_vector_stat: set-bit count mismatch");
    const IntVec r = get_int_vector(in, 64);
    if (r.words != rank_v5_words(v.words.data(), v.n)) throw std::runtime_error("bit_vector_stat: rank support mismatch");
    skip_select_mcl(in);
    return std::move(v.words);
}

// ------------------------------------------------------------------------------- W: wt_huff<>

// sdsl::wt_huff<> = wt_pc<huff_shape, bit_vector, rank_support_v<1>, select_support_mcl<1>,
// select_support_mcl<0>, byte_tree<>> (wt_huff.hpp; the bit_vector's rank_1_type / select_1_type /
// select_0_type).  wt_pc::serialize: u64 size, u64 sigma (symbols that occur), the concatenated
// node bit_vector, its rank_support_v<1>, select_support_mcl<1>, select_support_mcl<0>, then the
// byte_tree: u64 node count, per node u64 bv_pos, u64 bv_pos_rank, u16 parent, u16 child[2]
// (0xFFFF = none), u16 c_to_leaf[256], u64 path[256].
//
// Shape (huff_shape::construct_tree): a leaf per occurring symbol in symbol order (temp node ids
// 0..sigma-1), then repeatedly the two smallest (frequency, temp id) pairs of a min-priority queue
// become child[0] and child[1] of a new node (next temp id).  byte_tree's constructor numbers the
// nodes breadth first from the root (the last temp node), children in child[0], child[1] order;
// bv_pos = bits of the inner nodes before it in that order; a leaf's bv_pos_rank is its symbol, an
// inner node's the ones of the bit_vector before its bv_pos (init_node_ranks); path[c] = the code
// length << 56 | the code, the root's branch in bit 0 (1 = child[1]).  Every inner node's bits are
// its symbols' branch bits in text order.
struct HuffTree {
    struct Node {
        uint64_t bv_pos = 0, bv_pos_rank = 0;
        uint16_t parent = 0xFFFF, child[2] = {0xFFFF, 0xFFFF};
        uint64_t freq = 0;
    };
    std::vector<Node> nodes;
    uint16_t leaf[256];
    uint64_t path[256];
};

inline HuffTree huff_shape(const uint64_t freq[256]) {
    struct Temp {
        uint64_t freq, sym;
        int64_t parent = -1, child[2] = {-1, -1};
    };
    std::vector<Temp> t;
    typedef std::pair<uint64_t, uint64_t> PII;  // (freq, temp id), std::greater: smallest first
    std::vector<PII> heap;
    auto cmp = [](const PII &a, const PII &b) { return a > b; };
    for (int s = 0; s < 256; ++s)
        if (freq[s]) {
            heap.push_back({freq[s], t.size()});
            std::push_heap(heap.begin(), heap.end(), cmp);
            t.push_back(Temp{freq[s], (uint64_t)s});
        }
    while (heap.size() > 1) {
        std::pop_heap(heap.begin(), heap.end(), cmp);
        const PII v1 = heap.back();
        heap.pop_back();
        std::pop_heap(heap.begin(), heap.end(), cmp);
        const PII v2 = heap.back();
        heap.pop_back();
        t[v1.second].parent = (int64_t)t.size();
        t[v2.second].parent = (int64_t)t.size();
        Temp in{v1.first + v2.first, ~0ull};
        in.child[0] = (int64_t)v1.second;
        in.child[1] = (int64_t)v2.second;
        heap.push_back({in.freq, t.size()});
        std::push_heap(heap.begin(), heap.end(), cmp);
        t.push_back(in);
    }
    HuffTree h;
    std::fill(h.leaf, h.leaf + 256, (uint16_t)0xFFFF);
    std::fill(h.path, h.path + 256, 0ull);
    if (t.empty()) return h;
    // breadth first from the root; tmap[v] = the temp node of tree node v
    std::vector<int64_t> tmap{(int64_t)t.size() - 1};
    h.nodes.push_back(HuffTree::Node{});
    uint64_t bv = 0;
    for (size_t v = 0; v < h.nodes.size(); ++v) {
        const Temp &tv = t[tmap[v]];
        h.nodes[v].freq = tv.freq;
        h.nodes[v].bv_pos = bv;
        if (tv.child[0] >= 0) {
            bv += tv.freq;
            for (int c = 0; c < 2; ++c) {
                HuffTree::Node ch;
                ch.parent = (uint16_t)v;
                h.nodes[v].child[c] = (uint16_t)h.nodes.size();
                h.nodes.push_back(ch);
                tmap.push_back(tv.child[c]);
            }
        } else {
            h.nodes[v].bv_pos_rank = tv.sym;
            h.leaf[tv.sym] = (uint16_t)v;
        }
    }
    for (int s = 0; s < 256; ++s) {
        if (h.leaf[s] == 0xFFFF) continue;
        uint64_t w = 0, l = 0;
        for (uint16_t v = h.leaf[s]; v != 0; v = h.nodes[v].parent) {
            w <<= 1;
            if (h.nodes[h.nodes[v].parent].child[1] == v) w |= 1;
            ++l;
        }
        if (l > 56) throw std::runtime_error("wt_huff: code depth greater than 56");
        h.path[s] = w | l << 56;
    }
    return h;
}

inline void put_wt_huff(std::ostream &o, const uint8_t *W, uint64_t n) {
    uint64_t freq[256] = {0};
    for (uint64_t i = 0; i < n; ++i) ++freq[W[i]];
    uint64_t sigma = 0;
    for (int s = 0; s < 256; ++s) sigma += freq[s] != 0;
    put_raw<uint64_t>(o, n);
    put_raw<uint64_t>(o, sigma);
    HuffTree h = huff_shape(freq);
    uint64_t total = 0;
    for (const auto &v : h.nodes)
        if (v.child[0] != 0xFFFF) total += v.freq;
    std::vector<uint64_t> bv((total + 63) / 64, 0);
    std::vector<uint64_t> cur(h.nodes.size(), 0);
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t p = h.path[W[i]], len = p >> 56;
        uint16_t v = 0;
        for (uint64_t d = 0; d < len; ++d) {
            const uint64_t b = (p >> d) & 1, pos = h.nodes[v].bv_pos + cur[v]++;
            if (b) bv[pos >> 6] |= 1ull << (pos & 63);
            v = h.nodes[v].child[b];
        }
    }
    // inner nodes: the ones before bv_pos (init_node_ranks over the rank support)
    for (auto &v : h.nodes) {
        if (v.child[0] == 0xFFFF) continue;
        uint64_t c = 0;
        for (uint64_t q = 0; q < (v.bv_pos >> 6); ++q) c += popc(bv[q]);
        if (v.bv_pos & 63) c += popc(bv[v.bv_pos >> 6] & ((1ull << (v.bv_pos & 63)) - 1));
        v.bv_pos_rank = c;
    }
    put_bit_vector(o, bv.data(), total);
    put_u64_vector(o, rank_v_words(bv.data(), total));
    put_select_mcl(o, bv.data(), total, true);
    put_select_mcl(o, bv.data(), total, false);
    put_raw<uint64_t>(o, (uint64_t)h.nodes.size());
    for (const auto &v : h.nodes) {
        put_raw<uint64_t>(o, v.bv_pos);
        put_raw<uint64_t>(o, v.bv_pos_rank);
        put_raw<uint16_t>(o, v.parent);
        put_raw<uint16_t>(o, v.child[0]);
        put_raw<uint16_t>(o, v.child[1]);
    }
    o.write((const char *)h.leaf, sizeof(h.leaf));
    o.write((const char *)h.path, sizeof(h.path));
}

inline std::vector<uint8_t> get_wt_huff(std::istream &in) {
    const uint64_t n = get_raw<uint64_t>(in);
    get_raw<uint64_t>(in);  // sigma
    const IntVec bvv = get_int_vector(in, 1);
    const uint64_t total = bvv.n;
    const std::vector<uint64_t> &bv = bvv.words;
    const IntVec r = get_int_vector(in, 64);
    if (r.words != rank_v_words(bv.data(), total)) throw std::runtime_error("wt_huff: rank support mismatch");
    skip_select_mcl(in);
    skip_select_mcl(in);
    const uint64_t nn = get_raw<uint64_t>(in);
    if (nn > 511) throw std::runtime_error("wt_huff: bad tree");
    std::vector<HuffTree::Node> nodes(nn);
    for (auto &v : nodes) {
        v.bv_pos = get_raw<uint64_t>(in);
        v.bv_pos_rank = get_raw<uint64_t>(in);
        v.parent = get_raw<uint16_t>(in);
        v.child[0] = get_raw<uint16_t>(in);
        v.child[1] = get_raw<uint16_t>(in);
    }
    uint16_t leaf[256];
    uint64_t path[256];
    if (!in.read((char *)leaf, sizeof(leaf)) || !in.read((char *)path, sizeof(path)))
        throw std::runtime_error("truncated wt_huff");
    std::vector<uint8_t> W(n);
    std::vector<uint64_t> cur(nn, 0);
    for (uint64_t i = 0; i < n; ++i) {  // root -> leaf with one cursor per inner node
        uint16_t v = 0;
        while (nn && nodes[v].child[0] != 0xFFFF) {
            const uint64_t pos = nodes[v].bv_pos + cur[v]++;
            if (pos >= total) throw std::runtime_error("wt_huff: bits out of range");
            v = nodes[v].child[bit(bv.data(), pos)];
            if (v >= nn) throw std::runtime_error("wt_huff: bad child");
        }
        if (!nn || nodes[v].bv_pos_rank > 255 || leaf[nodes[v].bv_pos_rank] != v)
            throw std::runtime_error("wt_huff: leaf without symbol");
        W[i] = (uint8_t)nodes[v].bv_pos_rank;
    }
    return W;
}

// ----------------------------------------------------------------------- sd_vector<> (.edgemask)

// sd_vector<> (sd_vector.hpp: the sd_vector_builder constructor and serialize): u64 size, u8 wl, low
// (int_vector<0> of m entries of width wl: each set position's low wl bits), high (bit_vector of
// m + 2^logm bits: set position j goes to bit (pos >> wl) + j), select_support_mcl<1> and
// select_support_mcl<0> over high.  logm = hi(m) + 1, logn = hi(size) + 1, logm - 1 when equal,
// wl = logn - logm.
inline void put_sd_vector(std::ostream &o, const std::vector<uint64_t> &setpos, uint64_t size) {
    const uint64_t m = setpos.size();
    uint8_t logm = hi1(m), logn = hi1(size);
    if (logm == logn) --logm;
    const uint8_t wl = (uint8_t)(logn - logm);
    IntVec low(m, wl);
    const uint64_t hsize = m + (1ull << logm);
    std::vector<uint64_t> high((hsize + 63) / 64, 0);
    for (uint64_t j = 0; j < m; ++j) {
        low.set(j, setpos[j]);
        const uint64_t hp = (setpos[j] >> wl) + j;
        high[hp >> 6] |= 1ull << (hp & 63);
    }
    put_raw<uint64_t>(o, size);
    put_raw<uint8_t>(o, wl);
    put_int_vector(o, low);
    put_bit_vector(o, high.data(), hsize);
    put_select_mcl(o, high.data(), hsize, true);
    put_select_mcl(o, high.data(), hsize, false);
}
inline std::vector<uint64_t> get_sd_vector(std::istream &in, uint64_t *size) {
    *size = get_raw<uint64_t>(in);
    const uint8_t wl = get_raw<uint8_t>(in);
    const IntVec low = get_int_vector(in, 0);
    const IntVec high = get_int_vector(in, 1);
    skip_select_mcl(in);
    skip_select_mcl(in);
    std::vector<uint64_t> out((*size + 63) / 64, 0);
    uint64_t j = 0;
    for (uint64_t hp = 0; hp < high.n; ++hp) {
        if (!bit(high.words.data(), hp)) continue;
        if (j >= low.n) throw std::runtime_error("sd_vector: more high ones than low entries");
        const uint64_t pos = ((hp - j) << wl) | (wl ? low.get(j) : 0);
        if (pos >= *size) throw std::runtime_error("sd_vector: position out of range");
        out[pos >> 6] |= 1ull << (pos & 63);
        ++j;
    }
    if (j != low.n) throw std::runtime_error("sd_vector: high/low count mismatch");
    return out;
}

// ---------------------------------------------------------------------- rrr_vector<63> (.edgemask)

// rrr_vector<63, int_vector<>, 32> (rrr_vector.hpp constructor + serialize; rrr_helper.hpp's
// binomial coding): u64 size; bt (int_vector<0> of width 6: the ones of every 63-bit block, one
// more block when size % 63 == 0), btnr (bit_vector: each block's class offset in ceil(log2 C(63,
// bt)) bits, at least 64 bits), btnrp (int_vector<0>: btnr position of every 32nd block), rank
// (int_vector<0>: ones before every 32nd block, plus the total when size % (32 * 63) != 0), invert
// (bit_vector: a superblock of 32 blocks with more than 16 blocks over 31 ones stores 63 - bt).
// The class offset enumerates the block's bits LSB first: a one at a position with nn positions
// and k ones left adds C(nn - 1, k) (bin_to_nr).
struct Binomial63 {
    uint64_t C[64][64];
    uint8_t space[64];
    Binomial63() {
        std::memset(C, 0, sizeof(C));
        for (int nn = 0; nn < 64; ++nn) {
            C[nn][0] = 1;
            for (int k = 1; k <= nn; ++k) C[nn][k] = C[nn - 1][k - 1] + (k <= nn - 1 ? C[nn - 1][k] : 0);
        }
        for (int k = 0; k < 64; ++k) space[k] = C[63][k] <= 1 ? 0 : hi1(C[63][k] - 1);
    }
    uint64_t bin_to_nr(uint64_t bin) const {
        if (bin == 0 || bin == (1ull << 63) - 1) return 0;
        uint64_t nr = 0, k = popc(bin), nn = 63;
        while (bin) {
            if (bin & 1) {
                nr += C[nn - 1][k];
                --k;
            }
            bin >>= 1;
            --nn;
        }
        return nr;
    }
    uint64_t nr_to_bin(uint64_t k, uint64_t nr) const {
        if (k == 0) return 0;
        if (k == 63) return (1ull << 63) - 1;
        uint64_t bin = 0, nn = 63;
        for (uint64_t pos = 0; k && nn; ++pos, --nn) {
            const uint64_t c = C[nn - 1][k];
            if (nr >= c) {
                bin |= 1ull << pos;
                nr -= c;
                --k;
            }
        }
        return bin;
    }
};
inline const Binomial63 &binomial63() {
    static const Binomial63 b;
    return b;
}
inline uint64_t get_bits(const uint64_t *w, uint64_t pos, unsigned len) {  // len <= 64, pos + len within data
    if (!len) return 0;
    const uint64_t q = pos >> 6, b = pos & 63;
    uint64_t v = w[q] >> b;
    if (b + len > 64) v |= w[q + 1] << (64 - b);
    return len == 64 ? v : v & ((1ull << len) - 1);
}

inline void put_rrr_vector(std::ostream &o, const uint64_t *data, uint64_t size) {
    constexpr uint64_t BS = 63, K = 32;
    const Binomial63 &B = binomial63();
    const uint64_t nblocks = (size + BS) / BS;
    std::vector<uint64_t> bt(nblocks, 0), bin(nblocks, 0);
    uint64_t btnr_bits = 0, total = 0;
    for (uint64_t i = 0, pos = 0; pos < size; ++i, pos += BS) {
        const unsigned len = (unsigned)std::min<uint64_t>(BS, size - pos);
        bin[i] = get_bits(data, pos, len);
        bt[i] = popc(bin[i]);
        total += bt[i];
        btnr_bits += B.space[bt[i]];
    }
    const uint64_t nsuper = (nblocks + K - 1) / K;
    const uint64_t btnr_size = std::max<uint64_t>(btnr_bits, 64);
    std::vector<uint64_t> btnr((btnr_size + 63) / 64, 0);
    IntVec btnrp(nsuper, hi1(btnr_bits));
    IntVec rank(nsuper + ((size % (K * BS)) > 0), hi1(total));
    std::vector<uint64_t> invert((nsuper + 63) / 64, 0);
    IntVec btv(nblocks, hi1(BS));
    uint64_t bp = 0, sum = 0;
    for (uint64_t i = 0, pos = 0; pos < size; ++i, pos += BS) {
        const bool full = pos + BS <= size;
        if (i % K == 0) {
            btnrp.set(i / K, bp);
            rank.set(i / K, sum);
            if (full && i + K <= nblocks) {  // the superblock's blocks all exist
                uint64_t gt = 0;
                for (uint64_t j = i; j < i + K; ++j) gt += bt[j] > BS / 2;
                if (gt > K / 2) invert[(i / K) >> 6] |= 1ull << ((i / K) & 63);
            }
        }
        const uint64_t s = B.space[bt[i]];
        sum += bt[i];
        if (s) {
            const uint64_t nr = B.bin_to_nr(bin[i]);
            for (uint64_t b = 0; b < s; ++b)
                if ((nr >> b) & 1) btnr[(bp + b) >> 6] |= 1ull << ((bp + b) & 63);
        }
        bp += s;
    }
    // an inverted superblock stores 63 - bt for all its blocks
    for (uint64_t i = 0; i < nblocks; ++i) {
        const bool iv = (invert[(i / K) >> 6] >> ((i / K) & 63)) & 1;
        btv.set(i, iv ? BS - bt[i] : bt[i]);
    }
    rank.set(rank.n - 1, total);
    put_raw<uint64_t>(o, size);
    put_int_vector(o, btv);
    put_bit_vector(o, btnr.data(), btnr_size);
    put_int_vector(o, btnrp);
    put_int_vector(o, rank);
    put_bit_vector(o, invert.data(), nsuper);
}
inline std::vector<uint64_t> get_rrr_vector(std::istream &in, uint64_t *size) {
    constexpr uint64_t BS = 63, K = 32;
    const Binomial63 &B = binomial63();
    *size = get_raw<uint64_t>(in);
    const IntVec bt = get_int_vector(in, 0);
    const IntVec btnr = get_int_vector(in, 1);
    get_int_vector(in, 0);  // btnrp
    get_int_vector(in, 0);  // rank
    const IntVec invert = get_int_vector(in, 1);
    if (bt.n != (*size + BS) / BS) throw std::runtime_error("rrr_vector: block count mismatch");
    std::vector<uint64_t> out((*size + 63) / 64 + 1, 0);
    uint64_t bp = 0;
    for (uint64_t i = 0, pos = 0; pos < *size; ++i, pos += BS) {
        const uint64_t sp = i / K;
        const bool iv = sp < invert.n && bit(invert.words.data(), sp);
        const uint64_t k = iv ? BS - bt.get(i) : bt.get(i);
        const uint64_t s = B.space[k];
        if (bp + s > btnr.n) throw std::runtime_error("rrr_vector: btnr out of range");
        const uint64_t blk = B.nr_to_bin(k, get_bits(btnr.words.data(), bp, (unsigned)s));
        bp += s;
        for (uint64_t b = 0; b < BS && pos + b < *size; ++b)
            if ((blk >> b) & 1) out[(pos + b) >> 6] |= 1ull << ((pos + b) & 63);
    }
    out.resize((*size + 63) / 64);
    return out;
}

// --------------------------------------------------------------------------- bit_vector_small

// the space predictions smallest_representation compares (bit_vector_adaptive.hpp:309-317):
// bit_vector_sd::predict_size (bit_vector_sd.hpp:62-65; footprint_sd_vector,
// vector_algorithm.cpp:578-607) against bit_vector_rrr<>::predict_size (bit_vector_sdsl.hpp:81-86,
// 384-394).  The sizeof terms are this restatement's count of the x86-64 member layouts:
// bit_vector_sd = vptr + bool + sd_vector<> (size, wl, low, high, two select_support_mcl of 80 B,
// five reference members) + rank/select_1 support pointers + select_0_support_sd (a pointer and two
// int_vectors) = 352 B; rank_support_rrr, select_support_rrr<1> / <0> = one pointer each.
constexpr uint64_t kSizeofBitVectorSdBits = 352 * 8;
constexpr uint64_t kSizeofRrrSupportBits = 8 * 8;

inline double footprint_select_mcl(uint64_t size, uint64_t ones) {
    const uint64_t sb = (ones + 4095) / 4096;
    const double avg_diff = 1.0 * size / (double)sb * 4095 / 4096;
    uint64_t blocks = ((uint64_t)hi1((uint64_t)avg_diff) * 64 + 64 + 8) * (ones / 4096);
    uint64_t flags = 0;
    if (ones % 4096) {
        blocks += 4096 * (uint64_t)hi1(size - 1) + 64 + 8;
        flags += (sb + 63) / 64 * 64 + 64;
    } else {
        flags += 64;
    }
    const uint64_t offsets = (sb * (uint64_t)hi1(size) + 63) / 64 * 64 + 64 + 8;
    return 64.0 + (double)offsets + (double)flags + (double)blocks;
}
inline double predict_sd(uint64_t size, uint64_t ones) {
    ones = std::min(ones, size - ones);
    uint8_t logn = hi1(size), logm = hi1(ones);
    if (logm == logn) --logm;
    const uint64_t low = ones * (uint64_t)(uint8_t)(logn - logm);
    const uint64_t high = ones + (1ull << logm);
    return (double)kSizeofBitVectorSdBits + (double)low + (double)high + footprint_select_mcl(high, ones) +
           footprint_select_mcl(high, high - ones);
}
inline double predict_rrr(uint64_t size, uint64_t ones) {
    const double t_bs = 63, t_k = 32;
    auto logbinomial = [](double n, double m) {
        return (std::lgamma(n + 1) - std::lgamma(m + 1) - std::lgamma(n - m + 1)) / std::log(2.0);
    };
    const uint64_t bt = (size + 63) / 63;
    const uint64_t blocks = (uint64_t)((double)bt * logbinomial(t_bs, t_bs * (double)ones / (double)size));
    const uint64_t sk = (bt + 31) / 32;
    const uint64_t v = (bt * (uint64_t)hi1(63) + 63) / 64 * 64 + 64 + 8 + (blocks + 63) / 64 * 64 + 64 +
                       (sk * (uint64_t)hi1(blocks) + 63) / 64 * 64 + 64 + 8 +
                       ((sk + ((size % (32 * 63)) > 0)) * (uint64_t)hi1(ones) + 63) / 64 * 64 + 64 + 8;
    (void)t_k;
    return (double)v + 3.0 * kSizeofRrrSupportBits;
}

enum : uint64_t { kRrrVector = 0, kSdVector = 1, kStatVector = 2 };  // bit_vector_adaptive::VectorCode

// bit_vector_small from an sdsl::bit_vector (bit_vector_adaptive.hpp:244-261): the BE type tag, then
// bit_vector_sd (sd_vector<> over the ones, or over the zeros when ones > size / 2, + the inverted
// byte; bit_vector_sd.hpp:88-106, 267-271) or bit_vector_rrr<> (rrr_vector<63>; its rank/select
// supports write nothing)
inline void put_bit_vector_small(std::ostream &o, const uint64_t *w, uint64_t nbits) {
    uint64_t ones = 0;
    for (uint64_t q = 0; q < (nbits + 63) / 64; ++q) ones += popc(w[q]);
    if (predict_sd(nbits, ones) < predict_rrr(nbits, ones)) {
        put_be(o, kSdVector);
        const bool inverted = ones > nbits / 2;
        std::vector<uint64_t> pos;
        pos.reserve(inverted ? nbits - ones : ones);
        for (uint64_t i = 0; i < nbits; ++i)
            if (bit(w, i) != inverted) pos.push_back(i);
        put_sd_vector(o, pos, nbits);
        put_raw<uint8_t>(o, inverted ? 1 : 0);
    } else {
        put_be(o, kRrrVector);
        put_rrr_vector(o, w, nbits);
    }
}
inline std::vector<uint64_t> get_bit_vector_small(std::istream &in, uint64_t *nbits) {
    const uint64_t tag = get_be(in);
    if (tag == kSdVector) {
        std::vector<uint64_t> v = get_sd_vector(in, nbits);
        const uint8_t inverted = get_raw<uint8_t>(in);
        if (inverted) {
            for (auto &x : v) x = ~x;
            if (*nbits & 63) v.back() &= (1ull << (*nbits & 63)) - 1;
        }
        return v;
    }
    if (tag == kRrrVector) return get_rrr_vector(in, nbits);
    if (tag == kStatVector) return get_bit_vector_stat(in, nbits);
    throw std::runtime_error("bit_vector_small: unknown representation");
}

}  // namespace sdslio
}  // namespace mtg
