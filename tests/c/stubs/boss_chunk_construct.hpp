// Declaration-only stand-in for the reference's IBOSSChunkConstructor / BOSS::Chunk
// (graph/representation/succinct/boss_chunk_construct.hpp:18-34, base/dbg_construct.hpp:12-22,
// boss_chunk.hpp:19-104), plus the array constructor INTEGRATION.md section 3 adds.  Only
// signatures: tests/test_capi_c.py compiles the INTEGRATION.md adapter against it so its calls
// into include/mtg_boss.h and its overrides are type-checked.  Not used by any build.
#pragma once
#include <cstdint>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace mtg::graph::boss {

class BOSS {
  public:
    class Chunk {
      public:
        // a Chunk from the arrays mtg_boss_ctor_build_chunk returns
        Chunk(uint64_t alph_size, uint64_t k, const uint8_t *W, const uint64_t *last_bits,
              const uint64_t *F, const uint32_t *weights, uint64_t n, uint8_t bits_per_count);
    };
};

template <class GraphChunk>
class IGraphChunkConstructor {
  public:
    virtual ~IGraphChunkConstructor() {}
    virtual void add_sequence(std::string_view sequence, uint64_t count = 1) = 0;
    virtual void add_sequences(std::vector<std::string>&& sequences) = 0;
    virtual void add_sequences(std::vector<std::pair<std::string, uint64_t>>&& sequences) = 0;
    virtual GraphChunk build_chunk() = 0;
};

class IBOSSChunkConstructor : public IGraphChunkConstructor<BOSS::Chunk> {
  public:
    virtual ~IBOSSChunkConstructor() {}
    virtual uint64_t get_k() const = 0;
};

}  // namespace mtg::graph::boss
