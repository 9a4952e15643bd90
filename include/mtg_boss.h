/*
 * mtg_boss.h -- C ABI of the MI355X BOSS chunk constructor (libmtg_boss.so).
 *
 * Drop-in boundary for MetaGraph's in-memory succinct `build` path.  Each entry point replaces
 * one member of the reference's chunk-constructor interface (paths relative to
 * /root/reference/metagraph/src):
 *
 *   mtg_boss_ctor_create        IBOSSChunkConstructor::initialize
 *                               graph/representation/succinct/boss_chunk_construct.hpp:18-34,
 *                               boss_chunk_construct.cpp:1134-1178 (same 9 parameters + device)
 *   mtg_boss_ctor_add_sequences IBOSSChunkConstructor::add_sequences(vector<pair<string,u64>>&&)
 *                               boss_chunk_construct.hpp:26-30 (thread-safe, copies the input)
 *   mtg_boss_ctor_add_sequence  IBOSSChunkConstructor::add_sequence(string_view, u64 count)
 *   mtg_boss_ctor_build_chunk   IBOSSChunkConstructor::build_chunk -> BOSS::Chunk
 *                               (boss_chunk.hpp:19-104: W, last, F, weights, k, alph_size = 5)
 *   mtg_boss_ctor_get_k         IBOSSChunkConstructor::get_k (BOSS k = DBG k - 1)
 *   mtg_boss_chunk_free / mtg_boss_ctor_destroy   the destructors
 *   mtg_last_error              logger->error + exit(1) / throw of the reference become
 *                               negative return codes plus this message
 *
 * Beyond the reference's interface, for callers that already hold reads in HBM (benchmarks,
 * multi-GPU shards): mtg_boss_build_device runs the whole path on a device buffer and leaves
 * the BOSS arrays in device memory; mtg_boss_last_timings reports per-stage device times.
 *
 * Multi-GPU (one process per GPU, RCCL over xGMI): every rank calls the *_dist variant with its
 * own reads and gets the chunk of one range of BOSS order; the rank chunks concatenate in rank
 * order with BOSS::Chunk::extend (boss_chunk.cpp:230-270) into the chunk a single build of all
 * reads returns: one exchange-based build where the reference shards by suffix.
 *
 * The suffix-sharded route itself (`build --suffix-len`, `concatenate --clear-dummy`,
 * cli/build.cpp:102-155, 358-456) runs too: a constructor created with a filter_suffix builds the
 * chunk of that node suffix, and mtg_boss_write_dbg with mask_dummy = 2 prunes the concatenated
 * chunks' redundant source dummies.
 *
 * No torch types, no C++ types: plain pointers and sizes.  All functions are thread-safe
 * except that one constructor must not be built and added to at the same time.
 */
#ifndef MTG_BOSS_H
#define MTG_BOSS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MTG_BOSS_ABI_VERSION 8

/* container types of the reference (kmer::ContainerType) */
#define MTG_CONTAINER_VECTOR 0
#define MTG_CONTAINER_VECTOR_DISK 1

/* return codes */
#define MTG_OK 0
#define MTG_ERR_INVALID_K -1        /* k not in [1, 84]      (reference: exit(1)) */
#define MTG_ERR_COUNT_WIDTH -2      /* bits_per_count > 32   (reference: runtime_error) */
#define MTG_ERR_UNSUPPORTED -3      /* a multi-GPU build with a filter suffix */
#define MTG_ERR_DEVICE -4           /* HIP runtime / kernel failure */
#define MTG_ERR_ARGUMENT -5
#define MTG_ERR_NO_DEVICE -6        /* no MI355X visible: the product path never falls back */

typedef struct mtg_boss_params {
    uint64_t k;                  /* BOSS k (node length) = DBG k - 1, in [1, 84] */
    int both_strands;            /* canonical mode: add reverse complements */
    uint8_t bits_per_count;      /* 0 = no weights; else --count-width (<= 32) */
    const char *filter_suffix;   /* NULL / "": the full construction; else chars of "$ACGT", shorter
                                    than k + 1: the chunk of the (k+1)-mers whose node ends with it
                                    (boss_chunk_construct.cpp:946-1013); copied at create */
    uint64_t num_threads;        /* host threads for input staging */
    double memory_preallocated;  /* bytes of device memory the build may use (0 = all free HBM);
                                    larger inputs are built in key-range batches */
    int container_type;          /* MTG_CONTAINER_VECTOR, or MTG_CONTAINER_VECTOR_DISK (--disk-swap):
                                    the bounded-memory build, in key-range batches; when even the real
                                    edges would not fit memory_preallocated, build_chunk spills: one
                                    range's edges in HBM at a time, the rest in host memory / swap_dir */
    const char *swap_dir;        /* the disk container's spill files go here (copied at create) */
    uint64_t disk_cap_bytes;     /* at most this many bytes of spill files; further blocks stay in RAM */
    int device_id;               /* HIP device ordinal */
} mtg_boss_params;

typedef struct mtg_boss_ctor mtg_boss_ctor;

/* BOSS::Chunk in host memory (arrays of n entries including the leading row 0).  The arrays are
   pinned host blocks owned by the chunk: release them with mtg_boss_chunk_free. */
typedef struct mtg_boss_chunk {
    uint64_t k;
    uint64_t alph_size;          /* 5: $ACGT */
    uint64_t n;
    uint8_t *W;                  /* n labels 0..9 (int_vector width 4 in the reference) */
    uint64_t *last;              /* n bits, packed: row i is bit i % 64 of word i / 64 (the
                                    sdsl::bit_vector layout of the reference's last_) */
    uint32_t *weights;           /* n weights or NULL (bits_per_count == 0) */
    uint64_t F[5];
    uint8_t bits_per_count;
    uint64_t n_real;             /* real (non-dummy) edges */
    uint64_t n_dummy;            /* dummy edges incl. the main dummy row */
} mtg_boss_chunk;

/* BOSS::Chunk left in device memory (owned by the constructor, valid until its next build) */
typedef struct mtg_boss_device_chunk {
    uint64_t k;
    uint64_t n;
    uint8_t *W;                  /* device pointers */
    uint8_t *last;
    uint32_t *weights;
    uint64_t F[5];
    uint64_t n_real;
    uint64_t n_dummy;
} mtg_boss_device_chunk;

typedef struct mtg_boss_timings {
    double total_ms;             /* device time of the whole path (events on the build stream) */
    double extract_ms;           /* K1 */
    double sort_ms;              /* K2 over the extracted k-mers */
    double unique_ms;            /* K3 */
    double rc_ms;                /* K4 incl. its re-sort */
    double dummy_ms;             /* K5/K6 incl. dummy sort + unique */
    double merge_ms;             /* K7 */
    double emit_ms;              /* K8 */
    double radix_pass_ms;        /* K2's first partition pass (MSD) or average onesweep pass (LSD) */
    double radix_bytes;          /* algorithmic bytes of that launch: 2 n (key + count) */
    uint64_t radix_launches;     /* launches averaged into radix_pass_ms */
    uint64_t n_positions;        /* window starts offered to the extractor */
    uint64_t n_extracted;        /* valid k-mers extracted (N) */
    uint64_t n_unique;           /* distinct k-mers collected (U) */
    uint64_t n_real;             /* real edges after rc augmentation */
    uint64_t n_dummy;            /* dummy edges (sinks + all source levels) */
    uint64_t n_rows;             /* BOSS rows incl. row 0 */
    double exchange_ms;          /* multi-GPU: time inside the exchanges (RCCL) */
    uint64_t n_sent;             /* multi-GPU: elements sent to other ranks */
    uint64_t world;              /* ranks of the build (1 = single GPU) */
    /* host-buffer builds (mtg_boss_ctor_build_chunk): wall times of the host-side stages */
    double stage_ms;             /* add_* calls since the previous build (reads packed to 2-bit codes + a
                                    valid mask in pinned memory, DMA'd to HBM piece by piece meanwhile) */
    double h2d_ms;               /* the wait for the last read pieces + their unpack in HBM */
    double d2h_ms;               /* W, packed last, weights -> pinned host blocks */
    double host_total_ms;        /* the whole build_chunk call */
    uint64_t n_batches;          /* key-range batches of the build (1 = the input fit at once) */
    uint64_t peak_bytes;         /* device workspace held at the end of the build */
    double input_ms;             /* host-buffer builds: KMC decode + FASTA split on the device (incl. their copies) */
    uint64_t spilled_bytes;      /* bytes the build kept outside HBM (the disk container's spill; 0 = none) */
    uint64_t spec_levels;        /* speculative final MSD levels that completed (sample-sized buckets) */
    uint64_t spec_fine_levels;   /* of those, levels sampled per tile (the final level of 3-level plans) */
    uint64_t spec_fallbacks;     /* speculative levels that overflowed and reran as the exact level */
    uint64_t collect_mode;       /* how the real k-mers were collected: 0 one pass, 1 key ranges re-scanning
                                    the reads (both strands), 2 canonical rounds of the fused extraction */
    uint64_t sent_bytes;         /* multi-GPU: bytes this rank sent to the other ranks (every exchange) */
    uint64_t spec_l1;            /* 1: the fused extraction scattered into the speculative level-1 layout
                                    (a sampled histogram pass) */
    uint64_t cached_bytes;       /* device blocks the workspace keeps idle for the next build (counted in
                                    peak_bytes; freed when a build ends without reusing them, or by
                                    mtg_boss_ctor_trim) */
    double exchange_hidden_ms;   /* multi-GPU: exchange time spent while the build stream sorted (the pieces of
                                    exchange 1 in flight under the owner sort of the previous piece) */
    uint64_t coresident;         /* multi-GPU: ranks sharing this rank's GPU (same host name and PCI bus id);
                                    they split its free HBM when planning rounds */
} mtg_boss_timings;

int mtg_boss_abi_version(void);
const char *mtg_last_error(void);

mtg_boss_ctor *mtg_boss_ctor_create(const mtg_boss_params *params);
void mtg_boss_ctor_destroy(mtg_boss_ctor *ctor);
uint64_t mtg_boss_ctor_get_k(const mtg_boss_ctor *ctor);
/* frees the device memory the constructor holds between builds: the blocks its workspace keeps idle
   (timings' cached_bytes) and the last build's stage buffers; the last build's device chunk arrays
   (W, last, weights) stay valid.  A build also frees, when it ends, the kept blocks it did not reuse */
int mtg_boss_ctor_trim(mtg_boss_ctor *ctor);

/* n sequences, seqs[i] of lens[i] bytes, counts[i] (NULL = all 1).  Copies the input. */
int mtg_boss_ctor_add_sequences(mtg_boss_ctor *ctor, const char *const *seqs,
                                const uint64_t *lens, const uint64_t *counts, size_t n);
int mtg_boss_ctor_add_sequence(mtg_boss_ctor *ctor, const char *seq, uint64_t len,
                               uint64_t count);
/* one packed buffer: n sequences back to back, offsets[n + 1] */
int mtg_boss_ctor_add_packed(mtg_boss_ctor *ctor, const char *data, const uint64_t *offsets,
                             const uint64_t *counts, size_t n);

/*
 * A FASTA or FASTQ file (plain or gzip) as input, the reference's parse_sequences ->
 * read_fasta_file_critical path (cli/parse_sequences.hpp:103-151, seq_io/sequence_io.cpp:364-405)
 * and push_sequences' one-thread-per-file loop (cli/build.cpp:31-56): the calling thread reads and
 * inflates the file into pinned memory; at build time its bytes go to HBM in one copy and are split
 * into records on the device (kseq rules: FASTA header lines start with '>', sequence lines are
 * joined, line ends dropped; FASTQ four-line records).  Each record is one sequence of count 1.
 * Thread-safe; call it concurrently for different files.
 */
int mtg_boss_ctor_add_fasta(mtg_boss_ctor *ctor, const char *path);

/*
 * A KMC1 k-mer counter database (`<base>.kmc_pre` + `<base>.kmc_suf`; either name or the base) as
 * input: seq_io::read_kmers (seq_io/kmc_parser.cpp:27-62) + the build's KMC branch
 * (cli/parse_sequences.hpp:50-101).  Every k-mer with min_count <= count < max_count becomes a
 * one-k-mer sequence with that count; with call_both_from_canonical and a database of canonical
 * k-mers, its reverse complement too (the reference passes graph_mode != CANONICAL).  The
 * records are decoded on the device at build time.  Reference defaults: 1, 2^32 - 1.
 */
int mtg_boss_ctor_add_kmc(mtg_boss_ctor *ctor, const char *kmc_path, uint64_t min_count,
                          uint64_t max_count, int call_both_from_canonical);

/*
 * A KMC1 database decoded straight into device memory, as mtg_boss_ctor_add_kmc decodes it at build
 * time (k bases + '$' per record, its reverse complement after it with call_both_from_canonical on
 * a canonical database), with per-read starts and counts: the input of mtg_boss_build_device[_dist]
 * for a build whose KMC input is already resident in HBM (BASELINE config 5).  Free with
 * mtg_device_reads_free.
 */
typedef struct mtg_device_reads {
    uint8_t *seq;                /* device pointers */
    uint64_t seq_len;
    uint64_t *read_starts;
    uint32_t *counts;
    uint64_t n_reads;            /* records (x2 with reverse complements) */
    int device_id;
} mtg_device_reads;
int mtg_kmc_load_device(const char *kmc_path, uint64_t min_count, uint64_t max_count,
                        int call_both_from_canonical, int device_id, mtg_device_reads *out);
void mtg_device_reads_free(mtg_device_reads *reads);

/*
 * The builder's own k-mer counter: counts the k-mers (k <= 32; canonical = KMC's canonical form,
 * the lexicographically smaller strand) of device-resident reads on the constructor's device and
 * writes them as a KMC1 database <outbase>.kmc_pre / .kmc_suf (record order, prefix table and
 * header as KMC writes them; counts saturate at the counter_size-byte maximum).  Input generator
 * for BASELINE config 5 (the reference takes its KMC databases from KMC itself).  *n_written (may
 * be NULL) = records written.
 */
int mtg_kmc_write_device(mtg_boss_ctor *ctor, const uint8_t *d_seq, uint64_t seq_len, unsigned k,
                         int canonical, unsigned counter_size, unsigned lut_len, const char *outbase,
                         uint64_t *n_written);

/* builds from everything added so far, returns host arrays; clears the added input */
int mtg_boss_ctor_build_chunk(mtg_boss_ctor *ctor, mtg_boss_chunk *out);
void mtg_boss_chunk_free(mtg_boss_chunk *chunk);

/*
 * Device-resident input: `d_seq` holds the reads back to back, each followed by at least one
 * byte outside {A,C,G,T,U,a,c,g,t,u} (so no k-mer spans two reads).  d_read_starts/d_counts
 * (both NULL, or n_reads entries) give per-read counts for --count-kmers.  `stream` is a
 * hipStream_t (NULL = the constructor's own stream).  Arrays stay in device memory.
 */
int mtg_boss_build_device(mtg_boss_ctor *ctor, const uint8_t *d_seq, uint64_t seq_len,
                          const uint64_t *d_read_starts, const uint32_t *d_counts,
                          uint64_t n_reads, void *stream, mtg_boss_device_chunk *out);

int mtg_boss_last_timings(const mtg_boss_ctor *ctor, mtg_boss_timings *out);

/*
 * Multi-GPU exchange.  mtg_comm_get_unique_id on one rank, broadcast the 128 bytes (e.g. with
 * torch.distributed or MPI), then mtg_comm_create_rccl on every rank with its device.
 * mtg_comm_create_local makes `world` ranks inside one process sharing one device (each rank
 * builds from its own host thread) -- the same exchange semantics without RCCL, for tests.
 */
#define MTG_COMM_ID_BYTES 128
typedef struct mtg_comm mtg_comm;
int mtg_comm_get_unique_id(uint8_t *id /* MTG_COMM_ID_BYTES */);
mtg_comm *mtg_comm_create_rccl(const uint8_t *id, int world, int rank, int device_id);
int mtg_comm_create_local(int world, mtg_comm **comms /* world entries */);
void mtg_comm_destroy(mtg_comm *comm);
int mtg_comm_rank(const mtg_comm *comm);
int mtg_comm_size(const mtg_comm *comm);
/*
 * Local groups created with MTG_LOCAL_SERIAL=1 in the environment hand the device to one rank at a
 * time (from build start to its next exchange, and between exchanges): a step's wall time is then
 * the sum of the ranks' work.  Returns this rank's accumulated device time in ms (reset != 0 zeroes
 * it), -1 for other communicators.  A measurement aid (tools/dist_sim.py), not a build mode.
 */
double mtg_comm_local_held_ms(mtg_comm *comm, int reset);

/*
 * The same exchange over caller-supplied functions on HOST buffers (each returns 0 on success): the
 * library stages every step's device data through host memory and calls them from the building
 * thread.  Any transport carries the build this way (torch.distributed over gloo, MPI, sockets);
 * RCCL over xGMI stays the fast path.  alltoallv: the bytes for rank j are send[sum scnt[0..j)]..
 * (scnt[j] bytes), the bytes from rank i land at recv[sum rcnt[0..i)]...
 */
typedef struct mtg_comm_callbacks {
    void *user;
    int rank;
    int world;
    int (*allreduce_sum_u64)(void *user, uint64_t *buf, size_t n);
    int (*allgather_u64)(void *user, const uint64_t *send, uint64_t *recv, size_t n);
    int (*alltoallv)(void *user, const void *send, const uint64_t *scnt, void *recv, const uint64_t *rcnt);
} mtg_comm_callbacks;
mtg_comm *mtg_comm_create_callbacks(const mtg_comm_callbacks *callbacks);

/* this rank's chunk of the global build (host input staged with mtg_boss_ctor_add_*) */
int mtg_boss_ctor_build_chunk_dist(mtg_boss_ctor *ctor, mtg_comm *comm, mtg_boss_chunk *out);
/* the same on device-resident reads */
int mtg_boss_build_device_dist(mtg_boss_ctor *ctor, mtg_comm *comm, const uint8_t *d_seq,
                               uint64_t seq_len, const uint64_t *d_read_starts,
                               const uint32_t *d_counts, uint64_t n_reads, void *stream,
                               mtg_boss_device_chunk *out);
/* the range split: bounds[0..world] over n_prefixes buckets, balanced on hist (host) */
int mtg_dist_bounds(const uint64_t *hist, uint64_t n_prefixes, int world, uint64_t *bounds);
/* the identity a rank all-gathers to count the ranks sharing its GPU: a hash of the host name (or
   MTG_HOST_ID) and the device's PCI bus id; and that count for `rank` over every rank's identity
   (timings' coresident; the ranks on one GPU split its free HBM when they plan rounds) */
uint64_t mtg_device_identity(const char *host, const char *pci_bus_id);
uint32_t mtg_dist_coresident(const uint64_t *ids, int world, int rank);

/*
 * The graph files `metagraph build` writes from a chunk (cli/build.cpp:323-352; DBGSuccinct::serialize,
 * dbg_succinct.cpp:754-790): <outbase>.dbg (BOSS F / k / state, W, last, the graph mode, the
 * suffix-range index), <outbase>.edgemask with mask_dummy (1 = --mask-dummy: the valid edges of
 * mark_all_dummy_edges, dbg_succinct.cpp:839-870; 2 = concatenate --clear-dummy: the redundant
 * source dummies of suffix chunks erased first, boss.cpp:1443-1650, and no weights file, as
 * build_boss_from_chunks takes none), <outbase>.dbg.weights when the chunk has
 * weights (node_weights.cpp:62-68).  graph_mode: 0 basic, 1 canonical.  suffix_length < 0 = the
 * build's default min(10, k).  *n_valid (may be NULL) = edges left valid by the mask (`nodes (k)` of
 * `metagraph stats`), else n - 1.  Host code: needs no device.  The sdsl-lite containers inside
 * (wt_huff<> for W, bit_vector_stat for last, bit_vector_small for the mask, int_vector<> for the
 * weights) are written field by field as sdsl-lite 2.x serializes them (csrc/sdsl_io.hpp, DESIGN.md
 * §9); no reference-written file exists to pin their bytes.
 */
int mtg_boss_write_dbg(const mtg_boss_chunk *chunk, const char *outbase, int graph_mode, int mask_dummy,
                       int64_t suffix_length, uint64_t *n_valid);

/* One sdsl-lite container of the graph files written alone to `path` (the layout tests): kind 0
 * bit_vector_stat over `nbits` bits of `data`, 1 bit_vector_small (sd_vector or rrr_vector<63>,
 * whichever predict_size picks), 2 wt_huff<> over `nbits` bytes of `data`, 3 the sd_vector<> of the
 * set bits, 4 rrr_vector<63>. */
int mtg_sdsl_write(const char *path, int kind, const void *data, uint64_t nbits);

typedef struct mtg_dbg_file {
    uint64_t k;
    uint64_t n;                  /* rows incl. row 0 */
    uint64_t F[5];
    uint64_t state;              /* 3 = STAT */
    uint64_t mode;               /* 0 basic, 1 canonical */
    uint64_t suffix_length;
    uint64_t n_ranges;           /* 4^suffix_length */
    uint8_t *W;                  /* n labels */
    uint64_t *last;              /* n bits, packed */
    uint64_t *ranges;            /* 2 * n_ranges: first and last edge of each indexed suffix */
    uint64_t *valid;             /* packed .edgemask bits, NULL when there is none */
    uint64_t n_valid;
} mtg_dbg_file;
int mtg_boss_read_dbg(const char *outbase, mtg_dbg_file *out);
void mtg_dbg_file_free(mtg_dbg_file *file);

/* the library's pool of pinned host blocks (chunk arrays, staged FASTA files): bytes held by spare
   blocks (at most 4 GiB; blocks above that are unpinned when freed), and a trim that unpins them all */
uint64_t mtg_host_pool_bytes(void);
void mtg_host_pool_trim(void);

/* encode table of the extractor (kmer/alphabets.hpp:127-143) evaluated by the device function on
   the host: out[c] in {0, 1, 2, 3, 4 = invalid} for every byte c (256 entries) */
void mtg_dna_encode_table(uint8_t *out);

/* device-memory helpers for callers without their own HIP runtime (ctypes, cgo, JNI) */
void *mtg_device_alloc(int device_id, uint64_t bytes);
int mtg_device_free(void *ptr);
int mtg_memcpy_h2d(void *dst, const void *src, uint64_t bytes);
int mtg_memcpy_d2h(void *dst, const void *src, uint64_t bytes);
int mtg_device_count(void);
/* device-to-device copy of `bytes` (multiple of 16, 16-byte aligned) by a streaming 16-byte-lane
   kernel on `stream` (NULL = default): the bench's achievable-HBM-bandwidth probe */
int mtg_device_copy(void *dst, const void *src, uint64_t bytes, void *stream);
int mtg_device_synchronize(int device_id);

#ifdef __cplusplus
}
#endif

#endif /* MTG_BOSS_H */
