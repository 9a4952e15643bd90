// comm.hpp -- the exchange layer of the multi-GPU build: one rank per GPU.
//
// RcclComm drives RCCL (ROCm's NCCL) directly on device buffers over xGMI: an all-reduce of the
// splitter histogram, an all-gather of the send-count matrix and grouped ncclSend/ncclRecv for
// the all-to-all-v of k-mer runs.  RCCL is opened with dlopen on first use (soname
// librccl.so.1, the one a PyTorch-ROCm process has already mapped), so the single-GPU library
// has no link dependency on it.
//
// LocalComm runs P ranks as P host threads of one process on one device: the same exchange
// semantics with device-to-device copies and a host barrier.  It is what the GPU tests use to
// check the distributed build on a one-GPU box (RCCL refuses two ranks on one device).
#pragma once

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

namespace mtg {

#define COMM_HIP(x)                                                                         \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess)                                                               \
            throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e_) +    \
                                     " at " #x);                                            \
    } while (0)

class Comm {
  public:
    Comm(int rank, int size) : rank_(rank), size_(size) {}
    virtual ~Comm() = default;
    int rank() const { return rank_; }
    int size() const { return size_; }
    // in place, n u64 on the device, stream-ordered
    virtual void allreduce_sum_u64(uint64_t *d, size_t n, hipStream_t s) = 0;
    // d_recv[r * n + i] = rank r's d_send[i]
    virtual void allgather_u64(const uint64_t *d_send, uint64_t *d_recv, size_t n, hipStream_t s) = 0;
    // rank j receives scnt[j] elements from d_send + soff[j] (element units, host arrays of P);
    // the elements from rank i land at d_recv + roff[i]; counts the bytes that leave this rank
    void alltoallv(const void *d_send, const uint64_t *scnt, const uint64_t *soff, void *d_recv, const uint64_t *rcnt,
                   const uint64_t *roff, size_t esz, hipStream_t s) {
        for (int j = 0; j < size_; ++j)
            if (j != rank_) sent_bytes += scnt[j] * esz;
        alltoallv_impl(d_send, scnt, soff, d_recv, rcnt, roff, esz, s);
    }
    // the same exchange enqueued on stream s without blocking the host where the transport allows it
    // (RCCL: grouped send/recv; LocalComm: copies ordered after the senders' events on their streams), so
    // the caller can sort on another stream meanwhile; the caller orders every later use of d_send and
    // d_recv after s.  A transport that cannot (the host-staged callbacks) completes it before returning
    void alltoallv_async(const void *d_send, const uint64_t *scnt, const uint64_t *soff, void *d_recv,
                         const uint64_t *rcnt, const uint64_t *roff, size_t esz, hipStream_t s) {
        for (int j = 0; j < size_; ++j)
            if (j != rank_) sent_bytes += scnt[j] * esz;
        alltoallv_async_impl(d_send, scnt, soff, d_recv, rcnt, roff, esz, s);
    }
    uint64_t sent_bytes = 0;  // bytes this rank sent to others through alltoallv
    virtual void alltoallv_impl(const void *d_send, const uint64_t *scnt, const uint64_t *soff, void *d_recv,
                                const uint64_t *rcnt, const uint64_t *roff, size_t esz, hipStream_t s) = 0;
    virtual void alltoallv_async_impl(const void *d_send, const uint64_t *scnt, const uint64_t *soff, void *d_recv,
                                      const uint64_t *rcnt, const uint64_t *roff, size_t esz, hipStream_t s) {
        alltoallv_impl(d_send, scnt, soff, d_recv, rcnt, roff, esz, s);
    }
    // a build's device work starts / ends on stream s (LocalComm's serial mode hands the device over)
    virtual void begin_build(hipStream_t) {}
    virtual void end_build(hipStream_t) {}

  protected:
    int rank_, size_;
};

// ------------------------------------------------------------------------------------- RCCL
struct RcclApi {
    ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*AllReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*AllGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char *(*GetErrorString)(ncclResult_t) = nullptr;

    static RcclApi &get() {
        static RcclApi api;
        static std::once_flag once;
        static std::string err;
        std::call_once(once, [] {
            void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
            if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
            if (!h) {
                err = std::string("cannot load RCCL: ") + dlerror();
                return;
            }
            auto sym = [&](const char *n) {
                void *p = dlsym(h, n);
                if (!p) err = std::string("RCCL symbol missing: ") + n;
                return p;
            };
            api.GetUniqueId = (decltype(api.GetUniqueId))sym("ncclGetUniqueId");
            api.CommInitRank = (decltype(api.CommInitRank))sym("ncclCommInitRank");
            api.CommDestroy = (decltype(api.CommDestroy))sym("ncclCommDestroy");
            api.AllReduce = (decltype(api.AllReduce))sym("ncclAllReduce");
            api.AllGather = (decltype(api.AllGather))sym("ncclAllGather");
            api.Send = (decltype(api.Send))sym("ncclSend");
            api.Recv = (decltype(api.Recv))sym("ncclRecv");
            api.GroupStart = (decltype(api.GroupStart))sym("ncclGroupStart");
            api.GroupEnd = (decltype(api.GroupEnd))sym("ncclGroupEnd");
            api.GetErrorString = (decltype(api.GetErrorString))sym("ncclGetErrorString");
        });
        if (!err.empty()) throw std::runtime_error(err);
        return api;
    }
};

#define RCCL_CHECK(x)                                                                       \
    do {                                                                                    \
        ncclResult_t r_ = (x);                                                              \
        if (r_ != ncclSuccess)                                                              \
            throw std::runtime_error(std::string("RCCL error ") +                           \
                                     RcclApi::get().GetErrorString(r_) + " at " #x);        \
    } while (0)

class RcclComm : public Comm {
  public:
    RcclComm(const ncclUniqueId &id, int size, int rank, int device) : Comm(rank, size) {
        COMM_HIP(hipSetDevice(device));
        RCCL_CHECK(RcclApi::get().CommInitRank(&comm_, size, id, rank));
    }
    ~RcclComm() override {
        if (comm_) (void)RcclApi::get().CommDestroy(comm_);
    }
    void allreduce_sum_u64(uint64_t *d, size_t n, hipStream_t s) override {
        RCCL_CHECK(RcclApi::get().AllReduce(d, d, n, ncclUint64, ncclSum, comm_, s));
    }
    void allgather_u64(const uint64_t *d_send, uint64_t *d_recv, size_t n, hipStream_t s) override {
        RCCL_CHECK(RcclApi::get().AllGather(d_send, d_recv, n, ncclUint64, comm_, s));
    }
    void alltoallv_impl(const void *d_send, const uint64_t *scnt, const uint64_t *soff, void *d_recv,
                   const uint64_t *rcnt, const uint64_t *roff, size_t esz, hipStream_t s) override {
        const RcclApi &api = RcclApi::get();
        // messages go out in pieces of at most 1 GiB (counts are size_t, but bounded pieces keep
        // every transfer inside RCCL's well-trodden sizes); pieces of one peer match in order
        constexpr size_t PIECE = size_t(1) << 30;
        const char *src = (const char *)d_send;
        char *dst = (char *)d_recv;
        // own slice: a device copy
        if (scnt[rank_])
            COMM_HIP(hipMemcpyAsync(dst + roff[rank_] * esz, src + soff[rank_] * esz, scnt[rank_] * esz,
                                    hipMemcpyDeviceToDevice, s));
        RCCL_CHECK(api.GroupStart());
        for (int p = 0; p < size_; ++p) {
            if (p == rank_) continue;
            for (size_t o = 0; o < scnt[p] * esz; o += PIECE)
                RCCL_CHECK(api.Send(src + soff[p] * esz + o, std::min(PIECE, scnt[p] * esz - o), ncclInt8, p,
                                    comm_, s));
            for (size_t o = 0; o < rcnt[p] * esz; o += PIECE)
                RCCL_CHECK(api.Recv(dst + roff[p] * esz + o, std::min(PIECE, rcnt[p] * esz - o), ncclInt8, p,
                                    comm_, s));
        }
        RCCL_CHECK(api.GroupEnd());
    }
    // grouped send/recv only enqueue: the host returns at once, the transfers run on s
    void alltoallv_async_impl(const void *d_send, const uint64_t *scnt, const uint64_t *soff, void *d_recv,
                              const uint64_t *rcnt, const uint64_t *roff, size_t esz, hipStream_t s) override {
        alltoallv_impl(d_send, scnt, soff, d_recv, rcnt, roff, esz, s);
    }

  private:
    ncclComm_t comm_ = nullptr;
};

// ------------------------------------------------------------------- host-staged callbacks
//
// The exchange over caller-supplied functions on host buffers (mtg_comm_create_callbacks): every
// step stages its device data through host memory, calls the function, and copies the result back.
// Any transport a caller has can carry the build this way -- torch.distributed over gloo (the
// two-process GPU test), MPI, a socket -- at PCIe + network speed instead of xGMI.
struct CommCallbacks {
    void *user = nullptr;
    // in place, n u64
    int (*allreduce_sum_u64)(void *user, uint64_t *buf, size_t n) = nullptr;
    // recv[r * n + i] = rank r's send[i]
    int (*allgather_u64)(void *user, const uint64_t *send, uint64_t *recv, size_t n) = nullptr;
    // byte all-to-all-v: the bytes for rank j are send[sum(scnt[0..j)) ..) (scnt[j] bytes), those
    // from rank i land at recv[sum(rcnt[0..i)) ..)
    int (*alltoallv)(void *user, const void *send, const uint64_t *scnt, void *recv, const uint64_t *rcnt) = nullptr;
};

class CallbackComm : public Comm {
  public:
    CallbackComm(const CommCallbacks &cb, int rank, int size) : Comm(rank, size), cb_(cb) {}
    void allreduce_sum_u64(uint64_t *d, size_t n, hipStream_t s) override {
        std::vector<uint64_t> h(n);
        COMM_HIP(hipMemcpyAsync(h.data(), d, n * 8, hipMemcpyDeviceToHost, s));
        COMM_HIP(hipStreamSynchronize(s));
        check(cb_.allreduce_sum_u64(cb_.user, h.data(), n), "all-reduce");
        COMM_HIP(hipMemcpyAsync(d, h.data(), n * 8, hipMemcpyHostToDevice, s));
        COMM_HIP(hipStreamSynchronize(s));
    }
    void allgather_u64(const uint64_t *d_send, uint64_t *d_recv, size_t n, hipStream_t s) override {
        std::vector<uint64_t> h(n), all(n * size_);
        COMM_HIP(hipMemcpyAsync(h.data(), d_send, n * 8, hipMemcpyDeviceToHost, s));
        COMM_HIP(hipStreamSynchronize(s));
        check(cb_.allgather_u64(cb_.user, h.data(), all.data(), n), "all-gather");
        COMM_HIP(hipMemcpyAsync(d_recv, all.data(), all.size() * 8, hipMemcpyHostToDevice, s));
        COMM_HIP(hipStreamSynchronize(s));
    }
    void alltoallv_impl(const void *d_send, const uint64_t *scnt, const uint64_t *soff, void *d_recv,
                   const uint64_t *rcnt, const uint64_t *roff, size_t esz, hipStream_t s) override {
        std::vector<uint64_t> sb(size_), rb(size_);
        uint64_t st = 0, rt = 0;
        for (int p = 0; p < size_; ++p) {
            sb[p] = scnt[p] * esz;
            rb[p] = rcnt[p] * esz;
            st += sb[p];
            rt += rb[p];
        }
        std::vector<char> hs(std::max<uint64_t>(st, 1)), hr(std::max<uint64_t>(rt, 1));
        uint64_t o = 0;
        for (int p = 0; p < size_; ++p) {  // the slices, packed in rank order
            if (sb[p])
                COMM_HIP(hipMemcpyAsync(hs.data() + o, (const char *)d_send + soff[p] * esz, sb[p],
                                        hipMemcpyDeviceToHost, s));
            o += sb[p];
        }
        COMM_HIP(hipStreamSynchronize(s));
        check(cb_.alltoallv(cb_.user, hs.data(), sb.data(), hr.data(), rb.data()), "all-to-all");
        o = 0;
        for (int p = 0; p < size_; ++p) {
            if (rb[p])
                COMM_HIP(hipMemcpyAsync((char *)d_recv + roff[p] * esz, hr.data() + o, rb[p], hipMemcpyHostToDevice, s));
            o += rb[p];
        }
        COMM_HIP(hipStreamSynchronize(s));  // hr is a local
    }

  private:
    static void check(int rc, const char *what) {
        if (rc != 0) throw std::runtime_error(std::string("exchange callback failed: ") + what);
    }
    CommCallbacks cb_;
};

// ------------------------------------------------------------------- in-process rank threads
// the received slices of one local all-to-all in one launch (one workgroup row per source rank)
// instead of one copy per peer: a P = 8 build made ~270 copies per rank, each a launch
constexpr int kLocalCopyMax = 64;
struct LocalCopyBatch {
    const char *src[kLocalCopyMax];
    char *dst[kLocalCopyMax];
    uint64_t bytes[kLocalCopyMax];
};

__global__ __launch_bounds__(256) void local_copy_kernel(LocalCopyBatch b) {
    const int seg = blockIdx.y;
    const char *src = b.src[seg];
    char *dst = b.dst[seg];
    const uint64_t n = b.bytes[seg];
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, T = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t al = ((uint64_t)(uintptr_t)src | (uint64_t)(uintptr_t)dst | n);
    if ((al & 15) == 0) {
        for (uint64_t i = t; i < n / 16; i += T) ((uint4 *)dst)[i] = ((const uint4 *)src)[i];
    } else if ((al & 7) == 0) {
        for (uint64_t i = t; i < n / 8; i += T) ((uint64_t *)dst)[i] = ((const uint64_t *)src)[i];
    } else if ((al & 3) == 0) {
        for (uint64_t i = t; i < n / 4; i += T) ((uint32_t *)dst)[i] = ((const uint32_t *)src)[i];
    } else {
        for (uint64_t i = t; i < n; i += T) dst[i] = src[i];
    }
}

struct LocalGroup {
    explicit LocalGroup(int n) : size(n), slots(n), host(n), held_ms(n, 0.0) {}
    int size;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t generation = 0;
    struct Slot {
        const void *ptr = nullptr;
        std::vector<uint64_t> soff, scnt;
        hipEvent_t ready = nullptr;  // async all-to-all: the send buffer is complete on its rank's stream
        hipEvent_t done = nullptr;   // async all-to-all: this rank's copies out of its peers' buffers ended
    };
    std::vector<Slot> slots;
    std::vector<std::vector<uint64_t>> host;

    std::string failure;  // first error any rank reported: every barrier then throws it

    // serial mode (MTG_LOCAL_SERIAL=1, tools/dist_sim.py): one rank at a time owns the device, from
    // build start to its next exchange and from there to the next, so every rank's device time is
    // its own work (held_ms) and the step's wall time is the SUM of the ranks' work
    bool serial = false;
    std::mutex gpu;
    std::vector<double> held_ms;

    // a rank that failed says so (fail), and peers waiting in a barrier throw its message at once;
    // a rank that dies without failing never arrives, and the others give up after a minute
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (!failure.empty()) throw std::runtime_error(failure);
        const uint64_t gen = generation;
        if (++arrived == size) {
            arrived = 0;
            ++generation;
            cv.notify_all();
            return;
        }
        const bool ok = cv.wait_for(lk, std::chrono::seconds(60),
                                    [&] { return generation != gen || !failure.empty(); });
        if (generation != gen) return;
        --arrived;
        throw std::runtime_error(ok ? failure : std::string("local exchange group: a peer rank did not arrive"));
    }
    void fail(const std::string &msg) {
        std::lock_guard<std::mutex> lk(mu);
        if (failure.empty()) failure = msg;
        cv.notify_all();
    }
};

class LocalComm : public Comm {
  public:
    LocalComm(std::shared_ptr<LocalGroup> g, int rank) : Comm(rank, g->size), g_(std::move(g)) {}
    void begin_build(hipStream_t) override { hold(); }
    void end_build(hipStream_t s) override {
        if (!held_) return;
        (void)hipStreamSynchronize(s);
        drop();
    }
    // this rank's device time in serial mode (ms), optionally reset
    double held_ms(bool reset) {
        std::lock_guard<std::mutex> lk(g_->mu);
        const double v = g_->held_ms[rank_];
        if (reset) g_->held_ms[rank_] = 0;
        return v;
    }
    void allreduce_sum_u64(uint64_t *d, size_t n, hipStream_t s) override {
        auto &mine = g_->host[rank_];
        mine.resize(n);
        COMM_HIP(hipMemcpyAsync(mine.data(), d, n * 8, hipMemcpyDeviceToHost, s));
        COMM_HIP(hipStreamSynchronize(s));
        wait();
        std::vector<uint64_t> sum(n, 0);
        for (int r = 0; r < size_; ++r)
            for (size_t i = 0; i < n; ++i) sum[i] += g_->host[r][i];
        wait();
        hold();
        COMM_HIP(hipMemcpyAsync(d, sum.data(), n * 8, hipMemcpyHostToDevice, s));
        COMM_HIP(hipStreamSynchronize(s));
    }
    void allgather_u64(const uint64_t *d_send, uint64_t *d_recv, size_t n, hipStream_t s) override {
        auto &mine = g_->host[rank_];
        mine.resize(n);
        COMM_HIP(hipMemcpyAsync(mine.data(), d_send, n * 8, hipMemcpyDeviceToHost, s));
        COMM_HIP(hipStreamSynchronize(s));
        wait();
        std::vector<uint64_t> all(n * size_);
        for (int r = 0; r < size_; ++r) std::copy(g_->host[r].begin(), g_->host[r].end(), all.begin() + r * n);
        wait();
        hold();
        COMM_HIP(hipMemcpyAsync(d_recv, all.data(), all.size() * 8, hipMemcpyHostToDevice, s));
        COMM_HIP(hipStreamSynchronize(s));
    }
    void alltoallv_impl(const void *d_send, const uint64_t *scnt, const uint64_t *soff, void *d_recv,
                   const uint64_t *rcnt, const uint64_t *roff, size_t esz, hipStream_t s) override {
        COMM_HIP(hipStreamSynchronize(s));  // the send buffer is complete before peers read it
        auto &slot = g_->slots[rank_];
        slot.ptr = d_send;
        slot.soff.assign(soff, soff + size_);
        slot.scnt.assign(scnt, scnt + size_);
        wait();
        for (int i = 0; i < size_; ++i)
            if (g_->slots[i].scnt[rank_] != rcnt[i]) {
                const std::string msg = "local all-to-all: rank " + std::to_string(rank_) + " expects " +
                                        std::to_string(rcnt[i]) + " elements from rank " + std::to_string(i) +
                                        ", which sends " + std::to_string(g_->slots[i].scnt[rank_]);
                g_->fail(msg);  // peers in the next barrier throw this too, without waiting
                throw std::runtime_error(msg);
            }
        hold();
        if (size_ <= kLocalCopyMax) {
            LocalCopyBatch batch{};
            uint64_t most = 0;
            for (int i = 0; i < size_; ++i) {
                const auto &src = g_->slots[i];
                batch.src[i] = (const char *)src.ptr + src.soff[rank_] * esz;
                batch.dst[i] = (char *)d_recv + roff[i] * esz;
                batch.bytes[i] = rcnt[i] * esz;
                most = std::max<uint64_t>(most, rcnt[i] * esz);
            }
            if (most) {
                const unsigned gx = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((most + 16383) / 16384, 2048));
                local_copy_kernel<<<dim3(gx, (unsigned)size_), dim3(256), 0, s>>>(batch);
                COMM_HIP(hipGetLastError());
            }
        } else {
            for (int i = 0; i < size_; ++i) {
                const auto &src = g_->slots[i];
                if (rcnt[i])
                    COMM_HIP(hipMemcpyAsync((char *)d_recv + roff[i] * esz,
                                            (const char *)src.ptr + src.soff[rank_] * esz, rcnt[i] * esz,
                                            hipMemcpyDeviceToDevice, s));
            }
        }
        COMM_HIP(hipStreamSynchronize(s));
        wait();  // nobody reuses its send buffer while a peer still copies from it
        hold();
    }
    ~LocalComm() override {
        if (ev_ready_) (void)hipEventDestroy(ev_ready_);
        if (ev_done_) (void)hipEventDestroy(ev_done_);
    }
    // the all-to-all ordered by events instead of host waits: every rank publishes its send buffer with an
    // event recorded on its stream s at the call, each receiver's copy kernel waits for its senders'
    // events on ITS stream s, and each sender's s then waits for every receiver's copy-done event (its
    // send buffer stays valid until then).  The two host barriers only exchange pointers and event
    // handles, so the host returns with the copies still queued.  An event is re-recorded only in the
    // next call, after the barrier every peer passes once it has queued its waits on the old record.
    void alltoallv_async_impl(const void *d_send, const uint64_t *scnt, const uint64_t *soff, void *d_recv,
                              const uint64_t *rcnt, const uint64_t *roff, size_t esz, hipStream_t s) override {
        if (g_->serial || size_ > kLocalCopyMax) {  // serial mode times each rank's device work alone
            alltoallv_impl(d_send, scnt, soff, d_recv, rcnt, roff, esz, s);
            return;
        }
        if (!ev_ready_) {
            COMM_HIP(hipEventCreateWithFlags(&ev_ready_, hipEventDisableTiming));
            COMM_HIP(hipEventCreateWithFlags(&ev_done_, hipEventDisableTiming));
        }
        COMM_HIP(hipEventRecord(ev_ready_, s));
        auto &slot = g_->slots[rank_];
        slot.ptr = d_send;
        slot.soff.assign(soff, soff + size_);
        slot.scnt.assign(scnt, scnt + size_);
        slot.ready = ev_ready_;
        wait();
        LocalCopyBatch batch{};
        uint64_t most = 0;
        for (int i = 0; i < size_; ++i) {
            const auto &src = g_->slots[i];
            if (src.scnt[rank_] != rcnt[i]) {
                const std::string msg = "local all-to-all: rank " + std::to_string(rank_) + " expects " +
                                        std::to_string(rcnt[i]) + " elements from rank " + std::to_string(i) +
                                        ", which sends " + std::to_string(src.scnt[rank_]);
                g_->fail(msg);
                throw std::runtime_error(msg);
            }
            if (i != rank_ && rcnt[i]) COMM_HIP(hipStreamWaitEvent(s, src.ready, 0));
            batch.src[i] = (const char *)src.ptr + src.soff[rank_] * esz;
            batch.dst[i] = (char *)d_recv + roff[i] * esz;
            batch.bytes[i] = rcnt[i] * esz;
            most = std::max<uint64_t>(most, rcnt[i] * esz);
        }
        if (most) {
            const unsigned gx = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((most + 16383) / 16384, 2048));
            local_copy_kernel<<<dim3(gx, (unsigned)size_), dim3(256), 0, s>>>(batch);
            COMM_HIP(hipGetLastError());
        }
        COMM_HIP(hipEventRecord(ev_done_, s));
        slot.done = ev_done_;
        wait();
        for (int j = 0; j < size_; ++j)
            if (j != rank_ && scnt[j]) COMM_HIP(hipStreamWaitEvent(s, g_->slots[j].done, 0));
    }

  private:
    hipEvent_t ev_ready_ = nullptr, ev_done_ = nullptr;
    // serial mode: take / hand over the device (the stream is drained before every hand-over)
    void hold() {
        if (!g_->serial || held_) return;
        g_->gpu.lock();
        held_ = true;
        t0_ = std::chrono::steady_clock::now();
    }
    void drop() {
        if (!held_) return;
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0_).count();
        {
            std::lock_guard<std::mutex> lk(g_->mu);
            g_->held_ms[rank_] += ms;
        }
        held_ = false;
        g_->gpu.unlock();
    }
    void wait() {
        drop();
        g_->barrier();
    }
    std::shared_ptr<LocalGroup> g_;
    bool held_ = false;
    std::chrono::steady_clock::time_point t0_;
};

}  // namespace mtg
