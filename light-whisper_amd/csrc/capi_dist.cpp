// extern "C": the native multi-GPU collectives (north_star: "RCCL over xGMI used only to broadcast Q8
// weights and gather token streams").  One process per GPU; the host (Rust via the C ABI, or bench.py / qasr.dist
// over ctypes) exchanges the 128-byte unique id out of band, then every rank opens a communicator on its device.
//   * qasr_dist_broadcast_weights: ONE ncclBroadcast over the model's whole weight blob (rank 0 loaded or generated
//     it, the others hold shells of the identical layout, qasr_model_open_shell) — a single large message, the shape
//     a per-link-bound ring over xGMI wants — then a wrapping 64-bit checksum per rank, all-gathered and compared;
//   * qasr_dist_gather_tokens: every rank's per-segment token ids to every rank (two all-gathers: the counts, then
//     the ragged payload padded to the largest rank);
//   * qasr_dist_agree: one int32 all-gather of every rank's local status before a collective (failure agreement).
// Neither runs inside a timed step.  The reference has no multi-GPU path.
//
// Liveness: every call is waited for against a deadline (qasr_dist_init_deadline's timeout, default
// QASR_DIST_TIMEOUT_MS or 300 s): the init on a helper thread the caller stops waiting for, a collective's completion
// polled through hipStreamQuery and ncclCommGetAsyncError.  A rank that never joins
// (it crashed before init, or inside it) or never enters a collective makes the others return QASR_E_BACKEND at the
// deadline — the communicator is then aborted (ncclCommAbort) and every later call on it fails at once — instead of
// hanging the job (the reference's expectation: the engine process exits and the Rust host sees it,
// funasr_service.rs:1367-1385).
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "../../include/qasr.h"
#include "capi_handles.h"
#include "capi_util.h"

using namespace qasr;

struct qasr_comm {
    ncclComm_t c = nullptr;
    int rank = 0, world = 1, device = 0;
    hipStream_t st = nullptr;
    double timeout_ms = 300000.0;
    bool dead = false;   // aborted after a deadline or an asynchronous error: every later call fails
    ~qasr_comm() {
        if (c) (void)(dead ? ncclCommAbort(c) : ncclCommDestroy(c));
        if (st) (void)hipStreamDestroy(st);
    }
};

namespace {

#define QASR_NCCL(x)                                                                                              \
    do {                                                                                                          \
        const ncclResult_t r_ = (x);                                                                              \
        if (r_ != ncclSuccess) throw Error(QASR_E_BACKEND, std::string("RCCL: ") + #x + ": " + ncclGetErrorString(r_)); \
    } while (0)
// a call on the (non-blocking) communicator c, settled against deadline dl
#define QASR_NCCL_C(c, dline, x) comm_settle((c), (x), #x, (dline).t)

// wrapping 64-bit sum of a blob (bytes % 8 == 0): order-independent, so every rank's value is the same for the
// same bytes whatever the reduction order
__global__ void k_blob_checksum(const unsigned long long* __restrict__ p, size_t n, unsigned long long* out) {
    __shared__ unsigned long long part[256];
    unsigned long long s = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += p[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) atomicAdd(out, part[0]);
}

double env_timeout_ms() {
    const char* e = getenv("QASR_DIST_TIMEOUT_MS");
    const double v = e && *e ? atof(e) : 0.0;
    return v > 0 ? v : 300000.0;
}

// QASR_DIST_DEBUG=1: the deadline machinery's steps on stderr (ms since the process's first call)
void dbg(const char* fmt, ...) {
    static const bool on = getenv("QASR_DIST_DEBUG") && atoi(getenv("QASR_DIST_DEBUG")) != 0;
    if (!on) return;
    static const auto t0 = std::chrono::steady_clock::now();
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    fprintf(stderr, "[qasr dist %9.1f ms] ", ms);
    va_list ap;
    va_start(ap, fmt);
    vfprintf(stderr, fmt, ap);
    va_end(ap);
    fputc('\n', stderr);
    fflush(stderr);
}

// abort the communicator (it may have work in flight that will never complete) and fail
[[noreturn]] void comm_fail(qasr_comm* c, const std::string& what) {
    dbg("fail: %s; aborting the communicator", what.c_str());
    if (c->c && !c->dead) (void)ncclCommAbort(c->c);
    dbg("abort returned");
    c->c = nullptr;
    c->dead = true;
    throw Error(QASR_E_BACKEND, "RCCL: " + what);
}

// a non-blocking communicator's call returned: poll until it is no longer in progress, within the deadline
void comm_settle(qasr_comm* c, ncclResult_t r, const char* what, std::chrono::steady_clock::time_point t_end) {
    for (;;) {
        if (r == ncclSuccess) return;
        if (r != ncclInProgress) comm_fail(c, std::string(what) + ": " + ncclGetErrorString(r));
        if (std::chrono::steady_clock::now() > t_end)
            comm_fail(c, std::string(what) + ": timed out (a rank did not join; the communicator was aborted)");
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
        if (ncclCommGetAsyncError(c->c, &r) != ncclSuccess) comm_fail(c, std::string(what) + ": async error query");
    }
}

// wait for everything enqueued on the communicator's stream (its collectives), within the deadline; an asynchronous
// RCCL error (a peer gone) or the deadline aborts the communicator
void comm_wait(qasr_comm* c, const char* what, std::chrono::steady_clock::time_point t_end) {
    for (int spin = 0;; spin++) {
        const hipError_t q = hipStreamQuery(c->st);
        if (q == hipSuccess) return;
        if (q != hipErrorNotReady) throw Error(QASR_E_BACKEND, std::string("HIP: ") + what + ": " + hipGetErrorString(q));
        ncclResult_t ae = ncclSuccess;
        if (ncclCommGetAsyncError(c->c, &ae) != ncclSuccess || (ae != ncclSuccess && ae != ncclInProgress))
            comm_fail(c, std::string(what) + ": " + ncclGetErrorString(ae));
        if (std::chrono::steady_clock::now() > t_end)
            comm_fail(c, std::string(what) + ": timed out (a rank did not enter the collective; the communicator was "
                                             "aborted)");
        if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}

struct Deadline {
    std::chrono::steady_clock::time_point t;
    explicit Deadline(const qasr_comm* c)
        : t(std::chrono::steady_clock::now() +
            std::chrono::microseconds((int64_t)(c->timeout_ms * 1e3))) {}
};

uint64_t blob_checksum(const void* dev, size_t bytes, unsigned long long* scratch, hipStream_t st) {
    QASR_CHECK(bytes % 8 == 0, QASR_E_INVALID, "checksum: blob size must be a multiple of 8");
    QASR_HIP(hipMemsetAsync(scratch, 0, sizeof(unsigned long long), st));
    k_blob_checksum<<<1024, 256, 0, st>>>((const unsigned long long*)dev, bytes / 8, scratch);
    QASR_HIP(hipGetLastError());
    unsigned long long h = 0;
    QASR_HIP(hipMemcpyAsync(&h, scratch, sizeof h, hipMemcpyDeviceToHost, st));
    QASR_HIP(hipStreamSynchronize(st));
    return h;
}

template <class T>
struct DevBuf {
    T* p = nullptr;
    explicit DevBuf(size_t n) { QASR_HIP(hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T))); }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

}  // namespace

extern "C" {

QASR_API int qasr_dist_unique_id(uint8_t* out, size_t cap) {
    return guard([&] {
        QASR_CHECK(out && cap >= NCCL_UNIQUE_ID_BYTES, QASR_E_INVALID, "unique id buffer: 128 bytes");
        ncclUniqueId id;
        QASR_NCCL(ncclGetUniqueId(&id));
        memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
    });
}

QASR_API int qasr_dist_init_deadline(const uint8_t* id, int32_t rank, int32_t world, int32_t device,
                                     double timeout_ms, qasr_comm** out) {
    return guard([&] {
        QASR_CHECK(id && out && world >= 1 && rank >= 0 && rank < world, QASR_E_INVALID, "bad arguments");
        *out = nullptr;
        auto c = std::make_unique<qasr_comm>();
        c->timeout_ms = timeout_ms > 0 ? timeout_ms : env_timeout_ms();
        QASR_HIP(hipSetDevice(device));
        // ncclCommInitRank blocks until every rank has joined, and this RCCL's non-blocking config does not make the
        // calling thread return early (measured: ncclCommInitRankConfig with blocking = 0 stayed inside its bootstrap
        // with a rank missing, gpurun_out/r6b_nj.log).  So the init runs on a helper thread and this thread waits for
        // it against the deadline; at the deadline the helper is abandoned (detached: it aborts the communicator itself
        // if the missing rank ever arrives) and the caller gets QASR_E_BACKEND — the host is expected to exit.
        struct InitJob {
            std::mutex mu;
            std::condition_variable cv;
            bool done = false, abandoned = false;
            ncclResult_t r = ncclSuccess;
            ncclComm_t comm = nullptr;
        };
        auto job = std::make_shared<InitJob>();
        ncclUniqueId uid;
        memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
        dbg("init rank %d of %d, device %d, deadline %.0f ms", rank, world, device, c->timeout_ms);
        std::thread([job, uid, rank, world, device] {
            ncclComm_t cm = nullptr;
            ncclResult_t r = hipSetDevice(device) == hipSuccess ? ncclCommInitRank(&cm, world, uid, rank)
                                                                 : ncclUnhandledCudaError;
            std::lock_guard<std::mutex> lk(job->mu);
            job->r = r;
            job->comm = cm;
            job->done = true;
            if (job->abandoned && cm) (void)ncclCommAbort(cm);   // the caller gave up: nobody will use it
            job->cv.notify_all();
        }).detach();
        std::unique_lock<std::mutex> lk(job->mu);
        const auto t_end = Deadline(c.get()).t;
        if (!job->cv.wait_until(lk, t_end, [&] { return job->done; })) {
            job->abandoned = true;
            dbg("init timed out");
            throw Error(QASR_E_BACKEND, "RCCL: ncclCommInitRank: timed out after " +
                                            std::to_string((long)c->timeout_ms) +
                                            " ms (a rank did not join the communicator)");
        }
        dbg("ncclCommInitRank returned %d (%s)", (int)job->r, ncclGetErrorString(job->r));
        if (job->r != ncclSuccess) {
            if (job->comm) (void)ncclCommAbort(job->comm);
            throw Error(QASR_E_BACKEND, std::string("RCCL: ncclCommInitRank: ") + ncclGetErrorString(job->r));
        }
        c->c = job->comm;
        QASR_HIP(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
        c->rank = rank, c->world = world, c->device = device;
        *out = c.release();
    });
}

QASR_API int qasr_dist_init(const uint8_t* id, int32_t rank, int32_t world, int32_t device, qasr_comm** out) {
    return qasr_dist_init_deadline(id, rank, world, device, 0.0, out);
}

QASR_API void qasr_dist_close(qasr_comm* c) { delete c; }

QASR_API int qasr_dist_broadcast(qasr_comm* c, const void* send, void* recv, size_t bytes, int32_t root) {
    return guard([&] {
        QASR_CHECK(c && recv && root >= 0 && root < c->world, QASR_E_INVALID, "bad arguments");
        QASR_CHECK(!c->dead, QASR_E_BACKEND, "communicator aborted by an earlier failure");
        const Deadline ddl(c);
        QASR_NCCL_C(c, ddl, ncclBroadcast(send ? send : recv, recv, bytes, ncclUint8, root, c->c, c->st));
        comm_wait(c, "broadcast", ddl.t);
    });
}

QASR_API int qasr_dist_broadcast_weights(qasr_comm* c, qasr_model* m, int32_t root, qasr_dist_info* info) {
    return guard([&] {
        QASR_CHECK(c && m && root >= 0 && root < c->world, QASR_E_INVALID, "bad arguments");
        QASR_CHECK(!c->dead, QASR_E_BACKEND, "communicator aborted by an earlier failure");
        const Deadline ddl(c);
        Model& md = *m->m;
        QASR_CHECK(c->rank == root || md.weights_pending, QASR_E_INVALID,
                   "weight broadcast: non-root ranks receive into a shell (qasr_model_open_shell)");
        QASR_HIP(hipDeviceSynchronize());   // the root's load / generation has landed
        const auto t0 = std::chrono::steady_clock::now();
        QASR_NCCL_C(c, ddl, ncclBroadcast(md.mem.base, md.mem.base, md.mem.bytes, ncclUint8, root, c->c, c->st));
        comm_wait(c, "weight broadcast", ddl.t);
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        // every rank's checksum, all-gathered: the copy is verified before sessions may open
        DevBuf<unsigned long long> scratch(1);
        const uint64_t mine = blob_checksum(md.mem.base, md.mem.bytes, scratch.p, c->st);
        DevBuf<unsigned long long> all((size_t)c->world);
        QASR_HIP(hipMemcpyAsync(all.p + c->rank, &mine, sizeof mine, hipMemcpyHostToDevice, c->st));
        QASR_NCCL_C(c, ddl, ncclAllGather(all.p + c->rank, all.p, 1, ncclUint64, c->c, c->st));
        std::vector<uint64_t> sums((size_t)c->world);
        QASR_HIP(hipMemcpyAsync(sums.data(), all.p, sums.size() * 8, hipMemcpyDeviceToHost, c->st));
        comm_wait(c, "checksum gather", ddl.t);
        bool agree = true;
        for (uint64_t s : sums) agree = agree && s == sums[(size_t)root];
        if (info) {
            info->bytes = (uint64_t)md.mem.bytes;
            info->ms = ms;
            info->checksum = sums[(size_t)root];
            info->checksums_agree = agree ? 1 : 0;
        }
        QASR_CHECK(agree, QASR_E_BACKEND, "weight broadcast: checksums differ across ranks");
        if (c->rank != root) md.weights_pending = false;
    });
}

QASR_API int qasr_dist_gather_tokens(qasr_comm* c, const int32_t* lens, int32_t n_seg, const int32_t* tokens,
                                     int32_t* rank_segs, int32_t* all_lens, size_t lens_cap, int32_t* all_tokens,
                                     size_t tokens_cap, size_t* n_segs_out, size_t* n_tokens_out) {
    return guard([&] {
        QASR_CHECK(c && n_seg >= 0 && (lens || n_seg == 0) && rank_segs && n_segs_out && n_tokens_out,
                   QASR_E_INVALID, "bad arguments");
        int64_t ntok = 0;
        for (int i = 0; i < n_seg; i++) {
            QASR_CHECK(lens[i] >= 0, QASR_E_INVALID, "negative segment length");
            ntok += lens[i];
        }
        QASR_CHECK(ntok == 0 || tokens, QASR_E_INVALID, "tokens missing");
        QASR_CHECK(!c->dead, QASR_E_BACKEND, "communicator aborted by an earlier failure");
        const Deadline ddl(c);
        const int W = c->world;
        // (1) counts
        DevBuf<int64_t> cnt((size_t)2 * W);
        const int64_t mine[2] = {n_seg, ntok};
        QASR_HIP(hipMemcpyAsync(cnt.p + 2 * c->rank, mine, sizeof mine, hipMemcpyHostToDevice, c->st));
        QASR_NCCL_C(c, ddl, ncclAllGather(cnt.p + 2 * c->rank, cnt.p, 2, ncclInt64, c->c, c->st));
        std::vector<int64_t> counts((size_t)2 * W);
        QASR_HIP(hipMemcpyAsync(counts.data(), cnt.p, counts.size() * 8, hipMemcpyDeviceToHost, c->st));
        comm_wait(c, "count gather", ddl.t);
        int64_t max_seg = 1, max_tok = 1, tot_seg = 0, tot_tok = 0;
        for (int r = 0; r < W; r++) {
            max_seg = std::max(max_seg, counts[2 * r]);
            max_tok = std::max(max_tok, counts[2 * r + 1]);
            tot_seg += counts[2 * r];
            tot_tok += counts[2 * r + 1];
            rank_segs[r] = (int32_t)counts[2 * r];
        }
        *n_segs_out = (size_t)tot_seg;
        *n_tokens_out = (size_t)tot_tok;
        // every rank states what it does next — 0 size query, 1 payload, -1 its buffers are too small — and all ranks
        // decide together, so a caller error on one rank is an error on every rank instead of the others blocking in
        // the payload all-gather
        const bool query = !all_lens && !all_tokens;
        const int32_t st = query ? 0 : (all_lens && all_tokens && lens_cap >= (size_t)tot_seg &&
                                        tokens_cap >= (size_t)tot_tok) ? 1 : -1;
        DevBuf<int32_t> sts((size_t)W);
        QASR_HIP(hipMemcpyAsync(sts.p + c->rank, &st, sizeof st, hipMemcpyHostToDevice, c->st));
        QASR_NCCL_C(c, ddl, ncclAllGather(sts.p + c->rank, sts.p, 1, ncclInt32, c->c, c->st));
        std::vector<int32_t> every((size_t)W);
        QASR_HIP(hipMemcpyAsync(every.data(), sts.p, every.size() * 4, hipMemcpyDeviceToHost, c->st));
        comm_wait(c, "status gather", ddl.t);
        const int32_t lo = *std::min_element(every.begin(), every.end());
        const int32_t hi = *std::max_element(every.begin(), every.end());
        QASR_CHECK(lo >= 0, QASR_E_CAPACITY, "gather buffers too small (on this or another rank)");
        QASR_CHECK(lo == hi, QASR_E_INVALID, "ranks disagree on size query vs payload gather");
        if (query) return;
        // (2) the ragged payload, padded to the largest rank
        DevBuf<int32_t> dl((size_t)max_seg * W), dt((size_t)max_tok * W);
        QASR_HIP(hipMemsetAsync(dl.p + max_seg * c->rank, 0, (size_t)max_seg * 4, c->st));
        QASR_HIP(hipMemsetAsync(dt.p + max_tok * c->rank, 0, (size_t)max_tok * 4, c->st));
        if (n_seg) QASR_HIP(hipMemcpyAsync(dl.p + max_seg * c->rank, lens, (size_t)n_seg * 4, hipMemcpyHostToDevice, c->st));
        if (ntok) QASR_HIP(hipMemcpyAsync(dt.p + max_tok * c->rank, tokens, (size_t)ntok * 4, hipMemcpyHostToDevice, c->st));
        QASR_NCCL_C(c, ddl, ncclAllGather(dl.p + max_seg * c->rank, dl.p, (size_t)max_seg, ncclInt32, c->c, c->st));
        QASR_NCCL_C(c, ddl, ncclAllGather(dt.p + max_tok * c->rank, dt.p, (size_t)max_tok, ncclInt32, c->c, c->st));
        std::vector<int32_t> hl((size_t)max_seg * W), ht((size_t)max_tok * W);
        QASR_HIP(hipMemcpyAsync(hl.data(), dl.p, hl.size() * 4, hipMemcpyDeviceToHost, c->st));
        QASR_HIP(hipMemcpyAsync(ht.data(), dt.p, ht.size() * 4, hipMemcpyDeviceToHost, c->st));
        comm_wait(c, "token gather", ddl.t);
        size_t os = 0, ot = 0;
        for (int r = 0; r < W; r++) {
            memcpy(all_lens + os, hl.data() + (size_t)max_seg * r, (size_t)counts[2 * r] * 4);
            memcpy(all_tokens + ot, ht.data() + (size_t)max_tok * r, (size_t)counts[2 * r + 1] * 4);
            os += (size_t)counts[2 * r];
            ot += (size_t)counts[2 * r + 1];
        }
    });
}

QASR_API int qasr_dist_agree(qasr_comm* c, int32_t local_status, int32_t* any_failed) {
    return guard([&] {
        QASR_CHECK(c && any_failed, QASR_E_INVALID, "bad arguments");
        QASR_CHECK(!c->dead, QASR_E_BACKEND, "communicator aborted by an earlier failure");
        const Deadline ddl(c);
        const int32_t mine = local_status != 0 ? 1 : 0;
        DevBuf<int32_t> sts((size_t)c->world);
        QASR_HIP(hipMemcpyAsync(sts.p + c->rank, &mine, sizeof mine, hipMemcpyHostToDevice, c->st));
        QASR_NCCL_C(c, ddl, ncclAllGather(sts.p + c->rank, sts.p, 1, ncclInt32, c->c, c->st));
        std::vector<int32_t> every((size_t)c->world);
        QASR_HIP(hipMemcpyAsync(every.data(), sts.p, every.size() * 4, hipMemcpyDeviceToHost, c->st));
        comm_wait(c, "agreement", ddl.t);
        *any_failed = *std::max_element(every.begin(), every.end());
    });
}

}  // extern "C"
