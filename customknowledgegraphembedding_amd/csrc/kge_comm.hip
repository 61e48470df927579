// kge_comm.hip — the row-sharded forward step's host path in C++: an RCCL communicator of our own and an
// executor that issues one rank's whole step (plan of the next batch, query exchange, owner-computes
// scoring, score exchange, finish) from ONE C call.
//
// Why: the Python host path of ShardedKGE.step_forward (distributed.py) costs ~160 us per rank-step at
// W = 8 (profiles/r04_host_probe.txt: plan 81 us + step 78 us, collectives stubbed), and every
// torch.distributed all_to_all_single adds ~22 us of host time under RCCL (same file). The single-GPU
// C4 step is ~100 us of device time, so at 8 ranks the host, not the GPU, would set the step time. Here:
//   * collectives are ncclAllToAllv calls on the executor's communication stream (RCCL over xGMI; the
//     split sizes come from the plan's host summary, parsed in C++);
//   * the scoring of chunk k overlaps the exchanges of the other chunks through events (the stream graph
//     of distributed.py's async work handles, without any host wait);
//   * the NEXT batch's plan (kge_shard_plan + the summary's device-to-host copy) is made inside the same
//     call on a third stream, so the split sizes of step i + 1 are on the host before step i + 1 starts.
// Memory: every device buffer is carved from the caller's workspace, the summaries go to the caller's
// pinned host buffer (the library allocates nothing; it creates its streams and events once per executor).
// Reference: the strategy layer of tensorflow_codes/run.py:8-17 and the per-step call of supervisor.py:30
// (strategy.run once per step); SURVEY §8e owner-computes.
#include <dlfcn.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "kge_hip.h"

// In-process loopback group: W communicators of ONE process (one host thread per simulated rank, all on one
// device), whose all-to-alls are device copies between the ranks' buffers with the stream dependencies of a
// real collective: a rank's pieces are copied after their sender's data is ready, and the collective
// completes on every rank's stream only when every rank has received. It runs the W-rank native executor on
// a single GPU (tests), as ThreadComm does for the Python path.
struct kge_loop_group {
    int world = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    int64_t generation = 0;
    struct Post {
        const float* send = nullptr;
        const size_t* sc = nullptr;
        const size_t* sd = nullptr;
        hipEvent_t ready = nullptr;  // the sender's data
        hipEvent_t done = nullptr;   // this rank's incoming copies
    };
    std::vector<Post> post;
    bool broken = false;
};

struct kge_comm {
    ncclComm_t nccl = nullptr;
    kge_loop_group* loop = nullptr;
    hipEvent_t loop_ready = nullptr, loop_done = nullptr;
    int world = 0, rank = 0;
};


namespace kge_impl {
int set_error(int code, const char* msg);  // kge_abi.hip

namespace {

// RCCL entry points, resolved at run time from the RCCL already loaded into the process (PyTorch's, when
// torch.distributed is imported: one RCCL per process), else from librccl.so.1 on the library path.
struct Rccl {
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_to_allv)(const void*, const size_t*, const size_t*, void*, const size_t*, const size_t*,
                                ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
    ncclResult_t (*count)(const ncclComm_t, int*) = nullptr;
    bool ok = false;
};

const Rccl& rccl() {
    static const Rccl r = [] {
        Rccl x;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return x;
        auto sym = [&](const char* n) { return dlsym(h, n); };
        x.get_unique_id = reinterpret_cast<decltype(x.get_unique_id)>(sym("ncclGetUniqueId"));
        x.init_rank = reinterpret_cast<decltype(x.init_rank)>(sym("ncclCommInitRank"));
        x.destroy = reinterpret_cast<decltype(x.destroy)>(sym("ncclCommDestroy"));
        x.all_to_allv = reinterpret_cast<decltype(x.all_to_allv)>(sym("ncclAllToAllv"));
        x.all_reduce = reinterpret_cast<decltype(x.all_reduce)>(sym("ncclAllReduce"));
        x.error_string = reinterpret_cast<decltype(x.error_string)>(sym("ncclGetErrorString"));
        x.count = reinterpret_cast<decltype(x.count)>(sym("ncclCommCount"));
        x.ok = x.get_unique_id && x.init_rank && x.destroy && x.all_to_allv && x.all_reduce && x.error_string;
        return x;
    }();
    return r;
}

// a barrier of the loopback group's W threads (60 s: a rank that never arrives breaks the group instead of
// hanging the others)
int loop_barrier(kge_loop_group* g) {
    std::unique_lock<std::mutex> lk(g->mu);
    if (g->broken) return set_error(KGE_EHIP, "loopback group broken (a rank failed or timed out)");
    const int64_t gen = g->generation;
    if (++g->arrived == g->world) {
        g->arrived = 0;
        ++g->generation;
        g->cv.notify_all();
        return 0;
    }
    if (!g->cv.wait_for(lk, std::chrono::seconds(60), [&] { return g->generation != gen || g->broken; }) || g->broken) {
        g->broken = true;
        g->cv.notify_all();
        return set_error(KGE_EHIP, "loopback group: barrier timed out");
    }
    return 0;
}

int nccl_fail(const char* what, ncclResult_t r) {
    const char* s = rccl().error_string ? rccl().error_string(r) : "?";
    return set_error(KGE_EHIP, (std::string(what) + ": RCCL error " + std::to_string((int)r) + " (" + s + ")").c_str());
}

int hip_fail(const char* what, hipError_t e) {
    return set_error(KGE_EHIP, (std::string(what) + ": " + hipGetErrorString(e)).c_str());
}

#define KGE_HIP_TRY(what, call)                   \
    do {                                          \
        const hipError_t e_ = (call);             \
        if (e_ != hipSuccess) return hip_fail(what, e_); \
    } while (0)

constexpr int kMaxWorld = 64;
constexpr int kMaxChunks = 8;
// plan slots: the step being issued and up to two batches planned ahead, so the host can run two steps
// ahead of the device without ever waiting for a summary that is still being computed
constexpr int kSlots = 3;

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// Device layout of one plan slot and of the exchange buffers, for a forward plan (one exchanged query
// column): the sizes are upper bounds, so one workspace serves every batch of the shape.
struct Layout {
    size_t cnt, hpre, qown, qslot, summ, bucket, bstart, slot;  // offsets inside a slot; slot = its size
    size_t q_send, qidx, q_block, s_send, s_recv, total;       // offsets of the exchange buffers
    int64_t summ_ints;
};

Layout layout_for(int64_t Bg, int64_t N, int64_t ent_dim, int world, int chunks) {
    Layout L{};
    const int64_t W = world, K = chunks, Rk = Bg / K, homeB = Bg / W;
    L.summ_ints = W * W + K * W;
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t at = o;
        o += al256(bytes);
        return at;
    };
    L.cnt = take((size_t)W * Bg * 4);
    L.hpre = take((size_t)W * Bg * 4);
    L.qown = take((size_t)Bg * 4);
    L.qslot = take((size_t)Bg * 4);
    L.summ = take((size_t)L.summ_ints * 4);
    L.bucket = take((size_t)Bg * (N + 1) * 8);
    L.bstart = take((size_t)Bg * 9 * 4);
    L.slot = o;
    o = kSlots * L.slot;  // the current batch's plan slot and the ones planned ahead
    // query rows: each chunk's block of this rank's rows, W copies (the all-to-all's input), at most Rk rows;
    // the received blocks hold at most Rk rows each
    L.q_send = take((size_t)W * Bg * ent_dim * 4);
    L.qidx = take((size_t)Bg * 8);
    L.q_block = take((size_t)K * Rk * ent_dim * 4);
    // scores: chunk k's owned scores of its rows (at most Rk (N + 1)), the home's received ones
    L.s_send = take((size_t)K * Rk * (N + 1) * 4);
    L.s_recv = take((size_t)homeB * (N + 1) * 4);
    L.total = o;
    return L;
}

}  // namespace
}  // namespace kge_impl

using namespace kge_impl;

struct kge_shard_exec {
    kge_comm* comm = nullptr;
    int fn = 0, world = 1, rank = 0, chunks = 1, flags = 0;
    int64_t nentity = 0, shard_rows = 0, ent_dim = 0, D = 0, Bg = 0, N = 0;
    Layout L{};
    char* ws = nullptr;
    int* host = nullptr;  // [kSlots][summ_ints] pinned
    struct Slot {
        bool planned = false;
        int mode = 0;
        const int64_t* pos = nullptr;
        const int64_t* neg = nullptr;
        int64_t neg_ld = 0;
        hipEvent_t ready = nullptr;  // the summary's copy to the host has landed
        hipEvent_t freed = nullptr;  // the last step that read the slot's device arrays is done
    } slot[kSlots];
    int cur = 0;       // the slot the next step consumes (the oldest plan)
    int nplanned = 0;  // plans waiting, in slots cur, cur + 1, ... (mod kSlots)
    hipStream_t comm_st = nullptr, plan_st = nullptr;
    hipEvent_t ev_start = nullptr, ev_gather = nullptr, ev_q[kMaxChunks] = {}, ev_s[kMaxChunks] = {},
               ev_x = nullptr;
    std::vector<size_t> sc, sd, rc, rd;  // ncclAllToAllv counts / displacements (elements)
    double wait_us = 0;                  // host time spent waiting for plans' summaries (kge_shard_exec_host_wait_us)
    // KGE_EXEC_TIMING: timing events of the last step (kge_shard_exec_timings): t[0] its start, t[1] after the
    // query gather, per chunk k the query exchange (t[2 + 6k], t[3 + 6k]), the scoring (t[4 + 6k], t[5 + 6k]) and
    // the score exchange (t[6 + 6k], t[7 + 6k]), then the finish (t[2 + 6K], t[3 + 6K])
    static constexpr int kTimingEvents = 4 + 6 * kMaxChunks;
    hipEvent_t t[kTimingEvents] = {};
    bool timed = false;  // the last step recorded them
    bool broken = false;  // a step failed part-way: its plan slots and (under RCCL) its peers are in an unknown state

    int* slot_i(int s, size_t off) { return reinterpret_cast<int*>(ws + s * L.slot + off); }
};

namespace {

// `ids_ready`: recorded on the caller's stream after the work that made the batch's ids (for the plan made
// inside a step: at the step's start, so the plan of batch i + 1 overlaps step i)
int make_plan(kge_shard_exec* x, int s, const int64_t* pos, const int64_t* neg, int64_t neg_ld, int mode,
              hipEvent_t ids_ready) {
    kge_shard_exec::Slot& sl = x->slot[s];
    // the plan's stream waits for the ids and for the last step that read this slot's arrays
    KGE_HIP_TRY("kge_shard_exec plan", hipStreamWaitEvent(x->plan_st, ids_ready, 0));
    KGE_HIP_TRY("kge_shard_exec plan", hipStreamWaitEvent(x->plan_st, sl.freed, 0));
    int rc = kge_shard_plan(pos, neg, neg_ld, x->Bg, x->N, x->nentity, x->world, x->chunks, mode, 0, x->rank,
                            x->slot_i(s, x->L.cnt), x->slot_i(s, x->L.hpre), x->slot_i(s, x->L.qown),
                            x->slot_i(s, x->L.qslot), x->slot_i(s, x->L.summ), x->slot_i(s, x->L.bucket),
                            x->slot_i(s, x->L.bstart), x->plan_st);
    if (rc) return rc;
    int* h = x->host + (size_t)s * x->L.summ_ints;
    KGE_HIP_TRY("kge_shard_exec summary copy",
                hipMemcpyAsync(h, x->slot_i(s, x->L.summ), (size_t)x->L.summ_ints * 4, hipMemcpyDeviceToHost,
                               x->plan_st));
    KGE_HIP_TRY("kge_shard_exec plan", hipEventRecord(sl.ready, x->plan_st));
    sl.planned = true;
    sl.mode = mode;
    sl.pos = pos;
    sl.neg = neg;
    sl.neg_ld = neg_ld;
    return 0;
}

// all-to-all through a loopback group: post, barrier, copy the incoming pieces, barrier, wait for every rank
int loop_all_to_allv(kge_comm* c, const float* send, const size_t* sc, const size_t* sd, void* recv, const size_t* rc,
                     const size_t* rd, hipStream_t st) {
    kge_loop_group* g = c->loop;
    hipError_t e = hipEventRecord(c->loop_ready, st);
    if (e != hipSuccess) return hip_fail("loopback all-to-all", e);
    g->post[c->rank] = {send, sc, sd, c->loop_ready, c->loop_done};
    int rcode = loop_barrier(g);
    if (rcode) return rcode;
    for (int s = 0; s < c->world && e == hipSuccess; ++s) {
        const kge_loop_group::Post& p = g->post[s];
        if (!rc[s]) continue;
        e = hipStreamWaitEvent(st, p.ready, 0);
        if (e == hipSuccess)
            e = hipMemcpyAsync(static_cast<char*>(recv) + rd[s] * 4, p.send + p.sd[c->rank], rc[s] * 4,
                               hipMemcpyDeviceToDevice, st);
    }
    if (e == hipSuccess) e = hipEventRecord(c->loop_done, st);
    if (e != hipSuccess) {
        g->broken = true;
        return hip_fail("loopback all-to-all", e);
    }
    rcode = loop_barrier(g);
    if (rcode) return rcode;
    for (int s = 0; s < c->world && e == hipSuccess; ++s) e = hipStreamWaitEvent(st, g->post[s].done, 0);
    if (e != hipSuccess) return hip_fail("loopback all-to-all", e);
    return loop_barrier(g);  // no rank re-posts before every rank has read the posts
}

// one all-to-all of floats on the communication stream; without a communicator (world 1) the only piece is
// this rank's own, a device copy; KGE_EXEC_PROBE skips the collectives (host-cost probe only)
int exchange(kge_shard_exec* x, const float* send, void* recv, hipStream_t cs, const char* what) {
    if (x->flags & KGE_EXEC_PROBE) return 0;
    if (!x->comm) {
        if (x->sc[0]) KGE_HIP_TRY(what, hipMemcpyAsync(static_cast<char*>(recv) + x->rd[0] * 4, send + x->sd[0],
                                                       x->sc[0] * 4, hipMemcpyDeviceToDevice, cs));
        return 0;
    }
    if (x->comm->loop)
        return loop_all_to_allv(x->comm, send, x->sc.data(), x->sd.data(), recv, x->rc.data(), x->rd.data(), cs);
    const ncclResult_t r = rccl().all_to_allv(send, x->sc.data(), x->sd.data(), recv, x->rc.data(), x->rd.data(),
                                              ncclFloat32, x->comm->nccl, cs);
    if (r != ncclSuccess) return nccl_fail(what, r);
    return 0;
}

}  // namespace

extern "C" {

int kge_comm_unique_id(void* id) {
    if (!id) return set_error(KGE_EINVAL, "kge_comm_unique_id: null pointer");
    if (!rccl().ok) return set_error(KGE_ENOTSUP, "kge_comm_unique_id: RCCL (librccl.so.1) not found");
    ncclUniqueId u;
    const ncclResult_t r = rccl().get_unique_id(&u);
    if (r != ncclSuccess) return nccl_fail("ncclGetUniqueId", r);
    memcpy(id, &u, sizeof(u));
    return set_error(0, "");
}

int kge_comm_init(kge_comm** out, const void* id, int world, int rank) {
    if (!out || !id) return set_error(KGE_EINVAL, "kge_comm_init: null pointer");
    *out = nullptr;
    if (world < 1 || world > kMaxWorld || rank < 0 || rank >= world)
        return set_error(KGE_EINVAL, "kge_comm_init: bad world/rank");
    if (!rccl().ok) return set_error(KGE_ENOTSUP, "kge_comm_init: RCCL (librccl.so.1) not found");
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    kge_comm* c = new kge_comm;
    const ncclResult_t r = rccl().init_rank(&c->nccl, world, u, rank);
    if (r != ncclSuccess) {
        delete c;
        return nccl_fail("ncclCommInitRank", r);
    }
    c->world = world;
    c->rank = rank;
    *out = c;
    return set_error(0, "");
}

kge_loop_group* kge_comm_loopback_group(int world) {
    if (world < 1 || world > kMaxWorld) {
        set_error(KGE_EINVAL, "kge_comm_loopback_group: bad world");
        return nullptr;
    }
    kge_loop_group* g = new kge_loop_group;
    g->world = world;
    g->post.resize(world);
    set_error(0, "");
    return g;
}

int kge_comm_loopback_group_destroy(kge_loop_group* group) {
    delete group;
    return set_error(0, "");
}

int kge_comm_loopback_init(kge_comm** out, kge_loop_group* group, int rank) {
    if (!out || !group) return set_error(KGE_EINVAL, "kge_comm_loopback_init: null pointer");
    *out = nullptr;
    if (rank < 0 || rank >= group->world) return set_error(KGE_EINVAL, "kge_comm_loopback_init: bad rank");
    kge_comm* c = new kge_comm;
    c->loop = group;
    c->world = group->world;
    c->rank = rank;
    hipError_t e = hipEventCreateWithFlags(&c->loop_ready, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->loop_done, hipEventDisableTiming);
    if (e != hipSuccess) {
        kge_comm_destroy(c);
        return hip_fail("kge_comm_loopback_init", e);
    }
    *out = c;
    return set_error(0, "");
}

int kge_comm_destroy(kge_comm* comm) {
    if (!comm) return set_error(0, "");
    const ncclResult_t r = comm->nccl ? rccl().destroy(comm->nccl) : ncclSuccess;
    if (comm->loop_ready) (void)hipEventDestroy(comm->loop_ready);
    if (comm->loop_done) (void)hipEventDestroy(comm->loop_done);
    delete comm;
    return r == ncclSuccess ? set_error(0, "") : nccl_fail("ncclCommDestroy", r);
}

int kge_comm_all_to_allv(kge_comm* comm, const float* send, const int64_t* send_counts, float* recv,
                         const int64_t* recv_counts, void* stream) {
    if (!comm || !send_counts || !recv_counts) return set_error(KGE_EINVAL, "kge_comm_all_to_allv: null pointer");
    const int W = comm->world;
    std::vector<size_t> sc(W), sd(W), rc(W), rd(W);
    size_t a = 0, b = 0;
    for (int o = 0; o < W; ++o) {
        if (send_counts[o] < 0 || recv_counts[o] < 0) return set_error(KGE_EINVAL, "kge_comm_all_to_allv: negative count");
        sc[o] = (size_t)send_counts[o];
        sd[o] = a;
        a += sc[o];
        rc[o] = (size_t)recv_counts[o];
        rd[o] = b;
        b += rc[o];
    }
    if (comm->loop) {
        const int rcode = loop_all_to_allv(comm, send, sc.data(), sd.data(), recv, rc.data(), rd.data(), (hipStream_t)stream);
        return rcode ? rcode : set_error(0, "");
    }
    const ncclResult_t r = rccl().all_to_allv(send, sc.data(), sd.data(), recv, rc.data(), rd.data(), ncclFloat32,
                                              comm->nccl, (hipStream_t)stream);
    return r == ncclSuccess ? set_error(0, "") : nccl_fail("ncclAllToAllv", r);
}

int kge_comm_all_reduce_sum(kge_comm* comm, float* buf, int64_t n, void* stream) {
    if (!comm || (n > 0 && !buf) || n < 0) return set_error(KGE_EINVAL, "kge_comm_all_reduce_sum: bad arguments");
    if (comm->loop) return set_error(KGE_ENOTSUP, "kge_comm_all_reduce_sum: not on a loopback communicator");
    if (n == 0) return set_error(0, "");
    const ncclResult_t r = rccl().all_reduce(buf, buf, (size_t)n, ncclFloat32, ncclSum, comm->nccl, (hipStream_t)stream);
    return r == ncclSuccess ? set_error(0, "") : nccl_fail("ncclAllReduce", r);
}

int64_t kge_shard_exec_workspace_size(int64_t Bg, int64_t N, int64_t ent_dim, int world, int chunks) {
    if (Bg <= 0 || N < 0 || ent_dim <= 0 || world < 1 || world > kMaxWorld || chunks < 1 || chunks > kMaxChunks ||
        world % chunks || Bg % world)
        return set_error(KGE_EINVAL, "kge_shard_exec_workspace_size: bad shape");
    return (int64_t)layout_for(Bg, N, ent_dim, world, chunks).total;
}

int64_t kge_shard_exec_host_ints(int world, int chunks) {
    if (world < 1 || world > kMaxWorld || chunks < 1 || chunks > kMaxChunks)
        return set_error(KGE_EINVAL, "kge_shard_exec_host_ints: bad world/chunks");
    return kSlots * ((int64_t)world * world + (int64_t)chunks * world);
}

int kge_shard_exec_create(kge_shard_exec** out, kge_comm* comm, int flags, int fn, int64_t nentity, int64_t shard_rows,
                          int64_t ent_dim, int64_t D, int64_t Bg, int64_t N, int world, int rank, int chunks,
                          void* workspace, int64_t workspace_bytes, int* host_pinned, int64_t host_ints) {
    if (!out) return set_error(KGE_EINVAL, "kge_shard_exec_create: null pointer");
    *out = nullptr;
    const int64_t need = kge_shard_exec_workspace_size(Bg, N, ent_dim, world, chunks);
    if (need < 0) return (int)need;
    if (rank < 0 || rank >= world || shard_rows <= 0 || D <= 0 || nentity < world)
        return set_error(KGE_EINVAL, "kge_shard_exec_create: bad rank / shard / D");
    if (comm && (comm->world != world || comm->rank != rank))
        return set_error(KGE_EINVAL, "kge_shard_exec_create: the communicator's world / rank differ");
    if (!comm && world > 1 && !(flags & KGE_EXEC_PROBE))
        return set_error(KGE_EINVAL, "kge_shard_exec_create: world > 1 needs a communicator (or KGE_EXEC_PROBE)");
    if (!workspace || workspace_bytes < need) return set_error(KGE_EINVAL, "kge_shard_exec_create: workspace too small");
    if (!host_pinned || host_ints < kge_shard_exec_host_ints(world, chunks))
        return set_error(KGE_EINVAL, "kge_shard_exec_create: host buffer too small");
    if (((uintptr_t)workspace & 255) != 0) return set_error(KGE_EINVAL, "kge_shard_exec_create: workspace must be 256-B aligned");
    kge_shard_exec* x = new kge_shard_exec;
    x->comm = comm;
    x->flags = flags;
    x->fn = fn;
    x->nentity = nentity;
    x->shard_rows = shard_rows;
    x->ent_dim = ent_dim;
    x->D = D;
    x->Bg = Bg;
    x->N = N;
    x->world = world;
    x->rank = rank;
    x->chunks = chunks;
    x->L = layout_for(Bg, N, ent_dim, world, chunks);
    x->ws = static_cast<char*>(workspace);
    x->host = host_pinned;
    x->sc.resize(world);
    x->sd.resize(world);
    x->rc.resize(world);
    x->rd.resize(world);
    hipError_t e = hipStreamCreateWithFlags(&x->comm_st, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&x->plan_st, hipStreamNonBlocking);
    auto ev = [&](hipEvent_t* p) {
        if (e == hipSuccess) e = hipEventCreateWithFlags(p, hipEventDisableTiming);
    };
    ev(&x->ev_start);
    ev(&x->ev_gather);
    ev(&x->ev_x);
    for (int k = 0; k < chunks; ++k) {
        ev(&x->ev_q[k]);
        ev(&x->ev_s[k]);
    }
    for (auto& s : x->slot) {
        ev(&s.ready);
        ev(&s.freed);
    }
    if (flags & KGE_EXEC_TIMING)
        for (int i = 0; i < kge_shard_exec::kTimingEvents && e == hipSuccess; ++i) e = hipEventCreate(&x->t[i]);
    if (e == hipSuccess) {
        // the slots start free: their `freed` events complete at once
        for (int i = 0; i < kSlots && e == hipSuccess; ++i) e = hipEventRecord(x->slot[i].freed, x->plan_st);
    }
    if (e != hipSuccess) {
        kge_shard_exec_destroy(x);
        return hip_fail("kge_shard_exec_create", e);
    }
    *out = x;
    return set_error(0, "");
}

int kge_shard_exec_destroy(kge_shard_exec* x) {
    if (!x) return set_error(0, "");
    if (x->comm_st) (void)hipStreamSynchronize(x->comm_st);
    if (x->plan_st) (void)hipStreamSynchronize(x->plan_st);
    auto drop = [](hipEvent_t e) {
        if (e) (void)hipEventDestroy(e);
    };
    drop(x->ev_start);
    drop(x->ev_gather);
    drop(x->ev_x);
    for (int k = 0; k < kMaxChunks; ++k) {
        drop(x->ev_q[k]);
        drop(x->ev_s[k]);
    }
    for (auto& s : x->slot) {
        drop(s.ready);
        drop(s.freed);
    }
    for (auto& t : x->t) drop(t);
    if (x->comm_st) (void)hipStreamDestroy(x->comm_st);
    if (x->plan_st) (void)hipStreamDestroy(x->plan_st);
    delete x;
    return set_error(0, "");
}

int kge_comm_size(kge_comm* comm) {
    if (!comm) return set_error(KGE_EINVAL, "kge_comm_size: null pointer");
    if (comm->loop || !comm->nccl) return comm->world;
    if (!rccl().count) return set_error(KGE_ENOTSUP, "kge_comm_size: ncclCommCount not found");
    int n = 0;
    const ncclResult_t r = rccl().count(comm->nccl, &n);
    if (r != ncclSuccess) return nccl_fail("ncclCommCount", r);
    return n;
}

int kge_shard_exec_timings(kge_shard_exec* x, float* out, int n) {
    if (!x || !out) return set_error(KGE_EINVAL, "kge_shard_exec_timings: null pointer");
    if (!(x->flags & KGE_EXEC_TIMING)) return set_error(KGE_EINVAL, "kge_shard_exec_timings: made without KGE_EXEC_TIMING");
    if (!x->timed) return set_error(KGE_EINVAL, "kge_shard_exec_timings: no timed step yet");
    const int K = x->chunks;
    if (n < 3 + 3 * K) return set_error(KGE_EINVAL, "kge_shard_exec_timings: out needs 3 + 3 chunks floats");
    const int fin = 2 + 6 * K;
    KGE_HIP_TRY("kge_shard_exec_timings", hipEventSynchronize(x->t[fin + 1]));
    auto span = [&](int a, int b) {
        float ms = 0.f;
        return hipEventElapsedTime(&ms, x->t[a], x->t[b]) == hipSuccess ? ms * 1e3f : -1.f;
    };
    out[0] = span(0, fin + 1);  // the step, first kernel to last
    out[1] = span(0, 1);        // the query gather
    out[2] = span(fin, fin + 1);  // the finish
    for (int k = 0; k < K; ++k) {
        out[3 + 3 * k] = span(2 + 6 * k, 3 + 6 * k);  // query all-to-all
        out[4 + 3 * k] = span(4 + 6 * k, 5 + 6 * k);  // owner-computes scoring
        out[5 + 3 * k] = span(6 + 6 * k, 7 + 6 * k);  // score all-to-all
    }
    return set_error(0, "");
}

double kge_shard_exec_host_wait_us(kge_shard_exec* x, int reset) {
    if (!x) return -1.0;
    const double w = x->wait_us;
    if (reset) x->wait_us = 0;
    return w;
}

int kge_shard_exec_plan(kge_shard_exec* x, const int64_t* pos, const int64_t* neg, int64_t neg_ld, int mode,
                        void* stream) {
    if (!x || !pos || !neg) return set_error(KGE_EINVAL, "kge_shard_exec_plan: null pointer");
    if (mode != KGE_HEAD_BATCH && mode != KGE_TAIL_BATCH)
        return set_error(KGE_EINVAL, "kge_shard_exec_plan: mode must be 0 or 1");
    // the slot after the ones already planned
    if (x->nplanned >= kSlots) return set_error(KGE_EINVAL, "kge_shard_exec_plan: every plan slot is waiting");
    const int s = (x->cur + x->nplanned) % kSlots;
    KGE_HIP_TRY("kge_shard_exec_plan", hipEventRecord(x->ev_start, (hipStream_t)stream));
    const int rc = make_plan(x, s, pos, neg, neg_ld, mode, x->ev_start);
    if (!rc) ++x->nplanned;
    return rc;
}

static int exec_step(kge_shard_exec* x, const float* shard, int64_t shard_ld, int64_t shard_lo, const float* rel,
                     int64_t nrelation, int64_t rel_ld, int64_t rel_off, const int64_t* pos, const int64_t* neg,
                     int64_t neg_ld, int mode, float gamma, float emb_range, float modulus, float temperature,
                     int adversarial, const int64_t* next_pos, const int64_t* next_neg, int next_mode, float* scores,
                     int64_t ns_ld, float* out_neg, float* pos_scores, float* out_pos, void* stream);

// An error part-way through a step (a failed launch or collective, an inline plan) leaves the plan slots and,
// under RCCL, the other ranks (blocked in the collective) in an unknown state: the executor is marked broken and
// every later call fails at once. Argument errors found before any work (null pointers, the waiting plan made
// for another batch) leave it usable.
int kge_shard_exec_step(kge_shard_exec* x, const float* shard, int64_t shard_ld, int64_t shard_lo, const float* rel,
                        int64_t nrelation, int64_t rel_ld, int64_t rel_off, const int64_t* pos, const int64_t* neg,
                        int64_t neg_ld, int mode, float gamma, float emb_range, float modulus, float temperature,
                        int adversarial, const int64_t* next_pos, const int64_t* next_neg, int next_mode,
                        float* scores, int64_t ns_ld, float* out_neg, float* pos_scores, float* out_pos,
                        void* stream) {
    if (!x || !shard || !rel || !pos || !neg || !scores || !out_neg || !pos_scores || !out_pos)
        return set_error(KGE_EINVAL, "kge_shard_exec_step: null pointer");
    if (x->broken)
        return set_error(KGE_EHIP, "kge_shard_exec_step: an earlier step of this executor failed part-way; an exec "
                                   "error is fatal to the executor and its communicator");
    if (x->nplanned > 0) {
        const kge_shard_exec::Slot& sl = x->slot[x->cur];
        if (sl.pos != pos || sl.neg != neg || sl.neg_ld != neg_ld || sl.mode != mode)
            return set_error(KGE_EINVAL, "kge_shard_exec_step: the waiting plan was made for another batch or mode");
    }
    const int rc = exec_step(x, shard, shard_ld, shard_lo, rel, nrelation, rel_ld, rel_off, pos, neg, neg_ld, mode,
                             gamma, emb_range, modulus, temperature, adversarial, next_pos, next_neg, next_mode, scores,
                             ns_ld, out_neg, pos_scores, out_pos, stream);
    if (rc) x->broken = true;
    return rc;
}

static int exec_step(kge_shard_exec* x, const float* shard, int64_t shard_ld, int64_t shard_lo, const float* rel,
                     int64_t nrelation, int64_t rel_ld, int64_t rel_off, const int64_t* pos, const int64_t* neg,
                     int64_t neg_ld, int mode, float gamma, float emb_range, float modulus, float temperature,
                     int adversarial, const int64_t* next_pos, const int64_t* next_neg, int next_mode, float* scores,
                     int64_t ns_ld, float* out_neg, float* pos_scores, float* out_pos, void* stream) {
    const hipStream_t st = (hipStream_t)stream;
    int s = x->cur;
    kge_shard_exec::Slot* sl = &x->slot[s];
    // the work queued so far (the next batch's ids included) ends here: the next plan waits for no more
    KGE_HIP_TRY("kge_shard_exec_step", hipEventRecord(x->ev_start, st));
    if (x->nplanned == 0) {  // no plan made ahead: plan now (the host then waits for the split sizes)
        int rc = make_plan(x, s, pos, neg, neg_ld, mode, x->ev_start);
        if (rc) return rc;
        x->nplanned = 1;
    } else if (sl->pos != pos || sl->neg != neg || sl->neg_ld != neg_ld || sl->mode != mode) {
        return set_error(KGE_EINVAL, "kge_shard_exec_step: the waiting plan was made for another batch or mode");
    }
    {  // made a step ahead: normally landed already
        const auto t0 = std::chrono::steady_clock::now();
        KGE_HIP_TRY("kge_shard_exec_step summary", hipEventSynchronize(sl->ready));
        x->wait_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    }
    const int W = x->world, K = x->chunks, me = x->rank;
    const int64_t Rk = x->Bg / K, homeB = x->Bg / W, d = x->ent_dim;
    const int hpc = W / K, k_home = me / hpc;
    const int* h = x->host + (size_t)s * x->L.summ_ints;
    const int* tot = h;           // [W][W]
    const int* qtot = h + W * W;  // [K][W] (one query column)
    // device pointers of the slot and the exchange buffers
    const int* cnt = x->slot_i(s, x->L.cnt);
    const int* hpre = x->slot_i(s, x->L.hpre);
    const int* summ = x->slot_i(s, x->L.summ);
    const int* bucket = x->slot_i(s, x->L.bucket);
    const int* bstart = x->slot_i(s, x->L.bstart);
    float* q_send = reinterpret_cast<float*>(x->ws + x->L.q_send);
    int64_t* qidx = reinterpret_cast<int64_t*>(x->ws + x->L.qidx);
    float* q_block = reinterpret_cast<float*>(x->ws + x->L.q_block);
    float* s_send = reinterpret_cast<float*>(x->ws + x->L.s_send);
    float* s_recv = reinterpret_cast<float*>(x->ws + x->L.s_recv);
    // the step's stream graph: compute on `st`, collectives on comm_st (the plan's arrays are complete: the
    // host waited for its event above, so `st` needs no wait on it). KGE_EXEC_ONE_STREAM: the collectives on
    // `st` too, in step order: no cross-stream event hops (each costs the dependent queue a wake-up), no
    // overlap of exchanges with scoring
    const bool one = (x->flags & KGE_EXEC_ONE_STREAM) != 0;
    const hipStream_t cs = one ? st : x->comm_st;
    auto hop = [&](hipEvent_t ev, hipStream_t from, hipStream_t to) -> hipError_t {
        if (one) return hipSuccess;
        hipError_t e = hipEventRecord(ev, from);
        return e == hipSuccess ? hipStreamWaitEvent(to, ev, 0) : e;
    };
    const bool tm = (x->flags & KGE_EXEC_TIMING) != 0;
    auto mark = [&](int i, hipStream_t on) -> hipError_t { return tm ? hipEventRecord(x->t[i], on) : hipSuccess; };
    x->timed = false;
    KGE_HIP_TRY("kge_shard_exec_step", mark(0, st));
    int rc = kge_shard_gather_queries(shard, x->shard_rows, shard_ld, shard_lo, pos, x->Bg, K, -1, d, W, me, mode, 0,
                                      x->slot_i(s, x->L.qown), x->slot_i(s, x->L.qslot), summ, q_send, qidx, st);
    if (rc) return rc;
    KGE_HIP_TRY("kge_shard_exec_step", mark(1, st));
    KGE_HIP_TRY("kge_shard_exec_step", hop(x->ev_gather, st, cs));
    // 1. every chunk's query exchange: this rank's rows of the chunk (the same piece to every rank)
    size_t at = 0, qb = 0;
    size_t qb_at[kMaxChunks], q_rows[kMaxChunks];
    for (int k = 0; k < K; ++k) {
        const int64_t mine = qtot[k * W + me];
        size_t r = 0;
        for (int o = 0; o < W; ++o) {
            x->sc[o] = (size_t)(mine * d);
            x->sd[o] = at + (size_t)o * mine * d;
            x->rc[o] = (size_t)qtot[k * W + o] * d;
            x->rd[o] = r;
            r += x->rc[o];
        }
        qb_at[k] = qb;
        q_rows[k] = r / (size_t)d;
        KGE_HIP_TRY("kge_shard_exec_step", mark(2 + 6 * k, cs));
        rc = exchange(x, q_send, q_block + qb, cs, "kge_shard_exec_step query all-to-all");
        if (rc) return rc;
        KGE_HIP_TRY("kge_shard_exec_step", mark(3 + 6 * k, cs));
        if (!one) KGE_HIP_TRY("kge_shard_exec_step", hipEventRecord(x->ev_q[k], cs));
        at += (size_t)W * mine * d;
        qb += r;
    }
    // 2. owner-computes scoring per chunk, 3. each chunk's scores to their home ranks
    size_t sb = 0;
    for (int k = 0; k < K; ++k) {
        const int64_t row0 = k * Rk;
        size_t nsend = 0;
        for (int o = 0; o < W; ++o) {
            const bool in_chunk = o >= k * hpc && o < (k + 1) * hpc;
            x->sc[o] = in_chunk ? (size_t)tot[o * W + me] : 0;
            x->sd[o] = nsend;
            nsend += x->sc[o];
        }
        size_t nrecv = 0;
        for (int o = 0; o < W; ++o) {
            x->rc[o] = k == k_home ? (size_t)tot[me * W + o] : 0;
            x->rd[o] = nrecv;
            nrecv += x->rc[o];
        }
        if (!one) KGE_HIP_TRY("kge_shard_exec_step", hipStreamWaitEvent(st, x->ev_q[k], 0));
        KGE_HIP_TRY("kge_shard_exec_step", mark(4 + 6 * k, st));
        if (nsend) {
            rc = kge_shard_score(x->fn, mode, q_block + qb_at[k], (int64_t)q_rows[k], d, qidx + row0, rel, nrelation, rel_ld,
                                 rel_off, shard, x->shard_rows, shard_ld, shard_lo, pos + row0 * 3, Rk, x->N, x->D,
                                 gamma, emb_range, modulus, bucket + row0 * (x->N + 1) * 2, bstart + row0 * 9,
                                 hpre + (int64_t)me * x->Bg + row0, cnt + (int64_t)me * x->Bg + row0, summ, W, me,
                                 homeB, row0 / homeB, s_send + sb, st);
            if (rc) return rc;
        }
        KGE_HIP_TRY("kge_shard_exec_step", mark(5 + 6 * k, st));
        KGE_HIP_TRY("kge_shard_exec_step", hop(x->ev_s[k], st, cs));
        KGE_HIP_TRY("kge_shard_exec_step", mark(6 + 6 * k, cs));
        rc = exchange(x, s_send + sb, s_recv, cs, "kge_shard_exec_step score all-to-all");
        if (rc) return rc;
        KGE_HIP_TRY("kge_shard_exec_step", mark(7 + 6 * k, cs));
        sb += nsend;
    }
    KGE_HIP_TRY("kge_shard_exec_step", hop(x->ev_x, cs, st));
    // 4. the home rows: scatter, positives, reductions
    KGE_HIP_TRY("kge_shard_exec_step", mark(2 + 6 * K, st));
    rc = kge_shard_finish(s_recv, summ, hpre, pos, neg, neg_ld, x->Bg, x->N, x->nentity, W, me, mode, temperature,
                          adversarial, scores, ns_ld, out_neg, pos_scores, out_pos, st);
    if (rc) return rc;
    KGE_HIP_TRY("kge_shard_exec_step", mark(3 + 6 * K, st));
    x->timed = tm;
    KGE_HIP_TRY("kge_shard_exec_step", hipEventRecord(sl->freed, st));
    sl->planned = false;
    x->cur = (s + 1) % kSlots;
    --x->nplanned;
    // the batch after the planned ones, planned now (into the slot a step before this one freed) so that
    // its split sizes are on the host long before its step; its stream waits only for the work queued
    // before this step (ev_start), so it overlaps this step
    if (next_pos && next_neg) {
        if (next_mode != KGE_HEAD_BATCH && next_mode != KGE_TAIL_BATCH)
            return set_error(KGE_EINVAL, "kge_shard_exec_step: next_mode must be 0 or 1");
        if (x->nplanned >= kSlots) return set_error(KGE_EINVAL, "kge_shard_exec_step: every plan slot is waiting");
        rc = make_plan(x, (x->cur + x->nplanned) % kSlots, next_pos, next_neg, neg_ld, next_mode, x->ev_start);
        if (rc) return rc;
        ++x->nplanned;
    }
    return set_error(0, "");
}

}  // extern "C"
