// loopback_rccl.cpp — TEST DOUBLE, not part of the product.
//
// The nine RCCL entry points wsg_mgpu.cpp loads at run time (dlopen of
// $WSG_RCCL_LIB, wsg_mgpu.cpp's rccl()), implemented for ranks that are
// threads of one process sharing one GPU.  With it the rank-per-process form
// of wsg_mgpu_encode_gather (its status and chunk-size all-gathers and the
// grouped per-chunk Send/Recv into the root) runs at world sizes a real RCCL
// communicator cannot have on a one-GPU box (tests/mgpu_rank_job.py).
//
// Semantics kept from NCCL: a group's operations start at ncclGroupEnd;
// Send/Recv between a pair of ranks match in posting order and must agree on
// the byte count (a rank with nothing to move takes no part); AllGather is a
// collective of every rank and places rank k's block at k * count.  Each
// group is completed synchronously at ncclGroupEnd (the posting streams are
// drained first) — the test checks placement, pairing and ordering, not
// overlap.  Copies run on the receiving rank's stream and are complete when
// the group returns (a plain hipMemcpy between device buffers may return
// before the copy lands, unordered with the product's non-blocking streams:
// a kernel the root queued after the Recv then read stale offsets, seen once
// on the box).  A mismatch (a Recv with no Send, a size disagreement, a Send
// nobody received within 60 s, an AllGather count disagreement) fails the
// group on the rank that sees it with ncclInvalidUsage and is counted in
// loopback_rccl_errors().
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <deque>
#include <memory>
#include <condition_variable>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

struct Op {
    enum Kind { SEND, RECV, ALLGATHER } kind;
    const void* src;
    void* dst;
    size_t bytes;
    int peer;
    hipStream_t stream;
};

// A send waiting in a mailbox until its receiver has copied it
struct Posted {
    const void* src;
    size_t bytes;
    bool taken = false;
    bool ok = false;
};

struct Group {
    explicit Group(int w) : world(w), ag_src(size_t(w)), mail(size_t(w) * size_t(w)) {}
    const int world;
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t generation = 0;
    std::vector<Op> ag_src;                          // per rank, its current AllGather
    std::vector<std::deque<std::shared_ptr<Posted>>> mail;   // [src * world + dst], posting order
};

std::atomic<int> g_errors{0};
std::mutex g_registry_lock;
std::map<std::string, Group*> g_registry;   // by unique id; groups live until exit
std::atomic<uint64_t> g_next_id{1};

size_t type_size(ncclDataType_t t)
{
    switch (t) {
    case ncclInt8:
    case ncclUint8:
        return 1;
    case ncclFloat16:
    case ncclBfloat16:
        return 2;
    case ncclInt32:
    case ncclUint32:
    case ncclFloat32:
        return 4;
    case ncclInt64:
    case ncclUint64:
    case ncclFloat64:
        return 8;
    default:
        return 0;
    }
}

// every rank of the group arrives before any leaves
void barrier(Group* g)
{
    std::unique_lock<std::mutex> lk(g->m);
    const uint64_t gen = g->generation;
    if (++g->arrived == g->world) {
        g->arrived = 0;
        ++g->generation;
        g->cv.notify_all();
    } else {
        g->cv.wait(lk, [&] { return g->generation != gen; });
    }
}

} // namespace

struct ncclComm {
    Group* group;
    int rank;
};

namespace {

thread_local std::vector<Op> t_ops;
thread_local ncclComm* t_comm = nullptr;
thread_local int t_depth = 0;

constexpr auto kWait = std::chrono::seconds(60);   // a partner that never comes is a failure

// One rank's group, completed before returning: its sends go into the
// mailboxes, its receives take their partners' sends in posting order (and
// copy them), then it waits until its own sends have been taken.  An
// AllGather is a collective round: every rank deposits its block, then
// every rank copies all of them.
ncclResult_t run_group(ncclComm* c, const std::vector<Op>& ops)
{
    Group* g = c->group;
    const int me = c->rank, world = g->world;
    bool bad = false;
    for (const Op& op : ops)
        if (hipStreamSynchronize(op.stream) != hipSuccess)
            bad = true;
    std::vector<std::shared_ptr<Posted>> mine;
    {
        std::lock_guard<std::mutex> lk(g->m);
        for (const Op& op : ops)
            if (op.kind == Op::SEND) {
                mine.push_back(std::make_shared<Posted>(Posted{op.src, op.bytes}));
                g->mail[size_t(me) * size_t(world) + size_t(op.peer)].push_back(mine.back());
            }
        g->cv.notify_all();
    }
    for (const Op& op : ops) {
        if (op.kind == Op::RECV) {
            std::shared_ptr<Posted> s;
            {
                std::unique_lock<std::mutex> lk(g->m);
                auto& box = g->mail[size_t(op.peer) * size_t(world) + size_t(me)];
                if (!g->cv.wait_for(lk, kWait, [&] { return !box.empty(); })) {
                    bad = true;   // no send from that peer
                    continue;
                }
                s = box.front();
                box.pop_front();
            }
            // on the receiver's stream, complete before the group returns (the
            // product orders its next launch on that stream after the Recv)
            const bool ok = s->bytes == op.bytes &&
                            hipMemcpyAsync(op.dst, s->src, op.bytes, hipMemcpyDefault, op.stream) == hipSuccess &&
                            hipStreamSynchronize(op.stream) == hipSuccess;
            bad = bad || !ok;
            std::lock_guard<std::mutex> lk(g->m);
            s->ok = ok;
            s->taken = true;
            g->cv.notify_all();
        } else if (op.kind == Op::ALLGATHER) {
            {
                std::lock_guard<std::mutex> lk(g->m);
                g->ag_src[size_t(me)] = op;
            }
            barrier(g);   // every rank's block is posted and ready
            for (int k = 0; k < world; ++k) {
                const Op& src = g->ag_src[size_t(k)];
                if (src.kind != Op::ALLGATHER || src.bytes != op.bytes ||
                    hipMemcpyAsync(static_cast<uint8_t*>(op.dst) + size_t(k) * op.bytes, src.src, op.bytes,
                                   hipMemcpyDefault, op.stream) != hipSuccess)
                    bad = true;
            }
            if (hipStreamSynchronize(op.stream) != hipSuccess)
                bad = true;
            barrier(g);   // every rank has copied before any posts its next block
        }
    }
    {
        std::unique_lock<std::mutex> lk(g->m);
        for (auto& s : mine) {
            if (!g->cv.wait_for(lk, kWait, [&] { return s->taken; }))
                bad = true;   // nobody received it
            else if (!s->ok)
                bad = true;
        }
    }
    if (bad) {
        g_errors.fetch_add(1);
        return ncclInvalidUsage;
    }
    return ncclSuccess;
}

ncclResult_t post(const Op& op, ncclComm* c)
{
    if (!c)
        return ncclInvalidArgument;
    if (op.kind != Op::ALLGATHER && (op.peer < 0 || op.peer >= c->group->world || op.peer == c->rank))
        return ncclInvalidArgument;
    if (t_depth == 0)
        return run_group(c, std::vector<Op>{op});
    if (t_comm && t_comm != c)
        return ncclInvalidUsage;   // one communicator per group (all the product uses)
    t_comm = c;
    t_ops.push_back(op);
    return ncclSuccess;
}

} // namespace

extern "C" {

int loopback_rccl_errors() { return g_errors.load(); }

ncclResult_t ncclGetUniqueId(ncclUniqueId* id)
{
    if (!id)
        return ncclInvalidArgument;
    std::memset(id->internal, 0, sizeof(id->internal));
    const uint64_t n = g_next_id.fetch_add(1);
    std::memcpy(id->internal, "loopback", 8);
    std::memcpy(id->internal + 8, &n, sizeof(n));
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank)
{
    if (!comm || nranks <= 0 || rank < 0 || rank >= nranks)
        return ncclInvalidArgument;
    std::lock_guard<std::mutex> lk(g_registry_lock);
    Group*& g = g_registry[std::string(id.internal, sizeof(id.internal))];
    if (!g)
        g = new Group(nranks);
    if (g->world != nranks)
        return ncclInvalidUsage;
    *comm = new ncclComm{g, rank};
    return ncclSuccess;
}

ncclResult_t ncclCommInitAll(ncclComm_t*, int, const int*) { return ncclInvalidUsage; }

ncclResult_t ncclCommDestroy(ncclComm_t comm)
{
    delete comm;
    return ncclSuccess;
}

ncclResult_t ncclGroupStart()
{
    ++t_depth;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd()
{
    if (t_depth <= 0)
        return ncclInvalidUsage;
    if (--t_depth > 0)
        return ncclSuccess;
    std::vector<Op> ops;
    ops.swap(t_ops);
    ncclComm* c = t_comm;
    t_comm = nullptr;
    return c ? run_group(c, ops) : ncclSuccess;
}

ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t s)
{
    return post(Op{Op::SEND, buf, nullptr, count * type_size(t), peer, s}, comm);
}

ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t s)
{
    return post(Op{Op::RECV, nullptr, buf, count * type_size(t), peer, s}, comm);
}

ncclResult_t ncclAllGather(const void* send, void* recv, size_t count, ncclDataType_t t, ncclComm_t comm,
                           hipStream_t s)
{
    return post(Op{Op::ALLGATHER, send, recv, count * type_size(t), -1, s}, comm);
}

} // extern "C"
