// wsg_capi.hip — implementation of the C-ABI in include/wsg_capi.h: device
// context, scratch, batch launches, host-staged paths, timing hooks.
// Nothing here computes payload bytes on the CPU: every payload byte of
// every entry point is produced by a gfx950 kernel.
#include "wsg_internal.h"
#include "wsg_env.h"
#include "wsg_trace.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

// Encode scratch (scan partials, piece starts, piece -> frame map); the ctx
// has one for wsg_encode_batch and every pipeline slot its own.
struct wsg_enc_scratch {
    uint64_t* d_scan = nullptr;          // sums | piece sums | prefixes | piece prefixes
    uint64_t scan_cap = 0;               // entries
    uint32_t* d_piece_start = nullptr;   // n + 1 piece starts
    uint64_t piece_start_cap = 0;
    uint32_t* d_piece_frame = nullptr;   // piece -> frame
    uint64_t piece_frame_cap = 0;
};

struct wsg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    int num_cus = 256;
    int blocks_per_cu = 32;       // encode / fan-out / xor grids
    // k_encode_mask grid: one wave per piece up to 2^31 threads (137 GB of
    // frames), grid-stride beyond.  A grid capped at 1024 blocks/CU dealt C5's
    // 5.2 M pieces five per wave, grid-stride, so resident waves streamed five
    // regions GiB apart: 6.12 vs 5.43 ms for the 16 GiB job (tools/enc_ab.py,
    // round 3); at or under a grid's worth of pieces the two are the same
    int enc_blocks_per_cu = 32768;
    uint64_t enc_launch_pieces = 0;   // k_encode_mask: pieces per launch (0: all in one)
    uint64_t xor_direct_max = 64 << 10;   // per-call XOR off the lane: kernel on the pinned stage up to this size
    uint64_t seg_bytes = 32ull << 20;     // staged host pipelines: segment of about this many wire bytes ($WSG_STAGE_MB)
    bool multi_share = false;             // multi-context splits keep several contexts of one device ($WSG_HOST_MULTI_SHARE)
    // host batches up to this many wire bytes whose buffers are page-locked:
    // the kernels read and write them in place (one launch sequence and one
    // synchronize, no staging copies); $WSG_HOST_DIRECT_MAX
    uint64_t host_direct_max = 4 << 20;   // 1-4 MB batches 1.6-2x faster direct, 16 MB even (profiles/r3/host_direct_sizes.log)
    bool check = false;            // $WSG_CHECK=1: operand ranges validated before every device launch (debug)
    int dec_blocks_per_cu = 4096;  // k_decode grid cap: one 16 KiB tile per block up to 16 GiB of wire (tools/tune.py, round 2: C2 84.3 vs 85.1 us at 48 blocks/CU, 88.1 at two tiles per block; C3 ragged 0.685 vs 0.705 ms at 256, 0.783 at 48)
    int fan_waves_per_cu = 6;    // fan-out period path: waves per CU (tools/c4_ab.py, graph-replayed C4: 6 -> 8.10 us, 4 -> 8.16, 8 -> 8.32)
    // fan-out period path: waves per workgroup (A/B $WSG_FAN_WPB; one-wave
    // workgroups measured best: C4 8.5 us against 9.3 at 4 and 9.0 at 8-16,
    // tools/c4_ab.py with graph-replayed launches; an empty kernel of that
    // grid is 1.65 us either way)
    int fan_wpb = 1;
    uint64_t small_avg = wsg::SMALL_AVG;   // batch encode: k_encode_small when wire_cap <= n * small_avg
    unsigned long long* d_err = nullptr;        // latch of the caller-visible async entry points (wsg_sync)
    // latches of the host-staged pipelines (their own status): [0] the
    // decodes' (read back, re-armed after an error), [1] the encodes' (their
    // capacity is checked on the host, so nothing they latch is read: apart,
    // so that it never disables the decodes' latch read-back)
    unsigned long long* d_err_host = nullptr;
    unsigned long long* h_err_copy = nullptr;   // page-locked: d_err_host after a large in-place decode
    // scratch
    wsg_enc_scratch enc;
    // staging for host entry points
    uint8_t* d_stage = nullptr;
    uint8_t* h_stage = nullptr;
    uint64_t stage_cap = 0;
    uint64_t* d_fs = nullptr;
    wsg_recv_info* d_info = nullptr;
    uint64_t fs_cap = 0;
    // pipelined host path (wsg_decode_batch_host): one stream + staging per slot
    struct Slot {
        hipStream_t stream = nullptr;
        hipEvent_t done = nullptr;       // the segment's last copy back has finished
        hipEvent_t h2d_done = nullptr;   // role pipeline: inputs are in HBM
        hipEvent_t k_done = nullptr;     // role pipeline: kernels have finished
        uint8_t* d_wire = nullptr;       // segment, decoded in place
        uint64_t wire_cap = 0;
        uint8_t* h_in = nullptr;         // pinned staging for pageable callers
        uint8_t* h_out = nullptr;
        uint64_t host_cap = 0;
        uint64_t* h_fs = nullptr;        // rebased frame starts (pinned)
        wsg_recv_info* h_info = nullptr; // info staging (pinned)
        uint64_t* d_fs = nullptr;
        wsg_recv_info* d_info = nullptr;
        uint64_t frames_cap = 0;
        // encode (wsg_encode_batch_host): payload in, frames out in d_wire
        uint8_t* d_payload = nullptr;
        uint64_t payload_cap = 0;
        wsg_send_desc* d_desc = nullptr;
        uint64_t desc_cap = 0;
        wsg_send_desc* h_desc = nullptr;  // rebased descriptors (pinned)
        uint64_t h_desc_cap = 0;
        uint64_t* d_woff = nullptr;
        uint64_t woff_cap = 0;
        wsg_enc_scratch enc;
        // work to finish on the host once `done` has fired
        bool busy = false;
        uint8_t* out_dst = nullptr;      // pageable destination of h_out (null: DMA'd directly)
        uint64_t out_src = 0, out_len = 0;
        wsg_recv_info* info_dst = nullptr;
        uint32_t info_n = 0;
        uint64_t base = 0;               // wire offset of the segment's first byte
    };
    static constexpr int kSlots = 3;
    Slot slots[kSlots];
    // role streams of the host pipelines: every H2D copy on one stream, every
    // kernel on another, every D2H copy on a third, so the two copy directions
    // run concurrently while kernels run between them
    hipStream_t s_h2d = nullptr, s_kern = nullptr, s_d2h = nullptr;
    // the host lane (wsg_internal.h): page-locked host batches of at most
    // lane_max wire bytes (and per-call XORs of at most that many bytes) go to
    // the device's resident lane, shared by every context of the process,
    // through its mailboxes instead of a launch + synchronize ($WSG_LANE_MAX,
    // 0 = never)
    struct LaneServer* lane = nullptr;   // the device's (made on first use)
    uint64_t lane_max = 512 << 10;
    uint32_t lane_groups = wsg::LANE_GROUPS_MAX;   // most frame groups of one request ($WSG_LANE_GROUPS)
    uint64_t lane_requests = 0;          // requests this context put on the lane (wsg_lane_stats)
    bool dead = false;                   // a lane request neither answered nor drained: buffers may still be written
    // timing of the dominant kernel
    struct EvPair {
        hipEvent_t a, b;
    };
    int timing = 0;            // 0 off; k > 0: time every k-th dominant-kernel launch
    uint64_t timing_seq = 0;
    std::vector<EvPair> pending, pool;
    double acc_ms = 0.0;
    uint64_t launches = 0;
    double min_ms = 0.0, max_ms = 0.0;   // extremes of the launches since the last reset
};

namespace {

#define WSG_HIP(expr)                                                                                        \
    do {                                                                                                     \
        if ((expr) != hipSuccess)                                                                            \
            return WSG_EHIP;                                                                                 \
    } while (0)

constexpr unsigned long long kNoError = ~0ull;

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
// NULL selects HIP's default (null) stream, as in every HIP API.
inline hipStream_t pick(wsg_ctx*, void* s) { return static_cast<hipStream_t>(s); }
inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

int grid_for(const wsg_ctx* c, uint64_t tiles, int blocks_per_cu = 0)
{
    const uint64_t cap = uint64_t(c->num_cus) * uint64_t(blocks_per_cu ? blocks_per_cu : c->blocks_per_cu);
    return int(std::max<uint64_t>(1, std::min(tiles, cap)));
}

void free_enc(wsg_enc_scratch& e)
{
    (void)hipFree(e.d_scan);
    (void)hipFree(e.d_piece_start);
    (void)hipFree(e.d_piece_frame);
    e = wsg_enc_scratch{};
}

// grow a device array of T to at least `want` entries
template <class T>
int ensure_array(T*& ptr, uint64_t& cap, uint64_t want)
{
    want = std::max<uint64_t>(want, 1);
    if (want <= cap)
        return WSG_OK;
    WSG_HIP(hipDeviceSynchronize());
    if (ptr)
        WSG_HIP(hipFree(ptr));
    ptr = nullptr;
    cap = 0;
    if (hipMalloc(&ptr, want * sizeof(T)) != hipSuccess)
        return WSG_ENOMEM;
    cap = want;
    return WSG_OK;
}

int ensure_stage(wsg_ctx* c, uint64_t bytes, uint64_t frames)
{
    bytes = std::max<uint64_t>((bytes + 15) & ~uint64_t(15), 16);
    if (bytes > c->stage_cap) {
        WSG_HIP(hipDeviceSynchronize());
        if (c->d_stage)
            WSG_HIP(hipFree(c->d_stage));
        if (c->h_stage)
            WSG_HIP(hipHostFree(c->h_stage));
        c->d_stage = nullptr;
        c->h_stage = nullptr;
        c->stage_cap = 0;
        if (hipMalloc(&c->d_stage, bytes) != hipSuccess)
            return WSG_ENOMEM;
        if (hipHostMalloc(&c->h_stage, bytes, hipHostMallocDefault) != hipSuccess)
            return WSG_ENOMEM;
        c->stage_cap = bytes;
    }
    frames = std::max<uint64_t>(frames, 1);
    if (frames > c->fs_cap) {
        WSG_HIP(hipDeviceSynchronize());
        if (c->d_fs)
            WSG_HIP(hipFree(c->d_fs));
        if (c->d_info)
            WSG_HIP(hipFree(c->d_info));
        c->d_fs = nullptr;
        c->d_info = nullptr;
        c->fs_cap = 0;
        if (hipMalloc(&c->d_fs, frames * sizeof(uint64_t)) != hipSuccess ||
            hipMalloc(&c->d_info, frames * sizeof(wsg_recv_info)) != hipSuccess)
            return WSG_ENOMEM;
        c->fs_cap = frames;
    }
    return WSG_OK;
}

// Record the start event of a timed kernel; returns the pair index or -1.
int timing_begin(wsg_ctx* c, hipStream_t s)
{
    if (c->timing <= 0 || (c->timing_seq++ % uint64_t(c->timing)) != 0)
        return -1;
    wsg_ctx::EvPair ev;
    if (!c->pool.empty()) {
        ev = c->pool.back();
        c->pool.pop_back();
    } else {
        if (hipEventCreate(&ev.a) != hipSuccess || hipEventCreate(&ev.b) != hipSuccess)
            return -1;
    }
    (void)hipEventRecord(ev.a, s);
    c->pending.push_back(ev);
    return int(c->pending.size()) - 1;
}

void timing_end(wsg_ctx* c, hipStream_t s, int idx)
{
    if (idx >= 0)
        (void)hipEventRecord(c->pending[size_t(idx)].b, s);
}

int drain_timing(wsg_ctx* c)
{
    for (auto& ev : c->pending) {
        WSG_HIP(hipEventSynchronize(ev.b));
        float ms = 0.f;
        WSG_HIP(hipEventElapsedTime(&ms, ev.a, ev.b));
        c->acc_ms += ms;
        c->min_ms = c->launches ? std::min(c->min_ms, double(ms)) : double(ms);
        c->max_ms = c->launches ? std::max(c->max_ms, double(ms)) : double(ms);
        c->launches += 1;
        c->pool.push_back(ev);
    }
    c->pending.clear();
    return WSG_OK;
}

} // namespace

int wsg::ctx_device(const wsg_ctx* c) { return c ? c->device : 0; }
bool wsg::ctx_multi_share(const wsg_ctx* c) { return c && c->multi_share; }

namespace {

// Checked launches ($WSG_CHECK=1, a debug mode): [p, p + bytes) must lie in
// ONE device allocation (hipMemGetAddressRange), which every access of the
// kernel to that operand stays inside when the sizes passed are right.  GPU
// address sanitizers are not available on the target pool; this catches a
// short buffer or a wrong size on the host, before the kernel runs.
bool in_alloc(const void* p, uint64_t bytes)
{
    if (bytes == 0)
        return true;
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, const_cast<void*>(p)) != hipSuccess)
        return false;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p), b = reinterpret_cast<uintptr_t>(base);
    return a >= b && a - b <= size && bytes <= size - (a - b);
}

} // namespace

namespace {

// Page-locked host memory the kernels read and write in place (the session
// batches' buffers, the direct paths' tables): the runtime's default
// (mapped at the same address on the device).  The lane's system-scope
// acquire / release fences keep its reads and writes of it coherent.
unsigned host_alloc_flags() { return unsigned(hipHostMallocDefault); }

// The blocks wsg_host_alloc made (page-locked, mapped at the same address on
// the device): a host batch in one of them (the session batches' buffers
// always are) is recognised without a runtime query, whose few us per
// pointer were a visible share of a small batch's call (tools/lane_ab.py).
// A block leaves the table before it is freed.
std::mutex& host_blocks_lock()
{
    static std::mutex* m = new std::mutex;   // leaked: used from static destructors
    return *m;
}
std::map<uintptr_t, uint64_t>& host_blocks()
{
    static auto* b = new std::map<uintptr_t, uint64_t>;
    return *b;
}
void host_blocks_add(const void* p, uint64_t bytes)
{
    std::lock_guard<std::mutex> g(host_blocks_lock());
    host_blocks()[reinterpret_cast<uintptr_t>(p)] = bytes;
}
// Bumped by every removal: a thread's cached blocks (in_host_block) are
// trusted only while it is unchanged.
std::atomic<uint64_t> g_blocks_gen{0};
void host_blocks_remove(const void* p)
{
    std::lock_guard<std::mutex> g(host_blocks_lock());
    host_blocks().erase(reinterpret_cast<uintptr_t>(p));
    g_blocks_gen.fetch_add(1, std::memory_order_release);
}
// Each host call checks several pointers (wire, output, table, records):
// under one process-wide lock, eight IO threads queued on it; a thread
// remembers the last blocks it found, valid until a block is removed.
struct BlockHit {
    uintptr_t base = 0;
    uint64_t size = 0;
    uint64_t gen = ~uint64_t(0);
};
thread_local BlockHit t_hits[4] __attribute__((tls_model("initial-exec")));
thread_local uint32_t t_hit_next __attribute__((tls_model("initial-exec"))) = 0;
bool in_host_block(const void* p, uint64_t bytes = 1)
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint64_t gen = g_blocks_gen.load(std::memory_order_acquire);
    for (const BlockHit& h : t_hits)
        if (h.gen == gen && a - h.base < h.size && bytes <= h.size - (a - h.base))
            return true;
    std::lock_guard<std::mutex> g(host_blocks_lock());
    auto& m = host_blocks();
    auto it = m.upper_bound(a);
    if (it == m.begin())
        return false;
    --it;
    if (!(a - it->first < it->second && bytes <= it->second - (a - it->first)))
        return false;
    t_hits[t_hit_next++ & 3] = BlockHit{it->first, it->second, gen};
    return true;
}

} // namespace

// ---- the host lane --------------------------------------------------------

// One lane per device, shared by every context of the process on it
// (wsg_internal.h): its mailboxes, its stream and the launches of its
// resident kernel.  Servers are made on first use and live as long as the
// process (the at-exit handler stops their kernels).
struct LaneServer {
    int device = 0;
    wsg::LaneBell* bell = nullptr;   // page-locked, coherent, mapped
    hipStream_t stream = nullptr;
    uint32_t W = 8;                  // workgroups ($WSG_LANE_WGS)
    uint64_t idle_ticks = 0, yield_ticks = 0, delay_ticks = 0;
    int timeout_ms = 5000;           // a request unanswered this long: the lane is given up ($WSG_LANE_TIMEOUT_MS)
    int drain_ms = 2000;             // ... and waited for this long to leave ($WSG_LANE_DRAIN_MS)
    uint32_t delay_gens = ~0u;       // test hook: generations up to this one start late ($WSG_TEST_LANE_DELAY_GENS)
    std::mutex launch_lock;
    std::atomic<uint32_t> gen{0};        // the last launch's generation (0: none yet)
    std::atomic<bool> broken{false};     // given up: no launches until re-armed, every caller takes the launch paths
    // a lane given up is re-armed (lane_rearm) once its stream has drained and
    // this hold-off has passed: it doubles with every give-up in a row (from
    // kRearmFirstMs up to kRearmMaxMs) and resets once a re-armed lane answers
    std::atomic<int64_t> retry_at_ns{0};
    uint32_t backoff_ms = 0;             // (under launch_lock)
    std::atomic<bool> rearmed{false};    // re-armed and not yet answered a request since
    std::atomic<uint64_t> give_ups{0}, rearms{0};   // (wsg_lane_events)
    uint32_t delay_every = 0;            // test hook: every launch whose generation it divides starts late too ($WSG_TEST_LANE_DELAY_EVERY)
    std::atomic<uint64_t> tickets{0};    // next ticket
    std::atomic<int> inflight{0};        // requests posted and not yet answered
    std::atomic<uint64_t> launches{0};
    // per mailbox slot: the last ticket + 1 whose caller has read its answer
    // (a slot is reused only after that: its previous task done and read)
    std::atomic<uint64_t> released[wsg::LANE_WGS_MAX * wsg::LANE_RING];
};

namespace {

std::mutex& lane_servers_lock()
{
    static std::mutex* m = new std::mutex;   // leaked: used at exit
    return *m;
}
std::map<int, LaneServer*>& lane_servers()
{
    static auto* v = new std::map<int, LaneServer*>;
    return *v;
}

// Wait (at most ms) until every launch on the lane's stream has ended.
bool lane_drained(LaneServer* s, int ms)
{
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t q = hipStreamQuery(s->stream);
        if (q == hipSuccess)
            return true;
        if (q != hipErrorNotReady) {
            (void)hipGetLastError();
            return false;
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(ms))
            return false;
        std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
}

// Start the lane's mailboxes at ticket `base` (a multiple of W), with no
// launch running or queued and no request in flight: every workgroup resumes
// at its first ticket from `base` on, and every slot counts as answered and
// read, so the first W * LANE_RING tickets from `base` post without waiting.
// (Slots keep their old units: every tag in them is below base + 1, and
// every ticket from base on has a tag above that.)
void lane_set_frontier(LaneServer* s, uint64_t base)
{
    const uint64_t W = s->W, R = wsg::LANE_RING;
    for (uint32_t g = 0; g < s->W; ++g)
        __atomic_store_n(&s->bell->next_j[g], base / W, __ATOMIC_RELAXED);
    for (uint64_t t = base; t < base + W * R; ++t)
        s->released[(t % W) * R + (t / W) % R].store(t >= W * R ? t - W * R + 1 : 0, std::memory_order_relaxed);
    s->tickets.store(base);
}

int64_t steady_ns()
{
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// Every lane told to leave at process exit (a lane also leaves on its own
// after its idle limit); a lane already given up is not waited for again.
void lanes_at_exit()
{
    std::lock_guard<std::mutex> g(lane_servers_lock());
    for (auto& kv : lane_servers()) {
        LaneServer* s = kv.second;
        if (s->broken.load() || s->gen.load() == 0)
            continue;
        __atomic_store_n(&s->bell->ctl.stop, 1u, __ATOMIC_RELEASE);
        (void)lane_drained(s, 1000);
    }
}

// The device's lane, made on first use (nullptr: it cannot be made).
LaneServer* lane_server(int device)
{
    std::lock_guard<std::mutex> g(lane_servers_lock());
    auto& m = lane_servers();
    auto it = m.find(device);
    if (it != m.end())
        return it->second;
    auto* s = new (std::nothrow) LaneServer;
    if (!s)
        return nullptr;
    s->device = device;
    for (auto& r : s->released)
        r.store(0, std::memory_order_relaxed);
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || khz <= 0)
        khz = 100000;   // 100 MHz, the gfx9 constant clock
    long idle_us = 2000, yield_us = 2000, delay_us = 0;
    uint64_t ticket_base = 0;
    bool stale_xres = false;
    {
        std::lock_guard<std::recursive_mutex> eg(wsg::env_mutex());
        if (const char* e = wsg::envp("WSG_LANE_WGS")) {
            const long v = std::atol(e);
            if (v >= 1 && v <= long(wsg::LANE_WGS_MAX))
                s->W = uint32_t(v);
        }
        if (const char* e = wsg::envp("WSG_LANE_IDLE_US"))
            idle_us = std::max(1l, std::min(1000000l, std::atol(e)));
        if (const char* e = wsg::envp("WSG_LANE_YIELD_US"))
            yield_us = std::max(1l, std::min(1000000l, std::atol(e)));
        if (const char* e = wsg::envp("WSG_LANE_TIMEOUT_MS"))
            s->timeout_ms = int(std::max(1l, std::min(600000l, std::atol(e))));
        if (const char* e = wsg::envp("WSG_LANE_DRAIN_MS"))
            s->drain_ms = int(std::max(1l, std::min(600000l, std::atol(e))));
        if (const char* e = wsg::envp("WSG_TEST_LANE_DELAY_US"))   // test hook: the kernel starts late
            delay_us = std::max(0l, std::min(10000000l, std::atol(e)));
        if (const char* e = wsg::envp("WSG_TEST_LANE_DELAY_GENS"))   // ... only its first launches
            s->delay_gens = uint32_t(std::max(0l, std::min(1000000l, std::atol(e))));
        if (const char* e = wsg::envp("WSG_TEST_LANE_DELAY_EVERY")) {   // ... or every n-th (then only those
            s->delay_every = uint32_t(std::max(0l, std::min(1000000l, std::atol(e))));   //  and the first GENS)
            if (!wsg::envp("WSG_TEST_LANE_DELAY_GENS"))
                s->delay_gens = 0;
        }
        if (const char* e = wsg::envp("WSG_TEST_LANE_TICKET_BASE"))  // test hook: the ticket counter starts here
            ticket_base = std::strtoull(e, nullptr, 10);
        if (const char* e = wsg::envp("WSG_TEST_LANE_STALE_XRES"))   // ... with every inline answer unit stale
            stale_xres = *e == '1';
    }
    s->idle_ticks = uint64_t(idle_us) * uint64_t(khz) / 1000u;
    s->yield_ticks = uint64_t(yield_us) * uint64_t(khz) / 1000u;
    s->delay_ticks = uint64_t(delay_us) * uint64_t(khz) / 1000u;
    void* p = nullptr;
    int dev0 = 0;
    (void)hipGetDevice(&dev0);
    // A running lane holds the hardware queue its stream is on: every packet
    // queued behind it waits until the launch ends.  The runtime keeps streams
    // of each priority on their own queues, so the lane goes on a
    // high-priority stream (ahead of nothing but itself) and the contexts'
    // ordinary streams never queue behind it.
    int lo = 0, hi = 0;
    const bool ok = hipSetDevice(device) == hipSuccess &&
                    hipHostMalloc(&p, sizeof(wsg::LaneBell), hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
                    hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess &&
                    hipStreamCreateWithPriority(&s->stream, hipStreamNonBlocking, hi) == hipSuccess;
    (void)hipSetDevice(dev0);
    if (!ok) {
        if (p)
            (void)hipHostFree(p);
        delete s;
        return nullptr;
    }
    std::memset(p, 0, sizeof(wsg::LaneBell));
    s->bell = static_cast<wsg::LaneBell*>(p);
    if (ticket_base) {
        lane_set_frontier(s, ticket_base / s->W * s->W);
        if (stale_xres) {
            // every slot's inline answer units as a task 2^32 tickets before
            // its next one would have left them: the low 32 bits of the tag
            // are the next ticket's, the dword not its answer
            const uint64_t b = s->tickets.load();
            for (uint64_t t = b; t < b + uint64_t(s->W) * wsg::LANE_RING; ++t)
                for (uint64_t& u : s->bell->xres[t % s->W][(t / s->W) % wsg::LANE_RING].u)
                    u = (uint64_t(uint32_t(t + 1)) << 32) | 0xA5A5A5A5u;
        }
    }
    static std::once_flag once;
    std::call_once(once, [] { std::atexit(lanes_at_exit); });
    m[device] = s;
    return s;
}

constexpr uint32_t kRearmFirstMs = 50, kRearmMaxMs = 4000;

// (under launch_lock) No launch until re-armed, and every workgroup leaves at
// its next check without taking another task; the hold-off before a re-arm
// doubles with every give-up in a row.
void lane_break_locked(LaneServer* s)
{
    if (s->broken.load())
        return;
    s->backoff_ms = s->backoff_ms ? std::min(kRearmMaxMs, s->backoff_ms * 2) : kRearmFirstMs;
    s->retry_at_ns.store(steady_ns() + int64_t(s->backoff_ms) * 1000000);
    s->rearmed.store(false);
    s->give_ups.fetch_add(1);
    s->broken.store(true);
    __atomic_store_n(&s->bell->ctl.stop, 1u, __ATOMIC_RELEASE);
}

// Give the lane up (a request went unanswered).
void lane_give_up(LaneServer* s)
{
    std::lock_guard<std::mutex> g(s->launch_lock);
#ifdef WSG_DIAG_LANE   // (diagnostic build: where the mailboxes stand at a give-up)
    std::fprintf(stderr, "lane give-up: tickets %llu gen %u closing %u stop %u\n",
                 (unsigned long long)s->tickets.load(), s->gen.load(), s->bell->ctl.closing, s->bell->ctl.stop);
    for (uint32_t q = 0; q < s->W; ++q)
        std::fprintf(stderr, "  wg %u next_j %llu slot %llu tag0 %llu\n", q, (unsigned long long)s->bell->next_j[q],
                     (unsigned long long)(s->bell->next_j[q] % wsg::LANE_RING),
                     (unsigned long long)s->bell->box[q][s->bell->next_j[q] % wsg::LANE_RING].w[0].tag);
#endif
    lane_break_locked(s);
}

// Bring a given-up lane back: once its hold-off has passed, no request is in
// flight (every caller of the give-up has taken its fallback and released its
// slots) and its stream has drained (no workgroup left to write a request's
// buffers), the mailboxes restart past every ticket handed out so far —
// tasks posted to the old lane and never taken are skipped, not run — and
// the next request launches a new generation.  False: still given up.
bool lane_rearm(LaneServer* s)
{
    if (steady_ns() < s->retry_at_ns.load(std::memory_order_relaxed))
        return false;
    std::unique_lock<std::mutex> g(s->launch_lock, std::try_to_lock);
    if (!g.owns_lock())
        return false;
    if (!s->broken.load())
        return true;
    if (s->inflight.load() != 0)
        return false;
    const hipError_t q = hipStreamQuery(s->stream);
    if (q != hipSuccess) {
        if (q != hipErrorNotReady)
            (void)hipGetLastError();
        s->retry_at_ns.store(steady_ns() + int64_t(s->backoff_ms) * 1000000);
        return false;
    }
    const uint64_t W = s->W;
    lane_set_frontier(s, (s->tickets.load() + W - 1) / W * W);
    __atomic_store_n(&s->bell->ctl.stop, 0u, __ATOMIC_RELAXED);
    // the last generation counts as ended: the next request launches
    __atomic_store_n(&s->bell->ctl.closing, s->gen.load(), __ATOMIC_RELEASE);
    s->rearmed.store(true);
    s->rearms.fetch_add(1);
    s->broken.store(false);
    return true;
}

// Launch the next generation if generation `seen` is the last one (none yet,
// or it announced its end): queued behind it on the lane's stream, it starts
// once every workgroup of the old one has left, each mailbox where it was.
void lane_relaunch(LaneServer* s, uint32_t seen)
{
    std::lock_guard<std::mutex> g(s->launch_lock);
    if (s->broken.load() || s->gen.load() != seen)
        return;
    uint32_t next = seen + 1;
    if (next == 0)
        next = 1;
    if (wsg::launch_lane(s->stream, s->bell, s->W, s->idle_ticks, s->yield_ticks, next,
                         next <= s->delay_gens || (s->delay_every && next % s->delay_every == 0) ? s->delay_ticks
                                                                                                 : 0) != hipSuccess) {
        (void)hipGetLastError();
        lane_break_locked(s);
        return;
    }
    s->launches.fetch_add(1);
    s->gen.store(next);
}

// A launch running (or queued) that has not announced its end; else launch.
void lane_ensure_running(LaneServer* s)
{
    const uint32_t g = s->gen.load(std::memory_order_acquire);
    if (g == 0 || __atomic_load_n(&s->bell->ctl.closing, __ATOMIC_ACQUIRE) == g)
        lane_relaunch(s, g);
}

// The lane for this context's request, or nullptr (lane off for the context,
// the lane given up, or it cannot be made).
LaneServer* lane_for(wsg_ctx* c)
{
    if (!c->lane_max)
        return nullptr;
    if (!c->lane) {
        c->lane = lane_server(c->device);
        if (!c->lane) {
            c->lane_max = 0;
            return nullptr;
        }
    }
    if (c->lane->broken.load(std::memory_order_relaxed) && !lane_rearm(c->lane))
        return nullptr;
    return c->lane;
}

// A request's frame groups: runs of whole frames [f, f + cnt), each at most
// LANE_THREADS frames over the byte range [lo, hi) of its boundaries b(f) ..
// b(f + cnt) (b(0) = 0, b(n) = the request's end), about equal in bytes and
// about as many as the lane has idle workgroups (W shared among the requests
// in flight, at most the context's lane_groups).  A group's range is at most
// `limit` bytes: strict (decode: the range is staged in LDS) a frame larger
// than that does not fit the lane; otherwise (encode: the payload span is
// staged when it fits, read in place when not) such a frame is a group alone.
// Returns the group count; 0 when the request does not fit the lane (more
// than LANE_GROUPS_MAX groups, or a frame too large for a strict stage).
struct LaneGroup {
    uint32_t f, cnt;
    uint64_t lo, hi;
};

template <class Bound>
uint32_t lane_plan(const wsg_ctx* c, const LaneServer* s, uint32_t n, uint64_t limit, bool strict, Bound b,
                   LaneGroup* g)
{
    const uint32_t busy = uint32_t(std::max(0, s->inflight.load(std::memory_order_relaxed))) + 1;
    const uint32_t want = std::max<uint32_t>(1, std::min(s->W / busy, c->lane_groups));
    const uint64_t total = b(n);
    const uint64_t target = std::max<uint64_t>(1, (total + want - 1) / want);
    // b is non-decreasing: the first index in [a, z] whose bound is >= v (z if none)
    const auto first_at_least = [&b](uint32_t a, uint32_t z, uint64_t v) {
        while (a < z) {
            const uint32_t m = a + (z - a) / 2;
            if (b(m) >= v)
                z = m;
            else
                a = m + 1;
        }
        return a;
    };
    uint32_t k = 0;
    for (uint32_t f = 0; f < n;) {
        if (k == wsg::LANE_GROUPS_MAX)
            return 0;
        const uint64_t lo = b(f);
        if (strict && b(f + 1) - lo > limit)
            return 0;
        // the group ends at the first bound reaching the target, before the
        // first past the limit, after at most LANE_THREADS frames, and holds
        // at least one frame
        const uint32_t z = uint32_t(std::min<uint64_t>(n, uint64_t(f) + wsg::LANE_THREADS));
        const uint32_t e_target = first_at_least(f + 1, z, lo + target);
        uint32_t e_limit = first_at_least(f + 1, z, lo + limit + 1);
        if (b(e_limit) - lo > limit)
            --e_limit;
        const uint32_t e = std::max(f + 1, std::min(e_target, e_limit));
        g[k++] = LaneGroup{f, e - f, lo, b(e)};
        f = e;
    }
    return k;
}

// Requests of at most this many frames fit the lane (groups of at most
// LANE_THREADS frames, at most LANE_GROUPS_MAX groups).
constexpr uint32_t kLaneMaxFrames = wsg::LANE_GROUPS_MAX * wsg::LANE_THREADS;

enum LaneResult { LANE_DONE = 0, LANE_FALLBACK = 1, LANE_LOST = 2 };

// Post a request's groups (task words words[k], w[0] = op | n << 32) and wait
// for every answer.  LANE_DONE: answered (*errs: the frames with an error).
// LANE_FALLBACK: not done by the lane, which has left: the caller does the
// request on the launch path (*answered: groups the lane did finish before it
// was given up — their outputs are written).  LANE_LOST: given up and the lane
// did not leave in time: it may still write the request's buffers, so the
// caller must not reuse them (the context is marked dead).
// xwords > 0: one inline-XOR task, answered by its self-tagged units
// (wsg::LaneXres), whose dwords go to xout.
LaneResult lane_run(wsg_ctx* c, LaneServer* s, const uint64_t (*words)[wsg::LANE_WORDS], uint32_t groups,
                    uint64_t* errs, uint32_t* answered, uint32_t xwords = 0, uint32_t* xout = nullptr)
{
    *errs = 0;
    *answered = 0;
    // in flight before the check: a re-arm (which needs none in flight while
    // the lane is given up) never runs under a request that saw it working
    s->inflight.fetch_add(1);
    if (s->broken.load()) {
        s->inflight.fetch_sub(1);
        return LANE_FALLBACK;
    }
    const uint32_t W = s->W, R = wsg::LANE_RING;
    const uint64_t x = s->tickets.fetch_add(groups);
    ++c->lane_requests;
    const auto t0 = std::chrono::steady_clock::now();
    auto late = [&] { return std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(s->timeout_ms); };
    // post: every group's slot (its previous task answered and read first),
    // each unit's value then its tag, the first unit last
    for (uint32_t k = 0; k < groups; ++k) {
        const uint64_t tk = x + k;
        const uint32_t wg = uint32_t(tk % W), slot = uint32_t((tk / W) % R);
        if (tk >= uint64_t(W) * R) {
            const uint64_t prev = tk - uint64_t(W) * R + 1;
            for (uint64_t i = 1; s->released[wg * R + slot].load(std::memory_order_acquire) != prev; ++i) {
                if ((i & 1023) == 0 && late()) {   // (posted anyway: the lane is stopped)
                    lane_give_up(s);
                    break;
                }
                __builtin_ia32_pause();
            }
        }
#ifndef WSG_DIAG_NO_XRES_POISON   // (diagnostic build only: shows test_lane_inline_answers_across_the_tag_wrap failing)
        if (xwords) {
            // an inline answer's units carry only the low 32 bits of the
            // ticket, which recur in this slot every 2^32 tickets (W * R
            // divides 2^32), and the slot's last inline task may have been
            // that long ago: units that tag no ticket of this lap before the
            // task goes out (its answer has been read: `released`, above)
            for (uint32_t q = 0; q < xwords; ++q)
                __atomic_store_n(&s->bell->xres[wg][slot].u[q], uint64_t(~uint32_t(tk + 1)) << 32, __ATOMIC_RELAXED);
        }
#endif
        wsg::LaneTask* T = &s->bell->box[wg][slot];
        for (uint32_t u = wsg::LANE_WORDS; u-- > 0;) {
            T->w[u].v = words[k][u];
            __atomic_store_n(&T->w[u].tag, tk + 1, __ATOMIC_RELEASE);
        }
    }
    lane_ensure_running(s);
    // wait for the answers, group by group
    uint32_t k = 0;
    bool gave_up = false;
    for (uint64_t i = 1; k < groups; ++i) {
        while (k < groups) {
            const uint64_t tk = x + k;
            const uint32_t wg = uint32_t(tk % W), slot = uint32_t((tk / W) % R);
            if (xwords) {   // (one group) every unit shows the tag: the answer is complete
                const wsg::LaneXres& xr = s->bell->xres[wg][slot];
                uint32_t q = 0;
                for (; q < xwords; ++q) {
                    const uint64_t u = __atomic_load_n(&xr.u[q], __ATOMIC_ACQUIRE);
                    if (uint32_t(u >> 32) != uint32_t(tk + 1))
                        break;
                    xout[q] = uint32_t(u);
                }
                if (q < xwords)
                    break;
            } else {
                wsg::LaneResp& r = s->bell->resp[wg][slot];
                if (__atomic_load_n(&r.done, __ATOMIC_ACQUIRE) != tk + 1)
                    break;
                *errs += __atomic_load_n(&r.errs, __ATOMIC_RELAXED);
            }
            s->released[wg * R + slot].store(tk + 1, std::memory_order_release);
            ++k;
        }
        if (k == groups)
            break;
        if ((i & 255) == 0) {
            if (s->broken.load()) {
                gave_up = true;
                break;
            }
            lane_ensure_running(s);   // the launch announced its end before these tasks: the next one
            if (late()) {
                lane_give_up(s);
                gave_up = true;
                break;
            }
        }
        __builtin_ia32_pause();
    }
    if (!gave_up) {
        s->inflight.fetch_sub(1);
        if (s->rearmed.load(std::memory_order_relaxed)) {   // the re-armed lane works: the next give-up's hold-off starts over
            std::lock_guard<std::mutex> g(s->launch_lock);
            if (s->rearmed.exchange(false) && !s->broken.load())
                s->backoff_ms = 0;
        }
        return LANE_DONE;
    }
    // Given up: nothing of the request may be touched until the lane has
    // left (a workgroup that took a task before `stop` finishes it).
    const bool drained = lane_drained(s, s->drain_ms);
    for (uint32_t q = 0; q < groups; ++q) {
        const uint64_t tk = x + q;
        const uint32_t wg = uint32_t(tk % W), slot = uint32_t((tk / W) % R);
        if (xwords ? uint32_t(__atomic_load_n(&s->bell->xres[wg][slot].u[0], __ATOMIC_ACQUIRE) >> 32) == uint32_t(tk + 1)
                   : __atomic_load_n(&s->bell->resp[wg][slot].done, __ATOMIC_ACQUIRE) == tk + 1)
            ++*answered;
        s->released[wg * R + slot].store(tk + 1, std::memory_order_release);
    }
    s->inflight.fetch_sub(1);
    if (!drained) {
        c->dead = true;
        return LANE_LOST;
    }
    return LANE_FALLBACK;
}

} // namespace

extern "C" {

int wsg_abi_version(void) { return WSG_ABI_VERSION; }

}   // extern "C"

// The runtime's first initialization under the environment lock (wsg_env.h):
// every entry point that can be a process's first HIP call goes through here
// before touching HIP or reading a knob.
void wsg::hip_init_once()
{
    static std::once_flag once;
    std::call_once(once, [] {
        std::lock_guard<std::recursive_mutex> g(wsg::env_mutex());
        (void)hipInit(0);
    });
}

extern "C" {

const char* wsg_strerror(int code)
{
    switch (code) {
    case WSG_OK:
        return "ok";
    case WSG_EINVAL:
        return "invalid argument or overlapping frames";
    case WSG_ETRUNC:
        return "frame runs past the end of the wire";
    case WSG_ENOMEM:
        return "out of memory or output capacity too small";
    case WSG_EHIP:
        return "HIP runtime error";
    default:
        return "unknown error";
    }
}


}   // extern "C"

namespace {

// The knobs a context takes from the environment, read once per context in
// wsg_create (no environment read on any data path).
struct Knobs {
    bool check = false;             // $WSG_CHECK=1: checked launches (debug, see in_alloc)
    uint64_t lane_max = 512 << 10;  // $WSG_LANE_MAX: largest lane request (0: the launch paths only; tools/lane_ab.py sweep)
    uint32_t lane_groups = wsg::LANE_GROUPS_MAX;   // $WSG_LANE_GROUPS: most frame groups per lane request
    uint64_t host_direct_max = 4 << 20;            // $WSG_HOST_DIRECT_MAX: host batches read in place up to this
    uint64_t seg_bytes = 32ull << 20;              // $WSG_STAGE_MB: segment of the staged host pipelines
    int enc_blocks_per_cu = 0;                     // $WSG_ENC_BLOCKS_PER_CU: k_encode_mask grid cap (0: default)
    bool multi_share = false;                      // $WSG_HOST_MULTI_SHARE=1: multi-context splits keep contexts of one device
    uint64_t enc_launch_pieces = 0;                // $WSG_ENC_LAUNCH_PIECES: pieces per k_encode_mask launch
};

Knobs read_knobs()
{
    Knobs k;
    std::lock_guard<std::recursive_mutex> g(wsg::env_mutex());
    if (const char* e = wsg::envp("WSG_CHECK"))
        k.check = *e == '1';
    if (const char* e = wsg::envp("WSG_LANE_MAX"))
        k.lane_max = std::strtoull(e, nullptr, 10);
    if (const char* e = wsg::envp("WSG_LANE_GROUPS")) {
        const long v = std::atol(e);
        if (v >= 1 && v <= long(wsg::LANE_GROUPS_MAX))
            k.lane_groups = uint32_t(v);
    }
    if (const char* e = wsg::envp("WSG_HOST_DIRECT_MAX"))
        k.host_direct_max = std::strtoull(e, nullptr, 10);
    if (const char* e = wsg::envp("WSG_STAGE_MB"))
        k.seg_bytes = std::max<uint64_t>(1, std::strtoull(e, nullptr, 10)) << 20;
    if (const char* e = wsg::envp("WSG_ENC_BLOCKS_PER_CU")) {   // (tests: grid-stride launch shapes)
        const int v = std::atoi(e);
        if (v > 0 && v <= 32768)
            k.enc_blocks_per_cu = v;
    }
    if (const char* e = wsg::envp("WSG_ENC_LAUNCH_PIECES"))     // (tests: split launches)
        k.enc_launch_pieces = std::strtoull(e, nullptr, 10);
    if (const char* e = wsg::envp("WSG_HOST_MULTI_SHARE"))      // (one-GPU tests of the multi-device split)
        k.multi_share = *e == '1';
    return k;
}

} // namespace

extern "C" {

int wsg_create(int device, wsg_ctx** out)
{
    if (!out)
        return WSG_EINVAL;
    *out = nullptr;
    wsg::hip_init_once();
    const Knobs k = read_knobs();
    wsg_ctx* c = nullptr;
    hipDeviceProp_t prop;
    {
        // a device's first use edits the environment as the runtime's
        // initialization does (wsg_env.h): these calls under the environment
        // lock; the synchronize below, which waits for this stream only, not
        std::lock_guard<std::recursive_mutex> env_guard(wsg::env_mutex());
        int count = 0;
        if (hipGetDeviceCount(&count) != hipSuccess || count <= 0 || device < 0 || device >= count)
            return WSG_EHIP;
        c = new (std::nothrow) wsg_ctx();
        if (!c)
            return WSG_ENOMEM;
        c->device = device;
        if (hipSetDevice(device) != hipSuccess || hipGetDeviceProperties(&prop, device) != hipSuccess ||
            hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
            hipMalloc(&c->d_err, sizeof(unsigned long long)) != hipSuccess ||
            hipMalloc(&c->d_err_host, 2 * sizeof(unsigned long long)) != hipSuccess ||
            hipHostMalloc(&c->h_err_copy, sizeof(unsigned long long), hipHostMallocDefault) != hipSuccess) {
            wsg_destroy(c);
            return WSG_EHIP;
        }
    }
    if (hipMemsetAsync(c->d_err, 0xFF, sizeof(unsigned long long), c->stream) != hipSuccess ||
        hipMemsetAsync(c->d_err_host, 0xFF, 2 * sizeof(unsigned long long), c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
        wsg_destroy(c);
        return WSG_EHIP;
    }
    c->num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    c->check = k.check;
    c->lane_max = k.lane_max;
    c->lane_groups = k.lane_groups;
    c->host_direct_max = k.host_direct_max;
    c->seg_bytes = k.seg_bytes;
    if (k.enc_blocks_per_cu)
        c->enc_blocks_per_cu = k.enc_blocks_per_cu;
    c->enc_launch_pieces = k.enc_launch_pieces;
    c->multi_share = k.multi_share;
    *out = c;
    return WSG_OK;
}

int wsg_destroy(wsg_ctx* c)
{
    if (!c)
        return WSG_EINVAL;
    if (c->dead) {
        // a lane request of this context neither answered nor drained: the
        // lane may still write its page-locked buffers, and freeing device or
        // page-locked memory waits for a device that may never drain; its
        // memory is left to the process's end
        delete c;
        return WSG_OK;
    }
    (void)hipSetDevice(c->device);
    if (c->stream)
        (void)hipStreamSynchronize(c->stream);
    for (auto& ev : c->pending) {
        (void)hipEventDestroy(ev.a);
        (void)hipEventDestroy(ev.b);
    }
    for (auto& ev : c->pool) {
        (void)hipEventDestroy(ev.a);
        (void)hipEventDestroy(ev.b);
    }
    (void)hipFree(c->d_err);
    (void)hipFree(c->d_err_host);
    if (c->h_err_copy)
        (void)hipHostFree(c->h_err_copy);
    free_enc(c->enc);
    (void)hipFree(c->d_stage);
    (void)hipFree(c->d_fs);
    (void)hipFree(c->d_info);
    if (c->h_stage)
        (void)hipHostFree(c->h_stage);
    for (hipStream_t r : {c->s_h2d, c->s_kern, c->s_d2h})
        if (r) {
            (void)hipStreamSynchronize(r);
            (void)hipStreamDestroy(r);
        }
    for (auto& sl : c->slots) {
        if (sl.stream)
            (void)hipStreamSynchronize(sl.stream);
        (void)hipFree(sl.d_wire);
        (void)hipFree(sl.d_payload);
        (void)hipFree(sl.d_desc);
        (void)hipFree(sl.d_woff);
        if (sl.h_desc)
            (void)hipHostFree(sl.h_desc);
        free_enc(sl.enc);
        (void)hipFree(sl.d_fs);
        (void)hipFree(sl.d_info);
        if (sl.h_in)
            (void)hipHostFree(sl.h_in);
        if (sl.h_out)
            (void)hipHostFree(sl.h_out);
        if (sl.h_fs)
            (void)hipHostFree(sl.h_fs);
        if (sl.h_info)
            (void)hipHostFree(sl.h_info);
        if (sl.done)
            (void)hipEventDestroy(sl.done);
        if (sl.h2d_done)
            (void)hipEventDestroy(sl.h2d_done);
        if (sl.k_done)
            (void)hipEventDestroy(sl.k_done);
        if (sl.stream)
            (void)hipStreamDestroy(sl.stream);
    }
    if (c->stream)
        (void)hipStreamDestroy(c->stream);
    delete c;
    return WSG_OK;
}

void* wsg_stream(wsg_ctx* c) { return c ? static_cast<void*>(c->stream) : nullptr; }

int wsg_sync(wsg_ctx* c, void* stream)
{
    if (!c)
        return WSG_EINVAL;
    hipStream_t s = pick(c, stream);
    unsigned long long e = kNoError;
    WSG_HIP(hipMemcpyAsync(&e, c->d_err, sizeof(e), hipMemcpyDeviceToHost, s));
    WSG_HIP(hipStreamSynchronize(s));
    if (e == kNoError)
        return WSG_OK;
    WSG_HIP(hipMemsetAsync(c->d_err, 0xFF, sizeof(unsigned long long), s));
    WSG_HIP(hipStreamSynchronize(s));
    return -int(e & 0xFFu);
}

namespace {

// Device decode: one k_decode launch (the pipelined host path runs several
// of these concurrently, one per slot).
int decode_launch(wsg_ctx* c, const uint8_t* d_wire, uint64_t wire_len, const uint64_t* d_frame_start, uint32_t n,
                  uint8_t* d_out, wsg_recv_info* d_info, hipStream_t s, unsigned long long* err)
{
    if (n == 0) {
        if (wire_len && d_out != d_wire)
            WSG_HIP(hipMemcpyAsync(d_out, d_wire, wire_len, hipMemcpyDeviceToDevice, s));
        return WSG_OK;
    }
    // every tile, and at least one block per 256 frames so that the frames of
    // a short (or empty) wire are still checked
    const uint64_t tiles = ceil_div(wire_len, wsg::TILE);
    const int t = timing_begin(c, s);
    WSG_HIP(wsg::launch_decode(s, grid_for(c, std::max(tiles, ceil_div(n, wsg::BLOCK)), c->dec_blocks_per_cu), d_wire, d_out, wire_len,
                               d_frame_start, n, d_info, err));
    timing_end(c, s, t);
    return WSG_OK;
}

} // namespace

int wsg_decode_batch(wsg_ctx* c, const uint8_t* d_wire, uint64_t wire_len, const uint64_t* d_frame_start, uint32_t n,
                     uint8_t* d_out, wsg_recv_info* d_info, void* stream)
{
    if (!c || (wire_len && (!d_wire || !d_out)) || (n && (!d_frame_start || !d_info)))
        return WSG_EINVAL;
    if (!aligned16(d_wire) || !aligned16(d_out))
        return WSG_EINVAL;
    if (c->check && (!in_alloc(d_wire, (wire_len + 15) & ~uint64_t(15)) || !in_alloc(d_out, wire_len) ||
                     !in_alloc(d_frame_start, uint64_t(n) * 8) || !in_alloc(d_info, uint64_t(n) * sizeof(wsg_recv_info))))
        return WSG_EINVAL;
    return decode_launch(c, d_wire, wire_len, d_frame_start, n, d_out, d_info, pick(c, stream), c->d_err);
}

namespace {

// upper bound of the pieces: sum of ceil((size + 15) / PIECE) over frames
inline uint64_t pieces_bound(uint32_t n, uint64_t wire_cap) { return wire_cap / wsg::PIECE + 2 * uint64_t(n) + 1; }

// Small-frame batches (average frame <= small_avg) take k_encode_small,
// the rest the piece kernel.
bool small_path(const wsg_ctx* c, uint32_t n, uint64_t wire_cap) { return wire_cap <= uint64_t(n) * c->small_avg; }

// scratch for either path (the piece map only for the piece kernel; for
// both when c is null)
int ensure_enc(const wsg_ctx* c, wsg_enc_scratch& e, uint32_t n, uint64_t wire_cap)
{
    if (int rc = ensure_array(e.d_scan, e.scan_cap, 4 * ceil_div(n, wsg::SCAN_ITEMS)))
        return rc;
    if (int rc = ensure_array(e.d_piece_start, e.piece_start_cap, uint64_t(n) + 1))
        return rc;
    if (c && small_path(c, n, wire_cap))
        return WSG_OK;
    // pieces are indexed by u32 in the launch (q_begin / q_end): a bound past
    // that (a wire_cap of terabytes, far past any HBM) is refused, not wrapped
    if (pieces_bound(n, wire_cap) > UINT32_MAX)
        return WSG_EINVAL;
    return ensure_array(e.d_piece_frame, e.piece_frame_cap, pieces_bound(n, wire_cap));
}

int encode_launch(wsg_ctx* c, hipStream_t s, const uint8_t* d_payload, const wsg_send_desc* d_desc, uint32_t n,
                  uint8_t* d_wire, uint64_t wire_cap, uint64_t* d_wire_off, wsg_enc_scratch& e,
                  unsigned long long* err)
{
    if (small_path(c, n, wire_cap)) {   // sizes scan, then one block per group of frames
        WSG_HIP(wsg::launch_encode_scan_small(s, d_desc, n, d_wire_off, e.d_scan));
        const int t = timing_begin(c, s);
        WSG_HIP(wsg::launch_encode_small(s, d_payload, d_desc, n, d_wire_off, e.d_scan, d_wire, wire_cap, err));
        timing_end(c, s, t);
        return WSG_OK;
    }
    const uint64_t pieces_cap = pieces_bound(n, wire_cap);
    if (pieces_cap > UINT32_MAX)   // as ensure_enc: u32 piece indices below
        return WSG_EINVAL;
    WSG_HIP(wsg::launch_encode_scan(s, d_desc, n, d_wire_off, e.d_piece_start, e.d_scan, e.d_piece_frame, pieces_cap,
                                    wire_cap, err));
    // one launch per run of at most enc_launch_pieces pieces (0: one launch)
    const uint64_t per = c->enc_launch_pieces ? c->enc_launch_pieces : pieces_cap;
    const int t = timing_begin(c, s);
    for (uint64_t q0 = 0; q0 < pieces_cap; q0 += per) {
        const uint64_t q1 = std::min<uint64_t>(pieces_cap, q0 + per);
        WSG_HIP(wsg::launch_encode_mask(s, grid_for(c, ceil_div(q1 - q0, wsg::BLOCK / 64), c->enc_blocks_per_cu),
                                        d_payload, d_desc, n, d_wire_off, e.d_piece_start, e.d_piece_frame, d_wire,
                                        wire_cap, uint32_t(q0), uint32_t(q1)));
    }
    timing_end(c, s, t);
    return WSG_OK;
}

} // namespace

int wsg_encode_batch(wsg_ctx* c, const uint8_t* d_payload, const wsg_send_desc* d_desc, uint32_t n, uint8_t* d_wire,
                     uint64_t wire_cap, uint64_t* d_wire_off, void* stream)
{
    if (!c || !d_wire_off || (n && (!d_desc || !d_wire)))
        return WSG_EINVAL;
    if (!aligned16(d_wire))
        return WSG_EINVAL;
    hipStream_t s = pick(c, stream);
    if (n == 0) {
        WSG_HIP(hipMemsetAsync(d_wire_off, 0, sizeof(uint64_t), s));
        return WSG_OK;
    }
    if (c->check) {   // the descriptors come to the host: every payload range and the wire capacity
        if (!in_alloc(d_desc, uint64_t(n) * sizeof(wsg_send_desc)) || !in_alloc(d_wire, wire_cap) ||
            !in_alloc(d_wire_off, (uint64_t(n) + 1) * 8))
            return WSG_EINVAL;
        std::vector<wsg_send_desc> h;
        try {
            h.resize(n);
        } catch (...) {
            return WSG_ENOMEM;
        }
        WSG_HIP(hipMemcpyAsync(h.data(), d_desc, uint64_t(n) * sizeof(wsg_send_desc), hipMemcpyDeviceToHost, s));
        WSG_HIP(hipStreamSynchronize(s));
        for (const wsg_send_desc& d : h)
            if (d.len && (!d_payload || !in_alloc(d_payload + d.src_off, d.len)))
                return WSG_EINVAL;
    }
    if (int rc = ensure_enc(c, c->enc, n, wire_cap))
        return rc;
    return encode_launch(c, s, d_payload, d_desc, n, d_wire, wire_cap, d_wire_off, c->enc, c->d_err);
}

namespace {

// One fan-out message's k frames on the flat / piece kernels (frame sizes the
// period path does not take).
int fanout_one_flat(wsg_ctx* c, hipStream_t s, const uint8_t* d_payload, uint64_t len, const uint32_t* d_keys,
                    uint32_t k, uint8_t opcode, int mask, uint8_t* d_wire)
{
    const uint64_t fsize = wsg_frame_size(opcode, mask, len, 0);
    const uint64_t total = fsize * k;
    const uint64_t blocks = ceil_div(ceil_div(total, wsg::CHUNK), wsg::BLOCK * wsg::FAN_UNITS);
    WSG_HIP(wsg::launch_fanout(s, grid_for(c, blocks), d_payload, len, d_keys, k, opcode, mask ? 1u : 0u, fsize,
                               d_wire));
    return WSG_OK;
}

// m messages x k keys.  Messages of one geometry (length, opcode) whose frame
// size suits the period kernel go FAN_MSGS at a time into one launch
// (blockIdx.y = message); the others take one flat launch each.
int fanout_many(wsg_ctx* c, hipStream_t s, const uint8_t* d_payload, const uint64_t* src_off, const uint64_t* len,
                const uint8_t* opcode, uint32_t m, const uint32_t* d_keys, uint32_t k, int mask, uint8_t* d_wire,
                const uint64_t* wire_off)
{
    std::vector<char> done(m, 0);
    for (uint32_t i = 0; i < m; ++i) {
        if (done[i])
            continue;
        const uint64_t fsize = wsg_frame_size(opcode[i], mask, len[i], 0);
        wsg::FanMsgs g{};
        uint32_t cnt = 0;
        std::vector<uint32_t> members;
        for (uint32_t q = i; q < m; ++q) {
            if (done[q] || len[q] != len[i] || opcode[q] != opcode[i])
                continue;
            members.push_back(q);
        }
        for (size_t at = 0; at < members.size(); at += wsg::FAN_MSGS) {
            cnt = uint32_t(std::min<size_t>(wsg::FAN_MSGS, members.size() - at));
            for (uint32_t q = 0; q < cnt; ++q) {
                g.src[q] = src_off[members[at + q]];
                g.dst[q] = wire_off[members[at + q]];
            }
            hipError_t perr = hipSuccess;
            if (wsg::launch_fanout_period(s, c->num_cus, c->fan_waves_per_cu, c->fan_wpb, d_payload, len[i], d_keys, k, opcode[i],
                                          mask ? 1u : 0u, fsize, d_wire, g, cnt, &perr)) {
                WSG_HIP(perr);
            } else {
                for (uint32_t q = 0; q < cnt; ++q)
                    if (int rc = fanout_one_flat(c, s, d_payload + g.src[q], len[i], d_keys, k, opcode[i], mask,
                                                 d_wire + g.dst[q]))
                        return rc;
            }
        }
        for (uint32_t q : members)
            done[q] = 1;
    }
    return WSG_OK;
}

} // namespace

int wsg_fanout_encode(wsg_ctx* c, const uint8_t* d_payload, uint64_t len, const uint32_t* d_keys, uint32_t k,
                      uint8_t opcode, int mask, uint8_t* d_wire, uint64_t wire_cap, void* stream)
{
    if (!c || (k && (!d_keys || !d_wire)) || (len && !d_payload))
        return WSG_EINVAL;
    if (!aligned16(d_wire))
        return WSG_EINVAL;
    if (k == 0)
        return WSG_OK;
    const uint64_t total = wsg_frame_size(opcode, mask, len, 0) * k;
    if (total > wire_cap)
        return WSG_ENOMEM;
    if (c->check && (!in_alloc(d_payload, len) || !in_alloc(d_keys, uint64_t(k) * 4) || !in_alloc(d_wire, total)))
        return WSG_EINVAL;
    hipStream_t s = pick(c, stream);
    const uint64_t src = 0, off[2] = {0, total};
    const int t = timing_begin(c, s);
    if (int rc = fanout_many(c, s, d_payload, &src, &len, &opcode, 1, d_keys, k, mask, d_wire, off))
        return rc;
    timing_end(c, s, t);
    return WSG_OK;
}

int wsg_fanout_encode_many(wsg_ctx* c, const uint8_t* d_payload, const uint64_t* src_off, const uint64_t* len,
                           const uint8_t* opcode, uint32_t m, const uint32_t* d_keys, uint32_t k, int mask,
                           uint8_t* d_wire, uint64_t wire_cap, uint64_t* wire_off, void* stream)
{
    try {   // no C++ exception leaves the ABI (host vectors: WSG_ENOMEM)
        if (!c || !wire_off || (m && (!src_off || !len || !opcode)) || (m && k && (!d_keys || !d_wire)))
            return WSG_EINVAL;
        if (d_wire && !aligned16(d_wire))
            return WSG_EINVAL;
        // message i's frames from wire_off[i], line-aligned (whole-line store rows)
        uint64_t at = 0;
        bool any_payload = false;
        for (uint32_t i = 0; i < m; ++i) {
            at = (at + wsg::PIECE_ALIGN - 1) & ~(wsg::PIECE_ALIGN - 1);
            wire_off[i] = at;
            at += wsg_frame_size(opcode[i], mask, len[i], 0) * k;
            any_payload = any_payload || len[i] != 0;
        }
        wire_off[m] = at;
        if (at > wire_cap)
            return WSG_ENOMEM;
        if (m == 0 || k == 0)
            return WSG_OK;
        if (any_payload && !d_payload)
            return WSG_EINVAL;
        if (c->check) {
            if (!in_alloc(d_keys, uint64_t(k) * 4) || !in_alloc(d_wire, at))
                return WSG_EINVAL;
            for (uint32_t i = 0; i < m; ++i)
                if (len[i] && !in_alloc(d_payload + src_off[i], len[i]))
                    return WSG_EINVAL;
        }
        hipStream_t s = pick(c, stream);
        const int t = timing_begin(c, s);
        if (int rc = fanout_many(c, s, d_payload, src_off, len, opcode, m, d_keys, k, mask, d_wire, wire_off))
            return rc;
        timing_end(c, s, t);
        return WSG_OK;
    } catch (...) {
        return WSG_ENOMEM;
    }
}

int wsg_xor_host(wsg_ctx* c, const void* src, void* dst, size_t len, uint32_t key, uint32_t phase)
{
    const wsg::TraceRange trace_range("wsg.xor_host");
    if (!c || (len && (!src || !dst)))
        return WSG_EINVAL;
    if (c->dead)
        return WSG_EHIP;
    if (len == 0)
        return WSG_OK;
    if (int rc = ensure_stage(c, len, 0))
        return rc;
    if (len <= std::min<uint64_t>(c->lane_max, wsg::LANE_PSTAGE)) {
        if (LaneServer* ls = lane_for(c)) {
            // a message of the per-call path (PrepareSendFrame /
            // PrepareReceiveFrame outside a batch scope): one lane task on the
            // page-locked stage, no launch and no synchronize; a payload of
            // up to LANE_INLINE bytes (an echo's 32) travels in the task
            uint64_t w[1][wsg::LANE_WORDS] = {{wsg::LANE_XOR | (uint64_t(1) << 32),
                                               reinterpret_cast<uint64_t>(c->h_stage), uint64_t(len),
                                               uint64_t(key) | (uint64_t(phase & 3u) << 32), 0, 0, 0, 0, 0}};
            const bool inl = len <= wsg::LANE_INLINE;
            if (inl) {   // (the answer comes back in the slot's self-tagged units, no buffer)
                w[0][0] = wsg::LANE_XOR_INLINE | (uint64_t(1) << 32);
                std::memcpy(&w[0][4], src, len);
            } else {
                std::memcpy(c->h_stage, src, len);
            }
            uint64_t errs = 0;
            uint32_t answered = 0;
            uint32_t res[wsg::LANE_INLINE / 4];
            const LaneResult r = inl ? lane_run(c, ls, w, 1, &errs, &answered, uint32_t((len + 3) / 4), res)
                                     : lane_run(c, ls, w, 1, &errs, &answered);
            if (r == LANE_DONE) {
                std::memcpy(dst, inl ? static_cast<const void*>(res) : c->h_stage, len);
                return WSG_OK;
            }
            if (r == LANE_LOST)
                return WSG_EHIP;
            // (the lane has left: the launch path below, from the input)
        }
    }
    std::memcpy(c->h_stage, src, len);
    hipStream_t s = c->stream;
    const uint64_t chunks = ceil_div(len, wsg::CHUNK);
    if (len <= c->xor_direct_max) {
        // small payloads: the kernel reads and writes the page-locked stage
        // itself over PCIe, one launch and one sync instead of H2D + kernel + D2H
        WSG_HIP(wsg::launch_xor(s, grid_for(c, ceil_div(chunks, wsg::BLOCK)), c->h_stage, c->h_stage, len, key, phase));
    } else {
        WSG_HIP(hipMemcpyAsync(c->d_stage, c->h_stage, len, hipMemcpyHostToDevice, s));
        WSG_HIP(wsg::launch_xor(s, grid_for(c, ceil_div(chunks, wsg::BLOCK)), c->d_stage, c->d_stage, len, key, phase));
        WSG_HIP(hipMemcpyAsync(c->h_stage, c->d_stage, len, hipMemcpyDeviceToHost, s));
    }
    WSG_HIP(hipStreamSynchronize(s));   // (polling hipStreamQuery instead: same at 1 thread, -9 % at 4)
    std::memcpy(dst, c->h_stage, len);
    return WSG_OK;
}

#ifndef WSG_COPY_WORKERS
#define WSG_COPY_WORKERS 5   // worker threads of the staged pipelines' host copies (A/B: tools/pcie_pageable.py)
#endif

namespace {

// Large host copies of the staged pipelines (a pageable caller buffer to or
// from the page-locked staging): one core copies ~27 GB/s, and a decode from
// pageable memory makes two such copies per byte (in and out), so one thread
// held the pipeline to 12.9 GiB/s of payload against 40 for page-locked
// buffers (round 4's bench line).  Copies of at least two parts' worth are
// cut into parts done by the calling thread and a few workers (made on first
// use; they park on the queue and are left to the process's end).
class CopyPool
{
public:
    static CopyPool& get()
    {
        static CopyPool* p = new CopyPool;   // leaked: its workers stay parked until the process ends
        return *p;
    }
    void copy(void* dst, const void* src, size_t len)
    {
        const size_t parts = std::min<size_t>(kWorkers + 1, len / kPartMin);
        if (parts <= 1) {
            std::memcpy(dst, src, len);
            return;
        }
        start_workers();
        const size_t per = ((len + parts - 1) / parts + 63) & ~size_t(63);
        std::atomic<size_t> left{0};
        size_t n = 0;
        {
            std::lock_guard<std::mutex> g(m_);
            for (size_t at = per; at < len; at += per, ++n)
                q_.push_back(Job{static_cast<uint8_t*>(dst) + at, static_cast<const uint8_t*>(src) + at,
                                 std::min(per, len - at), &left});
            left.store(n, std::memory_order_relaxed);
        }
        cv_.notify_all();
        std::memcpy(dst, src, std::min(per, len));
        // then help with whatever is queued (this call's parts or another's)
        // and wait for this call's parts
        for (;;) {
            Job j{};
            {
                std::lock_guard<std::mutex> g(m_);
                if (q_.empty())
                    break;
                j = q_.back();
                q_.pop_back();
            }
            run(j);
        }
        while (left.load(std::memory_order_acquire) != 0)
            std::this_thread::yield();
    }

private:
    static constexpr size_t kWorkers = WSG_COPY_WORKERS;
    static constexpr size_t kPartMin = size_t(2) << 20;
    struct Job {
        uint8_t* dst;
        const uint8_t* src;
        size_t len;
        std::atomic<size_t>* left;
    };
    static void run(const Job& j)
    {
        std::memcpy(j.dst, j.src, j.len);
        j.left->fetch_sub(1, std::memory_order_acq_rel);
    }
    void start_workers()
    {
        std::call_once(once_, [this] {
            for (size_t i = 0; i < kWorkers; ++i)
                std::thread([this] {
                    for (;;) {
                        Job j;
                        {
                            std::unique_lock<std::mutex> g(m_);
                            cv_.wait(g, [this] { return !q_.empty(); });
                            j = q_.front();
                            q_.pop_front();
                        }
                        run(j);
                    }
                }).detach();
        });
    }
    std::once_flag once_;
    std::mutex m_;
    std::condition_variable cv_;
    std::deque<Job> q_;
};

void host_copy(void* dst, const void* src, size_t len) { CopyPool::get().copy(dst, src, len); }

bool host_pinned(const void* p)
{
    if (in_host_block(p))
        return true;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// Page-locked AND mapped at the same address on the device, so a kernel may
// take the host pointer as it is (hipHostMalloc memory).  Memory registered
// with hipHostRegister can have another device address; such buffers take
// the staged pipeline (hipMemcpyAsync handles any host pointer).
bool host_direct(const void* p)
{
    if (in_host_block(p))
        return true;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost && a.devicePointer == p;
}

int slot_init(wsg_ctx::Slot& sl)
{
    if (sl.stream)
        return WSG_OK;
    WSG_HIP(hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking));
    WSG_HIP(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
    WSG_HIP(hipEventCreateWithFlags(&sl.h2d_done, hipEventDisableTiming));
    WSG_HIP(hipEventCreateWithFlags(&sl.k_done, hipEventDisableTiming));
    return WSG_OK;
}

// The three streams one segment's work goes to, and the hand-offs between
// them: H2D copies, then kernels, then D2H copies.
struct Pipe {
    hipStream_t h2d, kern, d2h;
    bool roles;
};

int pipe_for(wsg_ctx* c, wsg_ctx::Slot& sl, Pipe& p)
{
    (void)sl;
    p.roles = true;
    for (hipStream_t* r : {&c->s_h2d, &c->s_kern, &c->s_d2h})
        if (!*r)
            WSG_HIP(hipStreamCreateWithFlags(r, hipStreamNonBlocking));
    p.h2d = c->s_h2d;
    p.kern = c->s_kern;
    p.d2h = c->s_d2h;
    return WSG_OK;
}

// inputs copied -> kernels may start; kernels done -> copies back may start
int pipe_to_kern(const Pipe& p, wsg_ctx::Slot& sl)
{
    if (p.roles) {
        WSG_HIP(hipEventRecord(sl.h2d_done, p.h2d));
        WSG_HIP(hipStreamWaitEvent(p.kern, sl.h2d_done, 0));
    }
    return WSG_OK;
}
int pipe_to_d2h(const Pipe& p, wsg_ctx::Slot& sl)
{
    if (p.roles) {
        WSG_HIP(hipEventRecord(sl.k_done, p.kern));
        WSG_HIP(hipStreamWaitEvent(p.d2h, sl.k_done, 0));
    }
    return WSG_OK;
}

int slot_reserve(wsg_ctx::Slot& sl, uint64_t bytes, uint64_t frames, bool need_host)
{
    if (int rc = slot_init(sl))
        return rc;
    if (int rc = ensure_array(sl.d_wire, sl.wire_cap, bytes + 32))
        return rc;
    if (frames > sl.frames_cap) {
        (void)hipFree(sl.d_fs);
        (void)hipFree(sl.d_info);
        if (sl.h_fs)
            (void)hipHostFree(sl.h_fs);
        if (sl.h_info)
            (void)hipHostFree(sl.h_info);
        sl.d_fs = nullptr;
        sl.d_info = nullptr;
        sl.h_fs = nullptr;
        sl.h_info = nullptr;
        sl.frames_cap = 0;
        if (hipMalloc(&sl.d_fs, frames * sizeof(uint64_t)) != hipSuccess ||
            hipMalloc(&sl.d_info, frames * sizeof(wsg_recv_info)) != hipSuccess ||
            hipHostMalloc(&sl.h_fs, frames * sizeof(uint64_t), host_alloc_flags()) != hipSuccess ||
            hipHostMalloc(&sl.h_info, frames * sizeof(wsg_recv_info), host_alloc_flags()) != hipSuccess)
            return WSG_ENOMEM;
        sl.frames_cap = frames;
    }
    if (need_host && bytes + 32 > sl.host_cap) {
        if (sl.h_in)
            (void)hipHostFree(sl.h_in);
        if (sl.h_out)
            (void)hipHostFree(sl.h_out);
        sl.h_in = sl.h_out = nullptr;
        sl.host_cap = 0;
        if (hipHostMalloc(&sl.h_in, bytes + 32, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc(&sl.h_out, bytes + 32, hipHostMallocDefault) != hipSuccess)
            return WSG_ENOMEM;
        sl.host_cap = bytes + 32;
    }
    return WSG_OK;
}

// Wait for a slot's previous segment and finish its host-side copies.
int slot_drain(wsg_ctx::Slot& sl)
{
    if (!sl.busy)
        return WSG_OK;
    WSG_HIP(hipEventSynchronize(sl.done));
    if (sl.out_dst && sl.out_len)
        host_copy(sl.out_dst, sl.h_out + sl.out_src, sl.out_len);
    for (uint32_t k = 0; k < sl.info_n; ++k) {
        wsg_recv_info r = sl.h_info[k];
        r.payload_off += sl.base;   // segment-relative -> wire offset
        sl.info_dst[k] = r;
    }
    sl.busy = false;
    return WSG_OK;
}

} // namespace

int wsg_host_alloc(size_t bytes, void** out)
{
    if (!out)
        return WSG_EINVAL;
    *out = nullptr;
    wsg::hip_init_once();
    if (hipHostMalloc(out, bytes ? bytes : 1, host_alloc_flags()) != hipSuccess)
        return WSG_ENOMEM;
    host_blocks_add(*out, bytes ? bytes : 1);
    return WSG_OK;
}

int wsg_host_free(void* p)
{
    if (!p)
        return WSG_OK;
    host_blocks_remove(p);
    if (hipHostFree(p) != hipSuccess)
        return WSG_EHIP;
    return WSG_OK;
}

namespace {

// The batch's frame errors as the one-context call states them: a frame that
// runs into the next one overlaps it (EINVAL) when its whole length lies
// inside the wire; the status is the lowest-indexed bad frame's.
int host_batch_status(wsg_ctx* c, const uint8_t* wire, uint64_t wire_len, const uint64_t* frame_start, uint32_t n,
                      wsg_recv_info* info)
{
    int first = WSG_OK;
    for (uint32_t i = 0; i < n; ++i) {
        wsg_recv_info& r = info[i];
        if (r.error == WSG_ETRUNC && i + 1 < n && frame_start[i] < wire_len) {
            wsg_recv_info h;
            if (wsg_header_unpack(wire + frame_start[i], wire_len - frame_start[i], &h) == WSG_OK &&
                h.len <= wire_len - frame_start[i] - h.hdr_len)
                r.error = int8_t(WSG_EINVAL);
        }
        if (r.error && !first)
            first = r.error;
    }
    if (first) {   // re-arm the host paths' latch, landed before the next call's kernels
        // (a plain hipMemset goes to the null stream, which the context's
        // non-blocking streams do not wait for, and may return before it lands)
        WSG_HIP(hipMemsetAsync(c->d_err_host, 0xFF, sizeof(unsigned long long), c->stream));
        WSG_HIP(hipStreamSynchronize(c->stream));
    }
    return first;
}

// A small host batch in page-locked buffers (a read's frames, echo size):
// k_decode reads the wire and writes the output where they are, over PCIe,
// on the context's stream — one launch and one synchronize instead of the
// pipeline's H2D + kernel + D2H on three streams with event hand-offs.
bool strictly_increasing(const uint64_t* v, uint32_t n)
{
    for (uint32_t i = 1; i < n; ++i)
        if (v[i] <= v[i - 1])
            return false;
    return true;
}

// In-place decodes of at least this many frames on the launch path read the
// error latch back instead of scanning every record for the status.
constexpr uint32_t kLatchFrames = 4096;

int decode_host_direct(wsg_ctx* c, const uint8_t* wire, uint64_t wire_len, const uint64_t* frame_start, uint32_t n,
                       uint8_t* out, wsg_recv_info* info)
{
    wsg_ctx::Slot& sl = c->slots[0];
    if (int rc = slot_reserve(sl, 0, n, false))
        return rc;
    // a table and records in wsg_host_alloc blocks (the batch classes') are
    // used where they are; others through the slot's page-locked copies
    const uint64_t* fs_dev = frame_start;
    if (!in_host_block(frame_start, uint64_t(n) * sizeof(uint64_t))) {
        std::memcpy(sl.h_fs, frame_start, size_t(n) * sizeof(uint64_t));
        fs_dev = sl.h_fs;
    }
    wsg_recv_info* info_dev =
        in_host_block(info, uint64_t(n) * sizeof(wsg_recv_info)) ? info : sl.h_info;
    LaneServer* ls = nullptr;
    LaneGroup grp[wsg::LANE_GROUPS_MAX];
    uint32_t groups = 0;
    if (wire_len <= c->lane_max && n > 0 && n <= kLaneMaxFrames && strictly_increasing(frame_start, n) &&
        (ls = lane_for(c)) &&
        (groups = lane_plan(c, ls, n, wsg::LANE_STAGE - 64, true, [&](uint32_t i) -> uint64_t {
             return i == 0 ? 0 : i < n ? std::min(frame_start[i], wire_len) : wire_len;
         }, grp))) {
        // an echo's read, up to a few MiB: the device's resident lane, no
        // launch; group k's wire range from its first start (0 for the first)
        // to the next group's (wire_len after the last), staged whole in LDS
        uint64_t w[wsg::LANE_GROUPS_MAX][wsg::LANE_WORDS];
        for (uint32_t k = 0; k < groups; ++k) {
            w[k][0] = wsg::LANE_DECODE | (uint64_t(n) << 32);
            w[k][1] = reinterpret_cast<uint64_t>(wire);
            w[k][2] = wire_len;
            w[k][3] = reinterpret_cast<uint64_t>(fs_dev);
            w[k][4] = reinterpret_cast<uint64_t>(out);
            w[k][5] = reinterpret_cast<uint64_t>(info_dev);
            w[k][6] = uint64_t(grp[k].f) | (uint64_t(grp[k].cnt) << 32);
            w[k][7] = grp[k].lo;
            w[k][8] = grp[k].hi;
        }
        uint64_t errs = 0;
        uint32_t answered = 0;
        const LaneResult r = lane_run(c, ls, w, groups, &errs, &answered);
        if (r == LANE_DONE) {
            if (info_dev != info)
                std::memcpy(info, info_dev, size_t(n) * sizeof(wsg_recv_info));
            // no frame erred (the lane's count): nothing for the status pass to
            // find, and the records the GPU just wrote stay out of this core's
            // caches unless the caller reads them
            return errs ? host_batch_status(c, wire, wire_len, frame_start, n, info) : WSG_OK;
        }
        // given up on the lane: its answered groups have unmasked their bytes
        // (in place: a second pass would mask them again), and a lane that did
        // not leave may still write the buffers
        if (r == LANE_LOST || (answered && out == wire))
            return WSG_EHIP;
    }
    hipStream_t s = c->stream;
    if (int rc = decode_launch(c, wire, wire_len, fs_dev, n, out, info_dev, s, c->d_err_host))
        return rc;
    // many frames: the latch read back beside the kernel (an 8-byte copy on
    // the same stream) says whether any frame erred; none did, and the status
    // pass over n records the GPU just wrote to host memory (~2 ns a frame,
    // 0.2 ms at 100 K frames) is skipped, as the lane's error count skips it
    const bool latch = n >= kLatchFrames;
    if (latch)
        WSG_HIP(hipMemcpyAsync(c->h_err_copy, c->d_err_host, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    WSG_HIP(hipStreamSynchronize(s));
    if (info_dev != info)
        std::memcpy(info, info_dev, size_t(n) * sizeof(wsg_recv_info));
    if (latch && *c->h_err_copy == ~0ull)
        return WSG_OK;
    return host_batch_status(c, wire, wire_len, frame_start, n, info);
}

} // namespace

int wsg_decode_batch_host(wsg_ctx* c, const uint8_t* wire, uint64_t wire_len, const uint64_t* frame_start,
                          uint32_t n, uint8_t* out, wsg_recv_info* info)
{
    const wsg::TraceRange trace_range("wsg.decode_batch_host");
    try {   // no C++ exception leaves the ABI (host vectors: WSG_ENOMEM)
        if (!c || (wire_len && (!wire || !out)) || (n && (!frame_start || !info)))
            return WSG_EINVAL;
        if (c->dead)
            return WSG_EHIP;
        if (n == 0) {
            if (wire_len && out != wire)
                std::memmove(out, wire, wire_len);
            return WSG_OK;
        }
        const uint64_t seg_bytes = c->seg_bytes;
        const bool in_pinned = host_pinned(wire), out_pinned = host_pinned(out);
        if (in_pinned && out_pinned && wire_len <= c->host_direct_max && aligned16(wire) && aligned16(out) &&
            host_direct(wire) && host_direct(out))
            return decode_host_direct(c, wire, wire_len, frame_start, n, out, info);

        // segments: runs of whole frames of about seg_bytes; segment k covers wire
        // bytes [start of its first frame, start of the next segment's first frame)
        std::vector<uint32_t> cut{0};
        {
            uint64_t from = 0;
            for (uint32_t i = 1; i < n; ++i) {
                if (frame_start[i] >= wire_len)
                    break;   // frames past the wire: error frames, kept with the last segment
                if (frame_start[i] > from && frame_start[i] - from >= seg_bytes) {
                    cut.push_back(i);
                    from = frame_start[i];
                }
            }
            cut.push_back(n);
        }
        const size_t nseg = cut.size() - 1;
        uint64_t max_bytes = 0, max_frames = 0;
        auto seg_lo = [&](size_t k) { return k == 0 ? uint64_t(0) : std::min(frame_start[cut[k]], wire_len); };
        auto seg_hi = [&](size_t k) { return k + 1 == nseg ? wire_len : std::min(frame_start[cut[k + 1]], wire_len); };
        for (size_t k = 0; k < nseg; ++k) {
            const uint64_t base = seg_lo(k) & ~uint64_t(15);
            max_bytes = std::max(max_bytes, std::max(seg_hi(k), seg_lo(k)) - base);
            max_frames = std::max<uint64_t>(max_frames, cut[k + 1] - cut[k]);
        }
        for (auto& sl : c->slots)
            if (int rc = slot_reserve(sl, max_bytes, max_frames, !in_pinned || !out_pinned))
                return rc;

        for (size_t k = 0; k < nseg; ++k) {
            wsg_ctx::Slot& sl = c->slots[k % wsg_ctx::kSlots];
            if (int rc = slot_drain(sl))
                return rc;
            const uint32_t i0 = cut[k], i1 = cut[k + 1], m = i1 - i0;
            const uint64_t lo = seg_lo(k), hi = std::max(seg_hi(k), lo);
            const uint64_t base = lo & ~uint64_t(15);   // 16-B aligned device copy of [base, hi)
            const uint64_t len = hi - base;
            for (uint32_t j = 0; j < m; ++j)
                sl.h_fs[j] = frame_start[i0 + j] >= base ? frame_start[i0 + j] - base : ~uint64_t(0);
            const uint8_t* src = wire + base;
            if (!in_pinned) {
                host_copy(sl.h_in, wire + base, len);
                src = sl.h_in;
            }
            Pipe pp;
            if (int rc = pipe_for(c, sl, pp))
                return rc;
            WSG_HIP(hipMemcpyAsync(sl.d_wire, src, len, hipMemcpyHostToDevice, pp.h2d));
            WSG_HIP(hipMemcpyAsync(sl.d_fs, sl.h_fs, m * sizeof(uint64_t), hipMemcpyHostToDevice, pp.h2d));
            if (int rc = pipe_to_kern(pp, sl))
                return rc;
            if (int rc = decode_launch(c, sl.d_wire, len, sl.d_fs, m, sl.d_wire, sl.d_info, pp.kern, c->d_err_host))
                return rc;
            if (int rc = pipe_to_d2h(pp, sl))
                return rc;
            // copy back [lo, hi): bytes before lo belong to the previous segment
            const uint64_t back = hi - lo;
            if (out_pinned) {
                WSG_HIP(hipMemcpyAsync(out + lo, sl.d_wire + (lo - base), back, hipMemcpyDeviceToHost, pp.d2h));
                sl.out_dst = nullptr;
            } else {
                WSG_HIP(hipMemcpyAsync(sl.h_out, sl.d_wire + (lo - base), back, hipMemcpyDeviceToHost, pp.d2h));
                sl.out_dst = out + lo;
                sl.out_src = 0;
            }
            sl.out_len = back;
            WSG_HIP(hipMemcpyAsync(sl.h_info, sl.d_info, m * sizeof(wsg_recv_info), hipMemcpyDeviceToHost, pp.d2h));
            sl.info_dst = info + i0;
            sl.info_n = m;
            sl.base = base;
            WSG_HIP(hipEventRecord(sl.done, pp.d2h));
            sl.busy = true;
        }
        for (auto& sl : c->slots)
            if (int rc = slot_drain(sl))
                return rc;
        // the pipeline's kernels latched into d_err_host (segment-relative frame
        // indices, meaningless to the caller); the status comes from the
        // per-frame errors below, and the caller's own latch is left alone.
        // Many frames: the latch (every kernel has finished: the slots have
        // drained) read back first, and an untouched one skips the pass
        if (n >= kLatchFrames) {
            WSG_HIP(hipMemcpyAsync(c->h_err_copy, c->d_err_host, sizeof(unsigned long long), hipMemcpyDeviceToHost,
                                   c->stream));
            WSG_HIP(hipStreamSynchronize(c->stream));
            if (*c->h_err_copy == ~0ull)
                return WSG_OK;
        }

        // batch semantics: a frame that runs into the next segment's first frame
        // overlaps it (EINVAL), it is not truncated; and the status is the error
        // of the lowest-indexed bad frame (every slot has drained)
        return host_batch_status(c, wire, wire_len, frame_start, n, info);
    } catch (...) {
        return WSG_ENOMEM;
    }
}

namespace {

int slot_reserve_enc(wsg_ctx::Slot& sl, uint64_t payload_bytes, uint64_t wire_bytes, uint32_t frames,
                     bool need_host)
{
    if (int rc = slot_init(sl))
        return rc;
    if (int rc = ensure_array(sl.d_payload, sl.payload_cap, payload_bytes + 32))
        return rc;
    if (int rc = ensure_array(sl.d_wire, sl.wire_cap, wire_bytes + 32))
        return rc;
    if (int rc = ensure_array(sl.d_desc, sl.desc_cap, frames))
        return rc;
    if (int rc = ensure_array(sl.d_woff, sl.woff_cap, uint64_t(frames) + 1))
        return rc;
    if (int rc = ensure_enc(nullptr, sl.enc, frames, wire_bytes))   // both paths: segments differ
        return rc;
    if (frames > sl.h_desc_cap) {
        if (sl.h_desc)
            (void)hipHostFree(sl.h_desc);
        sl.h_desc = nullptr;
        sl.h_desc_cap = 0;
        if (hipHostMalloc(&sl.h_desc, frames * sizeof(wsg_send_desc), host_alloc_flags()) != hipSuccess)
            return WSG_ENOMEM;
        sl.h_desc_cap = frames;
    }
    const uint64_t host = std::max(payload_bytes, wire_bytes) + 32;
    if (need_host && host > sl.host_cap) {
        if (sl.h_in)
            (void)hipHostFree(sl.h_in);
        if (sl.h_out)
            (void)hipHostFree(sl.h_out);
        sl.h_in = sl.h_out = nullptr;
        sl.host_cap = 0;
        if (hipHostMalloc(&sl.h_in, host, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc(&sl.h_out, host, hipHostMallocDefault) != hipSuccess)
            return WSG_ENOMEM;
        sl.host_cap = host;
    }
    return WSG_OK;
}

} // namespace

int wsg_encode_batch_host(wsg_ctx* c, const uint8_t* payload, uint64_t payload_len, const wsg_send_desc* desc,
                          uint32_t n, uint8_t* wire, uint64_t wire_cap, uint64_t* wire_off)
{
    const wsg::TraceRange trace_range("wsg.encode_batch_host");
    try {   // no C++ exception leaves the ABI (host vectors: WSG_ENOMEM)
        if (!c || !wire_off || (n && (!desc || !wire)) || (payload_len && !payload))
            return WSG_EINVAL;
        if (c->dead)
            return WSG_EHIP;
        // frame offsets on the host (the same arithmetic as k_encode_scan_*), so
        // that segments can be cut and copied back without a device round trip
        wire_off[0] = 0;
        for (uint32_t i = 0; i < n; ++i) {
            const wsg_send_desc& d = desc[i];
            if (d.len > payload_len || d.src_off > payload_len - d.len)
                return WSG_EINVAL;
            const wsg::SendGeom g = wsg::send_geom(d.opcode, d.mask != 0, d.len, d.status);   // = wsg_frame_size
            wire_off[i + 1] = wire_off[i] + g.hdr + g.body;
        }
        if (wire_off[n] > wire_cap)
            return WSG_ENOMEM;
        if (n == 0)
            return WSG_OK;
        const uint64_t seg_bytes = c->seg_bytes;
        const bool in_pinned = host_pinned(payload), out_pinned = host_pinned(wire);
        if (in_pinned && out_pinned && wire_off[n] <= c->host_direct_max && aligned16(wire) && n <= (1u << 20) &&
            host_direct(wire) && (payload_len == 0 || host_direct(payload))) {
            // a small batch in page-locked buffers (the frames a tick sends):
            // the kernels read the payloads and write the frames where they
            // are, one launch sequence and one synchronize
            wsg_ctx::Slot& sl = c->slots[0];
            if (int rc = slot_reserve_enc(sl, 0, wire_off[n], n, false))
                return rc;
            // descriptors and offsets in wsg_host_alloc blocks (the batch
            // classes') are read where they are; others through copies
            const wsg_send_desc* desc_dev = desc;
            if (!in_host_block(desc, uint64_t(n) * sizeof(wsg_send_desc))) {
                std::memcpy(sl.h_desc, desc, size_t(n) * sizeof(wsg_send_desc));
                desc_dev = sl.h_desc;
            }
            LaneServer* ls = nullptr;
            LaneGroup grp[wsg::LANE_GROUPS_MAX];
            uint32_t groups = 0;
            if (wire_off[n] <= c->lane_max && n <= kLaneMaxFrames && (ls = lane_for(c)) &&
                (groups = lane_plan(c, ls, n, wsg::LANE_PSTAGE - 64, false,
                                    [&](uint32_t i) -> uint64_t { return wire_off[i]; }, grp))) {
                // the replies of an echo's read, up to a few MiB: the device's
                // resident lane at the offsets computed above, no launch;
                // groups of about equal wire bytes, each group's payload span
                // for its staging
                const uint64_t* off_dev = wire_off;
                if (!in_host_block(wire_off, (uint64_t(n) + 1) * sizeof(uint64_t))) {
                    if (int rc = slot_reserve(sl, 0, uint64_t(n) + 1, false))
                        return rc;
                    std::memcpy(sl.h_fs, wire_off, (size_t(n) + 1) * sizeof(uint64_t));
                    off_dev = sl.h_fs;
                }
                uint64_t w[wsg::LANE_GROUPS_MAX][wsg::LANE_WORDS];
                for (uint32_t k = 0; k < groups; ++k) {
                    const uint32_t f = grp[k].f, cnt = grp[k].cnt;
                    uint64_t lo = UINT64_MAX, hi = 0;
                    for (uint32_t i = f; i < f + cnt; ++i)
                        if (desc[i].len) {
                            lo = std::min(lo, desc[i].src_off);
                            hi = std::max(hi, desc[i].src_off + desc[i].len);
                        }
                    w[k][0] = wsg::LANE_ENCODE | (uint64_t(n) << 32);
                    w[k][1] = reinterpret_cast<uint64_t>(payload);
                    w[k][2] = reinterpret_cast<uint64_t>(desc_dev);
                    w[k][3] = reinterpret_cast<uint64_t>(off_dev);
                    w[k][4] = reinterpret_cast<uint64_t>(wire);
                    w[k][5] = 0;
                    w[k][6] = uint64_t(f) | (uint64_t(cnt) << 32);
                    w[k][7] = hi ? lo : 0;
                    w[k][8] = hi;
                }
                uint64_t errs = 0;
                uint32_t answered = 0;
                const LaneResult r = lane_run(c, ls, w, groups, &errs, &answered);
                if (r == LANE_DONE)
                    return WSG_OK;
                if (r == LANE_LOST)
                    return WSG_EHIP;   // (the lane may still write the frames)
                // given up on the lane, which has left: the launch path writes every frame again
            }
            hipStream_t s = c->stream;
            if (int rc = encode_launch(c, s, payload, desc_dev, n, wire, wire_off[n], sl.d_woff, sl.enc,
                                       c->d_err_host + 1))
                return rc;
            WSG_HIP(hipStreamSynchronize(s));
            return WSG_OK;   // capacity was checked on the host: nothing for the latch to report
        }

        // segments of whole frames, ~seg_bytes of wire each
        struct Seg {
            uint32_t i0, i1;
            uint64_t lo, hi;   // payload source range [lo, hi) (16-B aligned lo)
            uint64_t sum;      // payload bytes of its frames
            bool gather;       // frames' payloads not one tight range: copy them together
        };
        std::vector<Seg> segs;
        for (uint32_t i0 = 0; i0 < n;) {
            Seg g{i0, i0, ~uint64_t(0), 0, 0, false};
            do {
                const wsg_send_desc& d = desc[g.i1];
                if (d.len) {
                    g.lo = std::min(g.lo, d.src_off);
                    g.hi = std::max(g.hi, d.src_off + d.len);
                }
                g.sum += d.len;
                ++g.i1;
            } while (g.i1 < n && wire_off[g.i1] - wire_off[i0] < seg_bytes);
            if (g.lo > g.hi)
                g.lo = g.hi = 0;
            g.lo &= ~uint64_t(15);
            g.gather = g.hi - g.lo > g.sum + 16 * uint64_t(g.i1 - g.i0) + 4096;
            segs.push_back(g);
            i0 = g.i1;
        }
        uint64_t max_payload = 0, max_wire = 0;
        uint32_t max_frames = 0;
        bool need_host = !out_pinned;
        for (const Seg& g : segs) {
            max_payload = std::max(max_payload, g.gather ? g.sum : g.hi - g.lo);
            max_wire = std::max(max_wire, wire_off[g.i1] - wire_off[g.i0]);
            max_frames = std::max(max_frames, g.i1 - g.i0);
            need_host = need_host || g.gather || !in_pinned;
        }
        for (auto& sl : c->slots)
            if (int rc = slot_reserve_enc(sl, max_payload, max_wire, max_frames, need_host))
                return rc;

        for (size_t k = 0; k < segs.size(); ++k) {
            const Seg& g = segs[k];
            wsg_ctx::Slot& sl = c->slots[k % wsg_ctx::kSlots];
            if (int rc = slot_drain(sl))
                return rc;
            const uint32_t m = g.i1 - g.i0;
            const uint8_t* src = payload + g.lo;
            uint64_t plen = g.hi - g.lo;
            if (g.gather) {
                uint64_t at = 0;
                for (uint32_t j = 0; j < m; ++j) {
                    wsg_send_desc d = desc[g.i0 + j];
                    if (d.len)
                        std::memcpy(sl.h_in + at, payload + d.src_off, d.len);
                    d.src_off = at;
                    sl.h_desc[j] = d;
                    at += d.len;
                }
                src = sl.h_in;
                plen = at;
            } else {
                for (uint32_t j = 0; j < m; ++j) {
                    wsg_send_desc d = desc[g.i0 + j];
                    d.src_off = d.len ? d.src_off - g.lo : 0;
                    sl.h_desc[j] = d;
                }
                if (!in_pinned && plen) {
                    host_copy(sl.h_in, src, plen);
                    src = sl.h_in;
                }
            }
            Pipe pp;
            if (int rc = pipe_for(c, sl, pp))
                return rc;
            if (plen)
                WSG_HIP(hipMemcpyAsync(sl.d_payload, src, plen, hipMemcpyHostToDevice, pp.h2d));
            WSG_HIP(hipMemcpyAsync(sl.d_desc, sl.h_desc, m * sizeof(wsg_send_desc), hipMemcpyHostToDevice, pp.h2d));
            if (int rc = pipe_to_kern(pp, sl))
                return rc;
            const uint64_t wlen = wire_off[g.i1] - wire_off[g.i0];
            if (int rc = encode_launch(c, pp.kern, sl.d_payload, sl.d_desc, m, sl.d_wire, wlen, sl.d_woff, sl.enc,
                                       c->d_err_host + 1))
                return rc;
            if (int rc = pipe_to_d2h(pp, sl))
                return rc;
            if (out_pinned) {
                WSG_HIP(hipMemcpyAsync(wire + wire_off[g.i0], sl.d_wire, wlen, hipMemcpyDeviceToHost, pp.d2h));
                sl.out_dst = nullptr;
            } else {
                WSG_HIP(hipMemcpyAsync(sl.h_out, sl.d_wire, wlen, hipMemcpyDeviceToHost, pp.d2h));
                sl.out_dst = wire + wire_off[g.i0];
                sl.out_src = 0;
            }
            sl.out_len = wlen;
            sl.info_n = 0;
            WSG_HIP(hipEventRecord(sl.done, pp.d2h));
            sl.busy = true;
        }
        for (auto& sl : c->slots)
            if (int rc = slot_drain(sl))
                return rc;
        // the encode kernels latch only capacity errors, and capacity was checked
        // on the host above: nothing for the pipeline's latch to report
        return WSG_OK;
    } catch (...) {
        return WSG_ENOMEM;
    }
}

uint64_t wsg_frame_size(uint8_t opcode, int mask, uint64_t len, int32_t status)
{
    const wsg::SendGeom g = wsg::send_geom(opcode, mask != 0, len, status);
    return g.hdr + g.body;
}

int wsg_header_pack(uint8_t opcode, int mask, uint64_t len, int32_t status, uint32_t key, uint8_t* out)
{
    if (!out)
        return WSG_EINVAL;
    const wsg::SendGeom g = wsg::send_geom(opcode, mask != 0, len, status);
    for (uint32_t r = 0; r < g.hdr; ++r)
        out[r] = wsg::header_byte(opcode, mask != 0, g.body, key, r);
    return int(g.hdr);
}

int wsg_header_unpack(const uint8_t* buf, uint64_t avail, wsg_recv_info* info)
{
    if (!info || (avail && !buf))
        return WSG_EINVAL;
    wsg_recv_info r = {};
    const int e = wsg::parse_header([&](uint32_t k) { return buf[k]; }, avail, r);
    if (e)
        return e;
    r.payload_off = r.hdr_len;
    *info = r;
    return WSG_OK;
}

int wsg_timing_enable(wsg_ctx* c, int on)
{
    if (!c)
        return WSG_EINVAL;
    c->timing = on > 0 ? on : 0;
    c->timing_seq = 0;
    return WSG_OK;
}

int wsg_timing_read(wsg_ctx* c, double* total_ms, uint64_t* launches, int reset)
{
    if (!c)
        return WSG_EINVAL;
    if (int rc = drain_timing(c))
        return rc;
    if (total_ms)
        *total_ms = c->acc_ms;
    if (launches)
        *launches = c->launches;
    if (reset) {
        c->acc_ms = 0.0;
        c->launches = 0;
        c->min_ms = c->max_ms = 0.0;
    }
    return WSG_OK;
}

int wsg_lane_stats(wsg_ctx* c, uint64_t* requests, uint64_t* launches, int* running)
{
    if (!c)
        return WSG_EINVAL;
    LaneServer* s = c->lane;
    if (requests)
        *requests = c->lane_requests;
    if (launches)
        *launches = s ? s->launches.load() : 0;
    if (running) {
        const uint32_t g = s ? s->gen.load() : 0;
        *running = !s ? 0 : s->broken.load() ? -1 : (g && __atomic_load_n(&s->bell->ctl.closing, __ATOMIC_ACQUIRE) != g) ? 1 : 0;
    }
    return WSG_OK;
}

int wsg_lane_events(wsg_ctx* c, uint64_t* give_ups, uint64_t* rearms)
{
    if (!c)
        return WSG_EINVAL;
    LaneServer* s = c->lane;
    if (give_ups)
        *give_ups = s ? s->give_ups.load() : 0;
    if (rearms)
        *rearms = s ? s->rearms.load() : 0;
    return WSG_OK;
}

int wsg_timing_minmax(wsg_ctx* c, double* min_ms, double* max_ms)
{
    if (!c)
        return WSG_EINVAL;
    if (int rc = drain_timing(c))
        return rc;
    if (min_ms)
        *min_ms = c->min_ms;
    if (max_ms)
        *max_ms = c->max_ms;
    return WSG_OK;
}

} // extern "C"
