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
#include <cstring>
#include <map>
#include <mutex>
#include <new>
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
    uint64_t xor_direct_max = 64 << 10;   // per-call XOR: kernel on the pinned stage up to this size (A/B: $WSG_XOR_DIRECT_MAX)
    // host batches up to this many wire bytes whose buffers are page-locked:
    // the kernels read and write them in place (one launch sequence and one
    // synchronize, no staging copies); $WSG_HOST_DIRECT_MAX
    uint64_t host_direct_max = 4 << 20;   // 1-4 MB batches 1.6-2x faster direct, 16 MB even (profiles/r3/host_direct_sizes.log)
    int dec_tiles_per_block = 0;   // 0: grid from dec_blocks_per_cu alone; k: ceil(tiles / k) blocks (A/B)
    bool check = false;            // $WSG_CHECK=1: operand ranges validated before every device launch (debug)
    int dec_blocks_per_cu = 4096;  // k_decode grid cap: one 16 KiB tile per block up to 16 GiB of wire (tools/tune.py, round 2: C2 84.3 vs 85.1 us at 48 blocks/CU, 88.1 at two tiles per block; C3 ragged 0.685 vs 0.705 ms at 256, 0.783 at 48)
    int fan_waves_per_cu = 6;    // fan-out period path: waves per CU (tools/c4_ab.py, graph-replayed C4: 6 -> 8.10 us, 4 -> 8.16, 8 -> 8.32)
    // fan-out period path: waves per workgroup (A/B $WSG_FAN_WPB; one-wave
    // workgroups measured best: C4 8.5 us against 9.3 at 4 and 9.0 at 8-16,
    // tools/c4_ab.py with graph-replayed launches; an empty kernel of that
    // grid is 1.65 us either way)
    int fan_wpb = 1;
    // fan-out grid path (k_fanout_tables + k_fanout_grid) for calls of at
    // least this many messages of one geometry; 0: never ($WSG_FAN_GRID, an
    // A/B knob, off: 16 x C4 in 203 us against the period kernel's 122, its
    // lanes' two dependent L2 round trips per 16-B store,
    // profiles/r4/fan_grid_ab.log)
    uint32_t fan_grid_min = 0;
    void* d_fan_tab = nullptr;   // its chunk-template table
    uint64_t fan_tab_bytes = 0;
    uint64_t small_avg = wsg::SMALL_AVG;   // batch encode: k_encode_small when wire_cap <= n * small_avg
    unsigned long long* d_err = nullptr;        // latch of the caller-visible async entry points (wsg_sync)
    unsigned long long* d_err_host = nullptr;   // latch of the host-staged pipelines (their own status)
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
    // run concurrently while kernels run between them ($WSG_PIPE=slots: one
    // stream per slot instead, the earlier design, kept for A/B runs)
    hipStream_t s_h2d = nullptr, s_kern = nullptr, s_d2h = nullptr;
    // the host lane (wsg_internal.h): page-locked host batches of at most
    // lane_max wire bytes go to a resident kernel of lane_wgs workgroups
    // through a doorbell instead of a launch + synchronize ($WSG_LANE_MAX,
    // 0 = never; $WSG_LANE_WGS)
    struct Lane {
        wsg::LaneBell* bell = nullptr;   // page-locked, coherent
        hipStream_t stream = nullptr;
        bool running = false;            // launched, not yet seen leaving
        bool broken = false;             // did not answer: the launch paths from now on
        bool declined = false;           // the process already holds lane_cap lanes: the launch paths
        uint64_t seq = 0;
        uint64_t launches = 0;           // kernel launches of the lane (wsg_lane_stats)
        uint32_t gen = 0;                // the running launch's number (exited[] holds it when it leaves)
    } lane;
    uint64_t lane_max = 64 << 10;
    uint32_t lane_wgs = 8;          // workgroups (CUs) sharing a request's reads and writes
    int lane_cap = 4;               // this context takes a lane only while the process holds fewer ($WSG_LANE_CAP)
    bool tables_in_place = true;    // the direct paths use tables in wsg_host_alloc blocks in place ($WSG_TABLES_IN_PLACE, A/B)
    uint32_t lane_idle_us = 2000;   // the lane leaves after this long without a request
    uint32_t lane_reqs = 256;       // ... and after every lane_reqs-th request ($WSG_LANE_REQS)
    // $WSG_LANE_PROFILE=1: where a lane request's time goes (host: before the
    // ring, the wait, after the answer; lane: pick-up to staged, to parsed /
    // heads built, to done, the release fence), printed when the lane stops
    bool lane_profile = false;
    double lane_prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t lane_prof_n = 0;
    int wall_khz = 100000;          // constant clock of the lane's idle limit
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
// batches' buffers, the direct paths' tables): coherent (fine-grained)
// when $WSG_HOST_COHERENT=1, else the runtime's default (A/B: the lane's
// PCIe reads of it, tools/lane_ab.py).
unsigned host_alloc_flags()
{
    static const unsigned f = [] {
        const char* e = wsg::envp("WSG_HOST_COHERENT");
        return (e && *e == '1') ? unsigned(hipHostMallocCoherent | hipHostMallocMapped) : unsigned(hipHostMallocDefault);
    }();
    return f;
}

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

namespace {

// Every context with a lane, so that a process ending without wsg_destroy
// still stops them (the lanes also leave on their own after lane_idle_us).
std::mutex& lane_registry_lock()
{
    static std::mutex* m = new std::mutex;   // leaked: used at exit
    return *m;
}
std::vector<wsg_ctx*>& lane_registry()
{
    static auto* v = new std::vector<wsg_ctx*>;
    return *v;
}

void lane_report(wsg_ctx* c)
{
    if (!c->lane_profile || !c->lane_prof_n)
        return;
    const double n = double(c->lane_prof_n);
    const double* p = c->lane_prof;
    std::fprintf(stderr,
                 "WSG_LANE_PROFILE {\"requests\": %llu, \"host_prep_us\": %.2f, \"host_wait_us\": %.2f, "
                 "\"host_post_us\": %.2f, \"lane_stage_us\": %.2f, \"lane_frames_us\": %.2f, \"lane_rest_us\": %.2f, "
                 "\"lane_fence_us\": %.2f, \"bell_us\": %.2f, \"launches\": %llu}\n",
                 (unsigned long long)c->lane_prof_n, p[0] / n, p[1] / n, p[2] / n, p[3] / n, p[4] / n, p[5] / n, p[6] / n,
                 p[7] / n, (unsigned long long)c->lane.launches);
    c->lane_prof_n = 0;
}

// Ask the lane to leave and wait until it has (its kernel has ended; a
// launch that ended after its last request may still be finishing).
void lane_stop(wsg_ctx* c)
{
    if (!c->lane.bell || !c->lane.launches)
        return;
    (void)hipSetDevice(c->device);
    __atomic_store_n(&c->lane.bell->stop, 1u, __ATOMIC_RELEASE);
    (void)hipStreamSynchronize(c->lane.stream);
    c->lane.running = false;
}

void lanes_at_exit()
{
    std::lock_guard<std::mutex> g(lane_registry_lock());
    for (wsg_ctx* c : lane_registry()) {
        lane_stop(c);
        lane_report(c);
    }
}

// Launch the lane if it is not running (first use, or it left idle).
int lane_start(wsg_ctx* c)
{
    if (!c->lane.bell) {
        void* p = nullptr;
        if (hipHostMalloc(&p, sizeof(wsg::LaneBell), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
            return WSG_ENOMEM;
        std::memset(p, 0, sizeof(wsg::LaneBell));
        c->lane.bell = static_cast<wsg::LaneBell*>(p);
        // A running lane holds the hardware queue its stream is on: every
        // packet queued behind it waits until the launch ends.  The runtime
        // keeps streams of each priority on their own queues, so the lanes
        // go on high-priority streams (ahead of nothing but other lanes) and
        // the contexts' ordinary streams never queue behind one
        // ($WSG_LANE_PRIORITY=0: the default priority, A/B)
        int lo = 0, hi = 0;
        const char* pe = wsg::envp("WSG_LANE_PRIORITY");
        const bool made = (!pe || *pe != '0') && hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess
                              ? hipStreamCreateWithPriority(&c->lane.stream, hipStreamNonBlocking, hi) == hipSuccess
                              : hipStreamCreateWithFlags(&c->lane.stream, hipStreamNonBlocking) == hipSuccess;
        if (!made) {   // (never a launch on the null stream: the doorbell goes, the next call tries again)
            c->lane.stream = nullptr;
            (void)hipHostFree(p);
            c->lane.bell = nullptr;
            return WSG_EHIP;
        }
        static std::once_flag once;
        std::call_once(once, [] { std::atexit(lanes_at_exit); });
        std::lock_guard<std::mutex> g(lane_registry_lock());
        lane_registry().push_back(c);
    }
    if (c->lane.running)
        return WSG_OK;
    wsg::LaneBell* b = c->lane.bell;
    b->stop = 0;
    // (queued behind the previous launch on the lane's stream when that one
    // is still ending: it starts from each workgroup's `done`)
    const uint64_t idle = uint64_t(c->lane_idle_us) * uint64_t(c->wall_khz) / 1000u;
    if (++c->lane.gen == 0)
        ++c->lane.gen;
    if (wsg::launch_lane(c->lane.stream, b, c->lane_wgs, idle, c->lane.gen, c->lane_reqs) != hipSuccess)
        return WSG_EHIP;
    c->lane.running = true;
    ++c->lane.launches;
    return WSG_OK;
}

// Frames per group for a request of n frames: the workgroups share the
// frames evenly, a group at most LANE_THREADS frames, and no workgroup takes
// more than LANE_GROUPS_PER_WG groups (n <= lane_max_frames).
uint32_t lane_max_frames(const wsg_ctx* c)
{
    return std::min<uint32_t>(wsg::LANE_GROUPS_MAX, c->lane_wgs * wsg::LANE_GROUPS_PER_WG) * wsg::LANE_THREADS;
}
uint32_t lane_group_size(const wsg_ctx* c, uint32_t n)
{
    uint32_t G = (n + c->lane_wgs - 1) / c->lane_wgs;
    G = std::max<uint32_t>(G, (n + c->lane_wgs * wsg::LANE_GROUPS_PER_WG - 1) / (c->lane_wgs * wsg::LANE_GROUPS_PER_WG));
    G = std::max<uint32_t>(G, (n + wsg::LANE_GROUPS_MAX - 1) / wsg::LANE_GROUPS_MAX);
    return std::max<uint32_t>(1, std::min<uint32_t>(G, wsg::LANE_THREADS));
}

// One request on the lane (the group ranges already in bell->grp); returns
// when every workgroup has answered.  WSG_EHIP when the lane does not answer
// within seconds (it is then not used again).
int lane_call(wsg_ctx* c, uint32_t op, uint32_t n, uint32_t G, const uint64_t (&a)[6])
{
    wsg::LaneBell* b = c->lane.bell;
    const uint64_t want = ++c->lane.seq;
    // every unit a workgroup reads gets this request's tag, each after its
    // value (x86 stores are seen in program order; the release stores keep
    // the compiler's order): the group ranges (the caller's values), then
    // the request words, the first one last (the lane polls its tag)
    for (uint32_t k = 0; k < wsg::LANE_GROUPS_MAX; ++k)
        for (int h = 0; h < 2; ++h)
            __atomic_store_n(&b->grp[k][h].tag, want, __ATOMIC_RELEASE);
    uint64_t w[wsg::LANE_WORDS] = {uint64_t(op) | (uint64_t(n) << 32), a[0], a[1], a[2], a[3], a[4], a[5],
                                   uint64_t(G) | (uint64_t(c->lane_profile ? 1 : 0) << 32)};
    for (uint32_t k = wsg::LANE_WORDS; k-- > 0;) {   // w[0] last: the lane polls its tag
        b->w[k].v = w[k];
        __atomic_store_n(&b->w[k].tag, want, __ATOMIC_RELEASE);
    }
    const auto t0 = std::chrono::steady_clock::now();
    const uint32_t nw = c->lane_wgs;
    uint32_t g = 0;   // workgroups [0, g) have answered
    for (uint64_t i = 1;; ++i) {
        while (g < nw && __atomic_load_n(&b->done[g], __ATOMIC_ACQUIRE) == want)
            ++g;
        if (g == nw) {
            if (want % c->lane_reqs == 0)
                c->lane.running = false;   // this launch ends after this request: the next call launches again
            if (c->lane_profile) {
                const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
                const double k = 1000.0 / double(c->wall_khz);   // us per tick
                const uint64_t* v = b->prof;
                c->lane_prof[1] += us;
                c->lane_prof[3] += double(v[1] - v[0]) * k;
                c->lane_prof[4] += double(v[2] - v[1]) * k;
                c->lane_prof[5] += double(v[3] - v[2]) * k;
                c->lane_prof[6] += double(v[4] - v[3]) * k;
                c->lane_prof[7] += us - double(v[4] - v[0]) * k;
            }
            return WSG_OK;
        }
        if ((i & 255) == 0) {
            bool left = false;
            for (uint32_t k = 0; k < nw; ++k)
                left = left || __atomic_load_n(&b->exited[k], __ATOMIC_ACQUIRE) == c->lane.gen;
            if (left) {
                // a workgroup of the running launch left (idle limit) before
                // it saw this request: launch again, behind it on the
                // stream (its other workgroups leave idle too); each new
                // workgroup starts from its own `done` and takes its share
                // if it is still owed
                c->lane.running = false;
                if (int rc = lane_start(c))
                    return rc;
            }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
                c->lane.broken = true;
                __atomic_store_n(&b->stop, 1u, __ATOMIC_RELEASE);
                return WSG_EHIP;
            }
        }
        __builtin_ia32_pause();
    }
}

// Contexts of this process holding a lane (its doorbell allocated), and the
// most it lets hold one ($WSG_LANE_CAP, default 4).  Every lane's
// workgroups poll host memory over PCIe; with eight lanes (a TCP echo's four
// server and four client threads) the polls cost more than the launches
// they save: 100 clients 23.5 M msg/s with a lane per context, 30.3 M with
// four, 39.4 M with none; one client 9.5 / 9.2 / 6.2 M; in memory, 100
// clients on 4 threads 43.7 / 43.8 / 28.8 M (profiles/r4/lane_cap_ab.log).
std::atomic<int>& lane_holders()
{
    static std::atomic<int> n{0};
    return n;
}

// The lane for a request, launched if it is not running; nullptr when it
// cannot be used (it did not answer before, its launch failed, or the
// process holds its cap of lanes already).
wsg::LaneBell* lane_ready(wsg_ctx* c)
{
    if (c->lane.broken || c->lane.declined)
        return nullptr;
    const bool fresh = !c->lane.bell;
    if (fresh && lane_holders().fetch_add(1) >= c->lane_cap) {
        lane_holders().fetch_sub(1);
        c->lane.declined = true;
        return nullptr;
    }
    if (lane_start(c) != WSG_OK) {
        if (fresh && !c->lane.bell)
            lane_holders().fetch_sub(1);
        return nullptr;
    }
    return c->lane.bell;
}

void lane_release(wsg_ctx* c)
{
    if (!c->lane.bell)
        return;
    lane_holders().fetch_sub(1);
    {
        std::lock_guard<std::mutex> g(lane_registry_lock());
        auto& reg = lane_registry();
        reg.erase(std::remove(reg.begin(), reg.end(), c), reg.end());
    }
    if (!c->lane.broken)
        lane_stop(c);
    lane_report(c);
    if (c->lane.stream)
        (void)hipStreamDestroy(c->lane.stream);
    if (!c->lane.running)   // (a lane that never answered may still read its doorbell)
        (void)hipHostFree(c->lane.bell);
    c->lane.bell = nullptr;
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


int wsg_create(int device, wsg_ctx** out)
{
    if (!out)
        return WSG_EINVAL;
    *out = nullptr;
    wsg::hip_init_once();
    std::lock_guard<std::recursive_mutex> env_guard(wsg::env_mutex());   // (wsg_env.h)
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0 || device < 0 || device >= count)
        return WSG_EHIP;
    wsg_ctx* c = new (std::nothrow) wsg_ctx();
    if (!c)
        return WSG_ENOMEM;
    c->device = device;
    hipDeviceProp_t prop;
    if (hipSetDevice(device) != hipSuccess || hipGetDeviceProperties(&prop, device) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&c->d_err, sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(c->d_err, 0xFF, sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&c->d_err_host, sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(c->d_err_host, 0xFF, sizeof(unsigned long long)) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess) {
        wsg_destroy(c);
        return WSG_EHIP;
    }
    c->num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    if (const char* e = wsg::envp("WSG_BLOCKS_PER_CU")) {
        const int v = std::atoi(e);
        if (v > 0 && v <= 4096)
            c->blocks_per_cu = c->dec_blocks_per_cu = c->enc_blocks_per_cu = v;   // A/B runs: every grid
    }
    if (const char* e = wsg::envp("WSG_XOR_DIRECT_MAX"))   // A/B measurements (per-call path)
        c->xor_direct_max = std::strtoull(e, nullptr, 10);
    if (const char* e = wsg::envp("WSG_HOST_DIRECT_MAX"))   // A/B measurements (small host batches)
        c->host_direct_max = std::strtoull(e, nullptr, 10);
    if (const char* e = wsg::envp("WSG_DEC_TILES_PER_BLOCK")) {   // A/B measurements (tools/tune.py)
        const int v = std::atoi(e);
        if (v >= 0 && v <= 64)
            c->dec_tiles_per_block = v;
    }
    if (const char* e = wsg::envp("WSG_CHECK"))   // debug: checked launches (see in_alloc)
        c->check = *e == '1';
    if (const char* e = wsg::envp("WSG_ENC_BLOCKS_PER_CU")) {   // A/B measurements (tools/tune_enc.py)
        const int v = std::atoi(e);
        if (v > 0 && v <= 32768)
            c->enc_blocks_per_cu = v;
    }
    if (const char* e = wsg::envp("WSG_ENC_LAUNCH_PIECES"))   // A/B measurements (tools/c5_split.py)
        c->enc_launch_pieces = std::strtoull(e, nullptr, 10);
    if (const char* e = wsg::envp("WSG_FAN_WPB")) {   // A/B measurements (tools/c4_ab.py)
        const int v = std::atoi(e);
        if (v == 1 || v == 2 || v == 4 || v == 8 || v == 16)
            c->fan_wpb = v;
    }
    if (const char* e = wsg::envp("WSG_FAN_WAVES_PER_CU")) {   // A/B measurements (tools/tune_enc.py)
        const int v = std::atoi(e);
        if (v > 0 && v <= 64)
            c->fan_waves_per_cu = v;
    }
    if (const char* e = wsg::envp("WSG_FAN_GRID"))   // A/B measurements (tools/fan_many_ab.py)
        c->fan_grid_min = uint32_t(std::strtoul(e, nullptr, 10));
    if (const char* e = wsg::envp("WSG_SMALL_AVG"))   // A/B measurements (tools/tune_enc.py)
        c->small_avg = std::strtoull(e, nullptr, 10);
    if (const char* e = wsg::envp("WSG_LANE_MAX"))   // A/B measurements (tools/echo_size.py, bench_echo)
        c->lane_max = std::strtoull(e, nullptr, 10);
    if (const char* e = wsg::envp("WSG_LANE_PROFILE"))
        c->lane_profile = *e == '1';
    // default: one lane per hardware queue the runtime gives a priority
    // ($GPU_MAX_HW_QUEUES, 4 unless set): past that, lanes share queues and
    // each launch of one waits behind another's resident kernel (TCP echo,
    // 4+4 threads: 26 M msg/s with 8 lanes on 4 queues, 55 M on 8 queues,
    // profiles/r4/lane_hwq_ab.log)
    if (const char* e = wsg::envp("GPU_MAX_HW_QUEUES")) {
        const long v = std::atol(e);
        if (v >= 1 && v <= 64)
            c->lane_cap = int(v);
    }
    if (const char* e = wsg::envp("WSG_LANE_CAP")) {
        const long v = std::atol(e);
        if (v >= 1 && v <= (1l << 20))
            c->lane_cap = int(v);
    }
    if (const char* e = wsg::envp("WSG_LANE_REQS")) {
        const long v = std::atol(e);
        if (v >= 1 && v <= (1l << 30))
            c->lane_reqs = uint32_t(v);
    }
    if (const char* e = wsg::envp("WSG_TABLES_IN_PLACE"))
        c->tables_in_place = *e != '0';
    if (const char* e = wsg::envp("WSG_LANE_WGS")) {
        const long v = std::atol(e);
        if (v >= 1 && v <= long(wsg::LANE_WGS_MAX))
            c->lane_wgs = uint32_t(v);
    }
    if (const char* e = wsg::envp("WSG_LANE_IDLE_US")) {
        const long v = std::atol(e);
        if (v > 0 && v <= 1000000)
            c->lane_idle_us = uint32_t(v);
    }
    {
        int khz = 0;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) == hipSuccess && khz > 0)
            c->wall_khz = khz;
    }
    *out = c;
    return WSG_OK;
}

int wsg_destroy(wsg_ctx* c)
{
    if (!c)
        return WSG_EINVAL;
    (void)hipSetDevice(c->device);
    lane_release(c);
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
    (void)hipFree(c->d_fan_tab);
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
    const uint64_t units = c->dec_tiles_per_block ? ceil_div(tiles, uint64_t(c->dec_tiles_per_block)) : tiles;
    WSG_HIP(wsg::launch_decode(s, grid_for(c, std::max(units, ceil_div(n, wsg::BLOCK)), c->dec_blocks_per_cu), d_wire, d_out, wire_len,
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
    const uint64_t pieces = uint64_t(k) * ((fsize + wsg::PIECE_ALIGN - 1 + wsg::PIECE - 1) / wsg::PIECE);
    const uint64_t blocks = wsg::fanout_flat ? ceil_div(ceil_div(total, wsg::CHUNK), wsg::BLOCK * wsg::FAN_UNITS)
                                             : ceil_div(pieces, wsg::BLOCK / 64);
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
            if (c->fan_grid_min && cnt >= c->fan_grid_min) {
                // many messages: the grid path, its table grown as needed
                const uint64_t need = wsg::fanout_grid_table_bytes(fsize, k, cnt);
                if (need && need > c->fan_tab_bytes) {
                    (void)hipFree(c->d_fan_tab);
                    c->d_fan_tab = nullptr;
                    c->fan_tab_bytes = 0;
                    if (hipMalloc(&c->d_fan_tab, need) == hipSuccess)
                        c->fan_tab_bytes = need;
                }
                if (need && wsg::launch_fanout_grid(s, d_payload, len[i], d_keys, k, opcode[i], mask ? 1u : 0u, fsize,
                                                    d_wire, g, cnt, c->d_fan_tab, c->fan_tab_bytes, &perr)) {
                    WSG_HIP(perr);
                    continue;
                }
            }
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
    if (len == 0)
        return WSG_OK;
    if (int rc = ensure_stage(c, len, 0))
        return rc;
    hipStream_t s = c->stream;
    std::memcpy(c->h_stage, src, len);
    const uint64_t chunks = ceil_div(len, wsg::CHUNK);
    if (len <= c->xor_direct_max) {
        // small payloads (a message of the per-call path): the kernel reads
        // and writes the page-locked stage itself over PCIe, one launch and
        // one sync instead of H2D + kernel + D2H
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

namespace {

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
    const char* e = wsg::envp("WSG_PIPE");
    p.roles = !(e && std::strcmp(e, "slots") == 0);
    if (!p.roles) {
        p.h2d = p.kern = p.d2h = sl.stream;
        return WSG_OK;
    }
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
        std::memcpy(sl.out_dst, sl.h_out + sl.out_src, sl.out_len);
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

int decode_host_direct(wsg_ctx* c, const uint8_t* wire, uint64_t wire_len, const uint64_t* frame_start, uint32_t n,
                       uint8_t* out, wsg_recv_info* info)
{
    const auto t_in = std::chrono::steady_clock::now();
    wsg_ctx::Slot& sl = c->slots[0];
    if (int rc = slot_reserve(sl, 0, n, false))
        return rc;
    // a table and records in wsg_host_alloc blocks (the batch classes') are
    // used where they are; others through the slot's page-locked copies
    const uint64_t* fs_dev = frame_start;
    if (!c->tables_in_place || !in_host_block(frame_start, uint64_t(n) * sizeof(uint64_t))) {
        std::memcpy(sl.h_fs, frame_start, size_t(n) * sizeof(uint64_t));
        fs_dev = sl.h_fs;
    }
    wsg_recv_info* info_dev =
        c->tables_in_place && in_host_block(info, uint64_t(n) * sizeof(wsg_recv_info)) ? info : sl.h_info;
    wsg::LaneBell* lb = nullptr;
    if (wire_len <= std::min<uint64_t>(c->lane_max, wsg::LANE_STAGE - 64) && n > 0 && n <= lane_max_frames(c) &&
        strictly_increasing(frame_start, n) && (lb = lane_ready(c))) {
        // a few KiB (an echo's read): the resident lane, no launch; group
        // k's wire range from its first start (0 for the first) to the next
        // group's (wire_len after the last)
        const uint32_t G = lane_group_size(c, n);
        for (uint32_t k = 0, f = 0; f < n; ++k, f += G) {
            lb->grp[k][0].v = k == 0 ? 0 : std::min(frame_start[f], wire_len);
            lb->grp[k][1].v = f + G < n ? std::min(frame_start[f + G], wire_len) : wire_len;
        }
        const uint64_t a[6] = {reinterpret_cast<uint64_t>(wire), wire_len, reinterpret_cast<uint64_t>(fs_dev),
                               reinterpret_cast<uint64_t>(out), reinterpret_cast<uint64_t>(info_dev), 0};
        const auto t_ring = std::chrono::steady_clock::now();
        if (lane_call(c, wsg::LANE_DECODE, n, G, a) == WSG_OK) {
            const auto t_back = std::chrono::steady_clock::now();
            if (info_dev != info)
                std::memcpy(info, info_dev, size_t(n) * sizeof(wsg_recv_info));
            // no frame erred (the lane's count): nothing for the status pass to
            // find, and the records the GPU just wrote stay out of this core's
            // caches unless the caller reads them
            uint64_t errs = 0;
            for (uint32_t g = 0; g < c->lane_wgs; ++g)
                errs += lb->errs[g];
            const int rc = errs ? host_batch_status(c, wire, wire_len, frame_start, n, info) : WSG_OK;
            if (c->lane_profile) {
                using us = std::chrono::duration<double, std::micro>;
                c->lane_prof[0] += us(t_ring - t_in).count();
                c->lane_prof[2] += us(std::chrono::steady_clock::now() - t_back).count();
                ++c->lane_prof_n;
            }
            return rc;
        }
        // the lane did not answer: the launch path below (from now on always)
    }
    hipStream_t s = c->stream;
    if (int rc = decode_launch(c, wire, wire_len, fs_dev, n, out, info_dev, s, c->d_err_host))
        return rc;
    WSG_HIP(hipStreamSynchronize(s));
    if (info_dev != info)
        std::memcpy(info, info_dev, size_t(n) * sizeof(wsg_recv_info));
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
        if (n == 0) {
            if (wire_len && out != wire)
                std::memmove(out, wire, wire_len);
            return WSG_OK;
        }
        uint64_t seg_bytes = 32ull << 20;
        if (const char* e = wsg::envp("WSG_STAGE_MB"))
            seg_bytes = std::max<uint64_t>(1, std::strtoull(e, nullptr, 10)) << 20;
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
                std::memcpy(sl.h_in, wire + base, len);
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
        // per-frame errors below, and the caller's own latch is left alone

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
        const auto t_in = std::chrono::steady_clock::now();   // ($WSG_LANE_PROFILE)
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
        uint64_t seg_bytes = 32ull << 20;
        if (const char* e = wsg::envp("WSG_STAGE_MB"))
            seg_bytes = std::max<uint64_t>(1, std::strtoull(e, nullptr, 10)) << 20;
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
            if (!c->tables_in_place || !in_host_block(desc, uint64_t(n) * sizeof(wsg_send_desc))) {
                std::memcpy(sl.h_desc, desc, size_t(n) * sizeof(wsg_send_desc));
                desc_dev = sl.h_desc;
            }
            wsg::LaneBell* lb = nullptr;
            if (wire_off[n] <= c->lane_max && n <= lane_max_frames(c) && (lb = lane_ready(c))) {
                // a few KiB (the replies of an echo's read): the resident
                // lane at the offsets computed above, no launch; group k's
                // payload span for its staging
                const uint64_t* off_dev = wire_off;
                if (!c->tables_in_place || !in_host_block(wire_off, (uint64_t(n) + 1) * sizeof(uint64_t))) {
                    if (int rc = slot_reserve(sl, 0, uint64_t(n) + 1, false))
                        return rc;
                    std::memcpy(sl.h_fs, wire_off, (size_t(n) + 1) * sizeof(uint64_t));
                    off_dev = sl.h_fs;
                }
                const uint32_t G = lane_group_size(c, n);
                for (uint32_t k = 0, f = 0; f < n; ++k, f += G) {
                    uint64_t lo = UINT64_MAX, hi = 0;
                    for (uint32_t i = f, e = std::min(n, f + G); i < e; ++i)
                        if (desc[i].len) {
                            lo = std::min(lo, desc[i].src_off);
                            hi = std::max(hi, desc[i].src_off + desc[i].len);
                        }
                    lb->grp[k][0].v = hi ? lo : 0;
                    lb->grp[k][1].v = hi;
                }
                const uint64_t a[6] = {reinterpret_cast<uint64_t>(payload), reinterpret_cast<uint64_t>(desc_dev),
                                       reinterpret_cast<uint64_t>(off_dev), reinterpret_cast<uint64_t>(wire), 0, 0};
                const auto t_ring = std::chrono::steady_clock::now();
                if (lane_call(c, wsg::LANE_ENCODE, n, G, a) == WSG_OK) {
                    if (c->lane_profile) {
                        c->lane_prof[0] += std::chrono::duration<double, std::micro>(t_ring - t_in).count();
                        ++c->lane_prof_n;
                    }
                    return WSG_OK;
                }
            }
            hipStream_t s = c->stream;
            if (int rc = encode_launch(c, s, payload, desc_dev, n, wire, wire_off[n], sl.d_woff, sl.enc,
                                       c->d_err_host))
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
                    std::memcpy(sl.h_in, src, plen);
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
                                       c->d_err_host))
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
    if (requests)
        *requests = c->lane.seq;
    if (launches)
        *launches = c->lane.launches;
    if (running)
        *running = c->lane.broken ? -1 : c->lane.running ? 1 : 0;
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
