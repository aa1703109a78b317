// xcd_probe.hip — does a resident poller's round trip to page-locked host
// memory depend on the XCD it runs on?  Standalone measurement tool, not the
// product.  A grid of BLOCKS one-wave blocks is launched; only block `which`
// stays (the others leave at once), reads its XCC id (hardware register) and
// serves a ping-pong: the host writes a sequence number into page-locked
// memory, the wave polls it and answers with a vector store, the host spins
// on the answer.  For which = 0 .. BLOCKS-1: the XCC id and the median /
// p10 / p90 round trip, one JSON line each.  With NOISE > 0, block 0 serves
// and blocks 1 .. NOISE poll page-locked words of their own the same way
// (pollers that never get a task: does their traffic slow the server?);
// OWN=1: the noise pollers read only their own word, not the server's.
// WAVES > 1: the server block has that many waves, each polling the bell
// and answering (staggered pollers of one word in one block).
// The waves always end: a stop value, and a wall-clock limit.
//   xcd_probe [BLOCKS=16] [ROUNDS=20000] [NOISE=0] [OWN=0] [WAVES=1]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                      \
        }                                                                                      \
    } while (0)

namespace {

// s_getreg_b32 of HW_REG_XCC_ID (id 20), bits [3:0]
__device__ __forceinline__ uint32_t xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 0xF; }

__global__ __launch_bounds__(1024) void k_worker(const uint64_t* bell, uint64_t* ans, uint64_t* where, uint32_t which,
                                                 uint32_t noise, uint32_t own, uint64_t ticks)
{
    if (noise && blockIdx.x >= 1 && blockIdx.x <= noise) {
        if (threadIdx.x >= 64)
            return;
        // a poller without tasks: its own word (one 4 KiB page apart), until
        // the server's bell says stop or the wall-clock limit
        const uint64_t* mine = bell + 512 * blockIdx.x;
        const uint64_t t0 = wall_clock64();
        for (uint32_t it = 0; it < (1u << 30); ++it) {
            const uint64_t v = __hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) |
                               (own ? uint64_t(0) : __hip_atomic_load(bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
            if (v == ~uint64_t(0))
                break;
            if ((it & 63) == 63 && wall_clock64() - t0 > 4 * ticks)
                break;
            if (own && (it & 255) == 255 &&
                __hip_atomic_load(bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == ~uint64_t(0))
                break;
            __builtin_amdgcn_s_sleep(1);
        }
        return;
    }
    if (blockIdx.x != which)
        return;
    if (threadIdx.x == 0)
        __hip_atomic_store(where, uint64_t(xcc_id()) + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // every wave of the server block polls and answers (lane 0 of each wave),
    // started a fraction of a round trip apart (~40 short sleeps)
    {
        const uint32_t w = threadIdx.x / 64, nw = blockDim.x / 64;
        for (uint32_t k = 0; k < 40 * w / nw; ++k)
            __builtin_amdgcn_s_sleep(1);
    }
    uint64_t seq = 1;
    uint64_t t0 = wall_clock64();
    for (uint32_t it = 0; it < (1u << 30); ++it) {
        const uint64_t v = __hip_atomic_load(bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (v == ~uint64_t(0))
            break;
        if (v >= seq && v != ~uint64_t(0)) {   // (a wave may have missed a ring another answered)
            seq = v;
            if ((threadIdx.x & 63) == 0)
                __hip_atomic_store(ans, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            ++seq;
            t0 = wall_clock64();
            continue;
        }
        if ((it & 63) == 63 && wall_clock64() - t0 > ticks)
            break;
        __builtin_amdgcn_s_sleep(1);
    }
}

} // namespace

int main(int argc, char** argv)
{
    const uint32_t blocks = argc > 1 ? uint32_t(std::atoi(argv[1])) : 16;
    const int rounds = argc > 2 ? std::atoi(argv[2]) : 20000;
    const uint32_t noise = argc > 3 ? uint32_t(std::atoi(argv[3])) : 0;
    const uint32_t own = argc > 4 ? uint32_t(std::atoi(argv[4])) : 0;
    const uint32_t waves = argc > 5 ? std::max(1u, std::min(16u, uint32_t(std::atoi(argv[5])))) : 1;
    CK(hipSetDevice(0));
    int khz = 0;
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    const uint64_t ticks = uint64_t(khz) * 1000;   // 1 s without a ring: the wave leaves
    uint64_t* h = nullptr;
    CK(hipHostMalloc(&h, 4096 * 64, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(h, 0, 4096 * 64);
    volatile uint64_t* bell = h;
    uint64_t* ans = h + 64;
    uint64_t* where = h + 128;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (uint32_t which = 0; which < (noise ? 1u : blocks); ++which) {
        *bell = 0;
        __atomic_store_n(ans, 0, __ATOMIC_SEQ_CST);
        __atomic_store_n(where, 0, __ATOMIC_SEQ_CST);
        hipLaunchKernelGGL(k_worker, dim3(std::max(blocks, noise + 1)), dim3(64 * waves), 0, s, h, ans, where, which,
                           noise, own, ticks);
        CK(hipGetLastError());
        std::vector<double> v;
        bool ok = true;
        for (int r = 1; r <= rounds; ++r) {
            const auto t = std::chrono::steady_clock::now();
            *bell = uint64_t(r);
            __atomic_thread_fence(__ATOMIC_SEQ_CST);
            bool got = false;
            for (uint64_t i = 0;; ++i) {
                if (__atomic_load_n(ans, __ATOMIC_ACQUIRE) == uint64_t(r)) {
                    got = true;
                    break;
                }
                if ((i & 4095) == 0 && std::chrono::steady_clock::now() - t > std::chrono::milliseconds(200))
                    break;
            }
            if (!got) {
                ok = false;
                break;
            }
            v.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count());
        }
        *bell = ~uint64_t(0);
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
        CK(hipStreamSynchronize(s));
        std::sort(v.begin(), v.end());
        const uint64_t w = __atomic_load_n(where, __ATOMIC_ACQUIRE);
        if (v.empty())
            std::printf("{\"block\": %u, \"xcc\": %lld, \"ok\": false}\n", which, (long long)w - 1);
        else
            std::printf("{\"block\": %u, \"xcc\": %lld, \"noise\": %u, \"own\": %u, \"waves\": %u, "
                        "\"us_median\": %.3f, \"us_p10\": %.3f, \"us_p90\": %.3f, \"ok\": %s}\n",
                        which, (long long)w - 1, noise, own, waves, v[v.size() / 2], v[v.size() / 10],
                        v[v.size() * 9 / 10], ok ? "true" : "false");
        std::fflush(stdout);
    }
    CK(hipStreamDestroy(s));
    CK(hipHostFree(h));
    return 0;
}
