// bar_probe.hip — can the host ring a resident kernel's doorbell in device
// memory (written over the PCIe BAR) instead of the kernel polling host
// memory over PCIe?  Standalone measurement tool, not the product.
//
//   1. fine-grained device memory (hipExtMallocWithFlags, Finegrained and
//      Uncached): its pointer attributes, and whether the host can store to
//      it and read it back (a host fault ends this process only);
//   2. ping-pong round trips, median of ROUNDS, microseconds: the host writes
//      a sequence number into the doorbell, one resident wave polls it and
//      answers with a vector store into page-locked host memory, the host
//      spins on the answer —
//        bell_host   doorbell in page-locked host memory (the lane's design)
//        bell_dev_F  doorbell in fine-grained device memory
//        bell_dev_U  doorbell in uncached device memory
//   3. the same with a lane-sized task instead of one word: the host writes
//      nine 16-byte units (value, then tag = sequence number; the first unit
//      last), the wave reads all nine in one 16-byte load per lane and
//      answers once every tag shows — task_host / task_dev_F / task_dev_U.
// The worker's wave always ends: a stop value, and a wall-clock limit.
//   bar_probe [ROUNDS=20000]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
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

__device__ __forceinline__ uint64_t ld8_sys(const uint64_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One wave: waits for bell == seq (seq = 1, 2, ...), answers ans = seq; ends
// on bell == ~0 (stop) or after `ticks` of the wall clock without a ring.
__global__ __launch_bounds__(64) void k_worker(const uint64_t* bell, uint64_t* ans, uint64_t ticks)
{
    uint64_t seq = 1;
    uint64_t t0 = wall_clock64();
    for (uint32_t it = 0; it < (1u << 30); ++it) {
        const uint64_t v = ld8_sys(bell);
        if (v == ~uint64_t(0))
            break;
        if (v == seq) {
            if (threadIdx.x == 0)
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

// bell: the host's view of the doorbell, dbell: the kernel's (the same
// address unless the allocation maps them apart)
// One wave: waits until the nine units of `task` all carry tag seq, answers
// ans = seq; ends on unit 0's value == ~0 with tag 0 (stop) or after `ticks`.
__global__ __launch_bounds__(64) void k_task_worker(const uint64_t* task, uint64_t* ans, uint64_t ticks)
{
    const uint32_t t = threadIdx.x;
    uint64_t seq = 1;
    uint64_t t0 = wall_clock64();
    for (uint32_t it = 0; it < (1u << 30); ++it) {
        uint64_t v = 0, tag = 0;
        if (t < 9) {
            v = __hip_atomic_load(task + 2 * t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            tag = __hip_atomic_load(task + 2 * t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        const uint64_t v0 = __shfl(v, 0), tag0 = __shfl(tag, 0);
        if (v0 == ~uint64_t(0) && tag0 == 0)
            break;
        if (__ballot(t < 9 && tag != seq) == 0) {
            if (t == 0)
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

// fenced: the lane's order (the nine values, a store fence, the nine tags,
// a store fence); else each value then its tag (compiler order only)
bool g_fenced = false;
double g_post_us = 0;   // median time of the host's task stores (last run)

double pingpong_task(volatile uint64_t* task, const uint64_t* dtask, uint64_t* ans, int rounds, bool* ok)
{
    int khz = 0;
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    const uint64_t ticks = uint64_t(khz) * 1000;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    __atomic_store_n(ans, 0, __ATOMIC_SEQ_CST);
    for (int u = 0; u < 18; ++u)
        task[u] = 0;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    hipLaunchKernelGGL(k_task_worker, dim3(1), dim3(64), 0, s, dtask, ans, ticks);
    CK(hipGetLastError());
    std::vector<double> v;
    *ok = true;
    std::vector<double> post;
    for (int r = 1; r <= rounds; ++r) {
        const auto t = std::chrono::steady_clock::now();
        if (g_fenced) {
            for (int u = 8; u >= 0; --u)
                task[2 * u] = uint64_t(r) * 1000 + u;
            __builtin_ia32_sfence();
            for (int u = 8; u >= 0; --u)
                task[2 * u + 1] = uint64_t(r);
            __builtin_ia32_sfence();
        } else {
            for (int u = 8; u >= 0; --u) {   // value, then tag; the first unit last
                task[2 * u] = uint64_t(r) * 1000 + u;
                __atomic_thread_fence(__ATOMIC_RELEASE);
                task[2 * u + 1] = uint64_t(r);
            }
            __atomic_thread_fence(__ATOMIC_SEQ_CST);
        }
        post.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count());
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
            *ok = false;
            break;
        }
        v.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count());
    }
    std::sort(post.begin(), post.end());
    g_post_us = post.empty() ? -1 : post[post.size() / 2];
    task[1] = 0;
    task[0] = ~uint64_t(0);
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    CK(hipStreamSynchronize(s));
    CK(hipStreamDestroy(s));
    if (v.empty())
        return -1;
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

double pingpong(volatile uint64_t* bell, const uint64_t* dbell, uint64_t* ans, int rounds, bool* ok)
{
    int khz = 0;
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    const uint64_t ticks = uint64_t(khz) * 1000;   // 1 s without a ring: the wave leaves
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    __atomic_store_n(ans, 0, __ATOMIC_SEQ_CST);
    *bell = 0;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    hipLaunchKernelGGL(k_worker, dim3(1), dim3(64), 0, s, dbell, ans, ticks);
    CK(hipGetLastError());
    std::vector<double> v;
    *ok = true;
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
            *ok = false;
            break;
        }
        v.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count());
    }
    *bell = ~uint64_t(0);
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    CK(hipStreamSynchronize(s));
    CK(hipStreamDestroy(s));
    if (v.empty())
        return -1;
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

} // namespace

int main(int argc, char** argv)
{
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 20000;
    CK(hipSetDevice(0));
    uint64_t* h_ans = nullptr;
    uint64_t* h_bell = nullptr;
    CK(hipHostMalloc(&h_ans, 4096, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostMalloc(&h_bell, 4096, hipHostMallocMapped | hipHostMallocCoherent));
    bool ok = false;
    const double host = pingpong(h_bell, h_bell, h_ans, rounds, &ok);
    std::printf("{\"bell_host_us\": %.3f, \"bell_host_ok\": %s", host, ok ? "true" : "false");
    for (int f = 0; f < 2; ++f) {
        g_fenced = f == 1;
        const double th = pingpong_task(h_bell, h_bell, h_ans, rounds, &ok);
        std::printf(", \"task_host%s_us\": %.3f, \"task_host%s_post_us\": %.3f, \"task_host%s_ok\": %s",
                    f ? "_fenced" : "", th, f ? "_fenced" : "", g_post_us, f ? "_fenced" : "", ok ? "true" : "false");
    }
    std::fflush(stdout);
    for (unsigned flags : {unsigned(hipDeviceMallocFinegrained), unsigned(hipDeviceMallocUncached)}) {
        const char* tag = flags == hipDeviceMallocFinegrained ? "F" : "U";
        void* d = nullptr;
        const hipError_t e = hipExtMallocWithFlags(&d, 4096, flags);
        if (e != hipSuccess) {
            std::printf(", \"dev_%s_alloc\": \"%s\"", tag, hipGetErrorString(e));
            continue;
        }
        hipPointerAttribute_t a{};
        const hipError_t ea = hipPointerGetAttributes(&a, d);
        std::printf(", \"dev_%s_attr\": {\"rc\": %d, \"type\": %d, \"host\": \"%p\", \"device\": \"%p\"}", tag, int(ea),
                    int(a.type), a.hostPointer, a.devicePointer);
        std::fflush(stdout);
        // the host touches the device pointer itself (BAR mapping) — a fault ends this process
        volatile uint64_t* p = static_cast<volatile uint64_t*>(a.hostPointer ? a.hostPointer : d);
        p[0] = 0x1234;
        const uint64_t back = p[0];
        std::printf(", \"dev_%s_host_rw\": %s", tag, back == 0x1234 ? "true" : "false");
        std::fflush(stdout);
        const double us = pingpong(p, static_cast<const uint64_t*>(a.devicePointer ? a.devicePointer : d), h_ans,
                                   rounds, &ok);
        std::printf(", \"bell_dev_%s_us\": %.3f, \"bell_dev_%s_ok\": %s", tag, us, tag, ok ? "true" : "false");
        for (int f = 0; f < 2; ++f) {
            g_fenced = f == 1;
            const double tu = pingpong_task(p, static_cast<const uint64_t*>(a.devicePointer ? a.devicePointer : d),
                                            h_ans, rounds, &ok);
            std::printf(", \"task_dev_%s%s_us\": %.3f, \"task_dev_%s%s_post_us\": %.3f, \"task_dev_%s%s_ok\": %s", tag,
                        f ? "_fenced" : "", tu, tag, f ? "_fenced" : "", g_post_us, tag, f ? "_fenced" : "",
                        ok ? "true" : "false");
        }
        std::fflush(stdout);
        CK(hipFree(d));
    }
    std::printf("}\n");
    CK(hipHostFree(h_ans));
    CK(hipHostFree(h_bell));
    return 0;
}
