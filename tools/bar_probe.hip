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
        std::fflush(stdout);
        CK(hipFree(d));
    }
    std::printf("}\n");
    CK(hipHostFree(h_ans));
    CK(hipHostFree(h_bell));
    return 0;
}
