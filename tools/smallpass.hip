// smallpass.hip — what one small host batch's GPU pass costs (VERDICT r3
// item 6: the C1 echo sends ~1000 x 38-byte frames per read, ~38 KB, and
// pays one GPU pass per read on each side).  Standalone measurement tool,
// not the product.  Times, median of many rounds, microseconds:
//   launch_sync     an empty kernel + hipStreamSynchronize
//   launch_flag     an empty kernel that stores a flag to host memory, the
//                   host spinning on the flag (no runtime synchronize)
//   xor_direct_B    one block XORs B bytes of page-locked host memory in
//                   place over PCIe (+ hipStreamSynchronize)
//   xor_direct_G    the same on G blocks
//   xor_staged      H2D copy, the XOR on device memory, D2H copy, one sync
//   bell_empty      a resident worker (one block) polling a host doorbell:
//                   host rings, worker answers, host spins on the answer
//   bell_xor        the same with the worker XORing the B bytes in place
// The worker's every wave ends: a stop flag, and an idle limit of its own.
//   smallpass [BYTES=38000] [ROUNDS=2000]
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
            std::exit(2);                                                                      \
        }                                                                                      \
    } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__global__ void k_empty() {}

__global__ void k_flag(uint64_t* flag, uint64_t v)
{
    if (threadIdx.x == 0)
        __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_xor(v4u* p, uint64_t chunks, uint32_t key)
{
    for (uint64_t c = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; c < chunks; c += uint64_t(gridDim.x) * blockDim.x)
        p[c] = p[c] ^ key;
}

struct Bell {
    uint64_t seq;        // host: request number
    uint64_t chunks;     // host: work of the request (16-B chunks, 0 = none)
    uint64_t pad0[6];
    uint64_t done;       // device: last request answered
    uint64_t pad1[7];
    uint64_t stop;       // host: leave
    uint64_t exited;     // device: the worker has left
};

// One block.  Thread 0 polls the doorbell (with sleeps), the block does the
// request, thread 0 answers.  Leaves on `stop`, or after `idle_ticks` of the
// constant clock without a request, or after max_iter polls: every wave
// reaches the end.
__global__ __launch_bounds__(1024) void k_worker(Bell* b, v4u* data, uint32_t key, uint64_t idle_ticks, uint32_t max_iter)
{
    __shared__ uint64_t s_seq, s_chunks;
    __shared__ int s_go;
    uint64_t last = 0;
    if (threadIdx.x == 0)
        last = __hip_atomic_load(&b->done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    for (;;) {
        if (threadIdx.x == 0) {
            int go = 0;
            uint64_t t0 = wall_clock64();
            for (uint32_t it = 0; it < max_iter; ++it) {
                const uint64_t s = __hip_atomic_load(&b->seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
                if (s != last) {
                    s_seq = s;
                    s_chunks = __hip_atomic_load(&b->chunks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    go = 1;
                    break;
                }
                if (__hip_atomic_load(&b->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) ||
                    wall_clock64() - t0 > idle_ticks)
                    break;
                __builtin_amdgcn_s_sleep(2);
            }
            s_go = go;
        }
        __syncthreads();
        if (!s_go)
            break;
        const uint64_t chunks = s_chunks;
        for (uint64_t c = threadIdx.x; c < chunks; c += blockDim.x)
            data[c] = data[c] ^ key;
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence_system();
            last = s_seq;
            __hip_atomic_store(&b->done, last, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    if (threadIdx.x == 0)
        __hip_atomic_store(&b->exited, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

using Clock = std::chrono::steady_clock;
static double us_since(Clock::time_point t) { return std::chrono::duration<double, std::micro>(Clock::now() - t).count(); }

template <class F>
static double median_us(int rounds, F f)
{
    std::vector<double> v;
    for (int i = 0; i < 50; ++i)
        f();
    for (int i = 0; i < rounds; ++i) {
        const auto t = Clock::now();
        f();
        v.push_back(us_since(t));
    }
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

static inline uint64_t ld_acq(const uint64_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }

int main(int argc, char** argv)
{
    const uint64_t bytes = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 38000;
    const int rounds = argc > 2 ? std::atoi(argv[2]) : 2000;
    const uint64_t chunks = (bytes + 15) / 16;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    v4u* h = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&h), chunks * 16, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(h, 0x5A, chunks * 16);
    v4u* d = nullptr;
    CK(hipMalloc(&d, chunks * 16));
    uint64_t* flag = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&flag), 64, hipHostMallocMapped | hipHostMallocCoherent));
    *flag = 0;
    Bell* bell = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&bell), sizeof(Bell), hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(bell, 0, sizeof(Bell));
    int dev = 0, khz = 100000;
    CK(hipGetDevice(&dev));
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);

    std::printf("{\"bytes\": %llu, \"rounds\": %d", (unsigned long long)bytes, rounds);
    std::printf(", \"launch_sync\": %.2f", median_us(rounds, [&] {
                    k_empty<<<1, 64, 0, s>>>();
                    CK(hipStreamSynchronize(s));
                }));
    uint64_t fv = 0;
    std::printf(", \"launch_flag\": %.2f", median_us(rounds, [&] {
                    ++fv;
                    k_flag<<<1, 64, 0, s>>>(flag, fv);
                    while (ld_acq(flag) != fv)
                        __builtin_ia32_pause();
                }));
    CK(hipStreamSynchronize(s));
    for (int g : {1, 4, 16, 64}) {
        std::printf(", \"xor_direct_%d\": %.2f", g, median_us(rounds, [&] {
                        k_xor<<<g, 256, 0, s>>>(h, chunks, 0x01020304u);
                        CK(hipStreamSynchronize(s));
                    }));
    }
    std::printf(", \"xor_direct_1x1024\": %.2f", median_us(rounds, [&] {
                    k_xor<<<1, 1024, 0, s>>>(h, chunks, 0x01020304u);
                    CK(hipStreamSynchronize(s));
                }));
    std::printf(", \"xor_staged\": %.2f", median_us(rounds, [&] {
                    CK(hipMemcpyAsync(d, h, chunks * 16, hipMemcpyHostToDevice, s));
                    k_xor<<<std::max<uint64_t>(1, (chunks + 255) / 256), 256, 0, s>>>(d, chunks, 0x01020304u);
                    CK(hipMemcpyAsync(h, d, chunks * 16, hipMemcpyDeviceToHost, s));
                    CK(hipStreamSynchronize(s));
                }));
    // the resident worker: idle limit 200 ms, at most 2^26 polls (~ seconds)
    hipStream_t ws;
    CK(hipStreamCreateWithFlags(&ws, hipStreamNonBlocking));
    const uint64_t idle = uint64_t(khz) * 200;   // 200 ms of the constant clock
    k_worker<<<1, 1024, 0, ws>>>(bell, h, 0x01020304u, idle, 1u << 26);
    CK(hipGetLastError());
    uint64_t seq = 0;
    bool dead = false;
    auto ring = [&](uint64_t c) {
        if (dead)
            return;
        bell->chunks = c;
        __atomic_store_n(&bell->seq, ++seq, __ATOMIC_RELEASE);
        const auto t = Clock::now();
        while (ld_acq(&bell->done) != seq) {
            __builtin_ia32_pause();
            if (us_since(t) > 1e6) {   // the worker left (idle limit) or never came
                dead = true;
                return;
            }
        }
    };
    std::printf(", \"bell_empty\": %.2f", median_us(rounds, [&] { ring(0); }));
    std::printf(", \"bell_xor\": %.2f", median_us(rounds, [&] { ring(chunks); }));
    __atomic_store_n(&bell->stop, 1, __ATOMIC_RELEASE);
    CK(hipStreamSynchronize(ws));
    std::printf(", \"worker_exited\": %s, \"worker_lost\": %s}\n", bell->exited ? "true" : "false",
                dead ? "true" : "false");
    CK(hipHostFree(h));
    CK(hipHostFree(flag));
    CK(hipHostFree(bell));
    CK(hipFree(d));
    return 0;
}
