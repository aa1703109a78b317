// decbench.hip — k_decode (through the C-ABI, wsg_decode_batch) against a
// bare 16 KiB-tile copy-with-XOR kernel compiled here, on the same buffers,
// the same stream and the same launch loop: separates the kernel's own cost
// from the harness around it (Python / torch launches, allocation).
// Diagnostic tool only.
//
//   decbench [frames=4096] [payload=65536] [lib.so]
#include <hip/hip_runtime.h>

#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <vector>

#include "wsg_capi.h"
#ifdef WITH_KERNELS   // k_decode linked into this binary (no library launch path)
#include "wsg_internal.h"
#endif

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t n16,
                                              uint32_t key)
{
    extern __shared__ uint32_t pad[];   // residency cap only (dynamic LDS), never touched
    if (key == 0xFFFFFFFFu)
        pad[threadIdx.x] = 0;
    const uint64_t tiles = n16 / 1024;
    for (uint64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            v[u] = __builtin_nontemporal_load(src + t * 1024 + u * 256 + threadIdx.x);
#pragma unroll
        for (int u = 0; u < 4; ++u)
            __builtin_nontemporal_store(v[u] ^ key, dst + t * 1024 + u * 256 + threadIdx.x);
    }
}

// Variants of the bare copy that isolate what k_decode's shell adds:
//  V 1: loads issued u0, u3, u1, u2 (the DIAG=6 build's order)
//  V 2: every load waited for before the first store (k_decode's stream path)
//  V 4: blocks 0-15 first run a k_decode-like per-frame slice (dependent
//       frame-table and header loads, 32 B info store per frame)
//  V 8: a k_decode-like metadata chain per tile: a 64-lane probe load of the
//       frame table issued before the data, then two dependent scalar loads
//       (table entry -> header) before the stores
template <int V>
__global__ __launch_bounds__(256) void k_copyv(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t n16,
                                               uint32_t key, const uint64_t* __restrict__ fs, uint32_t n,
                                               uint64_t* __restrict__ info)
{
    if (V & 4) {
        for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n && blockIdx.x < 16; i += 16 * 256) {
            const uint64_t s0 = fs[i];
            const uint64_t s1 = i + 1 < n ? fs[i + 1] : s0;
            const u32x4 h = src[s0 / 16];
            info[4 * i] = s0 + h.x;
            info[4 * i + 1] = s1 - s0;
            info[4 * i + 2] = h.y;
            info[4 * i + 3] = h.z;
        }
    }
    const uint64_t tiles = n16 / 1024;
    for (uint64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
        uint64_t probe = 0;
        if (V & 8) {
            const uint64_t g = t * n / tiles;
            probe = fs[std::min<uint64_t>(g + (threadIdx.x & 63), n - 1)];
            __builtin_amdgcn_sched_barrier(0);
        }
        u32x4 v[4];
        if (V & 1) {
            const int ord[4] = {0, 3, 1, 2};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                v[ord[k]] = __builtin_nontemporal_load(src + t * 1024 + ord[k] * 256 + threadIdx.x);
                __builtin_amdgcn_sched_barrier(0);
            }
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u)
                v[u] = __builtin_nontemporal_load(src + t * 1024 + u * 256 + threadIdx.x);
        }
        uint32_t k2 = key;
        if (V & 8) {
            // probe -> uniform table entry -> header word (scalar chain)
            const uint64_t e = __builtin_amdgcn_readfirstlane(uint32_t(__shfl(probe, 0)));
            const uint64_t f = fs[std::min<uint64_t>(e / 65550, n - 1)];
            k2 ^= reinterpret_cast<const uint32_t*>(src)[__builtin_amdgcn_readfirstlane(uint32_t(f / 4)) & 0xFFFFF] & 0;
        }
        if (V & 2)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int u = 0; u < 4; ++u)
            __builtin_nontemporal_store(v[u] ^ k2, dst + t * 1024 + u * 256 + threadIdx.x);
    }
}

struct Api {
    int (*create)(int, wsg_ctx**);
    int (*decode)(wsg_ctx*, const uint8_t*, uint64_t, const uint64_t*, uint32_t, uint8_t*, wsg_recv_info*, void*);
    int (*sync)(wsg_ctx*, void*);
};

template <class F>
double timed(F launch, int reps = 20)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i)
        launch(i);
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i)
        launch(i);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms / reps;
}

int main(int argc, char** argv)
{
    const uint32_t n = argc > 1 ? uint32_t(atoi(argv[1])) : 4096;
    const uint64_t size = argc > 2 ? strtoull(argv[2], 0, 10) : 65536;
    std::vector<const char*> libs;
    for (int i = 3; i < argc; ++i)
        libs.push_back(argv[i]);
    if (libs.empty())
        libs.push_back("cppserver_amd/_build/libwsg.so");
    const uint64_t hdr = size < 126 ? 6 : size < 65536 ? 8 : 14;
    const uint64_t fsz = hdr + size, wire_len = n * fsz;
    const uint64_t slot = (wire_len + 16383) / 16384 * 16384;
    // wire: masked binary frames, random payload bytes and keys
    std::vector<uint8_t> h(wire_len);
    std::vector<uint64_t> fs(n);
    uint64_t x = 7;
    auto rnd = [&]() {
        uint64_t z = (x += 0x9e3779b97f4a7c15ull);
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        return z ^ (z >> 31);
    };
    for (uint32_t i = 0; i < n; ++i) {
        uint8_t* f = h.data() + i * fsz;
        fs[i] = i * fsz;
        f[0] = 0x82;
        if (hdr == 6) {
            f[1] = uint8_t(0x80 | size);
        } else if (hdr == 8) {
            f[1] = 0x80 | 126;
            f[2] = uint8_t(size >> 8);
            f[3] = uint8_t(size);
        } else {
            f[1] = 0x80 | 127;
            for (int k = 0; k < 8; ++k)
                f[2 + k] = uint8_t(size >> (56 - 8 * k));
        }
        const uint32_t key = uint32_t(rnd());
        memcpy(f + hdr - 4, &key, 4);
        for (uint64_t k = 0; k < size; k += 8) {
            const uint64_t r = rnd();
            memcpy(f + hdr + k, &r, std::min<uint64_t>(8, size - k));
        }
    }
    uint8_t* base;
    CK(hipMalloc(&base, 4 * slot));
    uint64_t* d_fs;
    wsg_recv_info* d_info;
    CK(hipMalloc(&d_fs, n * 8));
    CK(hipMalloc(&d_info, (n + 1) * sizeof(wsg_recv_info)));   // + the linked-in leg's error latch
    CK(hipMemset(d_info + n, 0xFF, sizeof(wsg_recv_info)));
    CK(hipMemcpy(d_fs, fs.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(base, h.data(), wire_len, hipMemcpyHostToDevice));
    CK(hipMemcpy(base + 2 * slot, h.data(), wire_len, hipMemcpyHostToDevice));
    std::vector<Api> apis;
    std::vector<wsg_ctx*> ctxs;
    for (const char* lib : libs) {
        void* so = dlopen(lib, RTLD_NOW | RTLD_LOCAL);
        if (!so) {
            fprintf(stderr, "dlopen %s: %s\n", lib, dlerror());
            return 1;
        }
        Api a;
        a.create = (int (*)(int, wsg_ctx**))dlsym(so, "wsg_create");
        a.decode = (decltype(a.decode))dlsym(so, "wsg_decode_batch");
        a.sync = (int (*)(wsg_ctx*, void*))dlsym(so, "wsg_sync");
        wsg_ctx* c = nullptr;
        if (!a.create || !a.decode || !a.sync || a.create(0, &c) != 0) {
            fprintf(stderr, "%s: no wsg API\n", lib);
            return 1;
        }
        apis.push_back(a);
        ctxs.push_back(c);
    }
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int grid = p.multiProcessorCount * 48;
    printf("frames=%u payload=%llu wire=%llu B\n", n, (unsigned long long)size, (unsigned long long)wire_len);
    const double alg = 2.0 * wire_len;
    for (int rep = 0; rep < 5; ++rep) {
        for (size_t l = 0; l < apis.size(); ++l) {
            const double ms = timed([&](int i) {
                uint8_t* w = base + (i & 1) * 2 * slot;
                apis[l].decode(ctxs[l], w, wire_len, d_fs, n, w + slot, d_info, nullptr);
            });
            if (apis[l].sync(ctxs[l], nullptr) != 0)
                printf("decode error\n");
            printf("%-48s %8.1f us %7.1f GB/s\n", libs[l], ms * 1e3, alg / (ms * 1e-3) / 1e9);
        }
        const double ms = timed([&](int i) {
            uint8_t* w = base + (i & 1) * 2 * slot;
            k_copy<<<grid, 256>>>((const u32x4*)w, (u32x4*)(w + slot), wire_len / 16, 9u);
        });
        printf("%-48s %8.1f us %7.1f GB/s\n", "bare copy (16 KiB tiles, 48 blocks/CU)", ms * 1e3,
               2.0 * (wire_len / 16384 * 16384) / (ms * 1e-3) / 1e9);
#ifdef WITH_KERNELS
        {
            const double m = timed([&](int i) {
                uint8_t* w = base + (i & 1) * 2 * slot;
                wsg::launch_decode(nullptr, grid, w, w + slot, wire_len, d_fs, n, d_info,
                                   (unsigned long long*)(d_info + n));
            });
            printf("%-48s %8.1f us %7.1f GB/s\n", "k_decode linked in (launch_decode)", m * 1e3, alg / (m * 1e-3) / 1e9);
        }
#endif
        // the bare copy at fewer resident blocks per CU (dynamic LDS caps
        // residency: 160 KiB / lds): what k_decode's 5 waves/SIMD cost a copy
        for (int res : {5, 6, 8}) {
            const size_t lds = res == 8 ? 0 : (160 * 1024) / res - 1024;
            const double m = timed([&](int i) {
                uint8_t* w = base + (i & 1) * 2 * slot;
                k_copy<<<grid, 256, lds>>>((const u32x4*)w, (u32x4*)(w + slot), wire_len / 16, 9u);
            });
            printf("bare copy, %d blocks/CU resident %18s %8.1f us %7.1f GB/s\n", res, "", m * 1e3,
                   2.0 * (wire_len / 16384 * 16384) / (m * 1e-3) / 1e9);
        }
#define VAR(V, NAME)                                                                                          \
        {                                                                                                     \
            const double m = timed([&](int i) {                                                              \
                uint8_t* w = base + (i & 1) * 2 * slot;                                                       \
                k_copyv<V><<<grid, 256>>>((const u32x4*)w, (u32x4*)(w + slot), wire_len / 16, 9u, d_fs, n,   \
                                          (uint64_t*)d_info);                                                 \
            });                                                                                               \
            printf("%-48s %8.1f us %7.1f GB/s\n", NAME, m * 1e3, 2.0 * (wire_len / 16384 * 16384) / (m * 1e-3) / 1e9); \
        }
        VAR(0, "copy v0 (as bare, variant kernel)")
        VAR(1, "copy v1 (load order 0,3,1,2)")
        VAR(2, "copy v2 (all loads before stores)")
        VAR(4, "copy v4 (per-frame slice in blocks 0-15)")
        VAR(8, "copy v8 (probe + scalar metadata chain)")
        VAR(10, "copy v10 (chain + all loads before stores)")
#undef VAR
    }
    return 0;
}
