// membench.hip — streaming read+write ceiling on gfx950 for the access shape
// of the unmask kernel (16 B per lane, coalesced, out-of-place and in-place).
// Diagnostic tool only (not part of the product): tells which block size,
// steps-per-lane and cache policy reach the HBM roof for a copy-with-XOR.
//
//   hipcc --offload-arch=gfx950 -O3 -o membench membench.hip && ./membench [MiB]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int BLOCK, int U, int NT>
__global__ __launch_bounds__(BLOCK) void k_stream(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                  uint64_t n16, uint32_t key)
{
    const uint64_t per_tile = uint64_t(BLOCK) * U;
    const uint64_t tiles = n16 / per_tile;
    for (uint64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = t * per_tile + uint64_t(u) * BLOCK + threadIdx.x;
            if (NT & 1)
                v[u] = __builtin_nontemporal_load(src + i);
            else
                v[u] = src[i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = t * per_tile + uint64_t(u) * BLOCK + threadIdx.x;
            u32x4 w = v[u] ^ key;
            if (NT & 2)
                __builtin_nontemporal_store(w, dst + i);
            else
                dst[i] = w;
        }
    }
}

// Pattern of the encode kernel: each WAVE owns a contiguous piece of
// 64 x 16 x U bytes; pieces are dealt round-robin over all waves.
template <int BLOCK, int U, int NT>
__global__ __launch_bounds__(BLOCK) void k_wavepiece(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                     uint64_t n16, uint32_t key)
{
    const uint64_t per_piece = uint64_t(64) * U;
    const uint64_t pieces = n16 / per_piece;
    const uint64_t waves = uint64_t(gridDim.x) * (BLOCK / 64);
    const uint64_t lane = threadIdx.x & 63;
    for (uint64_t q = uint64_t(blockIdx.x) * (BLOCK / 64) + (threadIdx.x >> 6); q < pieces; q += waves) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            v[u] = __builtin_nontemporal_load(src + q * per_piece + u * 64 + lane);
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_nontemporal_store(v[u] ^ key, dst + q * per_piece + u * 64 + lane);
    }
}

// Tile -> block mappings for a streaming copy-with-XOR (16 KiB tiles):
//  MAP 0: grid-stride (tile t to block t % grid)
//  MAP 1: XCD-partitioned: blocks are dealt to the 8 XCDs round-robin
//         (block b runs on XCD b % 8), so XCD x streams the x-th eighth of
//         the buffer, grid-stride within it
//  MAP 2: block-contiguous runs (block b streams tiles [b*T/grid, (b+1)*T/grid))
template <int MAP>
__global__ __launch_bounds__(256) void k_map(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t n16,
                                             uint32_t key)
{
    constexpr int U = 4;
    const uint64_t per_tile = 256ull * U;
    const uint64_t tiles = n16 / per_tile;
    uint64_t t0, t1, stride;
    if (MAP == 0) {
        t0 = blockIdx.x;
        t1 = tiles;
        stride = gridDim.x;
    } else if (MAP == 1) {
        const uint64_t x = blockIdx.x % 8, per = gridDim.x / 8;
        t0 = x * tiles / 8 + blockIdx.x / 8;
        t1 = (x + 1) * tiles / 8;
        stride = per;
    } else {
        t0 = uint64_t(blockIdx.x) * tiles / gridDim.x;
        t1 = uint64_t(blockIdx.x + 1) * tiles / gridDim.x;
        stride = 1;
    }
    for (uint64_t t = t0; t < t1; t += stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            v[u] = __builtin_nontemporal_load(src + t * per_tile + uint64_t(u) * 256 + threadIdx.x);
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_nontemporal_store(v[u] ^ key, dst + t * per_tile + uint64_t(u) * 256 + threadIdx.x);
    }
}

// One 16 KiB tile per block; which tile block b takes: W-way interleave of
// W equal regions (W = 1: linear), i.e. W address streams advance together
template <int W>
__global__ __launch_bounds__(256) void k_ways(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t tiles,
                                              uint32_t key)
{
    const uint64_t per = tiles / W;
    const uint64_t t = (blockIdx.x % W) * per + blockIdx.x / W;
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
        v[u] = __builtin_nontemporal_load(src + t * 1024 + uint64_t(u) * 256 + threadIdx.x);
#pragma unroll
    for (int u = 0; u < 4; ++u)
        __builtin_nontemporal_store(v[u] ^ key, dst + t * 1024 + uint64_t(u) * 256 + threadIdx.x);
}

template <int MAP>
void run_map(const char* name, u32x4* const* srcs, u32x4* const* dsts, uint64_t n16, int grid)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 4; ++i)
        k_map<MAP><<<grid, 256>>>(srcs[i & 1], dsts[i & 1], n16, 7u);
    const int reps = 40;
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i)
        k_map<MAP><<<grid, 256>>>(srcs[i & 1], dsts[i & 1], n16, 7u);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    printf("%-28s grid=%6d  %8.1f us  %7.1f GB/s\n", name, grid, ms * 1e3, 2.0 * n16 * 16 / (ms * 1e-3) / 1e9);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

// Write-only stream (the fan-out's shape): every lane stores U chunks.
template <int BLOCK, int U, int NT>
__global__ __launch_bounds__(BLOCK) void k_fill(u32x4* __restrict__ dst, uint64_t n16, uint32_t key)
{
    const uint64_t per_tile = uint64_t(BLOCK) * U;
    for (uint64_t t = blockIdx.x; t * per_tile < n16; t += gridDim.x) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = t * per_tile + uint64_t(u) * BLOCK + threadIdx.x;
            if (i < n16) {
                const u32x4 w = u32x4{uint32_t(i), key, key, key};
                if (NT)
                    __builtin_nontemporal_store(w, dst + i);
                else
                    dst[i] = w;
            }
        }
    }
}

template <int BLOCK, int U, int NT>
void run_fill(u32x4* dst, uint64_t n16, int grid, bool single)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i)
        k_fill<BLOCK, U, NT><<<grid, BLOCK>>>(dst, n16, 7u);
    const int reps = single ? 1 : 20;
    float tot = 0;
    for (int r = 0; r < (single ? 20 : 1); ++r) {
        CK(hipEventRecord(a));
        for (int i = 0; i < reps; ++i)
            k_fill<BLOCK, U, NT><<<grid, BLOCK>>>(dst, n16, 7u);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        tot += ms;
    }
    const double ms = tot / 20;
    printf("fill %s U=%2d nt=%d grid=%6d  %8.2f us  %7.1f GB/s\n", single ? "single " : "b2b    ", U, NT, grid,
           ms * 1e3, n16 * 16 / (ms * 1e-3) / 1e9);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

template <int BLOCK, int U>
void run_wp(const char* name, const u32x4* src, u32x4* dst, uint64_t n16, int cus, int bpc)
{
    const uint64_t pieces = n16 / (64 * U);
    const int grid = int(std::min<uint64_t>(pieces / (BLOCK / 64), uint64_t(cus) * bpc));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i)
        k_wavepiece<BLOCK, U, 3><<<grid, BLOCK>>>(src, dst, n16, 0x12345678u);
    const int reps = 20;
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i)
        k_wavepiece<BLOCK, U, 3><<<grid, BLOCK>>>(src, dst, n16, 0x12345678u);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    printf("%-34s block=%4d U=%2d bpc=%2d grid=%6d  %8.1f us  %7.1f GB/s\n", name, BLOCK, U, bpc, grid, ms * 1e3,
           2.0 * n16 * 16 / (ms * 1e-3) / 1e9);
}

template <int BLOCK, int U, int NT>
void run(const char* name, const u32x4* src, u32x4* dst, uint64_t n16, int cus, int bpc)
{
    const uint64_t tiles = n16 / (uint64_t(BLOCK) * U);
    const int grid = int(std::min<uint64_t>(tiles, uint64_t(cus) * bpc));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i)
        k_stream<BLOCK, U, NT><<<grid, BLOCK>>>(src, dst, n16, 0x12345678u);
    const int reps = 20;
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i)
        k_stream<BLOCK, U, NT><<<grid, BLOCK>>>(src, dst, n16, 0x12345678u);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    const double gbs = 2.0 * n16 * 16 / (ms * 1e-3) / 1e9;
    printf("%-34s block=%4d U=%2d nt=%d bpc=%2d grid=%6d  %8.1f us  %7.1f GB/s\n", name, BLOCK, U, NT, bpc, grid,
           ms * 1e3, gbs);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

// Read-only stream: XOR-reduce into one dword per lane, stored only if it
// hits an impossible value (keeps the loads alive).
template <int U>
__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t n16)
{
    const uint64_t per_tile = 256ull * U;
    const uint64_t tiles = n16 / per_tile;
    u32x4 acc = {0, 0, 0, 0};
    for (uint64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
#pragma unroll
        for (int u = 0; u < U; ++u)
            acc ^= __builtin_nontemporal_load(src + t * per_tile + uint64_t(u) * 256 + threadIdx.x);
    }
    if (acc.x == 0xdeadbeefu && acc.y == 0x01234567u)
        dst[threadIdx.x] = acc;
}

// Streaming copy-with-XOR with the whole tile's loads issued before any
// store (same as k_stream U) but software-pipelined: the loads of tile t+grid
// are issued before the stores of tile t.
template <int U>
__global__ __launch_bounds__(256) void k_pipe(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t n16,
                                              uint32_t key)
{
    const uint64_t per_tile = 256ull * U;
    const uint64_t tiles = n16 / per_tile;
    uint64_t t = blockIdx.x;
    if (t >= tiles)
        return;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        v[u] = __builtin_nontemporal_load(src + t * per_tile + uint64_t(u) * 256 + threadIdx.x);
    for (;;) {
        const uint64_t nt = t + gridDim.x;
        const uint64_t lt = nt < tiles ? nt : t;   // last pass re-reads its own tile
        u32x4 w[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            w[u] = __builtin_nontemporal_load(src + lt * per_tile + uint64_t(u) * 256 + threadIdx.x);
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_nontemporal_store(v[u] ^ key, dst + t * per_tile + uint64_t(u) * 256 + threadIdx.x);
        if (nt >= tiles)
            break;
#pragma unroll
        for (int u = 0; u < U; ++u)
            v[u] = w[u];
        t = nt;
    }
}

// Cache-policy variants of the 16 KiB-tile copy (decode's shape): buffer
// loads/stores with the gfx950 cache-policy bits in `aux` (1 = sc0, 2 = nt,
// 16 = sc1); LA / SA = load / store policy; LA = 255 reads nothing (write-only),
// SA = 255 stores nothing (read-only, XOR-reduced).
template <int LA, int SA>
__global__ __launch_bounds__(256) void k_policy(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                uint64_t tiles, uint32_t key)
{
    constexpr uint64_t TB = 16384;
    u32x4 acc = {0, 0, 0, 0};
    for (uint64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
        u32x4 v[4];
        if (LA != 255) {
            const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(src) + t * TB, 0, TB, 0x00020000);
#pragma unroll
            for (int u = 0; u < 4; ++u)
                v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (u * 256 + threadIdx.x) * 16, 0, LA);
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u)
                v[u] = u32x4{uint32_t(t), uint32_t(u), threadIdx.x, key};
        }
        if (SA != 255) {
            const auto rd = __builtin_amdgcn_make_buffer_rsrc(dst + t * TB, 0, TB, 0x00020000);
#pragma unroll
            for (int u = 0; u < 4; ++u)
                __builtin_amdgcn_raw_buffer_store_b128(v[u] ^ key, rd, (u * 256 + threadIdx.x) * 16, 0, SA);
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u)
                acc ^= v[u];
        }
    }
    if (SA == 255 && acc.x == 0xdeadbeefu && acc.y == 0x01234567u)
        reinterpret_cast<u32x4*>(dst)[threadIdx.x] = acc;
}

// Write-only row patterns of the fan-out kernel: each wave stores RW
// consecutive 1 KiB rows (RW * 64 lanes... one 16-B chunk per lane per row)
// per pass, passes strided by the whole grid; SC1 = write-through stores.
// an (almost) empty kernel: the launch / wave start-up floor of a grid
// random source bytes (a 32-bit hash of the word index): the data the codec
// streams, against hipMemset's constant bytes
__global__ __launch_bounds__(256) void k_hashfill(uint32_t* __restrict__ dst, uint64_t words, uint32_t seed)
{
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < words; i += uint64_t(gridDim.x) * 256) {
        uint32_t x = uint32_t(i) ^ uint32_t(i >> 32) * 0x9E3779B1u ^ seed;
        x ^= x >> 16;
        x *= 0x7FEB352Du;
        x ^= x >> 15;
        x *= 0x846CA68Bu;
        x ^= x >> 16;
        dst[i] = x;
    }
}

__global__ void k_empty(uint32_t* out, uint32_t v)
{
    if (v == 0xFFFFFFFFu)
        out[threadIdx.x] = v;
}

template <int RW, bool SC1>
__global__ __launch_bounds__(64 * RW) void k_rows(uint8_t* __restrict__ dst, uint64_t rows, uint32_t key)
{
    const uint64_t wave_rows = uint64_t(gridDim.x) * RW;
    for (uint64_t r = uint64_t(blockIdx.x) * RW + threadIdx.x / 64; r < rows; r += wave_rows) {
        const u32x4 w = u32x4{uint32_t(r), key, threadIdx.x, key};
        uint8_t* row = dst + r * 1024;
        if (SC1) {
            const auto rs = __builtin_amdgcn_make_buffer_rsrc(row, 0, 1024, 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b128(w, rs, (threadIdx.x & 63) * 16, 0, 16);
        } else {
            __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(row) + (threadIdx.x & 63));
        }
    }
}


// Write runs: wave w of the grid (4-wave blocks) writes U consecutive 1 KiB
// rows [w U, w U + U), one 16-B store per lane per row (CONTIG = 1), or the
// block's 4U rows interleaved over its waves (CONTIG = 0: wave q of the
// block writes rows u * 4 + q, the fill's U-per-lane shape); every wave
// stores U times and leaves (a dense write front in grid order).
template <int U, int CONTIG>
__global__ __launch_bounds__(256) void k_wrun(uint8_t* __restrict__ dst, uint64_t rows, uint32_t key)
{
    const uint32_t q = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t r = CONTIG ? (uint64_t(blockIdx.x) * 4 + q) * U + u : uint64_t(blockIdx.x) * 4 * U + u * 4 + q;
        if (r < rows)
            __builtin_nontemporal_store(u32x4{uint32_t(r), key, lane, key}, reinterpret_cast<u32x4*>(dst + r * 1024) + lane);
    }
}

// LDS-DMA streaming copy-with-XOR: each wave owns pieces of U KiB (dealt
// round-robin over all waves of a resident grid) and loads them with
// global_load_lds_dwordx4 into a D-deep per-wave ring in LDS, so D-1 pieces
// stay in flight without holding VGPRs; ds_read_b128 -> XOR -> store.  vmcnt
// counts loads and stores in issue order, so the wait for piece q's DMA
// leaves exactly the ops issued after it outstanding (counted at run time).
// SP: 0 plain, 1 nontemporal, 2 write-through (sc1 buffer) stores.
__device__ __forceinline__ void wait_vm_le(int n)
{
    // s_waitcnt vmcnt(n) for n in multiples of 4 up to 60 (larger: 60 waits more: safe)
    switch (n >> 2) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(28)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(36)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(40)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(44)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(48)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(52)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(56)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(60)" ::: "memory"); break;
    }
}

template <int WPB, int D, int U, int SP>
__global__ __launch_bounds__(64 * WPB) void k_glds(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                   uint64_t pieces, uint32_t key)
{
    __shared__ u32x4 ring[WPB * D * U * 64];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t waves = uint64_t(gridDim.x) * WPB;
    const uint64_t q0 = uint64_t(blockIdx.x) * WPB + w;
    constexpr uint64_t PB = uint64_t(U) * 1024;
    u32x4* my = ring + w * (D * U * 64);
    auto issue = [&](uint64_t q, int slot) {
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_amdgcn_global_load_lds(
                (const void*)(src + q * PB + u * 1024 + lane * 16),
                (__attribute__((address_space(3))) void*)(my + (slot * U + u) * 64), 16, 0, 2);
    };
    int issued = 0;   // pieces issued ahead of the one being consumed
#pragma unroll
    for (int i = 0; i < D - 1; ++i)
        if (q0 + uint64_t(i) * waves < pieces) {
            issue(q0 + uint64_t(i) * waves, i);
            ++issued;
        }
    int stores_after = 0;   // stores issued after the oldest outstanding piece's loads
    int slot = 0;
    for (uint64_t q = q0; q < pieces; q += waves) {
        const uint64_t qn = q + uint64_t(D - 1) * waves;
        int loads_after = (issued - 1) * U;   // loads issued after piece q's
        if (qn < pieces) {
            issue(qn, (slot + D - 1) % D);
            loads_after += U;
        } else {
            --issued;
        }
        wait_vm_le(loads_after + stores_after);
        // ds_read in inline asm: hipcc otherwise waits vmcnt(0) before any
        // LDS read while a DMA is in flight (it cannot tell the ring slots
        // apart); the lgkmcnt wait takes the values as operands so nothing
        // uses them before it
        const uint32_t la = uint32_t(reinterpret_cast<uintptr_t>(
                                (__attribute__((address_space(3))) u32x4*)(my + slot * U * 64 + lane)));
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v[u]) : "v"(la), "i"(u * 1024));
        if (U == 2)
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[U > 1 ? 1 : 0]));
        else if (U == 4)
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[U > 2 ? 2 : 0]), "+v"(v[U > 3 ? 3 : 0]));
        else {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int u = 0; u < U; ++u)
                asm volatile("" : "+v"(v[u]));
        }
        if (SP == 2) {
            const auto rd = __builtin_amdgcn_make_buffer_rsrc(dst + q * PB, 0, uint32_t(PB), 0x00020000);
#pragma unroll
            for (int u = 0; u < U; ++u)
                __builtin_amdgcn_raw_buffer_store_b128(v[u] ^ key, rd, (u * 64 + lane) * 16, 0, 16);
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                u32x4* o = reinterpret_cast<u32x4*>(dst + q * PB) + u * 64 + lane;
                if (SP == 1)
                    __builtin_nontemporal_store(v[u] ^ key, o);
                else
                    *o = v[u] ^ key;
            }
        }
        // after the next piece's loads come these stores; older stores are
        // retired by the next wait with the loads they precede
        stores_after = min(stores_after + U, (D - 1) * U);
        slot = (slot + 1) % D;
    }
}

// Tail shaping: blocks [0, nbig) copy 16 KiB tiles in order, the blocks
// after them copy the rest in tiles of 256 x 16 x SU bytes, so the last
// blocks dispatched are short and the launch drains sooner.
template <int SU, bool REV = false>
__global__ __launch_bounds__(256) void k_tail(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t nbig,
                                              uint32_t key)
{
    uint64_t base;
    int units;
    // REV (control): the short tiles first, the 16 KiB tiles last
    const uint64_t nsmall = uint64_t(gridDim.x) - nbig;
    const uint64_t b = REV ? (blockIdx.x < nsmall ? nbig + blockIdx.x : blockIdx.x - nsmall) : blockIdx.x;
    if (b < nbig) {
        base = b * 1024;
        units = 4;
    } else {
        base = nbig * 1024 + (b - nbig) * 256 * SU;
        units = SU;
    }
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (u < units)
            v[u] = __builtin_nontemporal_load(src + base + uint64_t(u) * 256 + threadIdx.x);
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (u < units)
            __builtin_nontemporal_store(v[u] ^ key, dst + base + uint64_t(u) * 256 + threadIdx.x);
}

template <class F>
double time_kernel(F launch, int reps = 20)
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

// Ceiling exploration at a C2-sized footprint: read-only, write-only,
// out-of-place copy with the destination at several offsets from the source
// (channel/bank aliasing), in-place, software-pipelined copy.
static int explore(uint64_t bytes, int cus)
{
    const uint64_t n16 = bytes / 16;
    const uint64_t span = 4 * bytes + (64ull << 20);
    uint8_t* base;
    CK(hipMalloc(&base, span));
    CK(hipMemset(base, 5, span));
    auto P = [&](uint64_t off) { return (u32x4*)(base + off); };
    auto gbs = [&](double ms, double mult) { return mult * bytes / (ms * 1e-3) / 1e9; };
    for (int bpc : {8, 16, 32}) {
        const int grid = cus * bpc;
        double ms = time_kernel([&](int i) { k_read<4><<<grid, 256>>>(P((i & 1) * 2 * bytes), P(span - 4096), n16); });
        printf("read-only U=4 bpc=%2d      %8.1f us  %7.1f GB/s\n", bpc, ms * 1e3, gbs(ms, 1));
        ms = time_kernel([&](int i) { k_read<8><<<grid, 256>>>(P((i & 1) * 2 * bytes), P(span - 4096), n16); });
        printf("read-only U=8 bpc=%2d      %8.1f us  %7.1f GB/s\n", bpc, ms * 1e3, gbs(ms, 1));
        ms = time_kernel([&](int i) { k_fill<256, 4, 1><<<grid, 256>>>(P((i & 1) * 2 * bytes), n16, 7u); });
        printf("write-only U=4 bpc=%2d     %8.1f us  %7.1f GB/s\n", bpc, ms * 1e3, gbs(ms, 1));
    }
    // copy: src at 0 / 2*bytes alternating, dst = src + bytes + delta
    for (uint64_t delta : {0ull, 16ull, 80ull, 4096ull, 65536ull, 1ull << 20, (1ull << 20) + 4096, 3ull << 20,
                           7ull << 20, (32ull << 20) + 256}) {
        for (int bpc : {8, 32}) {
            const int grid = cus * bpc;
            double ms = time_kernel([&](int i) {
                const uint64_t s = (i & 1) * 2 * bytes;
                k_stream<256, 4, 3><<<grid, 256>>>(P(s), P(s + bytes + delta), n16, 9u);
            });
            printf("copy delta=%9llu bpc=%2d  %8.1f us  %7.1f GB/s\n", (unsigned long long)delta, bpc, ms * 1e3,
                   gbs(ms, 2));
        }
    }
    for (int bpc : {4, 8, 16, 32}) {
        const int grid = cus * bpc;
        double ms = time_kernel([&](int i) {
            const uint64_t s = (i & 1) * 2 * bytes;
            k_stream<256, 4, 3><<<grid, 256>>>(P(s), P(s), n16, 9u);
        });
        printf("inplace bpc=%2d              %8.1f us  %7.1f GB/s\n", bpc, ms * 1e3, gbs(ms, 2));
        ms = time_kernel([&](int i) {
            const uint64_t s = (i & 1) * 2 * bytes;
            k_pipe<4><<<grid, 256>>>(P(s), P(s + bytes), n16, 9u);
        });
        printf("pipelined U=4 bpc=%2d        %8.1f us  %7.1f GB/s\n", bpc, ms * 1e3, gbs(ms, 2));
        ms = time_kernel([&](int i) {
            const uint64_t s = (i & 1) * 2 * bytes;
            k_pipe<2><<<grid, 256>>>(P(s), P(s + bytes), n16, 9u);
        });
        printf("pipelined U=2 bpc=%2d        %8.1f us  %7.1f GB/s\n", bpc, ms * 1e3, gbs(ms, 2));
    }
    {
        double ms = time_kernel([&](int i) {
            const uint64_t s = (i & 1) * 2 * bytes;
            CK(hipMemcpyAsync(P(s + bytes), P(s), bytes, hipMemcpyDeviceToDevice));
        });
        printf("hipMemcpyDtoD               %8.1f us  %7.1f GB/s\n", ms * 1e3, gbs(ms, 2));
    }
    CK(hipFree(base));
    return 0;
}

int main(int argc, char** argv)
{
    const uint64_t mib = argc > 1 ? strtoull(argv[1], 0, 10) : 256;
    const uint64_t bytes = (mib ? mib : 64) << 20;   // 0 = write mode's fan-out size, in a 64 MiB buffer
    const uint64_t n16 = bytes / 16;
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    printf("device %s CUs=%d bytes=%llu MiB\n", p.gcnArchName, cus, (unsigned long long)mib);
    if (argc > 2 && std::string(argv[2]) == "explore")
        return explore(bytes, cus);
    if (argc > 2 && std::string(argv[2]) == "policy") {
        // cache-policy bits on loads/stores of the decode-shaped copy at the
        // C2 footprint (argv[1] MiB), two buffer pairs in turn, 48 blocks/CU;
        // then in place, then write-only / read-only per policy
        const uint64_t span = 4 * bytes;
        uint8_t* base;
        CK(hipMalloc(&base, span));
        CK(hipMemset(base, 5, span));
        const uint64_t tiles = bytes / 16384;
        auto gbs = [&](double ms, double mult) { return mult * bytes / (ms * 1e-3) / 1e9; };
#define POL(LA, SA, INPLACE, MULT)                                                                             \
    for (int bpc : {32, 48}) {                                                                                 \
        const int grid = int(std::min<uint64_t>(tiles, uint64_t(cus) * bpc));                                 \
        double ms = time_kernel([&](int i) {                                                                   \
            const uint64_t s = (i & 1) * 2 * bytes;                                                            \
            k_policy<LA, SA><<<grid, 256>>>(base + s, base + s + (INPLACE ? 0 : bytes), tiles, 9u);           \
        });                                                                                                    \
        printf("policy load=%3d store=%3d inplace=%d bpc=%2d %8.1f us %7.1f GB/s\n", LA, SA, INPLACE, bpc,      \
               ms * 1e3, gbs(ms, MULT));                                                                       \
    }
        for (int rep = 0; rep < 2; ++rep) {
            POL(2, 2, 0, 2) POL(0, 0, 0, 2) POL(2, 0, 0, 2) POL(2, 16, 0, 2) POL(2, 17, 0, 2) POL(2, 18, 0, 2)
            POL(2, 3, 0, 2) POL(2, 1, 0, 2) POL(16, 2, 0, 2) POL(18, 2, 0, 2) POL(3, 2, 0, 2)
            POL(2, 2, 1, 2) POL(2, 16, 1, 2) POL(2, 18, 1, 2)
            POL(255, 2, 0, 1) POL(255, 0, 0, 1) POL(255, 16, 0, 1) POL(255, 17, 0, 1) POL(255, 18, 0, 1)
            POL(2, 255, 0, 1) POL(0, 255, 0, 1) POL(16, 255, 0, 1) POL(18, 255, 0, 1)
        }
#undef POL
        CK(hipFree(base));
        return 0;
    }
    if (argc > 2 && std::string(argv[2]) == "empty") {
        // launch floor: back-to-back empty kernels of 64-thread and 256-thread blocks
        uint32_t* d;
        CK(hipMalloc(&d, 4096));
        for (int rep = 0; rep < 2; ++rep)
            for (int blocks : {256, 1024, 2048, 4096, 8192})
                for (int threads : {64, 256}) {
                    double ms = time_kernel([&](int) { k_empty<<<blocks, threads>>>(d, 1u); });
                    printf("empty blocks=%5d threads=%3d %8.2f us\n", blocks, threads, ms * 1e3);
                }
        CK(hipFree(d));
        return 0;
    }
    if (argc > 2 && std::string(argv[2]) == "wrun") {
        // write runs of U rows per wave (k_wrun), contiguous vs interleaved,
        // against the fill's one store per lane, on argv[1] MiB (626 =
        // ws_multicast's 16-message tick; 0 = one C4, 41,040,000 B)
        const uint64_t bytes41 = (mib ? n16 * 16 : 41040000ull) / 1024 * 1024;
        uint8_t* d;
        CK(hipMalloc(&d, 2 * bytes41 + 4096));
        const uint64_t rows = bytes41 / 1024;
#define WR(U, C)                                                                                                        \
    {                                                                                                                   \
        const int blocks = int((rows + 4 * U - 1) / (4 * U));                                                           \
        double ms = time_kernel([&](int i) { k_wrun<U, C><<<blocks, 256>>>(d + (i & 1) * bytes41, rows, 7u); });       \
        printf("wrun U=%2d contig=%d blocks=%7d  %8.2f us  %7.1f GB/s\n", U, C, blocks, ms * 1e3,                       \
               bytes41 / (ms * 1e-3) / 1e9);                                                                            \
    }
        for (int rep = 0; rep < 2; ++rep) {
            WR(1, 1) WR(2, 1) WR(4, 1) WR(8, 1) WR(16, 1) WR(2, 0) WR(4, 0) WR(8, 0)
            double ms = time_kernel([&](int i) { CK(hipMemsetAsync(d + (i & 1) * bytes41, i, bytes41)); });
            printf("hipMemsetAsync          %8.2f us  %7.1f GB/s\n", ms * 1e3, bytes41 / (ms * 1e-3) / 1e9);
        }
#undef WR
        CK(hipFree(d));
        return 0;
    }
    if (argc > 2 && std::string(argv[2]) == "wpattern") {
        // the fan-out's output (41,040,000 B) written by row patterns: one
        // 1 KiB row per wave per pass (the period kernel) vs 2 / 4 / 16
        // consecutive rows per block, nontemporal vs write-through, over
        // several wave counts; b2b = launches back to back
        // (argv[1] MiB > 0: that many bytes instead, e.g. 626 = ws_multicast's 16-message tick)
        const uint64_t bytes41 = (mib ? n16 * 16 : 41040000ull) / 1024 * 1024;
        uint8_t* d;
        CK(hipMalloc(&d, 2 * bytes41 + 4096));
        const uint64_t rows = bytes41 / 1024;
#define WP(RW, SC1)                                                                                                 for (int wpc : {4, 8, 16, 32}) {                                                                                    const int blocks = std::max(1, cus * wpc / RW);                                                                 double ms = time_kernel([&](int i) { k_rows<RW, SC1><<<blocks, 64 * RW>>>(d + (i & 1) * bytes41, rows, 7u); });         printf("rows RW=%2d sc1=%d waves/CU=%2d  %8.2f us  %7.1f GB/s\n", RW, int(SC1), wpc, ms * 1e3,                            bytes41 / (ms * 1e-3) / 1e9);                                                                        }
        for (int rep = 0; rep < 2; ++rep) {
            WP(1, false) WP(1, true) WP(2, true) WP(4, false) WP(4, true) WP(16, true)
        }
#undef WP
        CK(hipFree(d));
        return 0;
    }
    if (argc > 2 && std::string(argv[2]) == "tail") {
        // the last pct % of the bytes in short tiles (4 or 8 KiB) vs all 16 KiB
        // tiles; two buffer pairs in turn, interleaved settings, 3 rounds
        const uint64_t span = 4 * bytes;
        uint8_t* base;
        CK(hipMalloc(&base, span));
        CK(hipMemset(base, 5, span));
        auto P = [&](uint64_t off) { return (u32x4*)(base + off); };
        const uint64_t tiles = n16 / 1024;
        for (int rep = 0; rep < 3; ++rep)
            for (int su : {1, 2, -1})
                for (int pct : {0, 15, 25, 35, 50, 100}) {
                    const uint64_t nbig = tiles - tiles * pct / 100;
                    const uint64_t nsmall = (tiles - nbig) * 4 / (su < 0 ? 1 : su);
                    const int grid = int(nbig + nsmall);
                    double ms = time_kernel([&](int i) {
                        const uint64_t s = (i & 1) * 2 * bytes;
                        if (su == 1)
                            k_tail<1><<<grid, 256>>>(P(s), P(s + bytes), nbig, 9u);
                        else if (su == 2)
                            k_tail<2><<<grid, 256>>>(P(s), P(s + bytes), nbig, 9u);
                        else
                            k_tail<1, true><<<grid, 256>>>(P(s), P(s + bytes), nbig, 9u);
                    });
                    printf("tail su=%d pct=%2d grid=%6d %8.2f us %7.1f GB/s\n", su, pct, grid, ms * 1e3,
                           2.0 * tiles * 16384 / (ms * 1e-3) / 1e9);
                }
        CK(hipFree(base));
        return 0;
    }
    if (argc > 2 && std::string(argv[2]) == "ways") {
        // address streams: one tile per block, W-way interleaved regions,
        // against grid-stride loops of 1, 2 and 4 tiles per block; two pairs
        const uint64_t span = 4 * bytes;
        uint8_t* base;
        CK(hipMalloc(&base, span));
        CK(hipMemset(base, 5, span));
        auto P = [&](uint64_t off) { return (u32x4*)(base + off); };
        const uint64_t tiles = n16 / 1024;
        auto show = [&](const char* name, double ms) {
            printf("%-36s %8.1f us %7.1f GB/s\n", name, ms * 1e3, 2.0 * tiles * 16384 / (ms * 1e-3) / 1e9);
        };
#define WAYS(W)                                                                                                \
    show("one tile per block, " #W "-way", time_kernel([&](int i) {                                            \
             const uint64_t s = (i & 1) * 2 * bytes;                                                           \
             k_ways<W><<<int(tiles / W * W), 256>>>(P(s), P(s + bytes), tiles, 9u);                            \
         }));
        for (int rep = 0; rep < 2; ++rep) {
            WAYS(1) WAYS(2) WAYS(4) WAYS(8) WAYS(16)
            for (int per : {1, 2, 4}) {
                char name[64];
                snprintf(name, sizeof name, "grid-stride, %d tiles per block", per);
                show(name, time_kernel([&](int i) {
                         const uint64_t s = (i & 1) * 2 * bytes;
                         k_stream<256, 4, 3><<<int(tiles / per), 256>>>(P(s), P(s + bytes), n16, 9u);
                     }));
            }
            // 512- and 1024-thread blocks, one 32 / 64 KiB tile each (half /
            // a quarter of the blocks, nothing sequential inside a block)
            show("512-thread blocks, one 32 KiB tile", time_kernel([&](int i) {
                     const uint64_t s = (i & 1) * 2 * bytes;
                     k_stream<512, 4, 3><<<int(tiles / 2), 512>>>(P(s), P(s + bytes), n16, 9u);
                 }));
            show("1024-thread blocks, one 64 KiB tile", time_kernel([&](int i) {
                     const uint64_t s = (i & 1) * 2 * bytes;
                     k_stream<1024, 4, 3><<<int(tiles / 4), 1024>>>(P(s), P(s + bytes), n16, 9u);
                 }));
        }
#undef WAYS
        CK(hipFree(base));
        return 0;
    }
    if (argc > 2 && std::string(argv[2]) == "data") {
        // does the copy's rate depend on the bytes? the 16 KiB-tile copy at
        // 48 blocks/CU over two pairs, sources of constant bytes vs random
        // bytes (splitmix64), interleaved
        const uint64_t span = 4 * bytes;
        uint8_t* base;
        CK(hipMalloc(&base, span));
        std::vector<uint64_t> h(bytes / 8);
        uint64_t x = 12345;
        for (auto& w : h) {
            uint64_t z = (x += 0x9e3779b97f4a7c15ull);
            z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
            z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
            w = z ^ (z >> 31);
        }
        auto P = [&](uint64_t off) { return (u32x4*)(base + off); };
        const int grid = cus * 48;
        auto launch = [&](int i) {
            const uint64_t s = (i & 1) * 2 * bytes;
            k_stream<256, 4, 3><<<grid, 256>>>(P(s), P(s + bytes), n16, 9u);
        };
        for (int rep = 0; rep < 3; ++rep) {
            for (int kind = 0; kind < 3; ++kind) {
                // 0: constant 0x05, 1: zero, 2: random (both pairs' sources)
                for (int pr = 0; pr < 2; ++pr) {
                    if (kind == 2)
                        CK(hipMemcpy(base + pr * 2 * bytes, h.data(), bytes, hipMemcpyHostToDevice));
                    else
                        CK(hipMemset(base + pr * 2 * bytes, kind == 0 ? 5 : 0, bytes));
                }
                CK(hipDeviceSynchronize());
                const double ms = time_kernel(launch);
                printf("copy 16K tiles bpc=48 src=%-8s %8.1f us %7.1f GB/s\n",
                       kind == 0 ? "const05" : kind == 1 ? "zero" : "random", ms * 1e3,
                       2.0 * bytes / (ms * 1e-3) / 1e9);
            }
        }
        CK(hipFree(base));
        return 0;
    }
    if (argc > 2 && std::string(argv[2]) == "glds") {
        // LDS-DMA pipelined copy (k_glds) against the register copy at the
        // C2 footprint, two source/destination pairs in turn; resident grids.
        // After each timing, one launch on a cleared destination is checked
        // word for word (src ^ key).
        const uint64_t span = 4 * bytes;
        uint8_t* base;
        CK(hipMalloc(&base, span));
        CK(hipMemset(base, 5, span));
        {
            std::vector<uint32_t> h(bytes / 4);
            for (size_t k = 0; k < h.size(); ++k)
                h[k] = uint32_t(k * 2654435761u);
            CK(hipMemcpy(base, h.data(), bytes, hipMemcpyHostToDevice));
        }
        std::vector<uint32_t> hs(bytes / 4), hd(bytes / 4);
        CK(hipMemcpy(hs.data(), base, bytes, hipMemcpyDeviceToHost));
        auto P = [&](uint64_t off) { return (u32x4*)(base + off); };
        auto report = [&](const char* name, int grid, double ms, auto launch) {
            CK(hipMemset(base + bytes, 0, bytes));
            launch(0);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(hd.data(), base + bytes, bytes, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (size_t k = 0; k < hs.size(); ++k)
                bad += hd[k] != (hs[k] ^ 9u);
            printf("%-40s grid=%6d %8.1f us %7.1f GB/s%s\n", name, grid, ms * 1e3, 2.0 * bytes / (ms * 1e-3) / 1e9,
                   bad ? "  MISMATCH" : "");
        };
#define GL(WPB, D, U, SP, BPC)                                                                                 \
    {                                                                                                          \
        const uint64_t pieces = bytes / (U * 1024);                                                            \
        const int grid = cus * BPC;                                                                            \
        auto launch = [&](int i) {                                                                             \
            const uint64_t s = (i & 1) * 2 * bytes;                                                            \
            k_glds<WPB, D, U, SP><<<grid, 64 * WPB>>>(base + s, base + s + bytes, pieces, 9u);                 \
        };                                                                                                     \
        report("glds wpb=" #WPB " D=" #D " U=" #U " sp=" #SP " bpc=" #BPC, grid, time_kernel(launch), launch);  \
    }
        for (int rep = 0; rep < 2; ++rep) {
            {
                const int grid = cus * 48;
                auto launch = [&](int i) {
                    const uint64_t s = (i & 1) * 2 * bytes;
                    k_stream<256, 4, 3><<<grid, 256>>>(P(s), P(s + bytes), n16, 9u);
                };
                report("register copy 16K tiles nt/nt bpc=48", grid, time_kernel(launch), launch);
            }
            GL(4, 2, 4, 1, 5) GL(4, 2, 4, 2, 5) GL(4, 2, 4, 0, 5)
            GL(4, 3, 4, 1, 3) GL(4, 3, 4, 2, 3)
            GL(2, 4, 4, 1, 4) GL(2, 4, 4, 2, 4)
            GL(4, 2, 8, 1, 2) GL(4, 2, 8, 2, 2)
            GL(2, 3, 8, 1, 3) GL(2, 3, 8, 2, 3)
            GL(4, 2, 2, 1, 8) GL(4, 2, 2, 2, 8)
            GL(1, 4, 4, 1, 8) GL(1, 4, 4, 2, 8)
        }
#undef GL
        CK(hipFree(base));
        return 0;
    }
    if (argc > 2 && std::string(argv[2]) == "grid") {
        // copy ceiling against the grid: 16 KiB block tiles and 4 KiB wave
        // pieces, from grid-stride (8 blocks/CU) to one unit per block/wave;
        // two source/destination pairs used in turn (no warm Infinity Cache)
        const uint64_t span = 4 * bytes;
        uint8_t* base;
        CK(hipMalloc(&base, span));
        CK(hipMemset(base, 5, span));
        auto P = [&](uint64_t off) { return (u32x4*)(base + off); };
        const uint64_t tiles = n16 / (256 * 4), pieces = n16 / (64 * 4);
        for (int rep = 0; rep < 2; ++rep) {
            for (uint64_t bpc : {8ull, 32ull, 48ull, 64ull, 128ull, 1024ull}) {
                const int g1 = int(std::min<uint64_t>(tiles, cus * bpc));
                double ms = time_kernel([&](int i) {
                    const uint64_t s = (i & 1) * 2 * bytes;
                    k_stream<256, 4, 3><<<g1, 256>>>(P(s), P(s + bytes), n16, 9u);
                });
                printf("block-tile 16K bpc=%4llu grid=%6d %8.1f us %7.1f GB/s\n", (unsigned long long)bpc, g1, ms * 1e3,
                       2.0 * bytes / (ms * 1e-3) / 1e9);
                const int g2 = int(std::min<uint64_t>((pieces + 3) / 4, cus * bpc));
                ms = time_kernel([&](int i) {
                    const uint64_t s = (i & 1) * 2 * bytes;
                    k_wavepiece<256, 4, 3><<<g2, 256>>>(P(s), P(s + bytes), n16, 9u);
                });
                printf("wave-piece 4K  bpc=%4llu grid=%6d %8.1f us %7.1f GB/s\n", (unsigned long long)bpc, g2, ms * 1e3,
                       2.0 * bytes / (ms * 1e-3) / 1e9);
            }
        }
        CK(hipFree(base));
        return 0;
    }
    u32x4 *src, *dst;
    CK(hipMalloc(&src, bytes));
    CK(hipMalloc(&dst, bytes));
    CK(hipMemset(src, 1, bytes));
    CK(hipMemset(dst, 0, bytes));
    if (argc > 2 && std::string(argv[2]) == "pattern") {
        // block tiles (decode) vs wave pieces (encode), both nontemporal
        for (int rep = 0; rep < 2; ++rep) {
            run<256, 4, 3>("block-tile 16K", src, dst, n16, cus, 32);
            run_wp<256, 4>("wave-piece 4K", src, dst, n16, cus, 32);
            run_wp<256, 8>("wave-piece 8K", src, dst, n16, cus, 16);
            run_wp<256, 16>("wave-piece 16K", src, dst, n16, cus, 8);
        }
        CK(hipFree(src));
        CK(hipFree(dst));
        return 0;
    }
    if (argc > 2 && std::string(argv[2]) == "pcie") {
        // PCIe ceilings with pinned host memory: H2D alone, D2H alone, and both
        // directions at once on two streams (what a decode pipeline overlaps)
        void *h_in, *h_out;
        CK(hipHostMalloc(&h_in, bytes, hipHostMallocDefault));
        CK(hipHostMalloc(&h_out, bytes, hipHostMallocDefault));
        std::memset(h_in, 3, bytes);
        hipStream_t s1, s2;
        CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        auto timed = [&](const char* name, int mode, uint64_t seg) {
            for (int warm = 0; warm < 2; ++warm) {
                CK(hipDeviceSynchronize());
                auto t0 = std::chrono::steady_clock::now();
                for (uint64_t off = 0; off < bytes; off += seg) {
                    const uint64_t n = std::min(seg, bytes - off);
                    if (mode & 1)
                        CK(hipMemcpyAsync((uint8_t*)src + off, (uint8_t*)h_in + off, n, hipMemcpyHostToDevice, s1));
                    if (mode & 2)
                        CK(hipMemcpyAsync((uint8_t*)h_out + off, (uint8_t*)dst + off, n, hipMemcpyDeviceToHost, s2));
                }
                CK(hipDeviceSynchronize());
                const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                if (warm)
                    printf("%-12s seg=%5llu MiB  %6.1f GiB/s per direction\n", name, (unsigned long long)(seg >> 20),
                           bytes / sec / (1 << 30));
            }
        };
        for (uint64_t seg : {uint64_t(8) << 20, uint64_t(32) << 20, bytes}) {
            timed("H2D", 1, seg);
            timed("D2H", 2, seg);
            timed("H2D+D2H", 3, seg);
        }
        CK(hipHostFree(h_in));
        CK(hipHostFree(h_out));
        CK(hipFree(src));
        CK(hipFree(dst));
        return 0;
    }
    if (argc > 2 && std::string(argv[2]) == "map") {
        // C2-sized copy (argv[1] MiB per buffer), two buffer pairs alternating
        // so that no launch re-reads what the previous one left in the MALL
        u32x4 *s2, *d2;
        CK(hipMalloc(&s2, bytes));
        CK(hipMalloc(&d2, bytes));
        CK(hipMemset(s2, 2, bytes));
        u32x4* srcs[2] = {src, s2};
        u32x4* dsts[2] = {dst, d2};
        for (int rep = 0; rep < 2; ++rep)
            for (int bpc : {8, 16, 32}) {
                const int grid = cus * bpc;
                run_map<0>("grid-stride", srcs, dsts, n16, grid);
                run_map<1>("xcd-partitioned", srcs, dsts, n16, grid);
                run_map<2>("block-contiguous", srcs, dsts, n16, grid);
            }
        CK(hipFree(s2));
        CK(hipFree(d2));
        CK(hipFree(src));
        CK(hipFree(dst));
        return 0;
    }
    if (argc > 2 && std::string(argv[2]) == "power") {
        // C5's question, second part: per-launch times of a long back-to-back
        // run of the covering wave-piece copy on constant (hipMemset) vs
        // random source bytes; argv[3] launches (default 40)
        const int launches = argc > 3 ? atoi(argv[3]) : 40;
        const uint64_t pieces = n16 / 256;
        const int grid = int(pieces / 4);
        for (int random = 0; random < 2; ++random) {
            if (random)
                k_hashfill<<<cus * 64, 256>>>((uint32_t*)src, bytes / 4, 12345u);
            else
                CK(hipMemset(src, 1, bytes));
            CK(hipDeviceSynchronize());
            std::vector<hipEvent_t> ev(launches + 1);
            for (int i = 0; i <= launches; ++i)
                CK(hipEventCreate(&ev[i]));
            CK(hipEventRecord(ev[0]));
            for (int i = 0; i < launches; ++i) {
                k_wavepiece<256, 4, 3><<<grid, 256>>>(src, dst, n16, 0x12345678u);
                CK(hipEventRecord(ev[i + 1]));
            }
            CK(hipEventSynchronize(ev[launches]));
            printf("%s source, %d launches (us):", random ? "random" : "constant", launches);
            double first = 0, last = 0;
            for (int i = 0; i < launches; ++i) {
                float ms = 0;
                CK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
                printf(" %.0f", ms * 1e3);
                if (i < 5)
                    first += ms / 5;
                if (i >= launches - 5)
                    last += ms / 5;
            }
            printf("\n  first 5 avg %.1f us = %.1f GB/s, last 5 avg %.1f us = %.1f GB/s\n", first * 1e3,
                   2.0 * bytes / (first * 1e-3) / 1e9, last * 1e3, 2.0 * bytes / (last * 1e-3) / 1e9);
            for (int i = 0; i <= launches; ++i)
                CK(hipEventDestroy(ev[i]));
        }
        CK(hipFree(src));
        CK(hipFree(dst));
        return 0;
    }
    if (argc > 2 && std::string(argv[2]) == "footprint") {
        // C5's footprint question (round 3): the encode pattern (one 4 KiB
        // piece per wave) with a grid capped at 1024 blocks/CU — pieces dealt
        // grid-stride, so once the buffer has more pieces than the grid has
        // waves the resident waves work several regions GiB apart — against a
        // grid that covers every piece once (one pass, dispatch order = address
        // order), and the resident grid-stride copy (32 blocks/CU)
        for (int rep = 0; rep < 2; ++rep) {
            run_wp<256, 4>("wavepiece capped", src, dst, n16, cus, 1024);
            run_wp<256, 4>("wavepiece covering", src, dst, n16, cus, 1 << 22);
            run<256, 4, 3>("resident grid-stride", src, dst, n16, cus, 32);
        }
        CK(hipFree(src));
        CK(hipFree(dst));
        return 0;
    }
    if (argc > 2 && std::string(argv[2]) == "write") {
        // write-only floor for a fan-out-sized output (argv[1] MiB; 0 = 41,040,000 B)
        const uint64_t w16 = mib ? n16 : 41040000ull / 16;
        if (w16 > n16) {
            fprintf(stderr, "write size exceeds the buffer\n");
            return 1;
        }
        for (int single = 0; single < 2; ++single) {
            for (int grid : {cus * 4, cus * 8, cus * 16, int((w16 + 1023) / 1024)}) {
                run_fill<256, 4, 1>(dst, w16, grid, single);
                run_fill<256, 4, 0>(dst, w16, grid, single);
            }
            run_fill<256, 16, 1>(dst, w16, int((w16 + 4095) / 4096), single);
            run_fill<256, 1, 1>(dst, w16, int((w16 + 255) / 256), single);
            hipEvent_t a, b;
            CK(hipEventCreate(&a));
            CK(hipEventCreate(&b));
            CK(hipEventRecord(a));
            for (int i = 0; i < 20; ++i)
                CK(hipMemsetAsync(dst, i, w16 * 16));
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            printf("hipMemsetAsync b2b  %8.2f us\n", ms / 20 * 1e3);
        }
        CK(hipFree(src));
        CK(hipFree(dst));
        return 0;
    }
    if (argc > 2 && std::string(argv[2]) == "calib") {
        // PMC calibration: known bytes (read n16*16, write n16*16 per launch)
        run<256, 4, 0>("calib plain", src, dst, n16, cus, 8);
        run<256, 4, 3>("calib nt", src, dst, n16, cus, 8);
        CK(hipFree(src));
        CK(hipFree(dst));
        return 0;
    }
    for (int bpc : {4, 8, 16}) {
        run<256, 4, 0>("oop", src, dst, n16, cus, bpc);
        run<256, 4, 3>("oop", src, dst, n16, cus, bpc);
    }
    run<256, 8, 0>("oop", src, dst, n16, cus, 8);
    run<256, 8, 3>("oop", src, dst, n16, cus, 8);
    run<256, 8, 2>("oop", src, dst, n16, cus, 8);
    run<256, 8, 1>("oop", src, dst, n16, cus, 8);
    run<256, 16, 0>("oop", src, dst, n16, cus, 4);
    run<256, 16, 3>("oop", src, dst, n16, cus, 4);
    run<512, 4, 0>("oop", src, dst, n16, cus, 4);
    run<512, 8, 3>("oop", src, dst, n16, cus, 4);
    run<1024, 4, 0>("oop", src, dst, n16, cus, 2);
    run<1024, 4, 3>("oop", src, dst, n16, cus, 2);
    run<256, 4, 0>("oop grid=all tiles", src, dst, n16, cus, 1 << 20);
    run<256, 4, 3>("oop grid=all tiles", src, dst, n16, cus, 1 << 20);
    run<256, 8, 3>("oop grid=all tiles", src, dst, n16, cus, 1 << 20);
    run<256, 4, 0>("inplace", src, src, n16, cus, 8);
    run<256, 4, 3>("inplace", src, src, n16, cus, 8);
    run<256, 8, 3>("inplace", src, src, n16, cus, 8);
    CK(hipFree(src));
    CK(hipFree(dst));
    return 0;
}
