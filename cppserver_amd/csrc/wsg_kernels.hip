// wsg_kernels.hip — gfx950 (CDNA4) kernels for batched WebSocket frame
// decode (header unpack + payload unmask) and encode (header pack + payload
// mask), the per-byte hot path of CppServer's WebSocket codec
// (reference source/server/ws/ws.cpp:212-456).
//
// Layout in HBM:
//   decode: wire (concatenated frames) -> out (same geometry, payloads
//           unmasked where they sit); per-frame wsg_recv_info.
//   encode: payload arena + wsg_send_desc[] -> wire (frames back to back).
// Work unit: a 16 KiB tile of the OUTPUT byte range = 256 lanes x 16 B x 4.
// Every output byte is written exactly once by an aligned 16-byte
// nontemporal store (output is streamed, never re-read by the kernel).
//
// Decode is one launch (k_decode): each tile locates its frames itself with
// scalar loads and takes one of three block-uniform paths:
//   stream   - the tile lies inside one payload: 16-B load, XOR with the
//              tile-rotated key, 16-B store;
//   boundary - the tile touches <= MAXF frames: their payload segments are
//              held in scalar registers; a chunk inside a segment XORs with
//              its key word, the few chunks a segment edge cuts build masks;
//   staged   - more frames (small frames): segments staged in LDS, 256
//              frames per round.
// No MFMA: XOR is not a contraction; the bound is HBM bandwidth.
#include "wsg_internal.h"

namespace wsg {

namespace {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint64_t v4u64 __attribute__((ext_vector_type(4)));   // MAXF-wide frame fields

constexpr int MAXF = 4;   // frames a tile may touch and still take the boundary path

// Streaming loads/stores carry the nontemporal hint (measured faster for
// once-touched data on MI355X: tools/membench.hip); WSG_NT_LOAD/STORE=0
// builds the plain-policy variants for A/B runs.
#ifndef WSG_NT_LOAD
#define WSG_NT_LOAD 1
#endif
#ifndef WSG_ENC_NT_SRC
#define WSG_ENC_NT_SRC 0   // encode payload loads: plain policy measured 1-5% faster than nontemporal
#endif
#ifndef WSG_ENC_NT_HI
#define WSG_ENC_NT_HI 1    // ... including the funnel's second block (the next lane's line)
#endif
#ifndef WSG_DIAG_ENC
#define WSG_DIAG_ENC 0   // timing-only encode diagnostics: 1 skip edge chunks, 2 no funnel
#endif
#ifndef WSG_DIAG
#define WSG_DIAG 0   // 5: timing-only diagnostic build of k_decode (every tile streams; tools/)
#endif
#ifndef WSG_DIAG_FAN
#define WSG_DIAG_FAN 0   // timing-only fan-out diagnostics: 1 no key loads, 2 no payload loads, 4 stores only, 8 no edge blocks; period path: 16 no template loads, 32 no key loads, 64 no stores, 128 prologue only, 256 empty
#endif
#ifndef WSG_DIAG_NOINFO
#define WSG_DIAG_NOINFO 0   // timing-only: k_decode without its per-frame info slice (tools/)
#endif
#ifndef WSG_DEC_WAVES
#define WSG_DEC_WAVES 1   // k_decode minimum waves/SIMD (register cap); 6 and 8 spill and run slower
#endif
#ifndef WSG_DEC_RELOAD
#define WSG_DEC_RELOAD 1   // k_decode staged tiles re-read their bytes instead of holding them in registers
#endif
#ifndef WSG_FAN_PERIOD
#define WSG_FAN_PERIOD 1   // fan-out: period path (k_fanout_period) where the frame size allows; 0 = flat kernel only
#endif
#ifndef WSG_FAN_UNROLL
#define WSG_FAN_UNROLL 1   // fan-out period path: passes per loop iteration (A/B)
#endif
// Fan-out period path, many messages per launch (wsg_fanout_encode_many, the
// ws_multicast tick).  Round 5 capped the launch at 4 resident one-wave
// workgroups per CU (a dynamic LDS reserve the kernel does not use) with the
// single message's ~6 waves per CU per message: 16 x C4 in 111-113 us, 0.86-0.88
// of the runtime's fill of the same bytes (97 us).  Uncapped (register-limited
// residency) with ~46 waves per CU per message — 23 x Q = 11799 waves for
// C4, each 3-4 passes — it is 100.7-104 us, 0.93-0.97 of the fill; fewer or more
// waves lose it on both sides (24: 121 us, 36: 117, 56: 113, 64: 124, 96: 169,
// where one-wave workgroups come faster than the dispatcher launches them),
// and so does the cap at these counts (profiles/r6/fan_*_ab*.log).
#ifndef WSG_FAN_CAP
#define WSG_FAN_CAP 0   // workgroups per CU of a many-message launch (0: no cap)
#endif
#ifndef WSG_FAN_MANY_WPC
#define WSG_FAN_MANY_WPC 46   // waves per CU per message of a many-message launch (0: as one message)
#endif
#ifndef WSG_FAN_MANY_WPB
#define WSG_FAN_MANY_WPB 0   // ... and waves per workgroup (0: as one message)
#endif
#ifndef WSG_FAN_KV
#define WSG_FAN_KV 2   // fan-out period path: key registers per lane (64 pass-window slots each)
#endif
#ifndef WSG_NT_STORE
#define WSG_NT_STORE 1
#endif
__device__ __forceinline__ v4u ld16(const uint8_t* p) { return *reinterpret_cast<const v4u*>(p); }
// 16 bytes of host memory in one request past the GPU's caches (the system
// scope of the relaxed atomic loads, sc0 sc1): one snapshot of the 16 bytes.
__device__ __forceinline__ v4u ld16_sys(const void* p)
{
    v4u r;
    asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(r) : "v"(p) : "memory");
    return r;
}
__device__ __forceinline__ v4u ld16nt(const uint8_t* p)
{
    if (WSG_NT_LOAD)
        return __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
    return ld16(p);
}
__device__ __forceinline__ void st16nt(uint8_t* p, v4u v)
{
    if (WSG_NT_STORE)
        __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(p));
    else
        *reinterpret_cast<v4u*>(p) = v;
}

// Stores of a once-written output stream.  Write-through (sc1) buffer stores
// beat nontemporal ones in tools/membench.hip's copy (C2 footprint: 83.4-83.9
// vs 85.0-85.5 us) and write-only stream (43.6 vs 47.4 us), but NOT in
// k_decode: 90.7 vs 87.9 us on C2 and 0.825 vs 0.782 ms on C3's ragged
// frames, and 90.1 vs 86.3 us with buffer loads too (tools/tune.py, same box,
// interleaved, two boxes), so decode keeps nontemporal stores; the fan-out
// (write-only) takes them.  WSG_OUT_SC1=1 builds the decode variant for A/B.
#ifndef WSG_OUT_SC1
#define WSG_OUT_SC1 0
#endif
#ifndef WSG_OUT_AUX
#define WSG_OUT_AUX 16   // cache-policy bits of the write-through stores (16 = sc1, 17 = sc0 | sc1; A/B)
#endif
#ifndef WSG_ENC_SC1
#define WSG_ENC_SC1 0   // batch encode (piece kernel): write-through stores (A/B)
#endif
#ifndef WSG_FAN_SC1
#define WSG_FAN_SC1 1   // fan-out period path: write-through (sc1) stores, 13.0 vs 14.3 us nontemporal at C4 (tools/tune_enc.py CFG=c4)
#endif
struct OutTile {
    uint8_t* p;   // tile base (wave-uniform)
    bool sc1;
    __amdgpu_buffer_rsrc_t rs;
    __device__ __forceinline__ OutTile(uint8_t* base, uint32_t bytes, bool write_through = WSG_OUT_SC1 != 0)
        : p(base), sc1(write_through)
    {
        if (sc1)
            rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, bytes, 0x00020000);
    }
    // whole 16-B chunk at tile offset o (o + 16 <= bytes)
    __device__ __forceinline__ void put(uint32_t o, v4u v) const
    {
        if (sc1)
            __builtin_amdgcn_raw_buffer_store_b128(v, rs, o, 0, WSG_OUT_AUX);
        else
            st16nt(p + o, v);
    }
};

__device__ __forceinline__ uint32_t ab(uint32_t hi, uint32_t lo, uint32_t b)
{
    return __builtin_amdgcn_alignbyte(hi, lo, b);   // ({hi,lo} >> 8b)[31:0]
}

// Bytes [s, s+16) of the 32-byte little-endian window lo:hi (v_alignbyte_b32).
__device__ __forceinline__ v4u funnel(v4u lo, v4u hi, uint32_t s)
{
    const uint32_t b = s & 3u;
    v4u r;
    switch (s >> 2) {
    case 0:
        r = v4u{ab(lo.y, lo.x, b), ab(lo.z, lo.y, b), ab(lo.w, lo.z, b), ab(hi.x, lo.w, b)};
        break;
    case 1:
        r = v4u{ab(lo.z, lo.y, b), ab(lo.w, lo.z, b), ab(hi.x, lo.w, b), ab(hi.y, hi.x, b)};
        break;
    case 2:
        r = v4u{ab(lo.w, lo.z, b), ab(hi.x, lo.w, b), ab(hi.y, hi.x, b), ab(hi.z, hi.y, b)};
        break;
    default:
        r = v4u{ab(hi.x, lo.w, b), ab(hi.y, hi.x, b), ab(hi.z, hi.y, b), ab(hi.w, hi.z, b)};
        break;
    }
    return r;
}

// 16 source bytes at an arbitrary address, read as aligned 16-B blocks
// (never touching a 16-B block that holds no requested byte).
template <bool NT>
__device__ __forceinline__ v4u ld16_unaligned(const uint8_t* a)
{
    const uint32_t s = uint32_t(reinterpret_cast<uintptr_t>(a) & 15u);
    const uint8_t* a0 = a - s;
    const v4u lo = NT ? ld16nt(a0) : ld16(a0);
    if (s == 0)
        return lo;
    return funnel(lo, NT ? ld16nt(a0 + 16) : ld16(a0 + 16), s);
}

// Byte j (runtime) of a 16-byte value, through two 64-bit halves so that no
// register array is indexed at run time (that would spill to scratch).
__device__ __forceinline__ uint32_t lane_byte(v4u v, uint32_t j)
{
    const uint64_t lo = uint64_t(v.x) | (uint64_t(v.y) << 32);
    const uint64_t hi = uint64_t(v.z) | (uint64_t(v.w) << 32);
    return uint32_t((j < 8 ? lo >> (8u * j) : hi >> (8u * (j - 8))) & 0xFFu);
}

__device__ __forceinline__ void put_byte(v4u& w, uint32_t j, uint32_t b)
{
    const uint64_t m = uint64_t(b & 0xFFu) << (8u * (j & 7u));
    const uint64_t lo = j < 8 ? m : 0, hi = j < 8 ? 0 : m;
    w.x |= uint32_t(lo);
    w.y |= uint32_t(lo >> 32);
    w.z |= uint32_t(hi);
    w.w |= uint32_t(hi >> 32);
}

#ifndef WSG_STAGE_FPL
#define WSG_STAGE_FPL 2
#endif
constexpr int SPL = WSG_STAGE_FPL;   // staged frames per lane per round
constexpr int LDSF = BLOCK * SPL;    // frames per staged round (one round for tiles of 32-byte frames)

__device__ __forceinline__ uint64_t lane_bcast(uint64_t v, int src)
{
    const uint32_t lo = __builtin_amdgcn_readlane(uint32_t(v), src);
    const uint32_t hi = __builtin_amdgcn_readlane(uint32_t(v >> 32), src);
    return uint64_t(lo) | (uint64_t(hi) << 32);
}

// map[t] = frame for t in [lo, hi) (encode: piece -> frame), for every lane's range, with the
// whole wave storing each range (one lane per frame would serialise a large
// frame's thousands of tiles on a single lane).
__device__ __forceinline__ void fill_tiles_wave(uint32_t* tile_first, uint64_t lo, uint64_t hi, uint32_t frame)
{
    const uint32_t lane = threadIdx.x & 63;
    constexpr uint64_t kShort = 16;   // ranges up to this many entries: the lane stores its own
    if (hi > lo && hi - lo <= kShort)
        for (uint64_t t = lo; t < hi; ++t)
            tile_first[t] = frame;
    uint64_t pending = __ballot(hi > lo + kShort);
    while (pending) {
        const int j = __builtin_ctzll(pending);
        pending &= pending - 1;
        const uint64_t a = lane_bcast(lo, j), b = lane_bcast(hi, j);
        const uint32_t fj = __builtin_amdgcn_readlane(frame, j);
        for (uint64_t t = a + lane; t < b; t += 64)
            tile_first[t] = fj;
    }
}

__device__ __forceinline__ uint64_t lane_off(int u) { return (uint64_t(u) * BLOCK + threadIdx.x) * CHUNK; }

// ---- wave / block exclusive scan of uint64 (wave64) ----------------------
__device__ __forceinline__ uint64_t wave_inclusive_scan(uint64_t v)
{
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t u = __shfl_up(v, d, 64);
        if (lane >= d)
            v += u;
    }
    return v;
}

// Exclusive scan over the block (blockDim.x == BLOCK); *total = block sum.
__device__ uint64_t block_exclusive_scan(uint64_t v, uint64_t* total)
{
    __shared__ uint64_t wsum[BLOCK / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t inc = wave_inclusive_scan(v);
    if (lane == 63)
        wsum[wid] = inc;
    __syncthreads();
    uint64_t before = 0, all = 0;
#pragma unroll
    for (int k = 0; k < BLOCK / 64; ++k) {
        before += (k < wid) ? wsum[k] : 0;
        all += wsum[k];
    }
    __syncthreads();
    *total = all;
    return before + inc - v;
}

} // namespace

// ===========================================================================
// Decode in one launch: k_decode
// ===========================================================================
//
// Every tile finds its own frames.  The frame-start table is read-only and
// sorted, so the tile's first frame is located with uniform (scalar) loads:
// an interpolation guess, exact for equal-size frames, else a 16-ary search;
// the headers of the (at most MAXF) frames the tile touches are parsed from
// scalar loads of the wire.  Scalar loads do not queue behind the tile's
// vector data loads (those return in issue order), so this metadata chain
// overlaps the data's HBM latency.  The per-frame outputs (wsg_recv_info,
// error latch) come from a lane-per-frame slice of the same launch.  One
// launch instead of parse + unmask removes a kernel boundary: ~5 us per C2
// batch (tools/tune.py, a build that skipped the parse launch).
//
// Tile paths (block-uniform): stream (inside one payload), boundary (<= MAXF
// frames, records in scalar registers), staged (more frames: records staged
// in LDS, LDSF frames per round).

namespace {

// A wave-uniform value computed by vector instructions, moved to SGPRs.
__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
// (the builtins return int: each half goes through uint32_t, else a low half
// of 2^31 or more sign-extends over the high one)
__device__ __forceinline__ uint64_t uni(uint64_t x)
{
    return uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(x)))) |
           (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(x >> 32)))) << 32);
}

// Frame [s, limit) as PrepareReceiveFrame parses it when delivered whole
// (ws.cpp:320-386), with the batch checks of wsg_decode_batch.  Returns 0 or
// the frame's error; on error r describes an empty payload at s, so the
// frame's bytes are copied.
// (Block16: the aligned 16-byte block at a wire offset; global memory here,
// LDS for the host lane's staged wire.)
template <class Block16>
__device__ __forceinline__ int frame_parse_b(Block16 block, uint64_t wire_len, uint64_t s, uint64_t limit,
                                             wsg_recv_info& r)
{
    r = wsg_recv_info{};
    int e = WSG_ETRUNC;
    if (s < wire_len) {
        const uint64_t avail = wire_len - s;
        // wire[s .. s+16) as two u64 from the aligned 32-byte window, with
        // 64-bit shifts only (scalar instructions when s is wave-uniform)
        const uint64_t a0 = s & ~uint64_t(15);
        const v4u lo = block(a0);
        const v4u hi = (a0 + 16 < wire_len) ? block(a0 + 16) : v4u{0, 0, 0, 0};
        uint64_t q0 = uint64_t(lo.x) | (uint64_t(lo.y) << 32), q1 = uint64_t(lo.z) | (uint64_t(lo.w) << 32);
        const uint64_t q2 = uint64_t(hi.x) | (uint64_t(hi.y) << 32), q3 = uint64_t(hi.z) | (uint64_t(hi.w) << 32);
        uint64_t q2s = q2;
        if (s & 8) {
            q0 = q1;
            q1 = q2;
            q2s = q3;
        }
        const uint32_t b = 8u * uint32_t(s & 7);
        const uint64_t h0 = b ? (q0 >> b) | (q1 << (64u - b)) : q0;
        const uint64_t h1 = b ? (q1 >> b) | (q2s << (64u - b)) : q1;
        e = parse_header([&](uint32_t k) { return uint8_t(k < 8 ? h0 >> (8u * k) : h1 >> (8u * (k - 8))); }, avail, r);
        if (e == 0) {
            if (r.len > avail - r.hdr_len)
                e = WSG_ETRUNC;
            else if (limit < s || limit - s < r.hdr_len || r.len > limit - s - r.hdr_len)
                e = WSG_EINVAL;   // the next frame starts inside this one
        }
    }
    if (e != 0) {
        r = wsg_recv_info{};
        r.payload_off = s;
        r.error = int8_t(e);
    } else {
        r.payload_off = s + r.hdr_len;
    }
    return e;
}

__device__ __forceinline__ int frame_parse(const uint8_t* __restrict__ wire, uint64_t wire_len, uint64_t s,
                                           uint64_t limit, wsg_recv_info& r)
{
    return frame_parse_b([wire](uint64_t a) { return ld16(wire + a); }, wire_len, s, limit, r);
}

// wsg_recv_info as four 8-byte words (a struct store of the byte fields went
// through scratch).
__device__ __forceinline__ void store_info(wsg_recv_info* dst, const wsg_recv_info& r)
{
    static_assert(offsetof(wsg_recv_info, key) == 16 && offsetof(wsg_recv_info, opcode) == 20 &&
                      offsetof(wsg_recv_info, b0) == 24 && offsetof(wsg_recv_info, error) == 25 &&
                      sizeof(wsg_recv_info) == 32,
                  "wsg_recv_info layout");
    uint64_t* w = reinterpret_cast<uint64_t*>(dst);
    w[0] = r.payload_off;
    w[1] = r.len;
    w[2] = uint64_t(r.key) | (uint64_t(r.opcode) << 32) | (uint64_t(r.fin) << 40) | (uint64_t(r.masked) << 48) |
           (uint64_t(r.hdr_len) << 56);
    w[3] = uint64_t(r.b0) | (uint64_t(uint8_t(r.error)) << 8);
}

__device__ __forceinline__ uint64_t fs_at(const uint64_t* __restrict__ fs, uint32_t n, int64_t i)
{
    return fs[min<int64_t>(i, int64_t(n) - 1)];   // clamped: the load never depends on a compare
}

// Last index i < b with fs[i] <= p, or a - 1, given fs[a - 1] <= p < fs[b]
// (fs[-1] = -inf, fs[n] = +inf): 8 independent probes per round (one round
// of scalar loads when a/b are uniform); ends for any table.
__device__ __forceinline__ int64_t search8(const uint64_t* __restrict__ fs, uint32_t a, uint32_t b, uint64_t p)
{
    while (a < b) {
        const uint32_t step = (b - a + 8) / 9;   // probes a - 1 + step * k, k = 1..8 (< b)
        uint64_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
            v[k] = fs[min(a - 1 + step * (k + 1), b - 1)];
        uint32_t na = a, nb = b;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t ix = min(a - 1 + step * (k + 1), b - 1);
            if (ix >= na && ix < nb) {
                if (v[k] <= p)
                    na = ix + 1;
                else
                    nb = ix;
            }
        }
        a = na;
        b = nb;
    }
    return int64_t(a) - 1;
}

// The frames a tile touches: first = max(f0, 0), where f0 is the last frame
// starting at or before the tile's first byte (-1: none); st[k] = fs[first+k]
// (~0 past the table).
struct TileLoc {
    int64_t f0;
    uint32_t first;
    uint64_t st[MAXF + 1];
};

// The tile's first-frame guess (exact for equal-size frames).
__device__ __forceinline__ uint64_t tile_guess(uint32_t n, double frames_per_byte, uint64_t base)
{
    return uni(min(uint64_t(double(base) * frames_per_byte), uint64_t(n - 1)));
}

// Lane k's entry of the coarse probe around the guess g: fs[g + (k - 32) S].
__device__ __forceinline__ uint32_t probe_index(uint64_t g, uint32_t stride, uint32_t n, int k)
{
    const int64_t i = int64_t(g) + int64_t(k - 32) * int64_t(stride);
    return uint32_t(max<int64_t>(0, min<int64_t>(i, int64_t(n) - 1)));
}

// Locate the tile's frames.  `probe` is this lane's coarse-probe entry,
// loaded before the tile's data (so it is back first).  Equal-size frames
// hit the guess (one round of scalar loads); otherwise the probe brackets
// the answer to `stride` frames (a miss outside +-32 strides searches the
// rest of the table), and search8 finishes it.
__device__ __forceinline__ void locate(const uint64_t* __restrict__ fs, uint32_t n, uint64_t g, uint32_t stride,
                                       uint64_t probe, uint64_t base, TileLoc& L)
{
    uint64_t w[MAXF + 2];
#pragma unroll
    for (int k = 0; k < MAXF + 2; ++k) {
        const uint64_t x = fs_at(fs, n, int64_t(g) + k);
        w[k] = (g + k < n) ? x : ~uint64_t(0);
    }
    if (w[0] <= base && base < w[1]) {   // the guess (equal-size frames)
        L.f0 = int64_t(g);
        L.first = uint32_t(g);
#pragma unroll
        for (int k = 0; k <= MAXF; ++k)
            L.st[k] = w[k];
        return;
    }
    // candidates [a, b) for the last start <= base, fs[a - 1] <= base < fs[b];
    // the probe is consulted only here, so a hit of the guess never waits for it
    const uint64_t below = __ballot(probe <= base);   // a prefix of the lanes for a sorted table
    const int m = __builtin_popcountll(below);
    uint32_t a = m > 0 ? probe_index(g, stride, n, m - 1) + 1 : 0;
    uint32_t b = m < 64 ? probe_index(g, stride, n, m) : n;
    if (m == 0 && probe_index(g, stride, n, 0) == 0)
        b = 0;   // even fs[0] is past base: no frame starts at or before it
    L.f0 = search8(fs, a, b, base);
    L.first = uint32_t(L.f0 < 0 ? 0 : L.f0);
#pragma unroll
    for (int k = 0; k <= MAXF; ++k) {
        const uint64_t x = fs_at(fs, n, int64_t(L.first) + k);
        L.st[k] = (uint64_t(L.first) + k < n) ? x : ~uint64_t(0);
    }
}

// A frame's payload as seen from one tile: bytes [lo, hi) of the tile
// (tile-relative, clamped to the tile; for the frames of a tile in order,
// lo and hi are non-decreasing) XOR with kr, the frame's key rotated
// to the tile's phase — chunk offsets are multiples of 16, so one rotation
// serves every chunk of the tile (ws.cpp:403: byte i uses key[i % 4]).
struct Seg {
    uint32_t lo, hi, kr;
};

__device__ __forceinline__ Seg tile_seg(uint64_t po, uint64_t pe, uint32_t key, uint64_t base, uint32_t span)
{
    Seg s;
    s.lo = po <= base ? 0u : uint32_t(min<uint64_t>(po - base, span));
    s.hi = pe <= base ? 0u : uint32_t(min<uint64_t>(pe - base, span));
    if (s.hi < s.lo)
        s.hi = s.lo;   // empty stays at its place: segment ends stay sorted
    s.kr = key_rot(key, uint32_t(base - po));   // (base - po) mod 4, also when po > base
    return s;
}

// Bytes [0, k) of a dword as a mask (k <= 0: none, k >= 4: all).
__device__ __forceinline__ uint32_t low_bytes(int k)
{
    return k <= 0 ? 0u : k >= 4 ? ~0u : (1u << (8 * k)) - 1u;
}

// The XOR word of segment s for the chunk at tile offset o (zero outside s).
__device__ __forceinline__ v4u seg_xor(uint32_t o, const Seg& s)
{
    if (s.hi <= o || s.lo >= o + CHUNK)
        return v4u{0, 0, 0, 0};
    const int a = s.lo > o ? int(s.lo - o) : 0;
    const int b = s.hi < o + CHUNK ? int(s.hi - o) : int(CHUNK);
    v4u m;
#pragma unroll
    for (int d = 0; d < 4; ++d)
        m[d] = s.kr & low_bytes(b - 4 * d) & ~low_bytes(a - 4 * d);
    return m;
}

// A tile's inputs, issued before its metadata chain: the coarse probe of
// the frame table (vector load, first: loads return in issue order) and the
// tile's data.
struct TileIn {
    uint64_t base, g, probe;
    v4u v[UNROLL];
};

__device__ __forceinline__ void load_tile(TileIn& T, const uint8_t* __restrict__ wire, uint64_t wire_len,
                                          const uint64_t* __restrict__ fs, uint32_t n, double frames_per_byte,
                                          uint32_t stride, uint64_t base)
{
    T.base = base;
    T.g = tile_guess(n, frames_per_byte, base);
#if WSG_DIAG == 7   // timing-only: no coarse probe (right only where the guess is exact: equal-size frames)
    T.probe = 0;
#else
    T.probe = fs[probe_index(T.g, stride, n, int(threadIdx.x & 63))];
#endif
    __builtin_amdgcn_sched_barrier(0);
    // the tile's data does not depend on frame metadata: issue it next,
    // unconditionally, so that the metadata chain waits for the probe alone
    // (vmcnt(UNROLL)); loads behind a branch made the compiler wait vmcnt(0)
    // there, i.e. start the chain only once the whole tile had arrived.  The
    // wire's last, partial tile takes the staged path, which reads its bytes
    // itself: its loads here are clamped to the 16-B block holding the last
    // wire byte (readable by contract) and their values are not used.
    const uint64_t last_blk = (wire_len - 1) & ~uint64_t(CHUNK - 1);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
        T.v[u] = ld16nt(wire + min(base + lane_off(u), last_blk));
}

// The tile's frames located, their segments XORed into its bytes, stored.
__device__ __forceinline__ void process_tile(const TileIn& T, const uint8_t* __restrict__ wire, uint8_t* out,
                                             uint64_t wire_len, const uint64_t* __restrict__ fs, uint32_t n,
                                             uint32_t stride)
{
    const uint64_t base = T.base;
    const uint64_t tend = min(base + TILE, wire_len);
    const uint32_t span = uint32_t(tend - base);
    const bool full = span == TILE;
    const uint64_t g = T.g;
    const uint64_t probe = T.probe;
    const v4u* v = T.v;
    // Only a guess miss reads the probe.  Used on that path alone, the load
    // would be sunk into it, behind the data loads (vector loads return in
    // issue order: a ragged tile would wait for its data before searching),
    // so every path ends with keep_probe(): a test that is never true for a
    // batch the host launches (n > 0), after the tile's stores, where the
    // probe is long back.
    auto keep_probe = [&]() {
        if (n == 0 && probe == ~uint64_t(0))
            out[0] = 0;
    };
    TileLoc L;
    locate(fs, n, g, stride, probe, base, L);
    // frames touching the tile: a prefix of first, first + 1, ...
    int c = 0;
#pragma unroll
    for (int k = 0; k <= MAXF; ++k) {
        const bool touches = uint64_t(L.first) + k < n && (k == 0 ? L.f0 >= 0 || L.st[0] < tend : L.st[k] < tend);
        if (touches && c == k)
            c = k + 1;
    }

    if (WSG_DIAG == 5 || (full && c <= MAXF)) {
        // frames' payload segments in scalar registers (full tiles; the
        // wire's last, partial tile takes the staged path)
        Seg S[MAXF];
#pragma unroll
        for (int k = 0; k < MAXF; ++k) {
            S[k] = Seg{0, 0, 0};
            if (k < c) {
                wsg_recv_info r;
                const uint64_t lim = (uint64_t(L.first) + k + 1 < n) ? L.st[k + 1] : wire_len;
                frame_parse(wire, wire_len, L.st[k], lim, r);
                const Seg g = tile_seg(r.payload_off, r.payload_off + r.len, r.key, base, span);
                S[k] = Seg{uni(g.lo), uni(g.hi), uni(g.kr)};
            }
        }
#if WSG_DIAG == 5   // timing-only: every tile streams with its first frame's key (8-wave register budget)
        if (true) {
#else
        if (S[0].lo == 0 && S[0].hi == TILE) {
#endif
            // stream: the whole tile is payload of one frame
            const OutTile ot(out + base, uint32_t(TILE));
#pragma unroll
            for (int u = 0; u < UNROLL; ++u)
                ot.put(uint32_t(lane_off(u)), v[u] ^ S[0].kr);
            keep_probe();
            return;
        }
        const OutTile ot(out + base, uint32_t(TILE));
        // boundary: per chunk, the key word of the segment holding it;
        // the few chunks a segment edge cuts build byte masks
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint32_t o = uint32_t(lane_off(u));
            uint32_t kx = 0;
            bool cut = false;
#pragma unroll
            for (int k = 0; k < MAXF; ++k) {
                kx = (S[k].lo <= o && o + CHUNK <= S[k].hi) ? S[k].kr : kx;
                cut |= (S[k].lo > o && S[k].lo < o + CHUNK) || (S[k].hi > o && S[k].hi < o + CHUNK);
            }
            v4u x = v4u{kx, kx, kx, kx};
            if (cut) {
                x = seg_xor(o, S[0]);
#pragma unroll
                for (int k = 1; k < MAXF; ++k)
                    x |= seg_xor(o, S[k]);
            }
            ot.put(o, v[u] ^ x);
        }
        keep_probe();
        return;
    }

    // staged: payload segments in LDS, LDSF frames per round
    __shared__ uint32_t s_lo[LDSF], s_hi[LDSF], s_kr[LDSF];
    __shared__ uint32_t s_wcnt[BLOCK / 64];
    // stage the segments of frames r0, r0 + 1, ... that touch the tile;
    // more = frames past the stage touch it too (block-uniform)
    auto stage = [&](uint64_t r0, int& cnt, bool& more) {
        // slot q * BLOCK + lane holds frame r0 + q * BLOCK + lane
        uint64_t sj[SPL], lim[SPL];
        bool touch[SPL];
#pragma unroll
        for (int q = 0; q < SPL; ++q) {
            const uint64_t fi = r0 + uint64_t(q) * BLOCK + threadIdx.x;
            sj[q] = ~uint64_t(0);
            lim[q] = wire_len;
            if (fi < n) {
                sj[q] = fs[fi];
                lim[q] = fi + 1 < n ? fs[fi + 1] : wire_len;
            }
            // frame `first` touches (c > MAXF); the others when they start in the tile
            touch[q] = fi < n && (fi == L.first || sj[q] < tend);
        }
        // block-wide counts from wave ballots through LDS (the
        // __syncthreads_count / _or builtins cost ~40 VGPRs here,
        // tools/regs.py: 91 vs 53 for the whole kernel)
        uint32_t wc = 0;
#pragma unroll
        for (int q = 0; q < SPL; ++q)
            wc += uint32_t(__builtin_popcountll(__ballot(touch[q])));
        const bool last_more = __ballot(threadIdx.x == BLOCK - 1 && touch[SPL - 1] &&
                                        r0 + uint64_t(LDSF) < n && lim[SPL - 1] < tend) != 0;
        __syncthreads();   // the previous readers are done with the stage and the counts
        if ((threadIdx.x & 63) == 0)
            s_wcnt[threadIdx.x >> 6] = wc | (last_more ? 0x80000000u : 0u);
        __syncthreads();
        cnt = 0;
        more = false;
#pragma unroll
        for (int w = 0; w < BLOCK / 64; ++w) {
            const uint32_t x = s_wcnt[w];
            cnt += int(x & 0x7FFFFFFFu);
            more = more || (x >> 31) != 0;
        }
#pragma unroll 1
        for (int q = 0; q < SPL; ++q) {
            const int slot = q * BLOCK + int(threadIdx.x);
            if (slot < cnt) {
                wsg_recv_info r;
                frame_parse(wire, wire_len, sj[q], lim[q], r);
                const Seg g = tile_seg(r.payload_off, r.payload_off + r.len, r.key, base, span);
                s_lo[slot] = g.lo;
                s_hi[slot] = g.hi;
                s_kr[slot] = g.kr;
            }
        }
        __syncthreads();
    };
    // XOR words of the staged segments for the chunk at tile offset o
    auto chunk_xor = [&](uint32_t o, int cnt) {
        int lo = 0, hi = cnt;   // first segment ending after o (segment ends are non-decreasing)
#pragma unroll 1
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (s_hi[mid] <= o)
                lo = mid + 1;
            else
                hi = mid;
        }
        v4u x = {0, 0, 0, 0};
#pragma unroll 1
        for (int j = lo; j < cnt && s_lo[j] < o + CHUNK; ++j)
            x |= seg_xor(o, Seg{s_lo[j], s_hi[j], s_kr[j]});
        return x;
    };
    // rounds of LDSF frames (one for every tile but those of the tiniest
    // frames): each round ORs its segments' XOR words into the thread's
    // own LDS slots, then one pass reads the tile's bytes again (L2 /
    // Infinity-Cache warm), XORs and stores.  Nothing is carried in
    // registers across the staging: this path would otherwise set the
    // kernel's register budget (95 VGPRs with the tile held in registers
    // and a per-round store, 5 waves/SIMD; tools/regs.py).
    __shared__ v4u s_acc[UNROLL][BLOCK];
#pragma unroll 1
    for (uint64_t r0 = L.first;; r0 += LDSF) {
        int cnt;
        bool more;
        stage(r0, cnt, more);
#pragma unroll 1
        for (int u = 0; u < UNROLL; ++u) {
            const v4u x = chunk_xor(uint32_t(lane_off(u)), cnt);
            s_acc[u][threadIdx.x] = (r0 == L.first) ? x : (s_acc[u][threadIdx.x] | x);
        }
        if (!more)
            break;
    }
    {
        const OutTile ot(out + base, uint32_t(TILE));
#pragma unroll 1
        for (int u = 0; u < UNROLL; ++u) {
            const uint32_t o = uint32_t(lane_off(u));
            if (o + CHUNK <= span) {
                ot.put(o, ld16(wire + base + o) ^ s_acc[u][threadIdx.x]);
            } else if (o < span) {
                // the chunk the wire's end cuts: bytes only, through the
                // thread's LDS slot (no register byte shuffles)
                uint8_t* b = reinterpret_cast<uint8_t*>(&s_acc[u][threadIdx.x]);
#pragma unroll 1
                for (uint32_t k = 0; k < span - o; ++k)
                    out[base + o + k] = uint8_t(wire[base + o + k] ^ b[k]);
            }
        }
    }
    keep_probe();
}

} // namespace

// Decode (ws.cpp:320-406 over a batch): out = wire with every payload XORed
// by its key; info[i] and the error latch per frame.
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(WSG_DEC_WAVES))) void k_decode(const uint8_t* __restrict__ wire, uint8_t* out, uint64_t wire_len,
                                                  const uint64_t* __restrict__ fs, uint32_t n, double frames_per_byte,
                                                  uint32_t stride, wsg_recv_info* __restrict__ info,
                                                  unsigned long long* err, uint64_t num_tiles)
{
    // per-frame slice: header unpack + checks, one lane per frame (on the
    // grid's last blocks after their tiles instead: no faster, round 3)
    {
        const uint64_t fstride = uint64_t(gridDim.x) * BLOCK;
        for (uint64_t i0 = uint64_t(blockIdx.x) * BLOCK + (threadIdx.x & ~63u); i0 < n && !WSG_DIAG_NOINFO;
             i0 += fstride) {
            const uint64_t i = i0 + (threadIdx.x & 63u);
            if (i < n) {
                wsg_recv_info r;
                const int e = frame_parse(wire, wire_len, fs[i], i + 1 < n ? fs[i + 1] : wire_len, r);
                if (e != 0)
                    atomicMin(err, (static_cast<unsigned long long>(i) << 8) | static_cast<unsigned long long>(-e));
                store_info(info + i, r);
            }
        }
    }

#if WSG_DIAG == 6   // timing-only: the launch as a bare copy-with-XOR of the full tiles (no frame logic)
    for (uint64_t t = blockIdx.x; t < num_tiles; t += gridDim.x) {
        const uint64_t base = t * TILE;
        if (base + TILE > wire_len)
            break;
        v4u v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            v[u] = ld16nt(wire + base + lane_off(u));
#ifdef WSG_DIAG_ORD
            __builtin_amdgcn_sched_barrier(0);
#endif
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
            st16nt(out + base + lane_off(u), v[u] ^ 0x9u);
    }
    return;
#endif
    // (two tiles per block with both tiles' loads up front: 0.0900 vs 0.0875
    // ms at C2, round 2, dropped)
    for (uint64_t t = blockIdx.x; t < num_tiles; t += gridDim.x) {
        TileIn a;
        load_tile(a, wire, wire_len, fs, n, frames_per_byte, stride, t * TILE);
        process_tile(a, wire, out, wire_len, fs, n, stride);
    }
}

// ===========================================================================
// Encode: frame-aligned work pieces
// ===========================================================================
//
// A piece is at most PIECE = 4 KiB of ONE frame's wire bytes, cut at absolute
// 16-byte chunk boundaries: piece k of frame i covers
//     [max(off_i, A_i + k*PIECE), min(end_i, A_i + (k+1)*PIECE)),   A_i = off_i & ~127
// (line-aligned output rows).
// One wave encodes one piece, so the key, the key phase and the source shift
// are uniform over it: full data chunks stream (aligned 16-B loads,
// v_alignbyte_b32 funnel, XOR, 16-B nontemporal store).  Chunks holding
// header / close-status bytes, and the two edge chunks a frame shares with
// its neighbours, are built bytewise (edge chunks: each frame stores only
// its own bytes).  Piece counts are scanned together with frame sizes.

namespace {

// Everything a piece needs about its frame (wave-uniform).
struct FrameRec {
    uint64_t off;       // wire offset of the frame
    uint64_t pw;        // wire offset of the payload (status prefix included)
    uint64_t data_w;    // wire offset of the first data byte
    uint64_t end;       // wire offset one past the frame
    const uint8_t* src; // data bytes
    uint64_t body;
    uint32_t key;
    uint32_t hdr;
    uint32_t prefix;
    int32_t status;
    uint8_t opcode;
    bool mask;
};

__device__ __forceinline__ FrameRec make_rec(uint64_t off, const uint8_t* src, uint64_t len, uint32_t key,
                                             int32_t status, uint8_t opcode, bool mask)
{
    const SendGeom g = send_geom(opcode, mask, len, status);
    FrameRec r;
    r.off = off;
    r.pw = off + g.hdr;
    r.data_w = r.pw + g.prefix;
    r.end = r.pw + g.body;
    r.src = src;
    r.body = g.body;
    r.key = key;
    r.hdr = g.hdr;
    r.prefix = g.prefix;
    r.status = status;
    r.opcode = opcode;
    r.mask = mask;
    return r;
}

// A descriptor read as eight dwords: scalar loads cannot fetch the u8 fields
// on gfx9, and a vector load for them would bring an s_waitcnt vmcnt(0)
// that also waits for every data load in flight.
struct Desc {
    uint64_t src_off, len;
    uint32_t key;
    int32_t status;
    uint8_t opcode;
    bool mask;
};

__device__ __forceinline__ Desc load_desc(const wsg_send_desc* d)
{
    const uint32_t* w = reinterpret_cast<const uint32_t*>(d);
    Desc r;
    r.src_off = uint64_t(w[0]) | (uint64_t(w[1]) << 32);
    r.len = uint64_t(w[2]) | (uint64_t(w[3]) << 32);
    r.key = w[4];
    r.status = int32_t(w[5]);
    r.opcode = uint8_t(w[6]);
    r.mask = ((w[6] >> 8) & 0xFFu) != 0;
    return r;
}
static_assert(offsetof(wsg_send_desc, key) == 16 && offsetof(wsg_send_desc, opcode) == 24 &&
                  offsetof(wsg_send_desc, mask) == 25,
              "wsg_send_desc layout");

__device__ __forceinline__ uint32_t wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// 16 payload bytes as seen from a chunk: byte j = payload[c + j] where that
// offset is inside [0, len) (else 0).  Reads only aligned 16-B blocks that
// hold a wanted byte, at most two.
// The 16-B block at an aligned address: a global load, or (the lane) the
// block's copy staged in LDS.
struct GlobalBlocks {
    __device__ v4u operator()(const uint8_t* p) const { return ld16(p); }
};
struct StagedBlocks {
    const v4u* s;          // LDS copy of the aligned blocks from `base` on
    const uint8_t* base;   // 16-B aligned
    __device__ v4u operator()(const uint8_t* p) const { return s[(p - base) >> 4]; }
};

template <class Blocks = GlobalBlocks>
__device__ __forceinline__ v4u fan_window(const uint8_t* __restrict__ payload, uint64_t len, int64_t c,
                                          Blocks blk = Blocks{})
{
    // offsets relative to `payload`, loads through pointer arithmetic on it
    // (global_* loads; a pointer rebuilt from an integer loads flat_*)
    const uint32_t s = uint32_t((reinterpret_cast<uintptr_t>(payload) + uint64_t(c)) & 15u);
    const int64_t r0 = c - int64_t(s);   // aligned block holding byte c, relative to payload
    const int64_t n = int64_t(len);
    v4u lo = {0, 0, 0, 0}, hi = {0, 0, 0, 0};
    if (r0 < n && r0 + 16 > 0)
        lo = blk(payload + r0);
    if (s != 0 && r0 + 16 < n && r0 + 32 > 0)
        hi = blk(payload + r0 + 16);
    return s ? funnel(lo, hi, s) : lo;
}

// 128-bit byte shifts and byte masks (runtime counts) built on funnel().
__device__ __forceinline__ v4u shr_bytes(v4u x, uint64_t o)   // byte j = x[j + o]
{
    return o >= CHUNK ? v4u{0, 0, 0, 0} : funnel(x, v4u{0, 0, 0, 0}, uint32_t(o));
}
__device__ __forceinline__ v4u shl_bytes(v4u x, uint64_t s)   // byte j = x[j - s]
{
    return s == 0 ? x : s >= CHUNK ? v4u{0, 0, 0, 0} : funnel(v4u{0, 0, 0, 0}, x, uint32_t(CHUNK - s));
}
__device__ __forceinline__ v4u low_bytes(uint64_t n)   // bytes [0, n) = 0xFF
{
    const uint64_t lo = n >= 8 ? ~uint64_t(0) : (uint64_t(1) << (8 * n)) - 1;
    const uint64_t hi = n >= 16 ? ~uint64_t(0) : n <= 8 ? 0 : (uint64_t(1) << (8 * (n - 8))) - 1;
    return v4u{uint32_t(lo), uint32_t(lo >> 32), uint32_t(hi), uint32_t(hi >> 32)};
}

// Header + close-status bytes of frame R (<= 16, as PrepareSendFrame writes
// them, the status masked like payload bytes 0-1: SURVEY Q2/Q3), zero past
// them; wave-uniform.
__device__ __forceinline__ v4u frame_head(const FrameRec& R)
{
    v4u h = {0, 0, 0, 0};
#pragma unroll 1
    for (uint32_t r = 0; r < R.hdr; ++r)
        put_byte(h, r, header_byte(R.opcode, R.mask, R.body, R.key, r));
    if (R.prefix) {
        put_byte(h, R.hdr, uint32_t((R.status >> 8) & 0xFF) ^ key_byte(R.key, 0));
        put_byte(h, R.hdr + 1, uint32_t(R.status & 0xFF) ^ key_byte(R.key, 1));
    }
    return h;
}

// edge_chunk built with 16-byte vector operations instead of a byte loop:
// the head shifted into place, the data window XORed with the rotated key
// under its byte mask; stored whole when every byte is this frame's, else
// by dwords (bytes only where a dword is shared with a neighbour).
__device__ __forceinline__ void edge_chunk2(const FrameRec& R, v4u head, uint64_t p, uint8_t* __restrict__ wire)
{
    if (p + CHUNK <= R.off)
        return;   // a chunk of the piece's line before the frame: a neighbour's
    v4u w = p >= R.off ? shr_bytes(head, p - R.off) : shl_bytes(head, R.off - p);
    const int64_t data_len = int64_t(R.end - R.data_w);
    const int64_t rel = int64_t(p) - int64_t(R.data_w);   // source offset of chunk byte 0
    if (rel < data_len && rel + int64_t(CHUNK) > 0) {
        const v4u d = fan_window(R.src, uint64_t(data_len), rel);
        const uint32_t kw = key_rot(R.key, uint32_t(p - R.pw));   // (mod 4 also when p < pw)
        const uint64_t lo = p < R.data_w ? R.data_w - p : 0;
        const uint64_t hi = R.end - p < CHUNK ? R.end - p : CHUNK;
        w |= (d ^ v4u{kw, kw, kw, kw}) & (low_bytes(hi) & ~low_bytes(lo));
    }
    const uint32_t o_lo = p < R.off ? uint32_t(R.off - p) : 0u;
    const uint32_t o_hi = R.end - p < CHUNK ? uint32_t(R.end - p) : uint32_t(CHUNK);
    if ((o_lo == 0 && o_hi == CHUNK) || (WSG_DIAG_ENC & 4)) {
        st16nt(wire + p, w);
        return;
    }
    uint32_t* w32 = reinterpret_cast<uint32_t*>(wire + p);
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t b0 = 4 * k, b1 = b0 + 4;
        if (b0 >= o_lo && b1 <= o_hi) {
            w32[k] = w[k];
        } else {
            for (uint32_t j = max(b0, o_lo); j < min(b1, o_hi); ++j)
                wire[p + j] = uint8_t(w[k] >> (8 * (j - b0)));
        }
    }
}

// One wave's piece k of frame R, in two phases so that a wave can keep two
// pieces' loads in flight before storing either (load(), then store()).
template <bool NT>
struct Piece {
    FrameRec R;
    uint64_t lo = 0, hi = 0;
    uint32_t s = 0;        // source misalignment, uniform over the piece
    uint32_t kw = 0;       // key rotated to the piece's phase (uniform)
    bool live = false;
    uint32_t dmask = 0;   // bit u: chunk u of this lane is all data (a bool array would land in LDS)
    v4u a[EU], b[EU];

    __device__ __forceinline__ void load(const FrameRec& rec, uint64_t k, bool exists)
    {
        R = rec;
        const uint32_t lane = threadIdx.x & 63;
        lo = (R.off & ~(PIECE_ALIGN - 1)) + k * PIECE;
        live = exists && lo < R.end;   // piece counts are an upper bound
        hi = min(lo + PIECE, R.end);
        // source of wire byte q: R.src + (q - R.data_w), as pointer
        // arithmetic on the payload argument (global_* loads; a uintptr_t
        // round trip made them flat loads, whose lgkmcnt share turned every
        // scalar-load wait of the descriptor pipeline into a data-load wait)
        s = (WSG_DIAG_ENC & 2) ? 0u
                                : uint32_t((reinterpret_cast<uintptr_t>(R.src) + (lo - R.data_w)) & 15u);
        kw = key_rot(R.key, uint32_t(lo - R.pw));
#pragma unroll
        for (int u = 0; u < EU; ++u) {
            const uint64_t p = lo + (uint64_t(u) * 64 + lane) * CHUNK;
            const bool d = live && p < hi && p >= R.data_w && p + CHUNK <= R.end;
            dmask |= uint32_t(d) << u;
            const uint8_t* a0 = R.src + (int64_t(p - R.data_w) - int64_t(s));
            a[u] = d ? (NT ? ld16nt(a0) : ld16(a0)) : v4u{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < EU; ++u) {
            const uint64_t p = lo + (uint64_t(u) * 64 + lane) * CHUNK;
            const uint8_t* a0 = R.src + (int64_t(p - R.data_w) - int64_t(s));
            b[u] = ((dmask >> u) & 1u) && s ? ((NT && WSG_ENC_NT_HI) ? ld16nt(a0 + CHUNK) : ld16(a0 + CHUNK))
                                          : v4u{0, 0, 0, 0};
        }
    }

    __device__ __forceinline__ void store(uint8_t* __restrict__ wire) const
    {
        if (!live)
            return;
        const uint32_t lane = threadIdx.x & 63;
        const OutTile ot(wire + lo, uint32_t(PIECE), WSG_ENC_SC1 != 0);
        v4u head = {0, 0, 0, 0};
        if (lo < R.data_w)   // (wave-uniform) the piece holds header / status bytes
            head = frame_head(R);
#pragma unroll
        for (int u = 0; u < EU; ++u) {
            const uint64_t p = lo + (uint64_t(u) * 64 + lane) * CHUNK;
            if ((dmask >> u) & 1u) {
                ot.put(uint32_t(p - lo), (s ? funnel(a[u], b[u], s) : a[u]) ^ kw);
            } else if (p < hi && !(WSG_DIAG_ENC & 1)) {
                // header / status bytes, or a chunk shared with a neighbour
                // (built as a vector: the byte-at-a-time build it replaced
                // made C3's encode 0.730 ms against 0.701, round 4)
                edge_chunk2(R, head, p, wire);
            }
        }
    }
};

__device__ __forceinline__ uint64_t pieces_of(uint64_t frame_bytes)
{
    return (frame_bytes + PIECE_ALIGN - 1 + PIECE - 1) / PIECE;
}

} // namespace

// Per-block local exclusive scans of frame sizes and piece counts
// (SCAN_ITEMS frames per block).  Round k of a block reads frames
// k * BLOCK + t, so consecutive lanes read consecutive descriptors (a lane
// reading SCAN_PER_LANE adjacent descriptors touched 64 lines per load
// instruction); the rounds scan in frame order, carrying the running sums.
// PIECES = false (small-frame path): no piece counts.
template <bool PIECES>
__global__ __launch_bounds__(BLOCK) void k_encode_scan_local(const wsg_send_desc* __restrict__ desc, uint32_t n,
                                                             uint64_t* __restrict__ wire_off,
                                                             uint32_t* __restrict__ piece_start,
                                                             uint64_t* __restrict__ block_sums,
                                                             uint64_t* __restrict__ block_psums)
{
    const uint64_t first = uint64_t(blockIdx.x) * SCAN_ITEMS;
    uint64_t sz[SCAN_PER_LANE];
#pragma unroll
    for (int k = 0; k < SCAN_PER_LANE; ++k) {   // all descriptor loads first
        const uint64_t i = first + uint64_t(k) * BLOCK + threadIdx.x;
        sz[k] = 0;
        if (i < n) {
            const Desc d = load_desc(desc + i);
            const SendGeom g = send_geom(d.opcode, d.mask, d.len, d.status);
            sz[k] = g.hdr + g.body;
        }
    }
    uint64_t run = 0, run_p = 0;
#pragma unroll
    for (int k = 0; k < SCAN_PER_LANE; ++k) {
        const uint64_t i = first + uint64_t(k) * BLOCK + threadIdx.x;
        uint64_t tot, tot_p = 0;
        const uint64_t ex = block_exclusive_scan(sz[k], &tot);
        uint64_t ex_p = 0;
        if (PIECES)
            ex_p = block_exclusive_scan(sz[k] ? pieces_of(sz[k]) : 0, &tot_p);
        if (i < n) {
            wire_off[i] = run + ex;
            if (PIECES)
                piece_start[i] = uint32_t(run_p + ex_p);
        }
        run += tot;
        run_p += tot_p;
    }
    if (threadIdx.x == 0) {
        block_sums[blockIdx.x] = run;
        if (PIECES)
            block_psums[blockIdx.x] = run_p;
    }
}

// Single block: exclusive scans of the block sums; wire_off[n] = total bytes,
// piece_start[n] = total pieces.
__global__ __launch_bounds__(BLOCK) void k_encode_scan_blocks(const uint64_t* __restrict__ block_sums,
                                                              const uint64_t* __restrict__ block_psums, uint32_t nb,
                                                              uint64_t* __restrict__ block_prefix,
                                                              uint64_t* __restrict__ block_pprefix,
                                                              uint64_t* __restrict__ wire_off,
                                                              uint32_t* __restrict__ piece_start, uint32_t n)
{
    uint64_t carry = 0, carry_p = 0;
    for (uint32_t c = 0; c < nb; c += BLOCK) {
        const uint32_t i = c + threadIdx.x;
        uint64_t tot, tot_p;
        const uint64_t ex = block_exclusive_scan(i < nb ? block_sums[i] : 0, &tot);
        const uint64_t ex_p = block_exclusive_scan(i < nb ? block_psums[i] : 0, &tot_p);
        if (i < nb) {
            block_prefix[i] = carry + ex;
            block_pprefix[i] = carry_p + ex_p;
        }
        carry += tot;
        carry_p += tot_p;
    }
    if (threadIdx.x == 0) {
        wire_off[n] = carry;
        piece_start[n] = uint32_t(carry_p);
    }
}

// Add block prefixes, build the piece -> frame map, check capacity.
__global__ __launch_bounds__(BLOCK) void k_encode_finalize(const wsg_send_desc* __restrict__ desc, uint32_t n,
                                                           uint64_t* __restrict__ wire_off,
                                                           uint32_t* __restrict__ piece_start,
                                                           const uint64_t* __restrict__ block_prefix,
                                                           const uint64_t* __restrict__ block_pprefix,
                                                           uint32_t* __restrict__ piece_frame, uint64_t pieces_cap,
                                                           uint64_t wire_cap, unsigned long long* err)
{
    if (blockIdx.x * BLOCK + (threadIdx.x & ~63u) >= n)
        return;   // whole wave past the last frame
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    uint64_t lo = 0, hi = 0;
    if (i < n) {
        const wsg_send_desc d = desc[i];
        const SendGeom g = send_geom(d.opcode, d.mask != 0, d.len, d.status);
        const uint64_t off = wire_off[i] + block_prefix[i / SCAN_ITEMS];
        const uint64_t ps = piece_start[i] + block_pprefix[i / SCAN_ITEMS];
        const uint64_t end = off + g.hdr + g.body;
        wire_off[i] = off;
        piece_start[i] = uint32_t(ps);
        if (end > wire_cap)
            atomicMin(err, (static_cast<unsigned long long>(i) << 8) |
                               static_cast<unsigned long long>(-WSG_ENOMEM));
        lo = min(ps, pieces_cap);
        hi = min(ps + pieces_of(g.hdr + g.body), pieces_cap);
    }
    fill_tiles_wave(piece_frame, lo, hi, i);
}

__global__ __launch_bounds__(BLOCK) void k_encode_mask(const uint8_t* __restrict__ payload,
                                                       const wsg_send_desc* __restrict__ desc, uint32_t n,
                                                       const uint64_t* __restrict__ wire_off,
                                                       const uint32_t* __restrict__ piece_start,
                                                       const uint32_t* __restrict__ piece_frame,
                                                       uint8_t* __restrict__ wire, uint64_t wire_cap,
                                                       uint32_t q_begin, uint32_t q_end)
{
    const uint32_t waves = gridDim.x * (BLOCK / 64);
    uint32_t q = q_begin + blockIdx.x * (BLOCK / 64) + wave_id();
    if (wire_off[n] > wire_cap)
        return;   // capacity error latched by k_encode_finalize
    const uint32_t pieces = min(piece_start[n], q_end);   // this launch's pieces: [q_begin, min(all pieces, q_end))
    // Software pipeline over the wave's pieces: while piece q streams, the
    // descriptor of piece q + W (frame index already known) and the frame
    // index of piece q + 2W are in flight, so the dependent metadata loads
    // never sit between a piece's data loads and the previous piece's stores.
    struct Meta {
        Desc d;
        uint64_t off;
        uint32_t ps;
    };
    auto meta = [&](uint32_t i) { return Meta{load_desc(desc + i), wire_off[i], piece_start[i]}; };
    if (q >= pieces)
        return;
    Meta cur = meta(piece_frame[q]);
    uint32_t i_next = (q + waves < pieces) ? piece_frame[q + waves] : 0;
    for (;;) {
        Piece<WSG_ENC_NT_SRC != 0> pc;
        pc.load(make_rec(cur.off, payload + cur.d.src_off, cur.d.len, cur.d.key, cur.d.status, cur.d.opcode,
                         cur.d.mask),
                q - cur.ps, true);
        const uint32_t qn = q + waves;
        const bool more = qn < pieces;
        Meta nxt = cur;
        uint32_t i_after = 0;
        if (more) {
            nxt = meta(i_next);
            i_after = (qn + waves < pieces) ? piece_frame[qn + waves] : 0;
        }
        pc.store(wire);
        if (!more)
            break;
        cur = nxt;
        i_next = i_after;
        q = qn;
    }
}

// Fan-out, flat kernel (frame sizes the period path does not take): the k frames are one byte stream of k * fsize bytes, cut into
// 16-byte chunks; every lane builds whole chunks (both frames' bytes where a
// frame boundary falls inside one), so every store is a full 16-B store and
// no cache line is written in parts by two waves.  The frame of a chunk is
// p / fsize (a double-precision reciprocal, corrected by one).
constexpr int FU = FAN_UNITS;

__device__ __forceinline__ uint32_t fan_byte(const uint8_t* __restrict__ payload, const uint32_t* __restrict__ keys,
                                             uint8_t opcode, bool mask, const SendGeom& g, uint64_t fsize, uint64_t i,
                                             uint64_t r)
{
    const uint32_t key = keys[i];
    if (r < g.hdr)
        return header_byte(opcode, mask, g.body, key, uint32_t(r));
    const uint64_t k = r - g.hdr;
    if (k < g.prefix)
        return key_byte(key, k);   // status 0: both prefix bytes are 0
    return uint32_t(payload[k - g.prefix]) ^ key_byte(key, k);
}


// Frames of one fan-out differ only in their key: the header + status bytes
// (data0 <= 16 of them) are a constant vector plus the key bytes.
struct FanGeom {
    SendGeom g;
    uint32_t data0;   // frame offset of the first payload byte (<= 16)
    uint32_t kpos;    // frame offset of the mask key (2 + ext)
    bool mask;
    v4u hp0;          // header with the key bytes left 0; status bytes 0
};

__device__ __forceinline__ FanGeom fan_geom(uint8_t opcode, bool mask, uint64_t len)
{
    FanGeom f;
    f.g = send_geom(opcode, mask, len, 0);
    f.data0 = f.g.hdr + f.g.prefix;
    f.kpos = f.g.hdr - (mask ? 4u : 0u);
    f.mask = mask;
    f.hp0 = v4u{0, 0, 0, 0};
#pragma unroll 1
    for (uint32_t r = 0; r < f.kpos; ++r)
        put_byte(f.hp0, r, header_byte(opcode, mask, f.g.body, 0, r));
    return f;
}

// Bytes [o, o + 16) of the frame with key `key` (bytes past the frame are 0).
__device__ __forceinline__ v4u fan_frame_bytes(const uint8_t* __restrict__ payload, uint64_t len, const FanGeom& f,
                                               uint64_t fsize, uint32_t key, uint64_t o)
{
    v4u hp = f.hp0;
    if (f.mask)
        hp |= shl_bytes(v4u{key, 0, 0, 0}, f.kpos);
    if (f.g.prefix)
        hp |= shl_bytes(v4u{key & 0xFFFFu, 0, 0, 0}, f.g.hdr);   // status 0 ^ key
    v4u out = shr_bytes(hp, o);
    const uint64_t lo = o < f.data0 ? f.data0 - o : 0;               // chunk bytes [lo, hi) are payload
    const uint64_t hi = fsize - o < CHUNK ? fsize - o : CHUNK;
    if (lo < hi) {
        const v4u w = fan_window(payload, len, int64_t(o) - int64_t(f.data0));
        const v4u m = low_bytes(hi) & ~low_bytes(lo);
        out |= (w ^ key_rot(key, uint32_t(o - f.g.hdr))) & m;
    }
    return out;
}

// ---- batch encode of small frames -----------------------------------------
// The piece kernel spends one wave pass per frame whatever its size, so a
// batch of frames a few dozen bytes long (the reference's 32-byte echo
// messages) leaves most lanes idle.  Here a block owns fpb <= SMALL_F
// consecutive frames (about SMALL_RANGE wire bytes at the batch's average
// frame size), i.e. one contiguous wire range, and its lanes own the 16-B chunks
// of that range.  A chunk is ORed together from the frames it overlaps: each
// frame's head (header + close-status bytes, <= 16, built once per frame into
// LDS) shifted into place, plus its masked payload window.  The chunks at the
// two ends of the range, shared with the neighbouring blocks, get byte stores
// of this block's bytes only.  Correct for any sizes; the host picks it when
// the average frame is small (SMALL_AVG).
static_assert(SMALL_F <= BLOCK && SCAN_ITEMS % SMALL_F == 0, "k_encode_small: one frame per lane, one scan block");

struct SmallFrame {
    uint64_t src;   // offset of the first data byte in the payload arena (an
                    // offset, not an address: loads through a pointer rebuilt
                    // from an integer are flat loads)
    uint32_t key;
    uint32_t geo;   // head bytes (header + status) | header bytes << 8
};

// Bytes [o, o + 16) of a frame of fsize bytes (o < fsize), 0 past its end.
template <class Blocks = GlobalBlocks>
__device__ __forceinline__ v4u small_bytes(const uint8_t* __restrict__ payload, v4u head, const SmallFrame& f,
                                          uint64_t fsize, uint64_t o, Blocks blk = Blocks{})
{
    const uint32_t data0 = f.geo & 0xFFu, hdr = f.geo >> 8;
    v4u out = shr_bytes(head, o);
    const uint64_t lo = o < data0 ? data0 - o : 0;   // chunk bytes [lo, hi) are payload
    const uint64_t hi = fsize - o < CHUNK ? fsize - o : CHUNK;
    if (lo < hi) {
        const v4u w = fan_window(payload + f.src, fsize - data0, int64_t(o) - int64_t(data0), blk);
        out |= (w ^ key_rot(f.key, uint32_t(o - hdr))) & (low_bytes(hi) & ~low_bytes(lo));
    }
    return out;
}

// A frame's head (header bytes + close status, <= 16 bytes: SURVEY Q2/Q3)
// and record for the chunk builder; returns the frame's size.
__device__ __forceinline__ uint64_t small_head(const Desc& d, v4u& h, SmallFrame& fr)
{
    const SendGeom g = send_geom(d.opcode, d.mask, d.len, d.status);
    h = v4u{0, 0, 0, 0};
#pragma unroll 1
    for (uint32_t r = 0; r < g.hdr; ++r)
        put_byte(h, r, header_byte(d.opcode, d.mask, g.body, d.key, r));
    if (g.prefix) {   // close status, big-endian, masked like payload bytes 0-1
        put_byte(h, g.hdr, uint32_t((d.status >> 8) & 0xFF) ^ key_byte(d.key, 0));
        put_byte(h, g.hdr + 1, uint32_t(d.status & 0xFF) ^ key_byte(d.key, 1));
    }
    fr = SmallFrame{d.src_off, d.key, (g.hdr + g.prefix) | (g.hdr << 8)};
    return g.hdr + g.body;
}

// The 16-B chunks of a group's wire range [s_off[0], s_off[cnt]) (frames
// 0..cnt-1 of the group, LDS: offsets, heads, records), lanes t, t + nt, ...:
// each chunk ORs together the frames it overlaps; only the range's first and
// last chunk, shared with the neighbouring groups, get byte stores.
template <class Blocks = GlobalBlocks>
__device__ __forceinline__ void small_chunks(const uint8_t* __restrict__ payload, const uint64_t* s_off,
                                             const v4u* s_head, const SmallFrame* s_fr, uint32_t cnt,
                                             uint8_t* __restrict__ wire, uint32_t t, uint32_t nt,
                                             Blocks blk = Blocks{})
{
    const uint64_t r_lo = s_off[0], r_hi = s_off[cnt];
    for (uint64_t p = (r_lo & ~uint64_t(CHUNK - 1)) + uint64_t(t) * CHUNK; p < r_hi; p += uint64_t(nt) * CHUNK) {
        uint32_t a = 0, b = cnt - 1;   // last frame starting at or before p (frame 0 before the range)
        while (a < b) {
            const uint32_t m = (a + b + 1) >> 1;
            if (s_off[m] <= p)
                a = m;
            else
                b = m - 1;
        }
        v4u w = {0, 0, 0, 0};
        for (uint32_t j = a; j < cnt; ++j) {
            const uint64_t off = s_off[j];
            if (off >= p + CHUNK)
                break;
            const uint64_t fsize = s_off[j + 1] - off;
            if (p >= off)
                w |= small_bytes(payload, s_head[j], s_fr[j], fsize, p - off, blk);
            else
                w |= shl_bytes(small_bytes(payload, s_head[j], s_fr[j], fsize, 0, blk), off - p);
        }
        if (p >= r_lo && p + CHUNK <= r_hi) {
            st16nt(wire + p, w);
        } else {
            const uint32_t j0 = p < r_lo ? uint32_t(r_lo - p) : 0;
            const uint32_t j1 = r_hi - p < CHUNK ? uint32_t(r_hi - p) : CHUNK;
            for (uint32_t j = j0; j < j1; ++j)
                wire[p + j] = uint8_t(lane_byte(w, j));
        }
    }
}

// Also finishes the offsets scan (k_encode_scan_blocks and
// k_encode_finalize for the piece path): wire_off holds the block-local
// offsets of k_encode_scan_local<false>, block_sums its nb block totals; a
// block's frames share one scan block (fpb divides SCAN_ITEMS), whose prefix
// the block sums from the L2-resident totals itself.
__global__ __launch_bounds__(BLOCK) void k_encode_small(const uint8_t* __restrict__ payload,
                                                        const wsg_send_desc* __restrict__ desc, uint32_t n,
                                                        uint32_t fpb, uint64_t* __restrict__ wire_off,
                                                        const uint64_t* __restrict__ block_sums, uint32_t nb,
                                                        uint8_t* __restrict__ wire, uint64_t wire_cap,
                                                        unsigned long long* err)
{
    __shared__ uint64_t s_off[SMALL_F + 1];
    __shared__ v4u s_head[SMALL_F];
    __shared__ SmallFrame s_fr[SMALL_F];
    const uint32_t f_lo = blockIdx.x * fpb;   // fpb <= SMALL_F (host)
    if (f_lo >= n)
        return;
    const uint32_t sb = f_lo / uint32_t(SCAN_ITEMS);
    const uint32_t cnt = min(n - f_lo, fpb);
    const uint32_t t = threadIdx.x;   // frame f_lo + t (cnt <= BLOCK)
    // every load first (scan-block totals, descriptor, local offset), so that
    // their round trips overlap
    constexpr int PB = 4;   // totals per lane in one go (1 Mi frames); more in the loop below
    uint64_t bs[PB];
#pragma unroll
    for (int u = 0; u < PB; ++u) {
        const uint32_t k = t + uint32_t(u) * BLOCK;
        bs[u] = k < nb ? block_sums[k] : 0;
    }
    Desc d{};
    uint64_t off_local = 0;
    if (t < cnt) {
        d = load_desc(desc + f_lo + t);
        off_local = wire_off[f_lo + t];
    }
    uint64_t sz = 0;
    if (t < cnt)
        sz = small_head(d, s_head[t], s_fr[t]);
    uint64_t before = 0, all = 0;
#pragma unroll
    for (int u = 0; u < PB; ++u) {
        all += bs[u];
        before += t + uint32_t(u) * BLOCK < sb ? bs[u] : 0;
    }
    for (uint32_t k = t + PB * BLOCK; k < nb; k += BLOCK) {
        const uint64_t v = block_sums[k];
        all += v;
        before += k < sb ? v : 0;
    }
    uint64_t prefix, total;
    (void)block_exclusive_scan(before, &prefix);
    (void)block_exclusive_scan(all, &total);
    if (blockIdx.x == 0 && t == 0)
        wire_off[n] = total;
    const bool over = total > wire_cap;
    if (t < cnt) {
        const uint32_t i = f_lo + t;
        const uint64_t off = off_local + prefix;
        const uint64_t end = off + sz;
        wire_off[i] = off;
        s_off[t] = off;
        if (t + 1 == cnt)
            s_off[cnt] = end;   // not from wire_off[i + 1]: the next block may have finalized it already
        if (end > wire_cap)
            atomicMin(err, (static_cast<unsigned long long>(i) << 8) |
                               static_cast<unsigned long long>(-WSG_ENOMEM));
    }
    __syncthreads();
    if (over)
        return;   // offsets are final and the error latched; no frame bytes
    small_chunks(payload, s_off, s_head, s_fr, cnt, wire, threadIdx.x, BLOCK);
}

// ---- the host lane (wsg_internal.h) ----------------------------------------

// The lane reads its host inputs in whole, coalesced 16-byte blocks into
// LDS, every load of a step issued before any is waited for: one workgroup
// has few requests in flight, and each PCIe round trip costs microseconds
// (a lane-per-frame read of 32-byte descriptors or headers scattered over
// lines took several; one block per lane per round trip, three for an
// echo's read, $WSG_LANE_PROFILE).  `U` blocks per lane at most.
template <int U>
struct LaneLoads {
    v4u v[U];
    __device__ __forceinline__ void load(const uint8_t* __restrict__ src, uint64_t blocks, bool on)
    {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t k = threadIdx.x + uint64_t(u) * LANE_THREADS;
            if (on && k < blocks)
                v[u] = ld16(src + k * CHUNK);
        }
    }
    __device__ __forceinline__ void store(v4u* dst, uint64_t blocks, bool on) const
    {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t k = threadIdx.x + uint64_t(u) * LANE_THREADS;
            if (on && k < blocks)
                dst[k] = v[u];
        }
    }
};

// Encode of one frame group on the lane (frames [f_lo, f_lo + cnt)): its
// offsets and descriptors — and its frames' payload span [plo, phi) when that
// span's 16-B blocks fit LANE_PSTAGE — staged in one round trip, a lane per
// frame builds its head (small_head), then the group's chunks (small_chunks,
// payload windows from LDS): the bytes k_encode_small writes, at the host's
// offsets.  The range's first and last chunk, shared with the neighbouring
// groups (other workgroups), get byte stores.
__device__ __forceinline__ void lane_encode(const uint8_t* __restrict__ payload, uint64_t plo, uint64_t phi,
                                            const wsg_send_desc* __restrict__ desc, uint32_t f_lo, uint32_t cnt,
                                            const uint64_t* __restrict__ wire_off, uint8_t* __restrict__ wire,
                                            uint8_t* lds)
{
    uint64_t* s_off = reinterpret_cast<uint64_t*>(lds);                             // LANE_THREADS + 1 (+1 pad)
    v4u* s_head = reinterpret_cast<v4u*>(lds + 8 * (LANE_THREADS + 2));
    SmallFrame* s_fr = reinterpret_cast<SmallFrame*>(s_head + LANE_THREADS);
    v4u* s_desc = reinterpret_cast<v4u*>(s_fr + LANE_THREADS);                       // 2 blocks per descriptor
    v4u* s_pay = s_desc + 2 * LANE_THREADS;                                          // LANE_PSTAGE
    static_assert(sizeof(wsg_send_desc) == 32 && sizeof(SmallFrame) == 16, "lane LDS layout");
    static_assert(8 * (LANE_THREADS + 2) + 64 * LANE_THREADS + LANE_PSTAGE <= LANE_LDS, "lane LDS layout");
    const uint32_t t = threadIdx.x;
    // the span's aligned blocks (payload + plo rounded down)
    const uint8_t* p0 = payload + plo;
    p0 -= reinterpret_cast<uintptr_t>(p0) & (CHUNK - 1);
    const uint64_t pblocks = phi > plo ? (uint64_t(payload + phi - p0) + CHUNK - 1) / CHUNK : 0;
    const bool staged = pblocks <= LANE_PSTAGE / CHUNK;
    uint64_t off = 0, off_end = 0;
    if (t < cnt)
        off = wire_off[f_lo + t];
    if (t + 1 == cnt)
        off_end = wire_off[f_lo + cnt];
    LaneLoads<2> dl;
    dl.load(reinterpret_cast<const uint8_t*>(desc + f_lo), 2 * uint64_t(cnt), true);
    LaneLoads<LANE_PSTAGE / CHUNK / LANE_THREADS> pl;
    pl.load(p0, pblocks, staged);
    if (t < cnt)
        s_off[t] = off;
    if (t + 1 == cnt)
        s_off[cnt] = off_end;
    dl.store(s_desc, 2 * uint64_t(cnt), true);
    pl.store(s_pay, pblocks, staged);
    __syncthreads();
    if (t < cnt) {
        const Desc d = load_desc(reinterpret_cast<const wsg_send_desc*>(s_desc) + t);
        (void)small_head(d, s_head[t], s_fr[t]);
    }
    __syncthreads();
    if (staged)
        small_chunks(payload, s_off, s_head, s_fr, cnt, wire, t, LANE_THREADS, StagedBlocks{s_pay, p0});
    else
        small_chunks(payload, s_off, s_head, s_fr, cnt, wire, t, LANE_THREADS);
}

// Decode of one frame group on the lane (frame table strictly increasing,
// the group's range at most LANE_STAGE - 64 bytes): the group's frame starts and its
// wire range [lo, hi) — from its first frame's start (0 for the first group)
// to the next group's (wire_len for the last) — plus the 32 bytes a header
// read may look past hi, staged in one round trip; a lane per frame parses
// it (frame_parse_b: k_decode's rules) into LDS, the group's wsg_recv_info go
// out in whole blocks; then the range chunk by chunk: the wire bytes, the
// valid frames' payload bytes XORed with their keys.  Out-of-range and error
// frames' bytes are copied, as k_decode does.  (In place, a header that runs
// past hi — a table breaking the no-overlap contract — may read bytes the
// next group's workgroup has already unmasked, as k_decode's blocks may.)
__device__ __forceinline__ void lane_decode(const uint8_t* __restrict__ wire, uint64_t wire_len, uint64_t lo,
                                            uint64_t hi, const uint64_t* __restrict__ fs, uint32_t n, uint32_t f_lo,
                                            uint32_t cnt, uint8_t* out, wsg_recv_info* __restrict__ info,
                                            uint8_t* lds, uint32_t* s_err)
{
    v4u* s_wire = reinterpret_cast<v4u*>(lds);
    v4u* s_info = reinterpret_cast<v4u*>(lds + LANE_STAGE);                          // 2 blocks per record
    uint64_t* s_pl = reinterpret_cast<uint64_t*>(s_info + 2 * LANE_THREADS);
    uint64_t* s_pe = s_pl + LANE_THREADS;
    uint32_t* s_key = reinterpret_cast<uint32_t*>(s_pe + LANE_THREADS);
    uint64_t* s_fs = reinterpret_cast<uint64_t*>(s_key + LANE_THREADS);               // the group's starts + next
    static_assert(sizeof(wsg_recv_info) == 32, "lane LDS layout");
    static_assert(LANE_STAGE + 60 * LANE_THREADS + 8 <= LANE_LDS, "lane LDS layout");
    const uint32_t t = threadIdx.x;
    const uint64_t sb = lo & ~uint64_t(CHUNK - 1);
    const uint64_t se = min(hi + 32, wire_len);
    const uint64_t wblocks = se > sb ? (se - sb + CHUNK - 1) / CHUNK : 0;   // <= LANE_STAGE / CHUNK (host's groups)
    const auto block = [s_wire, sb](uint64_t a) { return s_wire[(a - sb) / CHUNK]; };
    uint64_t st = 0, nx = wire_len;
    if (t < cnt)
        st = fs[f_lo + t];
    if (t + 1 == cnt && f_lo + cnt < n)
        nx = fs[f_lo + cnt];
    LaneLoads<LANE_STAGE / CHUNK / LANE_THREADS> wl;
    wl.load(wire + sb, wblocks, true);
    if (t < cnt)
        s_fs[t] = st;
    if (t + 1 == cnt)
        s_fs[cnt] = nx;
    wl.store(s_wire, wblocks, true);
    __syncthreads();
    if (t < cnt) {
        const uint64_t st = s_fs[t];
        const uint64_t limit = s_fs[t + 1];   // the next frame's start, wire_len after the last
        wsg_recv_info r;
        const int e = frame_parse_b(block, wire_len, st, limit, r);
        store_info(reinterpret_cast<wsg_recv_info*>(s_info) + t, r);
        const uint64_t pl = e ? st : r.payload_off;
        s_pl[t] = pl;
        s_pe[t] = e ? st : pl + r.len;
        s_key[t] = (e == 0 && r.masked) ? r.key : 0u;
        if (e)
            atomicAdd(s_err, 1u);   // (the host skips its status pass over the records when no frame erred)
    }
    __syncthreads();
    {
        v4u* dst = reinterpret_cast<v4u*>(info + f_lo);
        for (uint32_t k = t; k < 2 * cnt; k += LANE_THREADS)
            dst[k] = s_info[k];
    }
    for (uint64_t p = sb + uint64_t(t) * CHUNK; p < hi; p += uint64_t(LANE_THREADS) * CHUNK) {
        const v4u wv = s_wire[(p - sb) / CHUNK];
        // last frame whose payload starts at or before p (frame 0 if none)
        uint32_t a = 0, b = cnt - 1;
        while (a < b) {
            const uint32_t m = (a + b + 1) >> 1;
            if (s_pl[m] <= p)
                a = m;
            else
                b = m - 1;
        }
        v4u m = {0, 0, 0, 0};
        for (uint32_t j = a; j < cnt; ++j) {
            const uint64_t pl = s_pl[j], pe = s_pe[j];
            if (pl >= p + CHUNK)
                break;
            const uint32_t key = s_key[j];
            if (key == 0 || pe <= p)
                continue;
            if (pl <= p && pe >= p + CHUNK) {   // the chunk lies in this payload
                const uint32_t kw = key_rot(key, uint32_t(p - pl));
                m ^= v4u{kw, kw, kw, kw};
            } else {   // the payload's bytes of the chunk: [max(pl, p), min(pe, p + 16))
                const uint32_t kw = key_rot(key, uint32_t(p - pl));   // (mod 4 also when p < pl)
                const uint64_t b0 = pl > p ? pl - p : 0, b1 = pe - p < CHUNK ? pe - p : CHUNK;
                m ^= v4u{kw, kw, kw, kw} & (low_bytes(b1) & ~low_bytes(b0));
            }
        }
        const v4u w = wv ^ m;
        if (p >= lo && p + CHUNK <= hi) {
            st16nt(out + p, w);
        } else {
            const uint32_t j0 = p < lo ? uint32_t(lo - p) : 0;
            const uint32_t j1 = hi - p < CHUNK ? uint32_t(hi - p) : CHUNK;
            for (uint32_t j = j0; j < j1; ++j)
                out[p + j] = uint8_t(lane_byte(w, j));
        }
    }
}

// Per-call XOR on the lane: the page-locked buffer [buf, buf + len) XORed in
// place, byte i with key byte (phase + i) % 4 (len <= LANE_PSTAGE, buf 16-B
// aligned: the context's stage); every load issued before any is waited for.
__device__ __forceinline__ void lane_xor(uint8_t* buf, uint64_t len, uint32_t key, uint32_t phase)
{
    const uint32_t t = threadIdx.x;
    const uint64_t chunks = len / CHUNK, tail = len & (CHUNK - 1);
    LaneLoads<LANE_PSTAGE / CHUNK / LANE_THREADS> v;
    v.load(buf, chunks, true);
    const uint64_t q = chunks * CHUNK + t;
    const uint32_t tb = t < tail ? uint32_t(buf[q]) : 0u;
    const uint32_t kw = key_rot(key, phase);
#pragma unroll
    for (int u = 0; u < int(LANE_PSTAGE / CHUNK / LANE_THREADS); ++u) {
        const uint64_t k = t + uint64_t(u) * LANE_THREADS;
        if (k < chunks)
            *reinterpret_cast<v4u*>(buf + k * CHUNK) = v.v[u] ^ kw;
    }
    if (t < tail)
        buf[q] = uint8_t(tb ^ key_byte(key, uint32_t(phase + q)));
}

// The lane: W = gridDim.x workgroups, workgroup g serving its mailbox
// (bell->box[g]: the tickets g, g + W, g + 2W, ... in order).  Wave 0 polls
// the next slot's units and the control word, all in one round trip; a
// `stop` there means no task is taken (a request the host gave up on: it
// waits for the lane to leave before it uses the buffers itself).  The workgroups
// never wait on each other: each stages, works and answers alone, so one
// request's PCIe reads and writes spread over as many CUs as it has groups
// (one CU has few requests in flight: one workgroup took ~5 us to stage a 38
// KB read and ~7 us to write it back, round 4).
// The lane's workgroups on the XCDs nearest the PCIe root: block b runs on
// XCC b mod 8 (round-robin dispatch), and a poller on XCCs 0-3 reaches
// page-locked host memory ~0.2 us sooner per round trip than one on 4-7
// (tools/xcd_probe.hip).  Blocks on the other XCCs leave at once; workgroup g
// of the lane is block (g / LANE_NEAR_XCCS) * 8 + g % LANE_NEAR_XCCS.
constexpr uint32_t LANE_XCCS = 8, LANE_NEAR_XCCS = 4;

__global__ __launch_bounds__(LANE_THREADS) void k_lane(LaneBell* __restrict__ bell, uint32_t W, uint64_t idle_ticks,
                                                       uint64_t yield_ticks, uint32_t gen, uint64_t delay_ticks)
{
    __shared__ uint64_t s_w[LANE_WORDS];
    __shared__ int s_go;         // 1: a task in s_w; 0: leave
    __shared__ uint32_t s_err;   // the task's frames with an error (decode)
    __shared__ v4u s_mem[LANE_LDS / 16];   // the op's staging (lane_decode / lane_encode layouts)
    const uint32_t t = threadIdx.x;
    const uint32_t x = blockIdx.x % LANE_XCCS, g = blockIdx.x / LANE_XCCS * LANE_NEAR_XCCS + x;
    if (x >= LANE_NEAR_XCCS || g >= W)
        return;   // (a block-uniform exit before any barrier or memory access)
    uint64_t j = 0;     // (wave 0) this workgroup's mailbox position: ticket g + j W
    uint32_t why = 0;   // (wave 0) why it leaves: 1 idle or yield (announced in `closing`), 2 stop, 3 closing seen
    const LaneTask* box = bell->box[g];
    const uint64_t t_start = wall_clock64();
    if (t < 64) {
        if (delay_ticks) {   // test hook: a lane that starts late (bounded: ~2^20 sleeps)
            for (uint32_t i = 0; i < (1u << 20) && wall_clock64() - t_start < delay_ticks; ++i)
                __builtin_amdgcn_s_sleep(64);
        }
        j = uni(__hip_atomic_load(&bell->next_j[g], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    }
    for (;;) {
        if (t < 64) {
            const uint64_t want = uint64_t(g) + j * W + 1;
            const LaneTask* task = &box[j % LANE_RING];
            int go = 0;
            if (wall_clock64() - t_start > yield_ticks)
                why = 1;   // running long enough: step aside (calls that wait for the device to drain)
            const uint64_t t0 = wall_clock64();
            // every poll reads all of the slot's units and the control word in
            // one round trip (lanes 0..LANE_WORDS): a task is taken the moment
            // its first unit shows, with no second read.  (A unit still
            // holding the slot's previous task — the reads may be served in
            // any order — is read again; the control word read with a task's
            // first unit: a `stop` set after it is covered by the host, which
            // waits for the lane to leave before it touches the buffers.)
            const void* src = t < LANE_WORDS ? static_cast<const void*>(&task->w[t])
                                             : t == LANE_WORDS ? static_cast<const void*>(&bell->ctl) : nullptr;
            uint64_t val = 0;
            // at most ~2^22 polls of >= 1 us each: ends even if the clock stalls
            for (uint32_t it = 0; !why && it < (1u << 22); ++it) {
                const v4u u = src ? ld16_sys(src) : v4u{0, 0, 0, 0};
                val = uint64_t(u.x) | (uint64_t(u.y) << 32);
                const uint64_t tag = uint64_t(u.z) | (uint64_t(u.w) << 32);
                const uint32_t stop = __builtin_amdgcn_readlane(u.x, LANE_WORDS);
                const uint32_t closing = __builtin_amdgcn_readlane(u.y, LANE_WORDS);
                if (stop) {
                    why = 2;   // given up on by the host (or teardown): no task taken
                    break;
                }
                if (closing == gen) {
                    why = 3;   // another workgroup of this launch left: follow
                    break;
                }
                // (through uint32_t: readlane returns int, and a tag whose low
                // word is 2^31 or more must not sign-extend — every ticket from
                // 2^31 - 1 on would never be taken)
                const uint64_t tag0 = uint64_t(uint32_t(__builtin_amdgcn_readlane(u.z, 0))) |
                                      (uint64_t(uint32_t(__builtin_amdgcn_readlane(u.w, 0))) << 32);
                if (tag0 == want) {
                    if (__ballot(t < LANE_WORDS && tag != want) == 0) {
                        go = 1;
                        break;
                    }
                    continue;   // (part of the slot still the old task: again, at once)
                }
                if ((it & 15) == 15) {
                    const uint64_t now = wall_clock64();
                    if (now - t0 > idle_ticks || now - t_start > yield_ticks)
                        why = 1;
                }
                if (it < 1024)
                    __builtin_amdgcn_s_sleep(1);
                else
                    __builtin_amdgcn_s_sleep(8);   // idle for a while: poll host memory less often
            }
            if (!go && !why)
                why = 1;
            if (go) {
                __atomic_thread_fence(__ATOMIC_ACQUIRE);   // (system scope: the task's host buffers)
                if (t < LANE_WORDS)
                    s_w[t] = val;
            }
            if (t == 0) {
                s_go = go;
                s_err = 0;
            }
        }
        __syncthreads();
        if (!s_go)
            break;
        const uint32_t op = uint32_t(s_w[0]);
        const uint32_t n = uint32_t(s_w[0] >> 32);
        const uint32_t f_lo = uint32_t(s_w[6]), cnt = uint32_t(s_w[6] >> 32);
        uint8_t* lds = reinterpret_cast<uint8_t*>(s_mem);
        if (op == LANE_DECODE && cnt >= 1 && cnt <= LANE_THREADS)
            lane_decode(reinterpret_cast<const uint8_t*>(s_w[1]), s_w[2], s_w[7], s_w[8],
                        reinterpret_cast<const uint64_t*>(s_w[3]), n, f_lo, cnt, reinterpret_cast<uint8_t*>(s_w[4]),
                        reinterpret_cast<wsg_recv_info*>(s_w[5]), lds, &s_err);
        else if (op == LANE_ENCODE && cnt >= 1 && cnt <= LANE_THREADS)
            lane_encode(reinterpret_cast<const uint8_t*>(s_w[1]), s_w[7], s_w[8],
                        reinterpret_cast<const wsg_send_desc*>(s_w[2]), f_lo, cnt,
                        reinterpret_cast<const uint64_t*>(s_w[3]), reinterpret_cast<uint8_t*>(s_w[4]), lds);
        else if (op == LANE_XOR && s_w[2] <= LANE_PSTAGE)
            lane_xor(reinterpret_cast<uint8_t*>(s_w[1]), s_w[2], uint32_t(s_w[3]), uint32_t(s_w[3] >> 32));
        else if (op == LANE_XOR_INLINE) {
            // the payload came with the task (w[4..8]) and the answer goes
            // back as self-tagged units (LaneXres): one dword per lane, one
            // 8-byte store each, no read of host memory and no fence
            if (s_w[2] <= LANE_INLINE && t < (s_w[2] + 3) / 4) {
                const uint32_t d = uint32_t(s_w[4 + t / 2] >> (32 * (t & 1)));
                const uint32_t tag = uint32_t(uint64_t(g) + j * W + 1);
                const uint64_t unit = uint64_t(d ^ key_rot(uint32_t(s_w[3]), uint32_t(s_w[3] >> 32))) |
                                      (uint64_t(tag) << 32);
                __hip_atomic_store(&bell->xres[g][j % LANE_RING].u[t], unit, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            }
            ++j;
            __syncthreads();   // (every wave has read this task's words before wave 0 polls the next)
            continue;          // (every thread: op is block-uniform)
        }
        __syncthreads();
        if (t == 0) {
            __threadfence_system();   // the task's stores are visible to the host before its answer
            LaneResp* r = &bell->resp[g][j % LANE_RING];
            __hip_atomic_store(&r->errs, uint64_t(s_err), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&r->done, uint64_t(g) + j * W + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        ++j;
    }
    if (t == 0) {
        // where the next launch resumes; then, leaving on its own, the launch
        // announces it ends (the others follow; a waiting caller launches the
        // next generation behind it on the lane's stream)
        __hip_atomic_store(&bell->next_j[g], j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (why == 1)
            __hip_atomic_store(&bell->ctl.closing, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Grid = `main_blocks` streaming blocks, then the edge blocks.
//  * Streaming waves own 64 x FU consecutive chunks and write every chunk
//    that is all payload of one frame (the frame index comes from one scalar
//    division per pass when frames are >= 1 KiB, else a per-lane reciprocal).
//  * Edge lanes own one (frame f, header chunk h) item each and write the
//    chunk(s) that hold frame f's start / header / status bytes, built from
//    frame f - 1's tail and frame f's head.  A chunk is written by exactly
//    one side (identical bytes if two edge items meet on one chunk), so the
//    streaming waves never branch into the header code.
//  * Frames shorter than a chunk: the streaming waves do every chunk byte by
//    byte and there are no edge blocks.
__device__ __forceinline__ void fan_locate(uint64_t p, uint64_t fsize, double inv, uint64_t& i, uint64_t& r)
{
    i = uint64_t(double(p) * inv);
    int64_t rr = int64_t(p - i * fsize);
    if (rr < 0) {
        --i;
        rr += int64_t(fsize);
    } else if (uint64_t(rr) >= fsize) {
        ++i;
        rr -= int64_t(fsize);
    }
    r = uint64_t(rr);
}

__device__ __forceinline__ void fan_store(uint8_t* __restrict__ wire, uint64_t c, uint64_t chunks, uint64_t total,
                                          v4u w)
{
    if (c + 1 < chunks || (total & (CHUNK - 1)) == 0) {
        st16nt(wire + c * CHUNK, w);
    } else {
#pragma unroll 1
        for (uint32_t j = 0; j < (total & (CHUNK - 1)); ++j)
            wire[c * CHUNK + j] = uint8_t(lane_byte(w, j));
    }
}

__global__ __launch_bounds__(BLOCK) void k_fanout_flat(const uint8_t* __restrict__ payload, uint64_t len,
                                                       const uint32_t* __restrict__ keys, uint32_t k, uint8_t opcode,
                                                       uint32_t mask, uint64_t fsize, double inv, uint32_t main_blocks,
                                                       uint8_t* __restrict__ wire)
{
    const FanGeom f = fan_geom(opcode, mask != 0, len);
    const SendGeom& g = f.g;
    const uint64_t total = fsize * k;
    const uint64_t chunks = (total + CHUNK - 1) / CHUNK;
    const uint64_t data0 = f.data0;
    const uint32_t lane = threadIdx.x & 63;

    // edge blocks come first in the grid so that their longer per-lane work
    // overlaps the streaming instead of trailing it
    const uint32_t edge_blocks = gridDim.x - main_blocks;
    if (blockIdx.x < edge_blocks) {
        // edge items: 2 per frame start (the last "start" is the wire's end)
        const uint64_t item = uint64_t(blockIdx.x) * BLOCK + threadIdx.x;
        const uint64_t fr = item >> 1, h = item & 1;
        if (fr > k || (WSG_DIAG_FAN & 8))
            return;
        const uint64_t start = fr * fsize;
        const uint64_t c = start / CHUNK + h;
        if (c >= chunks || (h && (start & (CHUNK - 1)) + data0 <= CHUNK) || (fr == k && h))
            return;
        uint64_t i, r;
        fan_locate(c * CHUNK, fsize, inv, i, r);
        v4u w = fan_frame_bytes(payload, len, f, fsize, keys[i], r);
        const uint64_t split = fsize - r;
        if (split < CHUNK && i + 1 < k)
            w |= shl_bytes(fan_frame_bytes(payload, len, f, fsize, keys[i + 1], 0), split);
        fan_store(wire, c, chunks, total, w);
        return;
    }

    const uint64_t step = uint64_t(main_blocks) * (BLOCK / 64) * (64 * FU);
    const bool big = fsize >= uint64_t(64) * CHUNK;   // a 1 KiB pass row spans at most 2 frames
    const uint32_t mb = blockIdx.x - edge_blocks;
    for (uint64_t base = (uint64_t(mb) * (BLOCK / 64) + wave_id()) * (64 * FU); base < chunks; base += step) {
        if (fsize < CHUNK) {
            // several frames per chunk: byte by byte
#pragma unroll 1
            for (int u = 0; u < FU; ++u) {
                const uint64_t c = base + uint64_t(u) * 64 + lane;
                if (c >= chunks)
                    break;
                uint64_t i, r;
                fan_locate(c * CHUNK, fsize, inv, i, r);
                v4u e = {0, 0, 0, 0};
#pragma unroll 1
                for (uint32_t j = 0; j < CHUNK; ++j, ++r) {
                    while (r >= fsize) {
                        r -= fsize;
                        ++i;
                    }
                    if (i < k)
                        put_byte(e, j, fan_byte(payload, keys, opcode, mask != 0, g, fsize, i, r));
                }
                fan_store(wire, c, chunks, total, e);
            }
            continue;
        }
        v4u v[FU];
        bool fast[FU];
        uint64_t i0 = 0, r0 = 0;
        if (big) {
            // frame of the pass row's first chunk: one scalar division per row
            i0 = uint32_t(__builtin_amdgcn_readfirstlane(uint32_t((base * CHUNK) / fsize)));
            r0 = base * CHUNK - i0 * fsize;
        }
#pragma unroll
        for (int u = 0; u < FU; ++u) {
            const uint64_t c = base + uint64_t(u) * 64 + lane;
            uint64_t i, r;
            if (big) {
                // row u starts at most (FU - 1) KiB + r0 past frame i0's start
                r = r0 + (uint64_t(u) * 64 + lane) * CHUNK;
                i = i0;
#pragma unroll
                for (int q = 0; q < FU + 1; ++q)
                    if (r >= fsize) {
                        r -= fsize;
                        ++i;
                    }
            } else {
                fan_locate(c * CHUNK, fsize, inv, i, r);
            }
            fast[u] = c < chunks && r >= data0 && r + CHUNK <= fsize;
            v[u] = v4u{0, 0, 0, 0};
            if (fast[u]) {
                const v4u d = (WSG_DIAG_FAN & 2) ? v4u{uint32_t(r), 1, 2, 3}
                                                 : fan_window(payload, len, int64_t(r) - int64_t(data0));
                v[u] = d ^ key_rot((WSG_DIAG_FAN & 1) ? uint32_t(i) : keys[i], uint32_t(r - g.hdr));
            }
        }
#pragma unroll
        for (int u = 0; u < FU; ++u)
            if (fast[u])
                st16nt(wire + (base + uint64_t(u) * 64 + lane) * CHUNK, v[u]);
    }
}

// ---- fan-out, period path ---------------------------------------------------
// The k frames of a fan-out are one template (header + status + payload) and
// differ only in the key XORed over fixed byte positions.  With the frame size
// F a multiple of 4, every P = 16 / gcd(F, 16) (<= 4) consecutive frames form a
// group of G = P * F / 16 whole chunks, so a chunk's bytes depend only on its
// position j within its group and on the keys of the (<= 2) frames it touches:
//     chunk = T[j] ^ (MA[j] & rot(key_a)) ^ (MB[j] & rot(key_b)).
// With W waves (one per 64-thread block: 4-wave blocks measured slower) and W * 64 a multiple of G, a lane's j
// is the same in every pass, so it builds T / MA / MB once (the only payload
// loads) and then only stores, pass after pass, its chunk of successive groups.
// The wave's keys for all its passes come in one vector load up front (lane
// q holds key P * (first group of pass q / 2P) + q % 2P) and are picked per
// pass with a lane shuffle.  Rows are 1 KiB-aligned, whole lines per wave.
//
// Many messages in one launch (wsg_fanout_encode_many, the ws_multicast tick):
// blockIdx.y picks message y of up to FAN_MSGS messages of one geometry
// (length, opcode), whose payload and output start come from the kernel
// arguments; the k frames of every message are written exactly as for one.
// Template and key mask of frame bytes [o, o + 16) (o < fsize): t = the
// bytes with a zero key (header with the key bytes 0, close status 0, raw
// payload; 0 past the frame), m = the bytes the key is XORed into ([kpos,
// fsize): mask key, status, payload), so the frame with key K is
// t ^ (m & key_rot(K, o - hdr)).
__device__ __forceinline__ void fan_tm(const uint8_t* __restrict__ payload, uint64_t len, const FanGeom& f,
                                       uint64_t fsize, uint64_t o, v4u& t, v4u& m)
{
    const uint64_t hi = fsize - o < CHUNK ? fsize - o : CHUNK;
    const uint64_t kl = o < f.kpos ? f.kpos - o : 0;
    const uint64_t lo = o < f.data0 ? f.data0 - o : 0;   // chunk bytes [lo, hi) are payload
    m = low_bytes(hi) & ~low_bytes(kl);
    t = shr_bytes(f.hp0, o);
    if (lo < hi)
        t |= fan_window(payload, len, int64_t(o) - int64_t(f.data0)) & (low_bytes(hi) & ~low_bytes(lo));
}

template <int P>
__global__ __launch_bounds__(1024) void k_fanout_period(const uint8_t* __restrict__ payload0, uint64_t len,
                                                      const uint32_t* __restrict__ keys, uint32_t k, uint8_t opcode,
                                                      uint32_t mask, uint64_t fsize, uint32_t G, uint32_t dm,
                                                      uint8_t* __restrict__ wire0, const FanMsgs msgs, v4u hp0,
                                                      uint32_t nwaves, uint32_t wpb)
{
    constexpr int KW = 2 * P;   // keys per pass: the row spans <= 2 groups (G >= 64)
    if (WSG_DIAG_FAN & 256)     // diagnostic: the launch of the grid alone
        return;
    const uint64_t src_off = msgs.src[blockIdx.y], dst_off = msgs.dst[blockIdx.y];
    // every kernel argument in SGPRs before anything else: left to the
    // compiler, the argument loads came in five dependent rounds (each
    // waiting on the last), a visible share of a 9 us kernel; this empty
    // asm consumes them all, so they are issued together and waited once
    asm volatile("" ::"s"(payload0), "s"(len), "s"(keys), "s"(k), "s"(fsize), "s"(G), "s"(dm), "s"(wire0),
                     "s"(nwaves), "s"(wpb), "s"(src_off), "s"(dst_off), "s"(uint32_t(opcode)), "s"(mask));
    const uint8_t* __restrict__ payload = payload0 + src_off;
    uint8_t* __restrict__ wire = wire0 + dst_off;
    FanGeom f;   // fan_geom() with the header bytes from the host (hp0)
    f.g = send_geom(opcode, mask != 0, len, 0);
    f.data0 = f.g.hdr + f.g.prefix;
    f.kpos = f.g.hdr - (mask ? 4u : 0u);
    f.mask = mask != 0;
    f.hp0 = hp0;
    const uint64_t total = fsize * k;
    const uint64_t chunks = (total + CHUNK - 1) / CHUNK;
    const uint32_t lane = threadIdx.x & 63;
    // one wave per block, W = nwaves of them (a kernel argument, not
    // gridDim: the dispatch packet is one more memory read before the first
    // store); rows are wave-uniform, so the write-through stores' buffer
    // resource sits in SGPRs (else every store becomes a waterfall loop)
    const uint32_t wid = blockIdx.x * wpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave of W
    if (wid >= nwaves)   // the last workgroup's spare waves
        return;
    const uint64_t row0 = uint64_t(wid) * 64;
    const uint64_t rstep = uint64_t(nwaves) * 64;   // W rows: a multiple of G (dm groups)
    const uint64_t m0 = uint32_t(row0) / G;              // first group of pass 0 (host: W < 2^22, row0 < 2^28)
    const uint32_t jw = uint32_t(row0 - m0 * G);         // group position of lane 0
    const uint32_t dl = (jw + lane) >= G ? 1u : 0u;      // lane's group: m0 + dl (+ it * dm)
    const uint32_t j = jw + lane - dl * G;

    // keys of every pass: slot it * KW + q -> key P * (m0 + it * dm) + q
    // (host: passes * KW <= 64 * WSG_FAN_KV).  Issued before the template's
    // payload loads, so the two arrive together: the kernel is short (41 MB
    // at C4), and a second dependent memory round trip before the first
    // store was a visible share of it
    uint32_t kv[WSG_FAN_KV];
#pragma unroll
    for (int h = 0; h < WSG_FAN_KV; ++h) {
        const uint32_t s = uint32_t(h) * 64 + lane;
        const uint64_t it = s / KW;
        const uint64_t idx = uint64_t(P) * (m0 + it * dm) + (s % KW);
        kv[h] = (WSG_DIAG_FAN & 32) ? uint32_t(idx) : (row0 + it * rstep < chunks && idx < k) ? keys[idx] : 0u;
    }

    // template of chunk j: its frame-a bytes, and the next frame's from byte
    // `split` on (the first 16 bytes of a frame: the same for every lane)
    const uint64_t o = uint64_t(j) * CHUNK;              // < P * fsize
    uint32_t qa = 0;                                     // frame of the group holding byte o
#pragma unroll
    for (int q = 1; q < P; ++q)
        qa += o >= uint64_t(q) * fsize ? 1u : 0u;
    const uint64_t r = o - uint64_t(qa) * fsize;
    v4u t, ma, mb = {0, 0, 0, 0};
    // a frame's first 16 bytes (the same for every lane), built by every
    // lane so that its payload loads go out with the chunk's own instead of
    // in a second round behind them; used where a frame starts in the chunk
    const uint64_t split = fsize - r;                    // the next frame starts at chunk byte `split`
    // (both windows issued together branch-free instead: +0.5 us per C4,
    // every lane then loads two more blocks; round 3)
    fan_tm(payload, len, f, fsize, r, t, ma);
    if (split < CHUNK) {
        v4u t0, m0v;
        fan_tm(payload, len, f, fsize, 0, t0, m0v);
        t |= shl_bytes(t0, split);
        mb = shl_bytes(m0v, split);
    }
    if (WSG_DIAG_FAN & 16) {
        t = v4u{j, 1, 2, 3};
        ma = v4u{~0u, ~0u, ~0u, ~0u};
    }
    const uint32_t pa = uint32_t(r - f.g.hdr), pb = uint32_t(0u - uint32_t(split) - f.g.hdr);
    const uint32_t ia = P * dl + qa;                     // key slots of this pass's window

    // Pass loop, kept lean (it is most of the kernel's instructions): running
    // row / pointer / shuffle-address registers instead of per-pass products,
    // rotations as one v_alignbit each, and a wave-uniform test for whole
    // rows, so a pass is ~2 shuffles, ~12 VALU and one 1 KiB store.
    const uint32_t sa = 8u * (pa & 3u), sbr = 8u * (pb & 3u);
    // rows below this are whole: 64 chunks, each all 16 bytes inside the
    // output (from whole chunks only: when the job's last chunk is partial
    // and ends a row, that row takes the byte-exact store below — counted
    // from `chunks`, its whole-chunk store wrote up to 15 bytes past the
    // last frame; profiles/r6/fan_gap_seed123.log)
    const uint64_t full_rows_end = (total / CHUNK) & ~uint64_t(63);
    // this wave's passes (rows row0 + it * rstep below chunks), the first
    // n_full of them whole rows: 32-bit scalar loop counters instead of
    // 64-bit row compares in the loop
    const uint32_t n_pass = row0 < chunks ? uint32_t((chunks - row0 + rstep - 1) / rstep) : 0u;
    const uint32_t n_full = row0 < full_rows_end ? uint32_t((full_rows_end - row0 + rstep - 1) / rstep) : 0u;
    const uint64_t wstep = rstep * CHUNK;
    const uint32_t addr = ia * 4;                           // shuffle address of key slot ia of pass 0
    if (WSG_DIAG_FAN & 128) {   // diagnostic: the prologue alone (its results kept live)
        const v4u w = t ^ ma ^ mb ^ v4u{kv[0], kv[WSG_FAN_KV - 1], addr, 0};
        if ((w[0] & w[1] & w[2] & w[3]) == 0xA5C3E1F7u && row0 + lane < chunks)
            st16nt(wire + (row0 + lane) * CHUNK, w);
        return;
    }
    // The keys of pass `it` for this lane: frame a's (slot ia) and, where a
    // frame starts inside the lane's chunk, frame b's (slot ia + 1).
    auto pass_keys = [&](uint32_t it, uint32_t& ka, uint32_t& kb, bool want_b) {
        const uint32_t slot = it * KW;                      // wave-uniform; KW divides 64
        uint32_t kreg = kv[0];
#pragma unroll
        for (int h = 1; h < WSG_FAN_KV; ++h)
            kreg = (slot >> 6) == uint32_t(h) ? kv[h] : kreg;
        const uint32_t sb = (slot & 63) * 4;
        ka = __builtin_amdgcn_ds_bpermute(int(addr + sb), int(kreg));
        kb = want_b ? __builtin_amdgcn_ds_bpermute(int(addr + sb + 4), int(kreg)) : 0u;
    };
    // The pass loop, in two forms: a frame starts inside a chunk at only
    // ~P positions of a group's G, so most waves hold no such lane (mb = 0
    // in every lane, fixed for all passes) and skip frame b's key and
    // masking; the loop is VALU-bound once the shuffles are off its chain.
    auto passes = [&](auto has_b) {
        constexpr bool B = decltype(has_b)::value;
        // a pass's keys are shuffled one pass ahead (in the pass itself:
        // C4 8.40 vs 8.32 us; v_readlane + per-lane selects 8.6, round 3)
        uint32_t ka_n = 0, kb_n = 0;
        pass_keys(0, ka_n, kb_n, B);
        auto word = [&](uint32_t it) {
            // this pass's keys were shuffled during the previous pass; the
            // next pass's go out now, ahead of this pass's store
            const uint32_t ka = ka_n, kb = kb_n;
            pass_keys(it + 1, ka_n, kb_n, B);   // (past the last pass: slots of kv, unused)
            const uint32_t ra = __builtin_amdgcn_alignbit(ka, ka, sa);
            v4u w = t ^ (ma & v4u{ra, ra, ra, ra});
            if constexpr (B) {
                const uint32_t rb = __builtin_amdgcn_alignbit(kb, kb, sbr);
                w ^= mb & v4u{rb, rb, rb, rb};
            }
            return w;
        };
        uint8_t* wrow = wire + row0 * CHUNK;
#pragma unroll WSG_FAN_UNROLL
        for (uint32_t it = 0; it < n_full; ++it) {
            const v4u w = word(it);
            if ((WSG_DIAG_FAN & 64) && (w[0] & w[1] & w[2] & w[3]) != 0xA5C3E1F7u) {
                // diagnostic: the computation without its stores
            } else if (WSG_FAN_SC1) {
                const OutTile ot(wrow, 64 * CHUNK, true);   // write-through (resource at the row)
                ot.put(lane * CHUNK, w);
            } else {
                st16nt(wrow + lane * CHUNK, w);
            }
            wrow += wstep;
        }
        if (n_pass > n_full) {   // the last, partial row (the job's final row only)
            const uint64_t row = row0 + uint64_t(n_full) * rstep;
            const v4u w = word(n_full);
            if (row + lane < chunks)
                fan_store(wire, row + lane, chunks, total, w);
        }
    };
    const bool any_b = __ballot((mb[0] | mb[1] | mb[2] | mb[3]) != 0u) != 0;   // wave-uniform
    if (any_b)
        passes(std::true_type{});
    else
        passes(std::false_type{});
}

// Single-buffer XOR used by the per-frame host path: dst[i] = src[i] ^
// key[(phase + i) % 4].  src/dst 16-byte aligned device staging buffers.
__global__ __launch_bounds__(BLOCK) void k_xor(const uint8_t* src, uint8_t* dst, uint64_t len, uint32_t key,
                                               uint32_t phase)
{
    const uint32_t k = key_rot(key, phase);
    const uint64_t chunks = len / CHUNK;
    for (uint64_t c = uint64_t(blockIdx.x) * BLOCK + threadIdx.x; c < chunks; c += uint64_t(gridDim.x) * BLOCK)
        *reinterpret_cast<v4u*>(dst + c * CHUNK) = ld16(src + c * CHUNK) ^ k;
    if (blockIdx.x == 0 && threadIdx.x < (len & (CHUNK - 1))) {
        const uint64_t q = chunks * CHUNK + threadIdx.x;
        dst[q] = src[q] ^ key_byte(key, phase + q);
    }
}

// ===========================================================================
// Host launchers
// ===========================================================================

hipError_t launch_decode(hipStream_t s, int grid, const uint8_t* wire, uint8_t* out, uint64_t wire_len,
                         const uint64_t* fs, uint32_t n, wsg_recv_info* info, unsigned long long* err)
{
    const uint64_t tiles = (wire_len + TILE - 1) / TILE;
    // frames per wire byte: the tile's first-frame guess (exact for equal-size frames)
    const double fpb = wire_len ? double(n) / double(wire_len) : 0.0;
    // coarse-probe stride: 64 probes span +-32 strides around the guess, a
    // power of two >= sqrt(n) / 32 frames (a random-walk deviation of frame
    // counts from the guess grows like sqrt(n): C3's 65536 ragged frames
    // deviate by ~100)
    uint32_t stride = 1;
    while (uint64_t(stride) * stride * 1024 < n)
        stride <<= 1;
    k_decode<<<grid, BLOCK, 0, s>>>(wire, out, wire_len, fs, n, fpb, stride, info, err, tiles);
    return hipGetLastError();
}

hipError_t launch_encode_scan(hipStream_t s, const wsg_send_desc* desc, uint32_t n, uint64_t* wire_off,
                              uint32_t* piece_start, uint64_t* scan, uint32_t* piece_frame, uint64_t pieces_cap,
                              uint64_t wire_cap, unsigned long long* err)
{
    const uint32_t nb = uint32_t((n + SCAN_ITEMS - 1) / SCAN_ITEMS);
    uint64_t* sums = scan;
    uint64_t* psums = scan + nb;
    uint64_t* prefix = scan + 2 * uint64_t(nb);
    uint64_t* pprefix = scan + 3 * uint64_t(nb);
    k_encode_scan_local<true><<<nb, BLOCK, 0, s>>>(desc, n, wire_off, piece_start, sums, psums);
    k_encode_scan_blocks<<<1, BLOCK, 0, s>>>(sums, psums, nb, prefix, pprefix, wire_off, piece_start, n);
    k_encode_finalize<<<(n + BLOCK - 1) / BLOCK, BLOCK, 0, s>>>(desc, n, wire_off, piece_start, prefix, pprefix,
                                                                piece_frame, pieces_cap, wire_cap, err);
    return hipGetLastError();
}

hipError_t launch_encode_mask(hipStream_t s, int grid, const uint8_t* payload, const wsg_send_desc* desc, uint32_t n,
                              const uint64_t* wire_off, const uint32_t* piece_start, const uint32_t* piece_frame,
                              uint8_t* wire, uint64_t wire_cap, uint32_t q_begin, uint32_t q_end)
{
    k_encode_mask<<<grid, BLOCK, 0, s>>>(payload, desc, n, wire_off, piece_start, piece_frame, wire, wire_cap, q_begin,
                                         q_end);
    return hipGetLastError();
}

hipError_t launch_encode_scan_small(hipStream_t s, const wsg_send_desc* desc, uint32_t n, uint64_t* wire_off,
                                    uint64_t* scan)
{
    const uint32_t nb = uint32_t((n + SCAN_ITEMS - 1) / SCAN_ITEMS);
    k_encode_scan_local<false><<<nb, BLOCK, 0, s>>>(desc, n, wire_off, nullptr, scan, nullptr);
    return hipGetLastError();
}

hipError_t launch_encode_small(hipStream_t s, const uint8_t* payload, const wsg_send_desc* desc, uint32_t n,
                               uint64_t* wire_off, const uint64_t* scan, uint8_t* wire, uint64_t wire_cap,
                               unsigned long long* err)
{
    // frames per block: as many as fit SMALL_RANGE wire bytes at the average
    // frame size (wire_cap / n), so that larger frames still fill the grid
    const uint64_t avg = wire_cap / n + 1;
    uint32_t fpb = SMALL_F;
    while (fpb > 1 && uint64_t(fpb) * avg > SMALL_RANGE)
        fpb >>= 1;
    const uint32_t nb = uint32_t((n + SCAN_ITEMS - 1) / SCAN_ITEMS);
    k_encode_small<<<(n + fpb - 1) / fpb, BLOCK, 0, s>>>(payload, desc, n, fpb, wire_off, scan, nb, wire, wire_cap,
                                                         err);
    return hipGetLastError();
}

hipError_t launch_fanout(hipStream_t s, int grid, const uint8_t* payload, uint64_t len, const uint32_t* keys,
                         uint32_t k, uint8_t opcode, uint32_t mask, uint64_t fsize, uint8_t* wire)
{
    // edge blocks: two items per frame start (k + 1 starts); none for
    // frames shorter than a chunk (the streaming waves do those)
    const uint64_t edge_blocks = fsize >= CHUNK ? (2 * (uint64_t(k) + 1) + BLOCK - 1) / BLOCK : 0;
    k_fanout_flat<<<dim3(uint32_t(grid + edge_blocks)), BLOCK, 0, s>>>(
        payload, len, keys, k, opcode, mask, fsize, 1.0 / double(fsize), uint32_t(grid), wire);
    return hipGetLastError();
}

// Period path (k_fanout_period) when the frame size allows it; returns false
// to leave the batch to k_fanout_flat.  Wave count W = Q * s with W * 64 a
// multiple of G (Q = G / gcd(G, 64)), about `waves` of them, and few enough
// passes per wave that one key load covers them (passes * 2P <= 64 * WSG_FAN_KV).
bool launch_fanout_period(hipStream_t s, int cus, int waves_per_cu, int wpb, const uint8_t* payload, uint64_t len,
                          const uint32_t* keys, uint32_t k, uint8_t opcode, uint32_t mask, uint64_t fsize,
                          uint8_t* wire, const FanMsgs& msgs, uint32_t nmsgs, hipError_t* err)
{
    if (nmsgs == 0 || nmsgs > uint32_t(FAN_MSGS))
        return false;
    if (!WSG_FAN_PERIOD || fsize % 4 != 0)
        return false;
    uint64_t g16 = 16;
    while (fsize % g16)
        g16 >>= 1;
    const uint32_t P = uint32_t(16 / g16);               // 1, 2 or 4
    const uint64_t G = uint64_t(P) * fsize / CHUNK;
    if (G < 64 || G > (1u << 20))
        return false;
    uint64_t g64 = 64;
    while (G % g64)
        g64 >>= 1;
    const uint64_t Q = G / g64;
    const uint64_t chunks = (fsize * k + CHUNK - 1) / CHUNK;
    const uint64_t max_passes = 64 * WSG_FAN_KV / (2 * P);
    if (Q * 64 > chunks * 2)   // even the fewest waves would mostly idle: leave it to the flat kernel
        return false;
    const uint64_t rows = (chunks + 63) / 64;
    if (WSG_FAN_MANY_WPC && nmsgs > 1)
        waves_per_cu = WSG_FAN_MANY_WPC;
    if (WSG_FAN_MANY_WPB && nmsgs > 1)
        wpb = WSG_FAN_MANY_WPB;
    uint64_t mult = std::max<uint64_t>(1, (uint64_t(cus) * waves_per_cu + Q / 2) / Q);
    mult = std::min(mult, (rows + Q - 1) / Q);                                                 // no idle waves
    mult = std::max(mult, (chunks + Q * 64 * max_passes - 1) / (Q * 64 * max_passes));   // every pass's keys in one load per lane
    const uint64_t W = Q * mult;
    if (W > (1u << 22))
        return false;
    const uint32_t dm = uint32_t(W * 64 / G);
    // workgroups of wpb waves (the last one's spare waves return at once):
    // dispatching one-wave workgroups was most of a C4 launch
    if (wpb < 1 || wpb > 16)
        wpb = 1;
    const uint32_t blocks = uint32_t((W + uint64_t(wpb) - 1) / uint64_t(wpb));
    // header bytes before the key (<= 10), the same in every frame
    const SendGeom sg = send_geom(opcode, mask != 0, len, 0);
    const uint32_t kpos = sg.hdr - (mask ? 4u : 0u);
    uint32_t hw[4] = {0, 0, 0, 0};
    for (uint32_t r = 0; r < kpos; ++r)
        hw[r / 4] |= uint32_t(header_byte(opcode, mask != 0, sg.body, 0, r)) << (8 * (r % 4));
    const v4u hp0 = v4u{hw[0], hw[1], hw[2], hw[3]};
    // (WSG_FAN_CAP: LDS reserved per workgroup only to bound the workgroups
    // resident per CU; the kernel uses none)
    // (many messages only: one message's waves are all resident anyway)
    const uint32_t lds = WSG_FAN_CAP && nmsgs > 1 ? uint32_t((160u << 10) / WSG_FAN_CAP) & ~255u : 0u;
    switch (P) {
    case 1:
        k_fanout_period<1><<<dim3(blocks, nmsgs), 64 * uint32_t(wpb), lds, s>>>(payload, len, keys, k, opcode, mask, fsize,
                                                                             uint32_t(G), dm, wire, msgs, hp0, uint32_t(W),
                                                                             uint32_t(wpb));
        break;
    case 2:
        k_fanout_period<2><<<dim3(blocks, nmsgs), 64 * uint32_t(wpb), lds, s>>>(payload, len, keys, k, opcode, mask, fsize,
                                                                             uint32_t(G), dm, wire, msgs, hp0, uint32_t(W),
                                                                             uint32_t(wpb));
        break;
    default:
        k_fanout_period<4><<<dim3(blocks, nmsgs), 64 * uint32_t(wpb), lds, s>>>(payload, len, keys, k, opcode, mask, fsize,
                                                                             uint32_t(G), dm, wire, msgs, hp0, uint32_t(W),
                                                                             uint32_t(wpb));
        break;
    }
    *err = hipGetLastError();
    return true;
}

// The job's wire offsets on the gather root: every chunk's frame offsets
// arrive relative to its sender's local wire.
// Multi-GPU gather root: the job's wire offsets from every rank's local
// frame offsets.  stage holds rank r's n_local(r) local offsets at
// [rank_base[r], rank_base[r + 1]) (one transfer per rank); global frame g
// is in chunk c = g / chunk, owned by rank c % world as its local chunk
// q = c / world, which the gather placed at goff[c] in the job's wire.
__global__ __launch_bounds__(BLOCK) void k_rebase_offsets(const uint64_t* __restrict__ stage,
                                                          const uint64_t* __restrict__ goff,
                                                          const uint64_t* __restrict__ rank_base, uint64_t n_total,
                                                          uint32_t chunk, uint32_t world, uint64_t* __restrict__ out_off,
                                                          uint64_t total)
{
    const uint64_t stride = uint64_t(gridDim.x) * BLOCK;
    for (uint64_t g = uint64_t(blockIdx.x) * BLOCK + threadIdx.x; g < n_total; g += stride) {
        const uint64_t c = g / chunk;
        const uint64_t r = c % world, q = c / world;
        const uint64_t* loc = stage + rank_base[r] + q * chunk;
        out_off[g] = loc[g - c * chunk] - loc[0] + goff[c];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0)
        out_off[n_total] = total;
}

hipError_t launch_rebase_offsets(hipStream_t s, const uint64_t* stage, const uint64_t* goff, const uint64_t* rank_base,
                                 uint64_t n_total, uint32_t chunk, uint32_t world, uint64_t* out_off, uint64_t total)
{
    const uint64_t blocks = std::min<uint64_t>(std::max<uint64_t>((n_total + BLOCK - 1) / BLOCK, 1), 8192);
    k_rebase_offsets<<<uint32_t(blocks), BLOCK, 0, s>>>(stage, goff, rank_base, n_total, chunk, world, out_off, total);
    return hipGetLastError();
}

// Test hook of the multi-GPU gather ($WSG_TEST_NULL_SPIN_US, wsg_mgpu.cpp):
// one wave that waits `ticks` of the constant-rate wall clock on the stream
// it is launched on.  The iteration cap ends it whatever the clock does
// (about 2 s at the most).
__global__ __launch_bounds__(64) void k_test_spin(uint64_t ticks)
{
    const uint64_t t0 = wall_clock64();
    for (uint32_t i = 0; i < (1u << 20); ++i) {
        if (wall_clock64() - t0 >= ticks)
            break;
        __builtin_amdgcn_s_sleep(64);
    }
}

hipError_t launch_test_spin(hipStream_t s, uint32_t us)
{
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0)
        khz = 100000;   // 100 MHz, the gfx9 constant clock
    k_test_spin<<<1, 64, 0, s>>>(uint64_t(std::min<uint32_t>(us, 200000u)) * uint64_t(khz) / 1000u);
    return hipGetLastError();
}

hipError_t launch_lane(hipStream_t s, LaneBell* bell, uint32_t workgroups, uint64_t idle_ticks,
                       uint64_t yield_ticks, uint32_t gen, uint64_t delay_ticks)
{
    if (workgroups < 1 || workgroups > LANE_WGS_MAX || gen == 0)
        return hipErrorInvalidValue;
    const uint32_t blocks = (workgroups + LANE_NEAR_XCCS - 1) / LANE_NEAR_XCCS * LANE_XCCS;
    k_lane<<<blocks, LANE_THREADS, 0, s>>>(bell, workgroups, idle_ticks, yield_ticks, gen, delay_ticks);
    return hipGetLastError();
}

hipError_t launch_xor(hipStream_t s, int grid, const uint8_t* src, uint8_t* dst, uint64_t len, uint32_t key,
                      uint32_t phase)
{
    k_xor<<<grid, BLOCK, 0, s>>>(src, dst, len, key, phase);
    return hipGetLastError();
}

} // namespace wsg
