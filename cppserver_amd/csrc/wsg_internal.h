// wsg_internal.h — kernel geometry and kernel declarations shared by
// wsg_kernels.hip and the C-ABI implementation.
#pragma once

#include "wsg_frame.h"

namespace wsg {

constexpr int BLOCK = 256;                  // 4 wave64s
constexpr int CHUNK = 16;                   // bytes per lane per step (dwordx4)
#ifndef WSG_UNROLL
#define WSG_UNROLL 4
#endif
constexpr int UNROLL = WSG_UNROLL;          // steps per lane per tile
constexpr uint64_t TILE = uint64_t(BLOCK) * CHUNK * UNROLL;   // 16 KiB of output
#ifndef WSG_EU
#define WSG_EU 4
#endif
constexpr int EU = WSG_EU;                              // encode: 16-B steps per lane per piece
constexpr uint64_t PIECE = uint64_t(64) * CHUNK * EU;   // encode work piece: 4 KiB of one frame
// Pieces start on 128-byte line boundaries of the OUTPUT, so every 1 KiB
// store row of a wave writes whole lines (a 16-B-aligned but line-misaligned
// streaming store costs 6-16 %: tools/membench.hip explore, delta 16/80).
constexpr uint64_t PIECE_ALIGN = 128;
#ifndef WSG_FAN_UNITS
#define WSG_FAN_UNITS 4
#endif
constexpr int FAN_UNITS = WSG_FAN_UNITS;                 // fan-out: 16-B chunks per lane per pass
constexpr uint32_t SMALL_F = BLOCK;                      // small-frame encode: most frames per block
                                                         // (512/1024 measured 10-40 % slower)
#ifndef WSG_SMALL_AVG
#define WSG_SMALL_AVG 4096
#endif
constexpr uint64_t SMALL_AVG = WSG_SMALL_AVG;            // ... used when wire_cap <= n * SMALL_AVG
#ifndef WSG_SMALL_RANGE
#define WSG_SMALL_RANGE 32768
#endif
constexpr uint64_t SMALL_RANGE = WSG_SMALL_RANGE;        // ... wire bytes per block (sets frames per block)
#ifndef WSG_SCAN_PER_LANE
#define WSG_SCAN_PER_LANE 4
#endif
constexpr int SCAN_PER_LANE = WSG_SCAN_PER_LANE;   // encode scan: frames per lane
constexpr uint64_t SCAN_ITEMS = uint64_t(BLOCK) * SCAN_PER_LANE;   // frames per scan block

__global__ void k_decode(const uint8_t* wire, uint8_t* out, uint64_t wire_len, const uint64_t* fs, uint32_t n,
                         double frames_per_byte, uint32_t stride, wsg_recv_info* info, unsigned long long* err,
                         uint64_t num_tiles);
__global__ void k_xor(const uint8_t* src, uint8_t* dst, uint64_t len, uint32_t key, uint32_t phase);

// Host launchers (defined in wsg_kernels.hip next to the kernels).
// One-launch decode (k_decode): grid blocks over the wire's tiles, per-frame
// info and the error latch from the same launch.
hipError_t launch_decode(hipStream_t s, int grid, const uint8_t* wire, uint8_t* out, uint64_t wire_len,
                         const uint64_t* fs, uint32_t n, wsg_recv_info* info, unsigned long long* err);
// Sizes + piece counts scan (scan: 4 * ceil(n / SCAN_ITEMS) words), wire
// offsets, piece starts (n + 1 each) and the piece -> frame map.
hipError_t launch_encode_scan(hipStream_t s, const wsg_send_desc* desc, uint32_t n, uint64_t* wire_off,
                              uint32_t* piece_start, uint64_t* scan, uint32_t* piece_frame, uint64_t pieces_cap,
                              uint64_t wire_cap, unsigned long long* err);
hipError_t launch_encode_mask(hipStream_t s, int grid, const uint8_t* payload, const wsg_send_desc* desc, uint32_t n,
                              const uint64_t* wire_off, const uint32_t* piece_start, const uint32_t* piece_frame,
                              uint8_t* wire, uint64_t wire_cap, uint32_t q_begin, uint32_t q_end);
// Small-frame batch encode: block-local sizes scan (scan: ceil(n /
// SCAN_ITEMS) block totals), then k_encode_small, which adds the block
// prefixes, writes the final wire_off[0..n] and latches capacity errors.
hipError_t launch_encode_scan_small(hipStream_t s, const wsg_send_desc* desc, uint32_t n, uint64_t* wire_off,
                                    uint64_t* scan);
hipError_t launch_encode_small(hipStream_t s, const uint8_t* payload, const wsg_send_desc* desc, uint32_t n,
                               uint64_t* wire_off, const uint64_t* scan, uint8_t* wire, uint64_t wire_cap,
                               unsigned long long* err);
// Messages of one fan-out launch (blockIdx.y): payload and output offsets.
constexpr int FAN_MSGS = 32;
struct FanMsgs {
    uint64_t src[FAN_MSGS];   // message payload offset from the payload base
    uint64_t dst[FAN_MSGS];   // wire offset of the message's first frame
};
// Period-path fan-out of nmsgs (<= FAN_MSGS) messages of one geometry; false:
// the frame size does not suit it (the caller takes launch_fanout per message).
bool launch_fanout_period(hipStream_t s, int cus, int waves_per_cu, int wpb, const uint8_t* payload, uint64_t len,
                          const uint32_t* keys, uint32_t k, uint8_t opcode, uint32_t mask, uint64_t fsize,
                          uint8_t* wire, const FanMsgs& msgs, uint32_t nmsgs, hipError_t* err);
hipError_t launch_fanout(hipStream_t s, int grid, const uint8_t* payload, uint64_t len, const uint32_t* keys,
                         uint32_t k, uint8_t opcode, uint32_t mask, uint64_t fsize, uint8_t* wire);
hipError_t launch_xor(hipStream_t s, int grid, const uint8_t* src, uint8_t* dst, uint64_t len, uint32_t key,
                      uint32_t phase);
// Multi-GPU gather (wsg_mgpu.cpp): the job's wire offsets from the ranks'
// local offsets, staged rank by rank at rank_base[r] (chunk c of the job is
// rank c % world's local chunk c / world, placed at goff[c]);
// out_off[n_total] = total.
hipError_t launch_rebase_offsets(hipStream_t s, const uint64_t* stage, const uint64_t* goff, const uint64_t* rank_base,
                                 uint64_t n_total, uint32_t chunk, uint32_t world, uint64_t* out_off, uint64_t total);
// Test hook only: one wave waiting `us` microseconds (at most 0.2 s) on `s`.
hipError_t launch_test_spin(hipStream_t s, uint32_t us);

// ---- the host lane: one resident kernel per device for small host batches
// A host batch of a few KiB (an echo's read: ~1000 frames of 38 B) costs a
// launch and a synchronize per pass (10 us for an empty kernel on MI355X,
// tools/smallpass.hip) on top of its PCIe round trips.  The lane is launched
// once per device and shared by every context of the process: W workgroups,
// each with a mailbox of LANE_RING task slots in page-locked host memory.
// A request is cut into frame groups; group k gets the ticket x + k of a
// process-wide ticket counter, i.e. slot (x + k) / W of workgroup (x + k) % W,
// so consecutive requests spread over the workgroups and one request's groups
// run side by side.  The host writes a slot's units (each value, then its
// tag = ticket + 1; the first unit last), the workgroup polls its next slot
// (every unit in one read), does the group on the host buffers in place and answers
// in the slot's response.  Every workgroup ends: on `stop` (teardown, or a
// request that timed out), or after idle_ticks without a task / yield_ticks of
// running, announced in `closing` so that the others follow at their next
// check; a caller waiting on an answer launches the next generation, which
// resumes each mailbox where the last one left it (next_j).
enum : uint32_t { LANE_DECODE = 1, LANE_ENCODE = 2, LANE_XOR = 3, LANE_XOR_INLINE = 4 };
constexpr uint64_t LANE_INLINE = 40;     // xor: payloads up to this size travel in the task (w[4..8])
constexpr uint32_t LANE_THREADS = 1024;   // one workgroup; frames per group (lane per frame)
constexpr uint64_t LANE_STAGE = 64 << 10;  // decode: wire bytes staged in LDS (one group's range limit)
constexpr uint64_t LANE_PSTAGE = 64 << 10; // encode: payload arena staged in LDS when its 16-B blocks fit
// LDS of the lane (one layout per op, the larger sized):
//   decode: staged wire | info blocks (32 B) | payload bounds (2 x 8 B), key (4 B), frame starts (8 B) per frame
//   encode: offsets (8 B) | heads (16 B) | records (16 B) | descriptors (32 B) per frame | staged payload
constexpr uint64_t LANE_LDS_DECODE = LANE_STAGE + 60 * LANE_THREADS + 64;
constexpr uint64_t LANE_LDS_ENCODE = 72 * LANE_THREADS + 64 + LANE_PSTAGE;
constexpr uint64_t LANE_LDS = LANE_LDS_DECODE > LANE_LDS_ENCODE ? LANE_LDS_DECODE : LANE_LDS_ENCODE;
static_assert(LANE_LDS <= 160 * 1024 - 1024, "the lane's workgroup LDS");
constexpr uint32_t LANE_WGS_MAX = 32;          // workgroups of the lane (each a CU's worth of LDS)
constexpr uint32_t LANE_GROUPS_MAX = 32;       // frame groups of a request (<= 32 Ki frames)
constexpr uint32_t LANE_RING = 64;             // task slots per workgroup mailbox
constexpr uint32_t LANE_WORDS = 9;             // task units (w[])
// A task word and the ticket it belongs to, + 1 (the host stores v, then
// tag; the lane reads the 16 bytes in one request).
struct alignas(16) LaneUnit {
    uint64_t v, tag;
};
// One frame group of a request (the host's, read by one workgroup):
//   w[0] = op | n << 32 (posted last: the workgroup polls its tag)
//   decode: w[1..5] = wire, wire_len, frame_start, out, info;
//           w[6] = f_lo | cnt << 32 (the group's frames [f_lo, f_lo + cnt));
//           w[7], w[8] = the group's wire range [lo, hi): its first start (0
//           for the first group) to the next group's (wire_len after the last),
//           clamped to wire_len — bit-identical to k_decode there; the table
//           strictly increasing (the caller checks), hi - lo + 64 <= LANE_STAGE
//   encode: w[1..4] = payload, desc, wire_off (n + 1, host-computed), wire;
//           w[6] = f_lo | cnt << 32; w[7], w[8] = the group's payload span
//           [lo, hi) ({0, 0}: none)
//   xor:    w[1..3] = buffer, length, key | phase << 32 (n = 1): the
//           page-locked buffer XORed in place, byte i with key byte
//           (phase + i) % 4; LANE_XOR_INLINE: the payload (<= LANE_INLINE
//           bytes) in w[4..8], the result in the slot's LaneXres (no write
//           to the buffer, no fence, no `done`)
struct LaneTask {
    LaneUnit w[LANE_WORDS];
    uint64_t pad[2];
};
// The lane's answer to a task: errs (decode: frames with an error), then
// done = the task's tag (release).
struct alignas(16) LaneResp {
    uint64_t done, errs;
};
// The answer of an inline XOR: result dword k beside the low 32 bits of the
// task's tag, one 8-byte unit each, written by one lane with one store and
// read by the host with one load — a unit showing the tag holds its dword,
// so the answer needs no release fence before it (the fence waits for the
// stores to be acknowledged over PCIe).
struct alignas(16) LaneXres {
    uint64_t u[LANE_INLINE / 4];
};
struct alignas(16) LaneCtl {
    uint32_t stop;      // host: every workgroup leaves at its next check
    uint32_t closing;   // lane: launch `closing` is ending (its workgroups leave at their next check)
    uint64_t pad;
};
struct LaneBell {
    LaneCtl ctl;
    uint64_t next_j[LANE_WGS_MAX];             // lane: workgroup g's next mailbox position (stored as it leaves)
    LaneResp resp[LANE_WGS_MAX][LANE_RING];    // lane: answers
    LaneXres xres[LANE_WGS_MAX][LANE_RING];    // lane: inline XOR answers
    LaneTask box[LANE_WGS_MAX][LANE_RING];     // host: mailboxes (ticket x: box[x % W][(x / W) % LANE_RING])
};
// A launch of `workgroups` (the server's W) workgroups of generation `gen`
// (>= 1): each leaves after idle_ticks without a task, after yield_ticks of
// running (at a task boundary), on `stop`, or when `closing` names its
// generation.  delay_ticks: a test hook, the workgroups wait that long before
// their first poll (a lane that starts late).
hipError_t launch_lane(hipStream_t s, LaneBell* bell, uint32_t workgroups, uint64_t idle_ticks,
                       uint64_t yield_ticks, uint32_t gen, uint64_t delay_ticks);

// HIP device a context is bound to (wsg_capi.hip)
int ctx_device(const wsg_ctx* c);
// $WSG_HOST_MULTI_SHARE as the context read it at wsg_create (wsg_mgpu.cpp)
bool ctx_multi_share(const wsg_ctx* c);

} // namespace wsg
