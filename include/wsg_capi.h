/*
 * wsg_capi.h — C-ABI boundary of the MI355X WebSocket frame codec.
 *
 * This is the drop-in boundary for CppServer's per-byte WebSocket hot path
 * (reference: chronoxor/CppServer 1.0.5.0, class CppServer::WS::WebSocket,
 * include/server/ws/ws.h:29, source/server/ws/ws.cpp:212-498).
 *
 * Plain C types only: pointers, sizes, fixed-layout structs.  No C++ types and
 * no torch types cross this boundary; no C++ exception ever leaves it.  Every
 * entry point returns an int status (WSG_OK = 0, negative on failure).
 *
 * Device ("d_") buffers are caller-owned and must already be resident in HBM.
 * Batch entry points are asynchronous on the given HIP stream (NULL = HIP's
 * default stream, as everywhere in HIP; wsg_stream() returns a non-blocking
 * stream owned by the context); the caller synchronizes (wsg_sync) before
 * reading outputs.  Data-dependent errors (a frame that overruns the wire, overlapping
 * frames) are latched in the context and reported by wsg_sync.
 *
 * Thread-safety: one wsg_ctx per host thread.  A ctx is not thread-safe.
 *
 * Debug: with $WSG_CHECK=1 at wsg_create, the device entry points check
 * before every launch that each operand range lies inside one device
 * allocation (encode: every descriptor's payload range too, read back from
 * the device) and return WSG_EINVAL instead of launching otherwise.
 */
#ifndef WSG_CAPI_H
#define WSG_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WSG_ABI_VERSION 3

/* ---- status codes ------------------------------------------------------ */
#define WSG_OK          0
#define WSG_EINVAL    (-22)  /* bad argument: NULL pointer, misaligned buffer, overlapping frames */
#define WSG_ETRUNC    (-61)  /* a frame header/payload runs past the end of the wire */
#define WSG_ENOMEM    (-12)  /* device or pinned allocation failed / output capacity too small */
#define WSG_EHIP      (-5)   /* HIP runtime error (no device, launch failure, ...) */

/* ---- opcode byte values (reference ws.h:33-43) ------------------------- */
#define WSG_FIN    0x80
#define WSG_TEXT   0x01
#define WSG_BINARY 0x02
#define WSG_CLOSE  0x08
#define WSG_PING   0x09
#define WSG_PONG   0x0A

/* Required alignment of wire/output device buffers in the batch decode/encode
 * entry points (hipMalloc and torch allocations satisfy it). */
#define WSG_ALIGN 16

/* One frame to encode (a batched PrepareSendFrame call, ws.cpp:212).
 * key is _ws_send_mask[0..3] read as a little-endian uint32, i.e.
 * byte j of the key is (key >> 8*j) & 0xFF (ws.cpp:244-247, :270). */
typedef struct wsg_send_desc {
    uint64_t src_off;   /* payload offset inside d_payload                    */
    uint64_t len;       /* payload length in bytes (excluding close status)   */
    uint32_t key;       /* per-connection send mask (ws.cpp:97 / :206)       */
    int32_t  status;    /* close status, ws.cpp:215 (0 = none)                */
    uint8_t  opcode;    /* whole first header byte, e.g. WSG_FIN|WSG_BINARY   */
    uint8_t  mask;      /* nonzero: set MASK bit and emit the 4 key bytes     */
    uint8_t  _pad[6];
} wsg_send_desc;        /* 32 bytes */

/* One decoded frame (the per-frame arithmetic of PrepareReceiveFrame,
 * ws.cpp:320-386). */
typedef struct wsg_recv_info {
    uint64_t payload_off; /* absolute offset of the payload in wire and output */
    uint64_t len;         /* payload length                                    */
    uint32_t key;         /* receive mask (little-endian), 0 if unmasked       */
    uint8_t  opcode;      /* b0 & 0x0F (raw; 0 = continuation, ws.cpp:320)     */
    uint8_t  fin;         /* b0 >> 7 (ws.cpp:321)                              */
    uint8_t  masked;      /* b1 >> 7 (ws.cpp:322)                              */
    uint8_t  hdr_len;     /* 2/4/10 (+4 when masked), ws.cpp:331/349/367       */
    uint8_t  b0;          /* raw first header byte (RSV bits kept)             */
    int8_t   error;       /* 0, or WSG_ETRUNC / WSG_EINVAL for this frame      */
    uint8_t  _pad[6];
} wsg_recv_info;        /* 32 bytes */

typedef struct wsg_ctx wsg_ctx;

/* ---- context ------------------------------------------------------------ */
/* Bind to HIP device `device`, create a non-blocking stream, small scratch.   */
int wsg_create(int device, wsg_ctx** out);
int wsg_destroy(wsg_ctx* ctx);
/* Synchronize `stream` (NULL = default stream) and return the first
 * data-dependent error latched since the last wsg_sync (then clear it).      */
int wsg_sync(wsg_ctx* ctx, void* stream);
/* HIP stream owned by the context (a hipStream_t). */
void* wsg_stream(wsg_ctx* ctx);
int wsg_abi_version(void);
/* Human-readable name of a status code. */
const char* wsg_strerror(int code);

/* ---- batch decode: unmask (PrepareReceiveFrame over many frames) -------- */
/* d_wire: `wire_len` bytes of concatenated frames.  d_frame_start[i]: wire
 * offset of frame i (strictly increasing, frames must not overlap; the host
 * framer produces it with RequiredReceiveFrameSize semantics, ws.cpp:458).
 * d_out: wire_len bytes; on return it is the wire with every frame's payload
 * unmasked in place (ws.cpp:399-406); header and gap bytes are copied
 * unchanged.  d_out may equal d_wire (in-place).  d_info[i] describes frame i
 * (payload at d_out + d_info[i].payload_off).  d_wire/d_out 16-byte aligned;
 * the kernel reads d_wire in whole 16-byte blocks, so the block holding the
 * last wire byte must be readable (hipMalloc / torch allocations are).       */
int wsg_decode_batch(wsg_ctx* ctx, const uint8_t* d_wire, uint64_t wire_len,
                     const uint64_t* d_frame_start, uint32_t n,
                     uint8_t* d_out, wsg_recv_info* d_info, void* stream);

/* ---- batch encode: header pack + mask (PrepareSendFrame over many frames) */
/* Frames are written back to back into d_wire (16-byte aligned, capacity
 * wire_cap bytes).  d_wire_off[0..n] receives each frame's offset;
 * d_wire_off[n] is the total wire length.  Byte-exact with ws.cpp:212-271,
 * including the close-status prefix on CLOSE/PING/PONG opcodes (ws.cpp:215)
 * and the XOR applied even when mask == 0 (ws.cpp:269-270).                  */
int wsg_encode_batch(wsg_ctx* ctx, const uint8_t* d_payload,
                     const wsg_send_desc* d_desc, uint32_t n,
                     uint8_t* d_wire, uint64_t wire_cap,
                     uint64_t* d_wire_off, void* stream);

/* ---- fan-out: one payload, k client keys (k x client-style SendBinary) -- */
/* Frame j = PrepareSendFrame(opcode, mask, payload, len) with
 * _ws_send_mask = d_keys[j]; frames back to back in d_wire, each
 * wsg_frame_size(opcode, mask, len, 0) bytes.  d_wire 16-byte aligned.        */
int wsg_fanout_encode(wsg_ctx* ctx, const uint8_t* d_payload, uint64_t len,
                      const uint32_t* d_keys, uint32_t k, uint8_t opcode,
                      int mask, uint8_t* d_wire, uint64_t wire_cap, void* stream);

/* ---- many messages x k keys in one call (a ws_multicast tick) ----------- */
/* The multicast driver sends `messages_rate` messages per tick to every
 * client (reference performance/ws_multicast_server.cpp:104-114, each through
 * WSServer::Multicast, source/server/ws/ws_server.cpp:36-64); this encodes
 * m messages for k client keys at once.  Frame (i, j) =
 * PrepareSendFrame(opcode[i], mask, message i, len[i]) with _ws_send_mask =
 * d_keys[j]; message i's payload is d_payload + src_off[i].  The k frames of
 * message i lie back to back from wire_off[i] (128-byte aligned; frame j at
 * wire_off[i] + j * wsg_frame_size(opcode[i], mask, len[i], 0)).
 * src_off / len / opcode are HOST arrays of m entries; wire_off (host, m + 1
 * entries) is filled, wire_off[m] = bytes used (checked against wire_cap).   */
int wsg_fanout_encode_many(wsg_ctx* ctx, const uint8_t* d_payload, const uint64_t* src_off, const uint64_t* len,
                           const uint8_t* opcode, uint32_t m, const uint32_t* d_keys, uint32_t k, int mask,
                           uint8_t* d_wire, uint64_t wire_cap, uint64_t* wire_off, void* stream);

/* ---- host-staged entry points (host buffers; PCIe in the path) ---------- */
/* XOR `len` bytes of host `src` into host `dst` with key byte (phase+i)%4 on
 * the GPU (H2D, kernel, D2H), synchronous.  src may equal dst.               */
int wsg_xor_host(wsg_ctx* ctx, const void* src, void* dst, size_t len,
                 uint32_t key, uint32_t phase);
/* Batch decode of a host wire buffer, synchronous, same results as
 * wsg_decode_batch with host pointers (payload_off are wire offsets).  The
 * batch is cut into ~32 MiB segments of whole frames ($WSG_STAGE_MB) that
 * flow through three stream slots, so H2D of one segment, decode of the next
 * and D2H of a third overlap.  Pinned buffers (wsg_host_alloc, or registered)
 * are DMA'd directly; pageable ones are staged through pinned memory.        */
int wsg_decode_batch_host(wsg_ctx* ctx, const uint8_t* wire, uint64_t wire_len,
                          const uint64_t* frame_start, uint32_t n,
                          uint8_t* out, wsg_recv_info* info);

/* Batch encode of host buffers, synchronous, the bytes wsg_encode_batch
 * produces: frames back to back in wire[0..wire_off[n]) (host pointers;
 * wire_off[0..n] is filled).  Segments of ~32 MiB of frames flow through the
 * same three stream slots; each segment's payloads are DMA'd as one range
 * (or gathered through pinned staging when its descriptors are scattered).  */
int wsg_encode_batch_host(wsg_ctx* ctx, const uint8_t* payload, uint64_t payload_len,
                          const wsg_send_desc* desc, uint32_t n,
                          uint8_t* wire, uint64_t wire_cap, uint64_t* wire_off);

/* Page-locked host memory for receive/send buffers (DMA without staging). */
int wsg_host_alloc(size_t bytes, void** out);
int wsg_host_free(void* p);

/* ---- single-frame header helpers (host; same code the kernels run) ------ */
/* Total frame size PrepareSendFrame produces (ws.cpp:215-252).               */
uint64_t wsg_frame_size(uint8_t opcode, int mask, uint64_t len, int32_t status);
/* Write the header (ws.cpp:222-248) into out[0..14); returns its length.     */
int wsg_header_pack(uint8_t opcode, int mask, uint64_t len, int32_t status,
                    uint32_t key, uint8_t* out);
/* Parse a complete header at buf[0..avail) (ws.cpp:320-386).  Returns WSG_OK,
 * or WSG_ETRUNC when avail is too short for the header.                       */
int wsg_header_unpack(const uint8_t* buf, uint64_t avail, wsg_recv_info* info);

/* ---- upgrade handshake (host; reference ws.cpp:26-210) ------------------ */
/* Sec-WebSocket-Accept for a Sec-WebSocket-Key: Base64(SHA-1(key + RFC 6455
 * GUID)), NUL-terminated in out[0..29).                                       */
int wsg_ws_accept(const char* key, size_t key_len, char* out, size_t out_cap);

/* ---- per-connection session (the WebSocket mix-in, ws.h:29) ------------- */
/* A session is the reference's per-connection codec state; its payload
 * mask/unmask runs on the GPU through the owning ctx.                         */
typedef struct wsg_session wsg_session;
/* Receive callback: kind is WSG_CB_* ; status is the close status.           */
#define WSG_CB_RECEIVED 1   /* onWSReceived (ws.cpp:445-450) */
#define WSG_CB_CLOSE    2   /* onWSClose    (ws.cpp:429-443) */
#define WSG_CB_PING     3   /* onWSPing     (ws.cpp:417-421) */
#define WSG_CB_PONG     4   /* onWSPong     (ws.cpp:423-427) */
typedef void (*wsg_receive_cb)(void* user, int kind, const uint8_t* data,
                               size_t size, int status);
int wsg_session_create(wsg_ctx* ctx, wsg_session** out);
int wsg_session_destroy(wsg_session* s);
/* _ws_send_mask as little-endian uint32 (ws.cpp:97 client / :206 server).   */
int wsg_session_set_send_key(wsg_session* s, uint32_t key);
/* PrepareSendFrame (ws.cpp:212): frame copied to out[0..*out_len).           */
int wsg_session_prepare_send(wsg_session* s, uint8_t opcode, int mask,
                             const void* buf, size_t size, int32_t status,
                             uint8_t* out, size_t out_cap, size_t* out_len);
/* PrepareReceiveFrame (ws.cpp:273): callbacks fire synchronously.            */
int wsg_session_prepare_receive(wsg_session* s, const void* buf, size_t size,
                                wsg_receive_cb cb, void* user);
/* RequiredReceiveFrameSize (ws.cpp:458).                                      */
size_t wsg_session_required(wsg_session* s);
/* ClearWSBuffers (ws.cpp:484).                                                */
int wsg_session_clear(wsg_session* s);

/* ---- batched receive over many sessions ---------- */
/* The host framer + session batcher: wsg_rx_feed runs a session's framing
 * state machine (PrepareReceiveFrame's header half, ws.cpp:292-397, the
 * split-header behaviour of SURVEY Q7 included) and appends each completed
 * frame to one page-locked batch; wsg_rx_flush unmasks the batch in one GPU
 * pass (wsg_decode_batch_host) and delivers the frames in arrival order
 * through each session's message logic (ws.cpp:399-452).  Every session sees
 * the callbacks wsg_session_prepare_receive would have fired, in the same
 * order.  Callback data stays valid until the next flush.  One thread.      */
typedef struct wsg_rx wsg_rx;
typedef void (*wsg_rx_cb)(void* user, wsg_session* s, int kind,
                          const uint8_t* data, size_t size, int status);
int wsg_rx_create(wsg_ctx* ctx, wsg_rx** out);
int wsg_rx_destroy(wsg_rx* rx);
int wsg_rx_feed(wsg_rx* rx, wsg_session* s, const void* buf, size_t size);
/* ClearWSBuffers (ws.cpp:484) for a batched session, in delivery order.       */
int wsg_rx_clear(wsg_rx* rx, wsg_session* s);
/* Drop a session's queued frames (before wsg_session_destroy).                */
int wsg_rx_forget(wsg_rx* rx, wsg_session* s);
/* Spread every flush's GPU pass over these devices' PCIe links (one context
 * per device, owned by rx; wsg_decode_batch_host_multi); n = 0: rx's own ctx.
 * Not from inside a flush (WSG_EINVAL).                                       */
int wsg_rx_set_devices(wsg_rx* rx, const int* devices, int n);
/* Complete frames and wire bytes queued for the next flush.                   */
int wsg_rx_pending(wsg_rx* rx, uint32_t* frames, uint64_t* bytes);
int wsg_rx_flush(wsg_rx* rx, wsg_rx_cb cb, void* user, uint32_t* delivered);

/* ---- batched send over many sessions ------------- */
/* wsg_tx_queue records PrepareSendFrame(opcode, mask, buf, size, status) for
 * session s with its current send key (read under its send lock) and copies
 * the payload; wsg_tx_flush encodes every queued frame in one pipelined GPU
 * pass (wsg_encode_batch_host) and hands each frame to `sink` in queue order.
 * The bytes are those wsg_session_prepare_send would produce.  One thread.  */
typedef struct wsg_tx wsg_tx;
typedef void (*wsg_tx_sink)(void* user, wsg_session* s, const uint8_t* frame,
                            size_t size);
int wsg_tx_create(wsg_ctx* ctx, wsg_tx** out);
int wsg_tx_destroy(wsg_tx* tx);
int wsg_tx_queue(wsg_tx* tx, wsg_session* s, uint8_t opcode, int mask,
                 const void* buf, size_t size, int32_t status);
/* Drop a session's queued frames (before wsg_session_destroy).                */
int wsg_tx_forget(wsg_tx* tx, wsg_session* s);
/* The same for the send batch (wsg_encode_batch_host_multi).                 */
int wsg_tx_set_devices(wsg_tx* tx, const int* devices, int n);
int wsg_tx_pending(wsg_tx* tx, uint32_t* frames, uint64_t* payload_bytes);
int wsg_tx_flush(wsg_tx* tx, wsg_tx_sink sink, void* user, uint32_t* sent);

/* ---- multi-GPU: shard, encode, gather to one rank */
/* BASELINE config C5 (1 Mi x 16 KiB frames on the 8 GPUs of a node): the
 * reference has no GPU and no collective; a C++ server that owns a node calls
 * this instead of encoding every frame on its IO threads.  Chunks of `chunk`
 * consecutive frames are dealt round-robin, chunk c to rank c % world; a
 * rank's local batch is its chunks in order (wsg_mgpu_shard_count frames).
 * The gather runs over RCCL (xGMI), loaded at run time.                      */
typedef struct wsg_mgpu wsg_mgpu;
#define WSG_MGPU_ID_BYTES 128
/* One process driving `ndev` GPUs (one ctx and stream per device). */
int wsg_mgpu_create(const int* devices, int ndev, wsg_mgpu** out);
/* One rank of a multi-process group (one process per GPU): rank 0 makes the
 * id with wsg_mgpu_unique_id and the caller hands it to every rank.        */
int wsg_mgpu_unique_id(uint8_t* id);
int wsg_mgpu_create_rank(int device, const uint8_t* id, int rank, int world, wsg_mgpu** out);
int wsg_mgpu_destroy(wsg_mgpu* g);
/* world size, ranks driven by this process, the first of them */
int wsg_mgpu_info(wsg_mgpu* g, int* world, int* nlocal, int* first_rank);
/* codec context of local rank i (its device; wsg_stream gives its stream) */
wsg_ctx* wsg_mgpu_ctx(wsg_mgpu* g, int i);
/* frames of an n_total-frame job that `rank` owns */
uint64_t wsg_mgpu_shard_count(uint64_t n_total, uint32_t chunk, int world, int rank);
/* Encode every local rank's shard and gather the job's frames, in global
 * frame order, to rank `root`.  Arrays of nlocal entries, one per local rank
 * (device buffers on that rank's GPU): d_payload / d_desc / n_local its
 * shard (as wsg_encode_batch), d_wire / wire_cap / d_wire_off its encoded
 * shard (n_local + 1 offsets).  On the root: d_out (capacity out_cap) gets
 * the whole job's wire, d_out_off (n_total + 1, or NULL) its frame offsets.
 * Synchronous; every rank of the group calls it with the same n_total,
 * chunk and root.  times (or NULL): {encode ms, gather ms}, max over the
 * local ranks.                                                              */
int wsg_mgpu_encode_gather(wsg_mgpu* g, uint64_t n_total, uint32_t chunk, const uint8_t* const* d_payload,
                           const wsg_send_desc* const* d_desc, const uint32_t* n_local, uint8_t* const* d_wire,
                           const uint64_t* wire_cap, uint64_t* const* d_wire_off, int root, uint8_t* d_out,
                           uint64_t out_cap, uint64_t* d_out_off, double* times);

/* ---- host batches over several GPUs (one process, no collective) -------- */
/* The host-staged path is PCIe-bound (one x16 link per GPU): a server whose
 * receive/send buffers live in host memory (asio socket buffers) spreads one
 * batch over its GPUs' links.  The frames are cut into contiguous runs
 * of about equal wire bytes; run i goes through ctxs[i]'s host pipeline
 * (wsg_decode_batch_host / wsg_encode_batch_host) on a thread of its own,
 * all runs at once.  Results and status are those of the one-context call
 * on the whole batch (a frame table that is not strictly increasing takes
 * that call on ctxs[0]).  Each context is used by this call alone meanwhile.
 * Only the first context of each device takes a run: two pipelines on one
 * GPU share its link and copy engines and run slower than one
 * ($WSG_HOST_MULTI_SHARE=1 splits over every context given).               */
int wsg_decode_batch_host_multi(wsg_ctx* const* ctxs, int nctx, const uint8_t* wire, uint64_t wire_len,
                                const uint64_t* frame_start, uint32_t n, uint8_t* out, wsg_recv_info* info);
int wsg_encode_batch_host_multi(wsg_ctx* const* ctxs, int nctx, const uint8_t* payload, uint64_t payload_len,
                                const wsg_send_desc* desc, uint32_t n, uint8_t* wire, uint64_t wire_cap,
                                uint64_t* wire_off);
/* The same over the GPUs a wsg_mgpu group drives in this process (its local
 * ranks' contexts).                                                          */
int wsg_mgpu_decode_batch_host(wsg_mgpu* g, const uint8_t* wire, uint64_t wire_len, const uint64_t* frame_start,
                               uint32_t n, uint8_t* out, wsg_recv_info* info);
int wsg_mgpu_encode_batch_host(wsg_mgpu* g, const uint8_t* payload, uint64_t payload_len, const wsg_send_desc* desc,
                               uint32_t n, uint8_t* wire, uint64_t wire_cap, uint64_t* wire_off);

/* ---- kernel timing (measurement hook used by bench.py) ------------------ */
/* on = k > 0: the ctx records HIP events around the dominant payload kernel of
 * every k-th batch call, on the stream it is launched on (k > 1 keeps the
 * event packets' own cost out of most steps); on = 0 disables.               */
int wsg_timing_enable(wsg_ctx* ctx, int on);
/* Sum of the dominant-kernel durations (ms) and launch count since the last
 * reset; synchronizes outstanding events.                                     */
int wsg_timing_read(wsg_ctx* ctx, double* total_ms, uint64_t* launches, int reset);
/* Shortest and longest of those durations (ms) since the last reset (0, 0
 * when none); synchronizes outstanding events, resets nothing.              */
int wsg_timing_minmax(wsg_ctx* ctx, double* min_ms, double* max_ms);

/* ---- the host lane (measurement / test hook) ----------------------------- */
/* Page-locked host batches of at most $WSG_LANE_MAX wire bytes (default 512
 * KiB) whose frame table is strictly increasing, and wsg_xor_host calls of at
 * most that many bytes (and 64 KiB), go to the device's resident lane instead
 * of a launch and a synchronize per call (the C1 echo's reads; the per-call
 * path).  One lane per device serves every context of the process:
 * $WSG_LANE_WGS workgroups (default 8) on a high-priority stream, a mailbox
 * each in host memory; a request is cut into frame groups of about equal
 * bytes (one per idle workgroup, at most $WSG_LANE_GROUPS), each a run of at
 * most 1024 whole frames; a decode with a frame larger than a group's 64 KiB
 * stage, or a request needing more than 32 groups, takes the launch path.
 * A launch ends after $WSG_LANE_IDLE_US (default 2000)
 * without a task and after $WSG_LANE_YIELD_US (default 2000) of running (a
 * running kernel holds up calls that wait for the device to drain); the next
 * call launches it again.  A request unanswered for $WSG_LANE_TIMEOUT_MS
 * (default 5000) gives the lane up: the caller waits up to
 * $WSG_LANE_DRAIN_MS (default 2000) for it to leave and then takes the
 * launch path, or, if it does not leave, returns WSG_EHIP without touching
 * the buffers (the lane may still write them) and the context returns
 * WSG_EHIP from then on (a device free in another context, e.g. its
 * wsg_destroy, waits for that lane to leave).  A lane given up comes back on
 * a later call once it has left, no request is in flight and a hold-off has
 * passed (50 ms, doubling with each give-up in a row up to 4 s); tasks the
 * old lane never took are skipped, not run.  The lane's settings are read
 * when a process first uses a device's lane.
 * Requests this context put on the lane, the launches of the device's lane,
 * and whether it runs now (1), has left (0) or is given up (-1: the launch
 * paths until it comes back).                                               */
int wsg_lane_stats(wsg_ctx* ctx, uint64_t* requests, uint64_t* launches, int* running);
/* How often the device's lane was given up (a request unanswered for
 * $WSG_LANE_TIMEOUT_MS, or a launch that failed) and brought back since the
 * process first used it.                                                    */
int wsg_lane_events(wsg_ctx* ctx, uint64_t* give_ups, uint64_t* rearms);

#ifdef __cplusplus
}
#endif

#endif /* WSG_CAPI_H */
