/*
 * ws_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of CppServer's WebSocket frame codec (reference
 * chronoxor/CppServer 1.0.5.0, source/server/ws/ws.cpp:212-498), used as the
 * parity checker for the HIP path and as the timed CPU baseline in bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it.  The product library (cppserver_amd/) never links or calls it.
 *
 * Parity pinning: the reference path cannot be compiled here without stand-in
 * headers (ws.h pulls CppCommon's system/uuid.h, absent from the image), so
 * there is no oracle/_ref build.  This restatement is pinned instead by the
 * known-answer vectors in tests/golden/kat.json: the reference's own
 * observed outputs recorded in SURVEY.md §8a (Q1-Q7, [probe]), the
 * reference tests' byte-count expectations (tests/test_ws.cpp:142,212-262)
 * and the RFC 6455 §5.7 examples.
 */
#ifndef WS_ORACLE_H
#define WS_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/wsg_capi.h"   /* wsg_send_desc / wsg_recv_info layouts */

#ifdef __cplusplus
extern "C" {
#endif

typedef struct wso_session wso_session;

/* Event kinds recorded by the receive path (same values as WSG_CB_*). */
#define WSO_EV_RECEIVED 1
#define WSO_EV_CLOSE    2
#define WSO_EV_PING     3
#define WSO_EV_PONG     4

wso_session* wso_new(void);
void   wso_free(wso_session* s);
void   wso_set_send_key(wso_session* s, uint32_t key);
void   wso_clear(wso_session* s);                                   /* ws.cpp:484 */
size_t wso_prepare_send(wso_session* s, uint8_t opcode, int mask,
                        const void* buf, size_t size, int32_t status); /* ws.cpp:212 */
const uint8_t* wso_send_buffer(wso_session* s, size_t* len);
void   wso_prepare_receive(wso_session* s, const void* buf, size_t size); /* ws.cpp:273 */
size_t wso_required(wso_session* s);                                /* ws.cpp:458 */
/* Callbacks (ws.cpp:415-452's onWS* calls) instead of recorded events: the
 * payload pointer is borrowed until the callback returns, as in the
 * reference.  Used by the CPU-reference echo loop (tools/bench_echo_ref).  */
typedef void (*wso_callback)(void* user, int kind, const uint8_t* data, size_t len, int status);
void   wso_set_callback(wso_session* s, wso_callback cb, void* user);
/* Recorded callbacks (copies of the delivered bytes). */
size_t wso_event_count(wso_session* s);
int    wso_event(wso_session* s, size_t i, int* kind, int* status,
                 const uint8_t** data, size_t* len);
void   wso_events_clear(wso_session* s);
/* Introspection used by parity tests. */
const uint8_t* wso_final_buffer(wso_session* s, size_t* len);
uint32_t wso_recv_key(wso_session* s);

/* Batch restatements with the same contracts as the wsg_* device calls.    */
int wso_encode_batch(const uint8_t* payload, const wsg_send_desc* desc, uint32_t n,
                     uint8_t* wire, uint64_t wire_cap, uint64_t* wire_off);
int wso_decode_batch(const uint8_t* wire, uint64_t wire_len,
                     const uint64_t* frame_start, uint32_t n,
                     uint8_t* out, wsg_recv_info* info);
int wso_fanout_encode(const uint8_t* payload, uint64_t len, const uint32_t* keys,
                      uint32_t k, uint8_t opcode, int mask, uint8_t* wire, uint64_t wire_cap);

/* CPU baseline timing: decode (PrepareReceiveFrame, one whole frame per
 * call, as a socket read delivering it) of frames [0,n) by `threads` threads,
 * each owning a contiguous slice of frames as an independent session.
 * Returns the median seconds per full pass over `iters` passes.             */
double wso_time_decode(const uint8_t* wire, uint64_t wire_len,
                       const uint64_t* frame_start, uint32_t n,
                       int threads, int iters);
/* Same for encode (PrepareSendFrame per frame + append to the wire).        */
double wso_time_encode(const uint8_t* payload, const wsg_send_desc* desc, uint32_t n,
                       int threads, int iters);

#ifdef __cplusplus
}
#endif

#endif
