// ws_session_impl.h — the C-ABI session object (wsg_session, include/wsg_capi.h):
// a WebSocket whose onWS* callbacks go to a C function pointer.  Shared by
// the per-connection entry points (ws.cpp) and the batched receive (ws_batch.cpp).
#pragma once

#include "server/ws/ws.h"

#include <mutex>
#include <vector>

// Callback target while wsg_rx_flush delivers frames on this thread: the
// batch's callback (which also gets the session) instead of the per-call one.
struct wsg_rx_dispatch {
    wsg_rx_cb cb = nullptr;
    void* user = nullptr;
};
extern thread_local wsg_rx_dispatch g_rx_dispatch;

struct wsg_session : public CppServer::WS::WebSocket {
    explicit wsg_session(wsg_ctx* c) : WebSocket(c) {}
    wsg_receive_cb cb = nullptr;
    void* user = nullptr;

    void emit(int kind, const void* b, size_t n, int status)
    {
        if (g_rx_dispatch.cb)
            g_rx_dispatch.cb(g_rx_dispatch.user, this, kind, static_cast<const uint8_t*>(b), n, status);
        else if (cb)
            cb(user, kind, static_cast<const uint8_t*>(b), n, status);
    }
    void onWSReceived(const void* b, size_t n) override { emit(WSG_CB_RECEIVED, b, n, 0); }
    void onWSClose(const void* b, size_t n, int status) override { emit(WSG_CB_CLOSE, b, n, status); }
    void onWSPing(const void* b, size_t n) override { emit(WSG_CB_PING, b, n, 0); }
    void onWSPong(const void* b, size_t n) override { emit(WSG_CB_PONG, b, n, 0); }

    std::mutex& send_lock() { return _ws_send_lock; }
    const std::vector<uint8_t>& send_buffer() const { return _ws_send_buffer; }
};
