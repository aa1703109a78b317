// ws_oracle.cpp — TEST INFRASTRUCTURE ONLY (see ws_oracle.h).
//
// A restatement, written from a reading of the reference, of CppServer's
// per-connection WebSocket codec: PrepareSendFrame (ws.cpp:212-271),
// PrepareReceiveFrame (ws.cpp:273-456), RequiredReceiveFrameSize
// (ws.cpp:458-482) and ClearWSBuffers (ws.cpp:484-498).  It keeps the
// reference's container behaviour (std::vector growth, byte-at-a-time XOR)
// because bench.py times it as the CPU baseline, and it keeps every quirk
// listed in SURVEY.md §8a (Q1-Q7) because the HIP path must be bit-exact with
// the reference, not with RFC 6455.
#include "ws_oracle.h"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <pthread.h>
#include <sched.h>
#include <thread>
#include <vector>

namespace {

struct Event {
    int kind;
    int status;
    std::vector<uint8_t> bytes;
};

// Per-connection codec state: the fields of ws.h:168-196.
struct Conn {
    // receive side
    uint8_t cur_opcode = 0;          // _ws_opcode (uninitialised in the reference; 0 here)
    bool frame_done = false;         // _ws_frame_received
    bool message_done = false;       // _ws_final_received
    size_t hdr_size = 0;             // _ws_header_size
    size_t body_size = 0;            // _ws_payload_size
    std::vector<uint8_t> frame;      // _ws_receive_frame_buffer (header + payload as received)
    std::vector<uint8_t> message;    // _ws_receive_final_buffer (unmasked payloads)
    uint8_t rkey[4] = {0, 0, 0, 0};  // _ws_receive_mask
    // send side
    std::vector<uint8_t> out;        // _ws_send_buffer
    uint8_t skey[4] = {0, 0, 0, 0};  // _ws_send_mask
    // recorded callbacks
    bool record = true;
    std::vector<Event> events;
    wso_callback cb = nullptr;       // set: callbacks instead of recorded events
    void* user = nullptr;
    size_t delivered = 0;            // byte counter used by the timing loop

    void reset_frame()
    {
        frame_done = false;
        hdr_size = 0;
        body_size = 0;
        frame.clear();
        std::memset(rkey, 0, 4);
    }
    void reset_message()
    {
        message_done = false;
        message.clear();
    }

    // ws.cpp:484-498
    void clear()
    {
        reset_frame();
        reset_message();
        out.clear();
        std::memset(skey, 0, 4);
    }

    // ws.cpp:212-271.  Status prefix test is (opcode & CLOSE) == CLOSE, which
    // also matches PING/PONG (Q2); the XOR runs even when mask == false (Q1).
    void encode(uint8_t opcode, bool mask, const uint8_t* data, size_t size, int status)
    {
        const bool prefix = ((opcode & WSG_CLOSE) == WSG_CLOSE) && (size > 0 || status != 0);
        const size_t body = size + (prefix ? 2 : 0);
        const uint8_t mbit = mask ? 0x80 : 0x00;

        out.clear();
        out.push_back(opcode);
        if (body < 126) {
            out.push_back(static_cast<uint8_t>(body) | mbit);
        } else if (body < 65536) {
            out.push_back(126 | mbit);
            out.push_back(static_cast<uint8_t>(body >> 8));
            out.push_back(static_cast<uint8_t>(body));
        } else {
            out.push_back(127 | mbit);
            for (int sh = 56; sh >= 0; sh -= 8)
                out.push_back(static_cast<uint8_t>(body >> sh));
        }
        if (mask)
            for (int j = 0; j < 4; ++j)
                out.push_back(skey[j]);

        const size_t base = out.size();
        out.resize(base + body);
        size_t pos = 0;
        if (prefix) {
            out[base + 0] = static_cast<uint8_t>((status >> 8) & 0xFF) ^ skey[0];
            out[base + 1] = static_cast<uint8_t>(status & 0xFF) ^ skey[1];
            pos = 2;
        }
        // key index counts payload positions from the frame's payload start,
        // status bytes included (Q3)
        for (; pos < body; ++pos)
            out[base + pos] = data[pos - (prefix ? 2 : 0)] ^ skey[pos % 4];
    }

    void deliver(int kind, const uint8_t* p, size_t n, int status)
    {
        delivered += n;
        if (cb) {   // the onWS* callback: a borrowed pointer, as the reference hands out
            cb(user, kind, p, n, status);
            return;
        }
        if (record)
            events.push_back(Event{kind, status, std::vector<uint8_t>(p, p + n)});
    }

    // Append exactly `want` more bytes of the input to the frame buffer, or
    // consume everything that is left and report failure.  Each header field
    // is pulled with its full width whatever the frame buffer already holds,
    // which is the reference's split-header behaviour (Q7, ws.cpp:312,340,358,378).
    bool pull(const uint8_t*& p, size_t& n, size_t want, uint8_t* mirror = nullptr)
    {
        for (size_t k = 0; k < want; ++k) {
            if (n == 0)
                return false;
            frame.push_back(*p);
            if (mirror)
                mirror[k] = *p;
            ++p;
            --n;
        }
        return true;
    }

    // ws.cpp:273-456
    void decode(const uint8_t* p, size_t n)
    {
        if (frame_done)
            reset_frame();
        if (message_done)
            reset_message();

        while (n > 0) {
            if (frame_done)
                reset_frame();
            if (message_done)
                reset_message();

            if (frame.size() < 2 && !pull(p, n, 2))
                return;

            const uint8_t b0 = frame[0], b1 = frame[1];
            const bool fin = (b0 & 0x80) != 0;
            const bool masked = (b1 & 0x80) != 0;
            const uint8_t op = b0 & 0x0F;
            size_t len = b1 & 0x7F;
            if (op != 0)
                cur_opcode = op;

            size_t field = 0;   // bytes of extended length
            if (len == 126)
                field = 2;
            else if (len == 127)
                field = 8;
            if (field != 0) {
                if (frame.size() < 2 + field && !pull(p, n, field))
                    return;
                len = 0;
                for (size_t k = 0; k < field; ++k)
                    len = (len << 8) | frame[2 + k];
            }
            hdr_size = 2 + field + (masked ? 4 : 0);
            body_size = len;
            frame.reserve(hdr_size + body_size);
            message.reserve(hdr_size + body_size);

            if (masked && frame.size() < hdr_size && !pull(p, n, 4, rkey))
                return;

            const size_t total = hdr_size + body_size;
            const size_t take = std::min(total - frame.size(), n);
            frame.insert(frame.end(), p, p + take);
            p += take;
            n -= take;

            if (frame.size() != total)
                continue;

            if (masked) {
                for (size_t i = 0; i < body_size; ++i)
                    message.push_back(frame[hdr_size + i] ^ rkey[i % 4]);
            } else {
                message.insert(message.end(), frame.begin() + hdr_size, frame.end());
            }
            frame_done = true;
            if (!fin)
                continue;
            message_done = true;
            switch (cur_opcode) {
            case WSG_PING:
                deliver(WSO_EV_PING, message.data(), message.size(), 0);
                break;
            case WSG_PONG:
                deliver(WSO_EV_PONG, message.data(), message.size(), 0);
                break;
            case WSG_CLOSE: {
                int st = 1000;
                size_t skip = 0;
                if (message.size() >= 2) {
                    st = (message[0] << 8) | message[1];
                    skip = 2;
                }
                deliver(WSO_EV_CLOSE, message.data() + skip, message.size() - skip, st);
                break;
            }
            case WSG_TEXT:
            case WSG_BINARY:
                deliver(WSO_EV_RECEIVED, message.data(), message.size(), 0);
                break;
            default:
                break;   // other opcodes: accumulated, no callback (Q6)
            }
        }
    }

    // ws.cpp:458-482
    size_t need() const
    {
        if (frame_done)
            return 0;
        if (frame.size() < 2)
            return 2 - frame.size();
        const bool masked = (frame[1] & 0x80) != 0;
        const size_t len7 = frame[1] & 0x7F;
        if (len7 == 126 && frame.size() < 4)
            return 4 - frame.size();
        if (len7 == 127 && frame.size() < 10)
            return 10 - frame.size();
        if (masked && frame.size() < hdr_size)
            return hdr_size - frame.size();
        return hdr_size + body_size - frame.size();
    }
};

inline uint32_t le32(const uint8_t k[4])
{
    return uint32_t(k[0]) | uint32_t(k[1]) << 8 | uint32_t(k[2]) << 16 | uint32_t(k[3]) << 24;
}
inline void set_le32(uint8_t k[4], uint32_t v)
{
    for (int j = 0; j < 4; ++j)
        k[j] = static_cast<uint8_t>(v >> (8 * j));
}

// Header validity of one frame of a batch, independent of any session:
// returns 0 and the total frame size, or an error code.
int frame_extent(const uint8_t* wire, uint64_t wire_len, uint64_t start, uint64_t limit,
                 uint64_t* total)
{
    if (start >= wire_len || wire_len - start < 2)
        return WSG_ETRUNC;
    const uint8_t b1 = wire[start + 1];
    uint64_t field = (b1 & 0x7F) == 126 ? 2 : (b1 & 0x7F) == 127 ? 8 : 0;
    uint64_t hdr = 2 + field + ((b1 & 0x80) ? 4 : 0);
    if (wire_len - start < hdr)
        return WSG_ETRUNC;
    uint64_t len = b1 & 0x7F;
    if (field) {
        len = 0;
        for (uint64_t k = 0; k < field; ++k)
            len = (len << 8) | wire[start + 2 + k];
    }
    if (len > wire_len - start - hdr)
        return WSG_ETRUNC;
    if (start + hdr + len > limit)
        return WSG_EINVAL;
    *total = hdr + len;
    return 0;
}

void pin_to_allowed_cpu(int idx)
{
    cpu_set_t allowed;
    if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0)
        return;
    int seen = 0;
    for (int c = 0; c < CPU_SETSIZE; ++c) {
        if (!CPU_ISSET(c, &allowed))
            continue;
        if (seen++ == idx) {
            cpu_set_t one;
            CPU_ZERO(&one);
            CPU_SET(c, &one);
            pthread_setaffinity_np(pthread_self(), sizeof(one), &one);
            return;
        }
    }
}

template <class Body>
double median_parallel_seconds(int threads, int iters, Body body)
{
    if (threads < 1)
        threads = 1;
    if (iters < 1)
        iters = 1;
    std::vector<double> samples;
    for (int it = 0; it < iters; ++it) {
        std::vector<std::thread> pool;
        std::vector<double> secs(threads, 0.0);
        for (int t = 0; t < threads; ++t) {
            pool.emplace_back([&, t]() {
                pin_to_allowed_cpu(t);
                auto t0 = std::chrono::steady_clock::now();
                body(t, threads);
                auto t1 = std::chrono::steady_clock::now();
                secs[t] = std::chrono::duration<double>(t1 - t0).count();
            });
        }
        for (auto& th : pool)
            th.join();
        samples.push_back(*std::max_element(secs.begin(), secs.end()));
    }
    std::sort(samples.begin(), samples.end());
    return samples[samples.size() / 2];
}

} // namespace

struct wso_session {
    Conn c;
};

extern "C" {

wso_session* wso_new(void) { return new wso_session(); }
void wso_free(wso_session* s) { delete s; }
void wso_set_send_key(wso_session* s, uint32_t key) { set_le32(s->c.skey, key); }

void wso_set_callback(wso_session* s, wso_callback cb, void* user)
{
    s->c.cb = cb;
    s->c.user = user;
}
void wso_clear(wso_session* s) { s->c.clear(); }

size_t wso_prepare_send(wso_session* s, uint8_t opcode, int mask, const void* buf, size_t size,
                        int32_t status)
{
    s->c.encode(opcode, mask != 0, static_cast<const uint8_t*>(buf), size, status);
    return s->c.out.size();
}

const uint8_t* wso_send_buffer(wso_session* s, size_t* len)
{
    *len = s->c.out.size();
    return s->c.out.data();
}

void wso_prepare_receive(wso_session* s, const void* buf, size_t size)
{
    s->c.decode(static_cast<const uint8_t*>(buf), size);
}

size_t wso_required(wso_session* s) { return s->c.need(); }
size_t wso_event_count(wso_session* s) { return s->c.events.size(); }

int wso_event(wso_session* s, size_t i, int* kind, int* status, const uint8_t** data, size_t* len)
{
    if (i >= s->c.events.size())
        return WSG_EINVAL;
    const Event& e = s->c.events[i];
    *kind = e.kind;
    *status = e.status;
    *data = e.bytes.data();
    *len = e.bytes.size();
    return 0;
}

void wso_events_clear(wso_session* s) { s->c.events.clear(); }

const uint8_t* wso_final_buffer(wso_session* s, size_t* len)
{
    *len = s->c.message.size();
    return s->c.message.data();
}

uint32_t wso_recv_key(wso_session* s) { return le32(s->c.rkey); }

int wso_encode_batch(const uint8_t* payload, const wsg_send_desc* desc, uint32_t n, uint8_t* wire,
                     uint64_t wire_cap, uint64_t* wire_off)
{
    Conn c;
    c.record = false;
    uint64_t at = 0;
    for (uint32_t i = 0; i < n; ++i) {
        set_le32(c.skey, desc[i].key);
        c.encode(desc[i].opcode, desc[i].mask != 0, payload + desc[i].src_off, desc[i].len,
                 desc[i].status);
        wire_off[i] = at;
        if (c.out.size() > wire_cap - std::min<uint64_t>(at, wire_cap))
            return WSG_ENOMEM;
        std::memcpy(wire + at, c.out.data(), c.out.size());
        at += c.out.size();
    }
    wire_off[n] = at;
    return 0;
}

int wso_decode_batch(const uint8_t* wire, uint64_t wire_len, const uint64_t* frame_start,
                     uint32_t n, uint8_t* out, wsg_recv_info* info)
{
    if (out != wire)
        std::memcpy(out, wire, wire_len);
    Conn c;
    c.record = false;
    int first_err = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t start = frame_start[i];
        const uint64_t limit = (i + 1 < n) ? frame_start[i + 1] : wire_len;
        wsg_recv_info r;
        std::memset(&r, 0, sizeof(r));
        uint64_t total = 0;
        int err = frame_extent(wire, wire_len, start, limit, &total);
        if (err) {
            r.payload_off = start;
            r.error = static_cast<int8_t>(err);
            info[i] = r;
            if (!first_err)
                first_err = err;
            c.reset_frame();
            c.reset_message();
            continue;
        }
        // frame the stream exactly as the sync receive loop does
        // (ws_client.cpp:139-151): reset, then feed RequiredReceiveFrameSize bytes
        c.decode(nullptr, 0);
        const size_t before = c.message.size();
        uint64_t at = start;
        while (!c.frame_done) {
            size_t want = c.need();
            c.decode(wire + at, want);
            at += want;
        }
        r.payload_off = start + c.hdr_size;
        r.len = c.body_size;
        r.key = le32(c.rkey);
        r.b0 = c.frame[0];
        r.opcode = c.frame[0] & 0x0F;
        r.fin = c.frame[0] >> 7;
        r.masked = c.frame[1] >> 7;
        r.hdr_len = static_cast<uint8_t>(c.hdr_size);
        info[i] = r;
        std::memcpy(out + r.payload_off, c.message.data() + before, c.body_size);
    }
    return first_err;
}

int wso_fanout_encode(const uint8_t* payload, uint64_t len, const uint32_t* keys, uint32_t k,
                      uint8_t opcode, int mask, uint8_t* wire, uint64_t wire_cap)
{
    Conn c;
    c.record = false;
    uint64_t at = 0;
    for (uint32_t j = 0; j < k; ++j) {
        set_le32(c.skey, keys[j]);
        c.encode(opcode, mask != 0, payload, len, 0);
        if (c.out.size() > wire_cap - std::min<uint64_t>(at, wire_cap))
            return WSG_ENOMEM;
        std::memcpy(wire + at, c.out.data(), c.out.size());
        at += c.out.size();
    }
    return 0;
}

double wso_time_decode(const uint8_t* wire, uint64_t wire_len, const uint64_t* frame_start,
                       uint32_t n, int threads, int iters)
{
    return median_parallel_seconds(threads, iters, [&](int t, int nt) {
        const uint32_t lo = uint32_t(uint64_t(n) * t / nt);
        const uint32_t hi = uint32_t(uint64_t(n) * (t + 1) / nt);
        Conn c;   // one session per thread: an independent connection
        c.record = false;
        for (uint32_t i = lo; i < hi; ++i) {
            const uint64_t end = (i + 1 < n) ? frame_start[i + 1] : wire_len;
            c.decode(wire + frame_start[i], end - frame_start[i]);
        }
        volatile size_t sink = c.delivered;
        (void)sink;
    });
}

double wso_time_encode(const uint8_t* payload, const wsg_send_desc* desc, uint32_t n, int threads,
                       int iters)
{
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i)
        total += desc[i].len + 16;
    std::vector<uint8_t> wire(total);
    return median_parallel_seconds(threads, iters, [&](int t, int nt) {
        const uint32_t lo = uint32_t(uint64_t(n) * t / nt);
        const uint32_t hi = uint32_t(uint64_t(n) * (t + 1) / nt);
        uint64_t at = 0;
        for (uint32_t i = 0; i < lo; ++i)
            at += desc[i].len + 16;
        Conn c;
        c.record = false;
        for (uint32_t i = lo; i < hi; ++i) {
            set_le32(c.skey, desc[i].key);
            c.encode(desc[i].opcode, desc[i].mask != 0, payload + desc[i].src_off, desc[i].len,
                     desc[i].status);
            std::memcpy(wire.data() + at, c.out.data(), c.out.size());
            at += c.out.size();
        }
    });
}

} // extern "C"
