// wsg_frame.h — RFC 6455 frame arithmetic as CppServer implements it, shared
// by the host entry points and the gfx950 kernels (one source of truth).
//
// Reference: source/server/ws/ws.cpp:212-271 (PrepareSendFrame) and
// :309-386 (header half of PrepareReceiveFrame).
#pragma once

#include <stdint.h>

#include "wsg_capi.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define WSG_HD __host__ __device__ __forceinline__
#else
// the host-only WebSocket classes (and their g++ sanitizer builds) use the
// same arithmetic without the HIP headers
#define WSG_HD inline
#endif

namespace wsg {

// Close-status prefix rule, ws.cpp:215: (opcode & CLOSE) == CLOSE also holds
// for PING (0x09) and PONG (0x0A) — reproduced on purpose.
WSG_HD bool has_status_prefix(uint8_t opcode, uint64_t len, int32_t status)
{
    return ((opcode & WSG_CLOSE) == WSG_CLOSE) && (len > 0 || status != 0);
}

// Geometry of one frame PrepareSendFrame would emit.
struct SendGeom {
    uint64_t body;     // payload length on the wire (status prefix included)
    uint32_t hdr;      // header bytes: 2/4/10 (+4 when masked)
    uint32_t prefix;   // 2 when the close status is prepended, else 0
};

WSG_HD SendGeom send_geom(uint8_t opcode, bool mask, uint64_t len, int32_t status)
{
    SendGeom g;
    g.prefix = has_status_prefix(opcode, len, status) ? 2u : 0u;
    g.body = len + g.prefix;
    g.hdr = (g.body < 126 ? 2u : g.body < 65536 ? 4u : 10u) + (mask ? 4u : 0u);
    return g;
}

WSG_HD uint8_t key_byte(uint32_t key, uint64_t pos) { return uint8_t(key >> (8u * uint32_t(pos & 3u))); }

// Key word for 4 payload bytes starting at a position congruent to `phase`
// (mod 4), little-endian: byte j uses key[(phase + j) % 4] (ws.cpp:270, :403).
WSG_HD uint32_t key_rot(uint32_t key, uint32_t phase)
{
    const uint32_t s = 8u * (phase & 3u);
    return s ? (key >> s) | (key << (32u - s)) : key;
}

// Byte r (< hdr) of the header PrepareSendFrame writes (ws.cpp:222-248).
WSG_HD uint8_t header_byte(uint8_t opcode, bool mask, uint64_t body, uint32_t key, uint32_t r)
{
    if (r == 0)
        return opcode;
    const uint8_t mbit = mask ? 0x80 : 0x00;
    const uint32_t ext = body < 126 ? 0u : body < 65536 ? 2u : 8u;
    if (r == 1)
        return uint8_t((ext == 0 ? uint8_t(body) : ext == 2 ? uint8_t(126) : uint8_t(127)) | mbit);
    if (r < 2 + ext)
        return uint8_t(body >> (8u * (ext - 1u - (r - 2u))));   // big-endian length
    return key_byte(key, r - 2u - ext);                          // mask key bytes
}

// Parse a complete header at h[0..avail).  Returns 0 or WSG_ETRUNC.
// Matches ws.cpp:320-386 for a header delivered whole.
template <class Load>
WSG_HD int parse_header(Load byte_at, uint64_t avail, wsg_recv_info& r)
{
    if (avail < 2)
        return WSG_ETRUNC;
    const uint8_t b0 = byte_at(0), b1 = byte_at(1);
    const uint32_t ext = (b1 & 0x7F) == 126 ? 2u : (b1 & 0x7F) == 127 ? 8u : 0u;
    const uint32_t masked = (b1 >> 7) & 1u;
    const uint32_t hdr = 2u + ext + 4u * masked;
    if (avail < hdr)
        return WSG_ETRUNC;
    uint64_t len = b1 & 0x7F;
    if (ext) {
        len = 0;
        for (uint32_t k = 0; k < ext; ++k)
            len = (len << 8) | byte_at(2 + k);
    }
    uint32_t key = 0;
    if (masked)
        for (uint32_t k = 0; k < 4; ++k)
            key |= uint32_t(byte_at(2 + ext + k)) << (8u * k);
    r.len = len;
    r.key = key;
    r.b0 = b0;
    r.opcode = b0 & 0x0F;
    r.fin = b0 >> 7;
    r.masked = uint8_t(masked);
    r.hdr_len = uint8_t(hdr);
    r.error = 0;
    return 0;
}

} // namespace wsg
