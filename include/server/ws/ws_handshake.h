/*
 * server/ws/ws_handshake.h — the arithmetic of the WebSocket upgrade
 * (reference ws.cpp:66-70, :155-159): Base64 (CppCommon::Encoding in the
 * reference) and the SHA-1 digest behind Sec-WebSocket-Accept.
 */
#ifndef CPPSERVER_AMD_WS_HANDSHAKE_H
#define CPPSERVER_AMD_WS_HANDSHAKE_H

#include <string>
#include <string_view>

namespace CppServer {
namespace WS {

std::string Base64Encode(std::string_view in);
//! Decodes the Base64 characters of `in`; anything else (padding, blanks) is skipped
std::string Base64Decode(std::string_view in);
//! SHA-1(key + "258EAFA5-E914-47DA-95CA-C5AB0DC85B11"), 20 raw bytes (RFC 6455 §1.3)
std::string WSAcceptDigest(std::string_view key);
//! Base64 of WSAcceptDigest: the Sec-WebSocket-Accept value for `key`
inline std::string WSAcceptKey(std::string_view key) { return Base64Encode(WSAcceptDigest(key)); }

} // namespace WS
} // namespace CppServer

#endif // CPPSERVER_AMD_WS_HANDSHAKE_H
