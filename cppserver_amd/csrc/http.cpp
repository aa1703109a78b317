// http.cpp — the HTTP request/response subset used by the WebSocket upgrade
// (include/server/http/*.h) and the handshake arithmetic: Base64 and the
// Sec-WebSocket-Accept digest (reference ws.cpp:66-70 / :155-159: SHA-1 of
// key + RFC 6455 GUID, OpenSSL as in the reference).  Host control plane.
#include "server/http/http_request.h"
#include "server/http/http_response.h"
#include "server/ws/ws_handshake.h"
#include "wsg_capi.h"

#include <openssl/evp.h>

#include <algorithm>
#include <cctype>
#include <cstring>
#include <map>

namespace CppServer {
namespace HTTP {

namespace {

std::string_view trim(std::string_view s)
{
    while (!s.empty() && (s.front() == ' ' || s.front() == '\t'))
        s.remove_prefix(1);
    while (!s.empty() && (s.back() == ' ' || s.back() == '\t'))
        s.remove_suffix(1);
    return s;
}

bool iequal(std::string_view a, std::string_view b)
{
    if (a.size() != b.size())
        return false;
    for (size_t i = 0; i < a.size(); ++i)
        if (std::tolower(static_cast<unsigned char>(a[i])) != std::tolower(static_cast<unsigned char>(b[i])))
            return false;
    return true;
}

// Header block [0, end) of `data` ("\r\n\r\n" included) or npos.
size_t header_end(std::string_view data)
{
    const size_t p = data.find("\r\n\r\n");
    return p == std::string_view::npos ? p : p + 4;
}

// Parse "Key: value" lines of `block` (starting after the first line) into
// spans relative to `base`; returns false on a line without ':'.
template <class Span>
bool parse_headers(std::string_view block, size_t base, std::vector<std::pair<Span, Span>>& out,
                   uint64_t& content_length)
{
    content_length = 0;
    size_t at = 0;
    while (at < block.size()) {
        const size_t eol = block.find("\r\n", at);
        const size_t end = eol == std::string_view::npos ? block.size() : eol;
        const std::string_view line = block.substr(at, end - at);
        if (!line.empty()) {
            const size_t colon = line.find(':');
            if (colon == std::string_view::npos || colon == 0)
                return false;
            const std::string_view key = trim(line.substr(0, colon));
            const std::string_view value = trim(line.substr(colon + 1));
            Span k{base + at + size_t(key.data() - line.data()), key.size()};
            Span v{base + at + size_t(value.data() - line.data()), value.size()};
            out.emplace_back(k, v);
            if (iequal(key, "Content-Length")) {
                content_length = 0;
                for (char c : value) {
                    if (c < '0' || c > '9')
                        return false;
                    content_length = content_length * 10 + uint64_t(c - '0');
                }
            }
        }
        at = end + 2;
    }
    return true;
}

const char* phrase_of(int status)
{
    static const std::map<int, const char*> table = {
        {100, "Continue"}, {101, "Switching Protocols"}, {102, "Processing"}, {103, "Early Hints"}, {200, "OK"},
        {201, "Created"}, {202, "Accepted"}, {203, "Non-Authoritative Information"}, {204, "No Content"},
        {205, "Reset Content"}, {206, "Partial Content"}, {207, "Multi-Status"}, {208, "Already Reported"},
        {226, "IM Used"}, {300, "Multiple Choices"}, {301, "Moved Permanently"}, {302, "Found"}, {303, "See Other"},
        {304, "Not Modified"}, {305, "Use Proxy"}, {306, "Switch Proxy"}, {307, "Temporary Redirect"},
        {308, "Permanent Redirect"}, {400, "Bad Request"}, {401, "Unauthorized"}, {402, "Payment Required"},
        {403, "Forbidden"}, {404, "Not Found"}, {405, "Method Not Allowed"}, {406, "Not Acceptable"},
        {407, "Proxy Authentication Required"}, {408, "Request Timeout"}, {409, "Conflict"}, {410, "Gone"},
        {411, "Length Required"}, {412, "Precondition Failed"}, {413, "Payload Too Large"}, {414, "URI Too Long"},
        {415, "Unsupported Media Type"}, {416, "Range Not Satisfiable"}, {417, "Expectation Failed"},
        {421, "Misdirected Request"}, {422, "Unprocessable Entity"}, {423, "Locked"}, {424, "Failed Dependency"},
        {425, "Too Early"}, {426, "Upgrade Required"}, {427, "Unassigned"}, {428, "Precondition Required"},
        {429, "Too Many Requests"}, {431, "Request Header Fields Too Large"}, {451, "Unavailable For Legal Reasons"},
        {500, "Internal Server Error"}, {501, "Not Implemented"}, {502, "Bad Gateway"}, {503, "Service Unavailable"},
        {504, "Gateway Timeout"}, {505, "HTTP Version Not Supported"}, {506, "Variant Also Negotiates"},
        {507, "Insufficient Storage"}, {508, "Loop Detected"}, {510, "Not Extended"},
        {511, "Network Authentication Required"}};
    const auto it = table.find(status);
    return it == table.end() ? "Unknown" : it->second;
}

} // namespace

// ---------------------------------------------------------------- request

std::tuple<std::string_view, std::string_view> HTTPRequest::header(size_t i) const noexcept
{
    if (i >= _headers.size())
        return {std::string_view(), std::string_view()};
    return {view(_headers[i].first), view(_headers[i].second)};
}

HTTPRequest& HTTPRequest::Clear()
{
    _error = false;
    _method = _url = _protocol = _body = Span{};
    _headers.clear();
    _cache.clear();
    return *this;
}

HTTPRequest& HTTPRequest::SetBegin(std::string_view method, std::string_view url, std::string_view protocol)
{
    Clear();
    _method = Span{_cache.size(), method.size()};
    _cache.append(method).append(" ");
    _url = Span{_cache.size(), url.size()};
    _cache.append(url).append(" ");
    _protocol = Span{_cache.size(), protocol.size()};
    _cache.append(protocol).append("\r\n");
    return *this;
}

HTTPRequest& HTTPRequest::SetHeader(std::string_view key, std::string_view value)
{
    Span k{_cache.size(), key.size()};
    _cache.append(key).append(": ");
    Span v{_cache.size(), value.size()};
    _cache.append(value).append("\r\n");
    _headers.emplace_back(k, v);
    return *this;
}

HTTPRequest& HTTPRequest::SetBody(std::string_view body)
{
    SetHeader("Content-Length", std::to_string(body.size()));
    _cache.append("\r\n");
    _body = Span{_cache.size(), body.size()};
    _cache.append(body);
    return *this;
}

size_t HTTPRequest::Parse(std::string_view data)
{
    Clear();
    const size_t hend = header_end(data);
    if (hend == std::string_view::npos)
        return 0;
    const size_t eol = data.find("\r\n");
    const std::string_view line = data.substr(0, eol);
    const size_t s1 = line.find(' '), s2 = line.rfind(' ');
    if (s1 == std::string_view::npos || s2 == s1) {
        _error = true;
        return hend;
    }
    uint64_t clen = 0;
    std::vector<std::pair<Span, Span>> hdrs;
    if (!parse_headers(data.substr(eol + 2, hend - 4 - eol), eol + 2, hdrs, clen)) {
        _error = true;
        return hend;
    }
    if (data.size() - hend < clen)
        return 0;
    _cache.assign(data.substr(0, hend + clen));
    _method = Span{0, s1};
    _url = Span{s1 + 1, s2 - s1 - 1};
    _protocol = Span{s2 + 1, line.size() - s2 - 1};
    _headers = std::move(hdrs);
    _body = Span{hend, size_t(clen)};
    return hend + size_t(clen);
}

// ---------------------------------------------------------------- response

std::tuple<std::string_view, std::string_view> HTTPResponse::header(size_t i) const noexcept
{
    if (i >= _headers.size())
        return {std::string_view(), std::string_view()};
    return {view(_headers[i].first), view(_headers[i].second)};
}

HTTPResponse& HTTPResponse::Clear()
{
    _error = false;
    _status = 0;
    _protocol = _phrase = _body = Span{};
    _headers.clear();
    _cache.clear();
    return *this;
}

HTTPResponse& HTTPResponse::SetBegin(int status, std::string_view protocol)
{
    return SetBegin(status, phrase_of(status), protocol);
}

HTTPResponse& HTTPResponse::SetBegin(int status, std::string_view status_phrase, std::string_view protocol)
{
    Clear();
    _protocol = Span{_cache.size(), protocol.size()};
    _cache.append(protocol).append(" ");
    _cache.append(std::to_string(status)).append(" ");
    _status = status;
    _phrase = Span{_cache.size(), status_phrase.size()};
    _cache.append(status_phrase).append("\r\n");
    return *this;
}

HTTPResponse& HTTPResponse::SetHeader(std::string_view key, std::string_view value)
{
    Span k{_cache.size(), key.size()};
    _cache.append(key).append(": ");
    Span v{_cache.size(), value.size()};
    _cache.append(value).append("\r\n");
    _headers.emplace_back(k, v);
    return *this;
}

HTTPResponse& HTTPResponse::SetBody(std::string_view body)
{
    SetHeader("Content-Length", std::to_string(body.size()));
    _cache.append("\r\n");
    _body = Span{_cache.size(), body.size()};
    _cache.append(body);
    return *this;
}

HTTPResponse& HTTPResponse::MakeErrorResponse(int status, std::string_view content, std::string_view content_type)
{
    Clear();
    SetBegin(status);
    if (!content_type.empty())
        SetHeader("Content-Type", content_type);
    SetBody(content);
    return *this;
}

size_t HTTPResponse::Parse(std::string_view data)
{
    Clear();
    const size_t hend = header_end(data);
    if (hend == std::string_view::npos)
        return 0;
    const size_t eol = data.find("\r\n");
    const std::string_view line = data.substr(0, eol);
    const size_t s1 = line.find(' ');
    const size_t s2 = s1 == std::string_view::npos ? s1 : line.find(' ', s1 + 1);
    int status = 0;
    bool ok = s1 != std::string_view::npos && s1 > 0;
    const size_t st_end = s2 == std::string_view::npos ? line.size() : s2;
    for (size_t i = s1 + 1; ok && i < st_end; ++i) {
        ok = line[i] >= '0' && line[i] <= '9';
        status = status * 10 + (line[i] - '0');
    }
    ok = ok && st_end - s1 - 1 == 3;
    uint64_t clen = 0;
    std::vector<std::pair<Span, Span>> hdrs;
    if (!ok || !parse_headers(data.substr(eol + 2, hend - 4 - eol), eol + 2, hdrs, clen)) {
        _error = true;
        return hend;
    }
    if (data.size() - hend < clen)
        return 0;
    _cache.assign(data.substr(0, hend + clen));
    _status = status;
    _protocol = Span{0, s1};
    _phrase = s2 == std::string_view::npos ? Span{line.size(), 0} : Span{s2 + 1, line.size() - s2 - 1};
    _headers = std::move(hdrs);
    _body = Span{hend, size_t(clen)};
    return hend + size_t(clen);
}

} // namespace HTTP

// ---------------------------------------------------------------- handshake arithmetic

namespace WS {

std::string Base64Encode(std::string_view in)
{
    static const char* abc = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    std::string out;
    out.reserve((in.size() + 2) / 3 * 4);
    size_t i = 0;
    for (; i + 3 <= in.size(); i += 3) {
        const uint32_t v = uint32_t(uint8_t(in[i])) << 16 | uint32_t(uint8_t(in[i + 1])) << 8 | uint8_t(in[i + 2]);
        out.push_back(abc[v >> 18]);
        out.push_back(abc[(v >> 12) & 63]);
        out.push_back(abc[(v >> 6) & 63]);
        out.push_back(abc[v & 63]);
    }
    if (const size_t rest = in.size() - i) {
        const uint32_t v = uint32_t(uint8_t(in[i])) << 16 | (rest == 2 ? uint32_t(uint8_t(in[i + 1])) << 8 : 0u);
        out.push_back(abc[v >> 18]);
        out.push_back(abc[(v >> 12) & 63]);
        out.push_back(rest == 2 ? abc[(v >> 6) & 63] : '=');
        out.push_back('=');
    }
    return out;
}

std::string Base64Decode(std::string_view in)
{
    auto val = [](char c) -> int {
        if (c >= 'A' && c <= 'Z')
            return c - 'A';
        if (c >= 'a' && c <= 'z')
            return c - 'a' + 26;
        if (c >= '0' && c <= '9')
            return c - '0' + 52;
        if (c == '+')
            return 62;
        if (c == '/')
            return 63;
        return -1;
    };
    std::string out;
    uint32_t acc = 0;
    int bits = 0;
    for (char c : in) {
        const int v = val(c);
        if (v < 0)
            continue;   // padding and whitespace carry no bits
        acc = (acc << 6) | uint32_t(v);
        bits += 6;
        if (bits >= 8) {
            bits -= 8;
            out.push_back(char((acc >> bits) & 0xFF));
        }
    }
    return out;
}

std::string WSAcceptDigest(std::string_view key)
{
    static const char guid[] = "258EAFA5-E914-47DA-95CA-C5AB0DC85B11";   // RFC 6455 §1.3
    std::string s(key);
    s.append(guid);
    unsigned char md[EVP_MAX_MD_SIZE];
    unsigned int n = 0;
    if (EVP_Digest(s.data(), s.size(), md, &n, EVP_sha1(), nullptr) != 1 || n != 20)
        return std::string();
    return std::string(reinterpret_cast<const char*>(md), n);
}

} // namespace WS
} // namespace CppServer

extern "C" int wsg_ws_accept(const char* key, size_t key_len, char* out, size_t out_cap)
{
    if ((key_len && !key) || !out)
        return WSG_EINVAL;
    const std::string a = CppServer::WS::WSAcceptKey(std::string_view(key ? key : "", key_len));
    if (a.empty())
        return WSG_EINVAL;
    if (out_cap < a.size() + 1)
        return WSG_ENOMEM;
    std::memcpy(out, a.c_str(), a.size() + 1);
    return WSG_OK;
}
