/*
 * server/http/http_request.h — the subset of CppServer's HTTPRequest the
 * WebSocket upgrade uses (reference include/server/http/http_request.h:30-140):
 * request line + headers + body kept in one serialized cache, with views
 * into it.  The rest of the reference HTTP module (sessions, caching,
 * cookies, incremental ReceiveHeader/ReceiveBody) is out of scope.
 */
#ifndef CPPSERVER_AMD_HTTP_REQUEST_H
#define CPPSERVER_AMD_HTTP_REQUEST_H

#include <cstddef>
#include <string>
#include <string_view>
#include <tuple>
#include <vector>

namespace CppServer {
namespace HTTP {

class HTTPRequest
{
public:
    HTTPRequest() { Clear(); }
    HTTPRequest(std::string_view method, std::string_view url, std::string_view protocol = "HTTP/1.1")
    {
        SetBegin(method, url, protocol);
    }

    bool empty() const noexcept { return _cache.empty(); }
    bool error() const noexcept { return _error; }
    std::string_view method() const noexcept { return view(_method); }
    std::string_view url() const noexcept { return view(_url); }
    std::string_view protocol() const noexcept { return view(_protocol); }
    size_t headers() const noexcept { return _headers.size(); }
    std::tuple<std::string_view, std::string_view> header(size_t i) const noexcept;
    std::string_view body() const noexcept { return view(_body); }
    //! The serialized request (what goes on the wire)
    const std::string& cache() const noexcept { return _cache; }
    std::string string() const { return _cache; }

    HTTPRequest& Clear();
    HTTPRequest& SetBegin(std::string_view method, std::string_view url, std::string_view protocol = "HTTP/1.1");
    HTTPRequest& SetHeader(std::string_view key, std::string_view value);
    //! Content-Length header, the blank line, then the body
    HTTPRequest& SetBody(std::string_view body = "");

    //! Parse one request from the start of `data`: returns the bytes it
    //! spans (header block + Content-Length body), 0 if incomplete; sets
    //! error() on a malformed request line or header.
    size_t Parse(std::string_view data);

private:
    struct Span {
        size_t at = 0, size = 0;
    };
    std::string_view view(Span s) const noexcept { return std::string_view(_cache.data() + s.at, s.size); }
    bool _error = false;
    Span _method, _url, _protocol, _body;
    std::vector<std::pair<Span, Span>> _headers;
    std::string _cache;
};

} // namespace HTTP
} // namespace CppServer

#endif // CPPSERVER_AMD_HTTP_REQUEST_H
