/*
 * server/http/http_response.h — the subset of CppServer's HTTPResponse the
 * WebSocket upgrade uses (reference include/server/http/http_response.h:30-160):
 * status line + headers + body in one serialized cache.  SetBegin(status)
 * takes the reference's status phrases; MakeErrorResponse matches
 * http_response.cpp:367-375.
 */
#ifndef CPPSERVER_AMD_HTTP_RESPONSE_H
#define CPPSERVER_AMD_HTTP_RESPONSE_H

#include <cstddef>
#include <string>
#include <string_view>
#include <tuple>
#include <vector>

namespace CppServer {
namespace HTTP {

class HTTPResponse
{
public:
    HTTPResponse() { Clear(); }
    HTTPResponse(int status, std::string_view protocol = "HTTP/1.1") { SetBegin(status, protocol); }

    bool empty() const noexcept { return _cache.empty(); }
    bool error() const noexcept { return _error; }
    int status() const noexcept { return _status; }
    std::string_view status_phrase() const noexcept { return view(_phrase); }
    std::string_view protocol() const noexcept { return view(_protocol); }
    size_t headers() const noexcept { return _headers.size(); }
    std::tuple<std::string_view, std::string_view> header(size_t i) const noexcept;
    std::string_view body() const noexcept { return view(_body); }
    const std::string& cache() const noexcept { return _cache; }
    std::string string() const { return _cache; }

    HTTPResponse& Clear();
    HTTPResponse& SetBegin(int status, std::string_view protocol = "HTTP/1.1");
    HTTPResponse& SetBegin(int status, std::string_view status_phrase, std::string_view protocol);
    HTTPResponse& SetHeader(std::string_view key, std::string_view value);
    HTTPResponse& SetBody(std::string_view body = "");
    HTTPResponse& MakeErrorResponse(int status, std::string_view content = "",
                                    std::string_view content_type = "text/plain; charset=UTF-8");

    //! Parse one response from the start of `data` (see HTTPRequest::Parse)
    size_t Parse(std::string_view data);

private:
    struct Span {
        size_t at = 0, size = 0;
    };
    std::string_view view(Span s) const noexcept { return std::string_view(_cache.data() + s.at, s.size); }
    bool _error = false;
    int _status = 0;
    Span _protocol, _phrase, _body;
    std::vector<std::pair<Span, Span>> _headers;
    std::string _cache;
};

} // namespace HTTP
} // namespace CppServer

#endif // CPPSERVER_AMD_HTTP_RESPONSE_H
