/*
 * server/ws/ws_common.h — the two CppCommon value types the reference WS API
 * names in its signatures: CppCommon::Timespan (the timeout overloads of
 * Send* / Receive*, reference include/server/ws/ws_client.h:55-96,
 * ws_session.h:48-89) and CppCommon::UUID (the connection id of
 * PerformClientUpgrade, reference include/server/ws/ws.h:62).
 *
 * A program that already builds against CppCommon keeps its own types (its
 * headers are found on the include path and used as they are).  Without
 * CppCommon, minimal value types with the same names, constructors and
 * accessors stand in, so that code written against the reference compiles
 * unchanged.  $WSG_NO_CPPCOMMON (a -D flag) forces the stand-ins.
 */
#ifndef CPPSERVER_AMD_WS_COMMON_H
#define CPPSERVER_AMD_WS_COMMON_H

#if !defined(WSG_NO_CPPCOMMON) && __has_include("time/timespan.h") && __has_include("system/uuid.h")
#include "system/uuid.h"
#include "time/timespan.h"
#else
#include <array>
#include <chrono>
#include <cstdint>
#include <random>
#include <string>

namespace CppCommon {

//! Time span in nanoseconds (CppCommon/time/timespan.h)
class Timespan
{
public:
    Timespan() noexcept : _duration(0) {}
    explicit Timespan(int64_t duration) noexcept : _duration(duration) {}
    template <class Rep, class Period>
    explicit Timespan(const std::chrono::duration<Rep, Period>& d) noexcept
        : _duration(std::chrono::duration_cast<std::chrono::nanoseconds>(d).count())
    {
    }

    int64_t days() const noexcept { return _duration / (24 * 3600 * 1000000000ll); }
    int64_t hours() const noexcept { return _duration / (3600 * 1000000000ll); }
    int64_t minutes() const noexcept { return _duration / (60 * 1000000000ll); }
    int64_t seconds() const noexcept { return _duration / 1000000000; }
    int64_t milliseconds() const noexcept { return _duration / 1000000; }
    int64_t microseconds() const noexcept { return _duration / 1000; }
    int64_t nanoseconds() const noexcept { return _duration; }
    int64_t total() const noexcept { return _duration; }
    std::chrono::nanoseconds chrono() const noexcept { return std::chrono::nanoseconds(_duration); }

    static Timespan days(int64_t v) noexcept { return Timespan(v * 24 * 3600 * 1000000000ll); }
    static Timespan hours(int64_t v) noexcept { return Timespan(v * 3600 * 1000000000ll); }
    static Timespan minutes(int64_t v) noexcept { return Timespan(v * 60 * 1000000000ll); }
    static Timespan seconds(int64_t v) noexcept { return Timespan(v * 1000000000); }
    static Timespan milliseconds(int64_t v) noexcept { return Timespan(v * 1000000); }
    static Timespan microseconds(int64_t v) noexcept { return Timespan(v * 1000); }
    static Timespan nanoseconds(int64_t v) noexcept { return Timespan(v); }
    static Timespan zero() noexcept { return Timespan(0); }

    friend bool operator==(const Timespan& a, const Timespan& b) noexcept { return a._duration == b._duration; }
    friend bool operator!=(const Timespan& a, const Timespan& b) noexcept { return a._duration != b._duration; }
    friend bool operator<(const Timespan& a, const Timespan& b) noexcept { return a._duration < b._duration; }

private:
    int64_t _duration;
};

//! 128-bit universally unique identifier (CppCommon/system/uuid.h)
class UUID
{
public:
    UUID() noexcept : _data{} {}
    explicit UUID(const std::array<uint8_t, 16>& data) noexcept : _data(data) {}

    const std::array<uint8_t, 16>& data() const noexcept { return _data; }
    std::string string() const
    {
        static const char hex[] = "0123456789abcdef";
        std::string s;
        for (size_t i = 0; i < 16; ++i) {
            if (i == 4 || i == 6 || i == 8 || i == 10)
                s.push_back('-');
            s.push_back(hex[_data[i] >> 4]);
            s.push_back(hex[_data[i] & 15]);
        }
        return s;
    }

    static UUID Nil() noexcept { return UUID(); }
    //! Version 4 (random) UUID
    static UUID Random()
    {
        thread_local std::mt19937_64 gen{std::random_device{}()};
        std::array<uint8_t, 16> d{};
        for (size_t i = 0; i < 16; i += 8) {
            const uint64_t v = gen();
            for (size_t j = 0; j < 8; ++j)
                d[i + j] = uint8_t(v >> (8 * j));
        }
        d[6] = uint8_t((d[6] & 0x0F) | 0x40);
        d[8] = uint8_t((d[8] & 0x3F) | 0x80);
        return UUID(d);
    }

    friend bool operator==(const UUID& a, const UUID& b) noexcept { return a._data == b._data; }
    friend bool operator!=(const UUID& a, const UUID& b) noexcept { return a._data != b._data; }

private:
    std::array<uint8_t, 16> _data;
};

} // namespace CppCommon
#endif

#endif // CPPSERVER_AMD_WS_COMMON_H
