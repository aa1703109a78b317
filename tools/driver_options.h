// driver_options.h — the reference drivers' command-line options
// (performance/ws_echo_client.cpp:96-102, ws_multicast_server.cpp:54-57,
// ws_multicast_client.cpp:64-69: -a/--address -p/--port -t/--threads
// -c/--clients -m/--messages -s/--size -z/--seconds), so the in-memory
// drivers run with the reference's flags; --mode and --tls pick this repo's
// variants.  -a and -p are accepted and unused (no sockets here).
#pragma once

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>

struct DriverOptions {
    std::string mode;
    int threads = std::max(1u, std::thread::hardware_concurrency() / 2);   // reference: physical cores
    int clients = 100;
    long messages = 1000;
    long size = 32;
    double seconds = 10;
    bool tls = false;
};

// Flags as the reference takes them (long forms with "=" too); returns
// false on an unknown flag or a missing value.
inline bool parse_driver_options(int argc, char** argv, DriverOptions& o)
{
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i], v;
        const size_t eq = a.find('=');
        if (a.rfind("--", 0) == 0 && eq != std::string::npos) {
            v = a.substr(eq + 1);
            a = a.substr(0, eq);
        }
        auto value = [&]() -> const char* {
            if (!v.empty())
                return v.c_str();
            return i + 1 < argc ? argv[++i] : nullptr;
        };
        const char* x = nullptr;
        if (a == "--tls") {
            o.tls = true;
            continue;
        }
        if (!(x = value()))
            return false;
        if (a == "--mode")
            o.mode = x;
        else if (a == "-t" || a == "--threads")
            o.threads = std::max(1, std::atoi(x));
        else if (a == "-c" || a == "--clients")
            o.clients = std::max(1, std::atoi(x));
        else if (a == "-m" || a == "--messages")
            o.messages = std::max(1L, std::atol(x));
        else if (a == "-s" || a == "--size")
            o.size = std::max(0L, std::atol(x));
        else if (a == "-z" || a == "--seconds")
            o.seconds = std::atof(x);
        else if (a != "-a" && a != "--address" && a != "-p" && a != "--port")
            return false;
    }
    return true;
}
