// lane_rtt.cpp — one lane task's round trip as the per-call path sees it:
// wsg_xor_host of SIZE bytes (<= 40: the payload travels in the task and the
// answer in self-tagged units), CALLS times back to back on one thread.
// Median / p10 / p90 microseconds, one JSON line.  Measurement tool only;
// $WSG_LANE_DOOR picks the mailboxes' memory as in the product.
//   lane_rtt [SIZE=32] [CALLS=20000]
#include "wsg_capi.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv)
{
    const size_t size = argc > 1 ? size_t(std::atol(argv[1])) : 32;
    const int calls = argc > 2 ? std::atoi(argv[2]) : 20000;
    wsg_ctx* c = nullptr;
    if (wsg_create(0, &c) != WSG_OK) {
        std::fprintf(stderr, "wsg_create failed\n");
        return 1;
    }
    std::vector<unsigned char> src(size), dst(size), back(size);
    for (size_t i = 0; i < size; ++i)
        src[i] = (unsigned char)(i * 37 + 11);
    const uint32_t key = 0xA1B2C3D4u;
    std::vector<double> v;
    v.reserve(size_t(calls));
    bool ok = true;
    for (int r = 0; r < calls + 200; ++r) {
        const auto t = std::chrono::steady_clock::now();
        const int rc = wsg_xor_host(c, src.data(), dst.data(), size, key, 0);
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count();
        if (rc != WSG_OK) {
            std::fprintf(stderr, "wsg_xor_host rc=%d\n", rc);
            return 1;
        }
        if (r >= 200)
            v.push_back(us);
    }
    // the XOR twice is the identity, and once changes every byte of this key
    ok = wsg_xor_host(c, dst.data(), back.data(), size, key, 0) == WSG_OK &&
         std::equal(back.begin(), back.end(), src.begin()) && !std::equal(dst.begin(), dst.end(), src.begin());
    uint64_t req = 0, launches = 0;
    int running = 0;
    wsg_lane_stats(c, &req, &launches, &running);
    std::sort(v.begin(), v.end());
    std::printf("{\"size\": %zu, \"calls\": %d, \"us_median\": %.3f, \"us_p10\": %.3f, \"us_p90\": %.3f, "
                "\"lane_requests\": %llu, \"lane_launches\": %llu, \"bytes_ok\": %s}\n",
                size, calls, v[v.size() / 2], v[v.size() / 10], v[v.size() * 9 / 10], (unsigned long long)req,
                (unsigned long long)launches, ok ? "true" : "false");
    wsg_destroy(c);
    return ok ? 0 : 2;
}
