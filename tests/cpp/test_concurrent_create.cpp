// test_concurrent_create.cpp — eight threads released together by a barrier
// each create a codec context (wsg_create) and run one host batch on it, in a
// fresh process: the pattern of a server whose IO threads build their
// contexts on their first connection.  Round 4 saw getenv crash in
// wsg_create when threads created contexts while the HIP runtime edited the
// environment (profiles/r4/getenv_race.log); every knob is now read once per
// context under the environment lock (wsg_env.h).
//
// With a GPU (tests/test_gpu_cpp_api.py): every context is made, and every
// thread's masked frames decode to their payloads (the device's lane).
// Without one (the ThreadSanitizer build, tests/test_sanitize.py): every
// wsg_create fails cleanly with WSG_EHIP, the same way on every thread.
#include "wsg_capi.h"

#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

int main(int argc, char** argv)
{
    const bool expect_gpu = argc > 1 && std::strcmp(argv[1], "gpu") == 0;
    constexpr int kThreads = 8, kFrames = 200, kLen = 40;
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    std::atomic<int> created{0}, failed_create{0}, exact{0}, wrong{0};
    std::vector<std::thread> th;
    for (int t = 0; t < kThreads; ++t)
        th.emplace_back([&, t] {
            {
                std::unique_lock<std::mutex> g(m);
                if (++arrived == kThreads)
                    cv.notify_all();
                cv.wait(g, [&] { return arrived == kThreads; });
            }
            wsg_ctx* c = nullptr;
            const int rc = wsg_create(0, &c);
            if (rc != WSG_OK) {
                if (rc == WSG_EHIP && !c)
                    ++failed_create;
                return;
            }
            ++created;
            // kFrames masked frames of kLen bytes (82 | 80+len | key | payload ^ key)
            const size_t fsz = 2 + 4 + kLen;
            uint8_t *wire = nullptr, *out = nullptr;
            uint64_t* fs = nullptr;
            wsg_recv_info* info = nullptr;
            if (wsg_host_alloc(fsz * kFrames, reinterpret_cast<void**>(&wire)) ||
                wsg_host_alloc(fsz * kFrames, reinterpret_cast<void**>(&out)) ||
                wsg_host_alloc(sizeof(uint64_t) * kFrames, reinterpret_cast<void**>(&fs)) ||
                wsg_host_alloc(sizeof(wsg_recv_info) * kFrames, reinterpret_cast<void**>(&info))) {
                ++wrong;
                return;
            }
            std::vector<uint8_t> payload(size_t(kFrames) * kLen);
            for (size_t i = 0; i < payload.size(); ++i)
                payload[i] = uint8_t(i * 7 + t * 31);
            for (int f = 0; f < kFrames; ++f) {
                uint8_t* p = wire + fsz * f;
                const uint32_t key = 0x9E3779B9u * uint32_t(f + 1) ^ uint32_t(t);
                p[0] = 0x82;
                p[1] = uint8_t(0x80 | kLen);
                std::memcpy(p + 2, &key, 4);
                for (int i = 0; i < kLen; ++i)
                    p[6 + i] = payload[size_t(f) * kLen + i] ^ uint8_t(key >> (8 * (i & 3)));
                fs[f] = fsz * f;
            }
            const int d = wsg_decode_batch_host(c, wire, fsz * kFrames, fs, kFrames, out, info);
            bool ok = d == WSG_OK;
            for (int f = 0; ok && f < kFrames; ++f)
                ok = info[f].payload_off == fsz * f + 6 && info[f].len == uint64_t(kLen) &&
                     std::memcmp(out + fsz * f + 6, &payload[size_t(f) * kLen], kLen) == 0;
            ++(ok ? exact : wrong);
            wsg_host_free(wire);
            wsg_host_free(out);
            wsg_host_free(fs);
            wsg_host_free(info);
            wsg_destroy(c);
        });
    for (auto& x : th)
        x.join();
    std::printf("{\"created\": %d, \"failed_create\": %d, \"exact\": %d, \"wrong\": %d}\n", created.load(),
                failed_create.load(), exact.load(), wrong.load());
    const bool pass = expect_gpu ? (created == kThreads && exact == kThreads && wrong == 0)
                                 : (failed_create + created == kThreads && wrong == 0);
    return pass ? 0 : 1;
}
