// Measurement tool (not part of the product): a SIGPROF sampling profiler
// linked into a benchmark binary. Every tick of the process CPU clock records
// the interrupted instruction address; at exit the samples are written as
// "module offset count" lines (to $WSG_SAMPLER_OUT, default sampler.txt) for
// tools/sampler_report.py to symbolize with addr2line. Enabled by setting
// $WSG_SAMPLER (the period in microseconds, e.g. 200).
#include <signal.h>
#include <sys/time.h>
#include <ucontext.h>
#include <dlfcn.h>
#include <link.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>

namespace {

constexpr size_t kMax = 1 << 22;
uintptr_t g_pc[kMax];
std::atomic<size_t> g_n{0};

void on_prof(int, siginfo_t*, void* ctx) {
    auto* uc = static_cast<ucontext_t*>(ctx);
    size_t i = g_n.fetch_add(1, std::memory_order_relaxed);
    if (i < kMax) g_pc[i] = static_cast<uintptr_t>(uc->uc_mcontext.gregs[REG_RIP]);
}

void dump() {
    struct itimerval off = {};
    setitimer(ITIMER_PROF, &off, nullptr);
    size_t n = g_n.load();
    if (n > kMax) n = kMax;
    std::map<std::pair<std::string, uintptr_t>, size_t> hist;
    for (size_t i = 0; i < n; ++i) {
        Dl_info info;
        std::string mod = "?";
        uintptr_t off = g_pc[i];
        if (dladdr(reinterpret_cast<void*>(g_pc[i]), &info) && info.dli_fname) {
            mod = info.dli_fname;
            off = g_pc[i] - reinterpret_cast<uintptr_t>(info.dli_fbase);
        }
        ++hist[{mod, off}];
    }
    const char* path = std::getenv("WSG_SAMPLER_OUT");
    FILE* f = std::fopen(path ? path : "sampler.txt", "w");
    if (!f) return;
    for (auto& kv : hist)
        std::fprintf(f, "%s %lx %zu\n", kv.first.first.c_str(),
                     static_cast<unsigned long>(kv.first.second), kv.second);
    std::fclose(f);
    std::fprintf(stderr, "sampler: %zu samples\n", n);
}

struct Start {
    Start() {
        const char* p = std::getenv("WSG_SAMPLER");
        if (!p) return;
        long us = std::atol(p);
        if (us <= 0) us = 200;
        struct sigaction sa = {};
        sa.sa_sigaction = on_prof;
        sa.sa_flags = SA_SIGINFO | SA_RESTART;
        sigaction(SIGPROF, &sa, nullptr);
        struct itimerval it = {};
        it.it_interval.tv_usec = us;
        it.it_value.tv_usec = us;
        setitimer(ITIMER_PROF, &it, nullptr);
        std::atexit(dump);
    }
} g_start;

}  // namespace
