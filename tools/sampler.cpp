// Measurement tool (not part of the product): a SIGPROF sampling profiler
// linked into a benchmark binary. Every tick of the process CPU clock records
// the interrupted instruction address; at exit the samples are written as
// "module offset count" lines (to $WSG_SAMPLER_OUT, default sampler.txt) for
// tools/sampler_report.py to symbolize with addr2line. Enabled by setting
// $WSG_SAMPLER (the period in microseconds, e.g. 200).  A host crash
// (SIGSEGV / SIGABRT) prints a backtrace to stderr ($WSG_CRASH_TRACE=0: not).
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>
#include <sys/time.h>
#include <ucontext.h>
#include <dlfcn.h>
#include <link.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <map>
#include <string>

namespace {

constexpr size_t kMax = 1 << 22;
uintptr_t g_pc[kMax];
std::atomic<size_t> g_n{0};
// $WSG_SAMPLER_STACKS=1: also the callers (backtrace() from the handler: not
// async-signal-safe in general; preloaded at start, a measurement tool only)
constexpr int kDepth = 10;
constexpr size_t kStackMax = 1 << 16;
uintptr_t g_stack[kStackMax][kDepth];
int g_stack_n[kStackMax];
std::atomic<size_t> g_sn{0};
bool g_stacks = false;

void on_prof(int, siginfo_t*, void* ctx) {
    auto* uc = static_cast<ucontext_t*>(ctx);
    size_t i = g_n.fetch_add(1, std::memory_order_relaxed);
    if (i < kMax) g_pc[i] = static_cast<uintptr_t>(uc->uc_mcontext.gregs[REG_RIP]);
    if (g_stacks) {
        const size_t k = g_sn.fetch_add(1, std::memory_order_relaxed);
        if (k < kStackMax) {
            void* fr[kDepth + 2];
            const int n = backtrace(fr, kDepth + 2);   // [0] this handler, [1] the signal frame
            int m = 0;
            g_stack[k][m++] = static_cast<uintptr_t>(uc->uc_mcontext.gregs[REG_RIP]);
            for (int j = 2; j < n && m < kDepth; ++j)
                g_stack[k][m++] = reinterpret_cast<uintptr_t>(fr[j]);
            g_stack_n[k] = m;
        }
    }
}

std::string where(uintptr_t pc)
{
    Dl_info info;
    char buf[32];
    if (dladdr(reinterpret_cast<void*>(pc), &info) && info.dli_fname) {
        std::snprintf(buf, sizeof(buf), "%lx", static_cast<unsigned long>(pc - reinterpret_cast<uintptr_t>(info.dli_fbase)));
        return std::string(info.dli_fname) + "@" + buf;
    }
    std::snprintf(buf, sizeof(buf), "%lx", static_cast<unsigned long>(pc));
    return std::string("?@") + buf;
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
    if (g_stacks) {
        const size_t sn = std::min(g_sn.load(), kStackMax);
        std::map<std::string, size_t> st;
        for (size_t k = 0; k < sn; ++k) {
            std::string line;
            for (int j = 0; j < g_stack_n[k]; ++j)
                line += (j ? ";" : "") + where(g_stack[k][j]);
            ++st[line];
        }
        std::string sp = std::string(path ? path : "sampler.txt") + ".stacks";
        if (FILE* g = std::fopen(sp.c_str(), "w")) {
            for (auto& kv : st)
                std::fprintf(g, "%zu %s\n", kv.second, kv.first.c_str());
            std::fclose(g);
        }
    }
}

void on_crash(int sig)
{
    void* frames[64];
    const int n = backtrace(frames, 64);
    const char msg[] = "sampler: fatal signal, backtrace:\n";
    (void)!write(2, msg, sizeof(msg) - 1);
    backtrace_symbols_fd(frames, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

struct Start {
    Start() {
        const char* ct = std::getenv("WSG_CRASH_TRACE");
        if (!ct || *ct != '0') {   // a backtrace on SIGSEGV / SIGABRT (host code); $WSG_CRASH_TRACE=0: off
            signal(SIGSEGV, on_crash);
            signal(SIGABRT, on_crash);
        }
        const char* p = std::getenv("WSG_SAMPLER");
        if (!p) return;
        if (const char* q = std::getenv("WSG_SAMPLER_STACKS")) {
            g_stacks = *q == '1';
            void* fr[4];
            (void)backtrace(fr, 4);   // load the unwinder now, not in the handler
        }
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
