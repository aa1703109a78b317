// wsg_env.h — the library's reads of its environment knobs ($WSG_*).
//
// The HIP runtime edits the process environment while it initializes, and
// getenv on another thread meanwhile can read freed memory: four threads
// creating their codec contexts at once crashed in getenv inside wsg_create
// (tools/calls_r4/gpu_r4ah.sh, backtrace in profiles/r4/getenv_race.log).
// So every read goes through env() under one lock, and the library's first
// HIP call (hip_init_once, wsg_capi.hip) and context creation (wsg_create,
// whose HIP calls may initialize the device) run under the same lock.
#pragma once

#include <cstdlib>
#include <mutex>
#include <string>

namespace wsg {

// (recursive: wsg_create holds it over its HIP calls and reads knobs inside)
inline std::recursive_mutex& env_mutex()
{
    static std::recursive_mutex* m = new std::recursive_mutex;   // leaked: used from static destructors
    return *m;
}

// $name's value copied under the lock; false when unset.
inline bool env(const char* name, std::string& out)
{
    std::lock_guard<std::recursive_mutex> g(env_mutex());
    const char* e = std::getenv(name);
    if (!e)
        return false;
    out = e;
    return true;
}

// getenv(name) through env(): a per-thread copy, valid until this thread's
// next envp call (each call site reads one knob at a time).
inline const char* envp(const char* name)
{
    thread_local std::string v;
    return env(name, v) ? v.c_str() : nullptr;
}

// The HIP runtime initialized once, under env_mutex (its environment edits
// then never overlap an env() on another thread).  Defined in wsg_capi.hip.
void hip_init_once();

} // namespace wsg
