// kmp_threads.hpp — the host thread pools behind the C ABI.  A pool that cannot start a thread
// (std::system_error from std::thread) must not throw across an extern "C" entry point: the
// parts that got no thread run on the calling thread after the others, so the call still
// completes (more slowly) instead of terminating the host process.
#pragma once
#include <system_error>
#include <thread>
#include <vector>

namespace kmp {

// f(0) .. f(T-1), f(0) on the calling thread, the rest on their own threads where possible
template <class F>
void run_parts(int T, F&& f) {
    std::vector<std::thread> pool;
    int started = 1;
    try {
        pool.reserve(T > 1 ? T - 1 : 0);
        for (; started < T; ++started) pool.emplace_back(f, started);
    } catch (const std::exception&) {
        // out of threads (or memory): the parts [started, T) run inline below
    }
    f(0);
    for (auto& th : pool) th.join();
    for (int t = started; t < T; ++t) f(t);
}

}  // namespace kmp
