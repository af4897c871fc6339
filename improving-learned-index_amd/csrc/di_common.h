// di_common.h -- shared host-side plumbing of libdeepimpact_hip.so:
// error reporting across the C ABI, HIP checks, device buffers, per-kernel
// HIP-event timing.  gfx950 only.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <map>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/deepimpact.h"

namespace di {

// thread-local last error (di_last_error)
void set_error(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
const char *last_error();
int n_cu();  // compute units of the current device

struct Error {
    int code;
};

// Host worker threads of the library's host-side passes (index build, synthetic
// collections): DI_HOST_THREADS, else OMP_NUM_THREADS (16 on the GPU box), else the
// hardware count; at most 64.
inline int host_threads() {
    const char *e = std::getenv("DI_HOST_THREADS");
    if (!e) e = std::getenv("OMP_NUM_THREADS");
    const int t = e ? std::atoi(e) : (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(t > 0 ? t : 1, 64));
}

// f(lo, hi, thread) over [0, n) split in `threads` contiguous ranges (thread t always
// gets the same range for the same n and threads).  A worker's exception -- a
// di::Error with its thread-local message, std::bad_alloc, anything -- is carried to
// the calling thread and rethrown there after every worker has joined (the lowest
// thread's), so the C-ABI guard turns it into a status code instead of
// std::terminate.
template <class F>
void parallel_for_threads(int64_t n, int threads, F &&f) {
    const int T = (int)std::min<int64_t>(std::max(threads, 1), std::max<int64_t>(n, 1));
    if (T == 1) {
        f((int64_t)0, n, 0);
        return;
    }
    std::vector<std::exception_ptr> err((size_t)T);
    std::vector<int> code((size_t)T, 0);
    std::vector<std::string> msg((size_t)T);
    std::vector<std::thread> th;
    th.reserve((size_t)T);
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            try {
                f(n * t / T, n * (t + 1) / T, t);
            } catch (const Error &e) {
                code[(size_t)t] = e.code;
                msg[(size_t)t] = last_error();
                err[(size_t)t] = std::current_exception();
            } catch (...) {
                err[(size_t)t] = std::current_exception();
            }
        });
    for (auto &x : th) x.join();
    for (int t = 0; t < T; ++t)
        if (err[(size_t)t]) {
            if (code[(size_t)t]) {
                set_error("%s", msg[(size_t)t].c_str());
                throw Error{code[(size_t)t]};
            }
            std::rethrow_exception(err[(size_t)t]);
        }
}

template <class F>
void parallel_for(int64_t n, F &&f) {
    parallel_for_threads(n, host_threads(), std::forward<F>(f));
}

// parallel_for over n chunks whose bodies may throw di::Error: f(chunk, thread).  The
// lowest-index failing chunk's error (code and message -- di_last_error is thread-local)
// is rethrown on the calling thread, the one a serial loop would have raised first.
template <class F>
void parallel_chunks(int64_t n, F &&f) {
    std::vector<int> code((size_t)std::max<int64_t>(n, 1), 0);
    std::vector<std::string> msg((size_t)std::max<int64_t>(n, 1));
    parallel_for(n, [&](int64_t lo, int64_t hi, int t) {
        for (int64_t c = lo; c < hi; ++c) {
            try {
                f(c, t);
            } catch (const Error &e) {
                code[(size_t)c] = e.code;
                msg[(size_t)c] = last_error();
                return;  // (later chunks of this thread come after the failure)
            } catch (...) {
                code[(size_t)c] = DI_ENOMEM;
                msg[(size_t)c] = "host allocation failed";
                return;
            }
        }
    });
    for (int64_t c = 0; c < n; ++c)
        if (code[(size_t)c]) {
            set_error("%s", msg[(size_t)c].c_str());
            throw Error{code[(size_t)c]};
        }
}

// body(); a di::Error it throws gets "line N: " in front of its message, N = line_of()
// (1-based; evaluated on the error path only, so it may rescan the input).
template <class Body, class LineOf>
void with_line_context(Body &&body, LineOf &&line_of) {
    try {
        body();
    } catch (const Error &) {
        const std::string m = last_error();
        set_error("line %lld: %s", (long long)line_of(), m.c_str());
        throw;
    }
}

[[noreturn]] inline void fail(int code, const char *msg) {
    set_error("%s", msg);
    throw Error{code};
}

#define DI_HIP(expr)                                                                    \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess) {                                                         \
            ::di::set_error("%s:%d %s: %s", __FILE__, __LINE__, #expr,                  \
                            hipGetErrorString(e_));                                     \
            throw ::di::Error{e_ == hipErrorOutOfMemory ? DI_ENOMEM : DI_EHIP};         \
        }                                                                               \
    } while (0)

#define DI_REQUIRE(cond, code, ...)                                                     \
    do {                                                                                \
        if (!(cond)) {                                                                  \
            ::di::set_error(__VA_ARGS__);                                               \
            throw ::di::Error{code};                                                    \
        }                                                                               \
    } while (0)

// Run a C-ABI body, translating exceptions into status codes.
template <class F>
int guard(F &&f) {
    try {
        f();
        return DI_OK;
    } catch (const Error &e) {
        return e.code;
    } catch (const std::bad_alloc &) {
        set_error("host allocation failed");
        return DI_ENOMEM;
    } catch (...) {
        set_error("unexpected C++ exception");
        return DI_EINVAL;
    }
}

// Owning device buffer (grows, never shrinks).
struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    void reserve(size_t n) {
        if (n <= bytes) return;
        if (p) DI_HIP(hipFree(p));
        p = nullptr;
        bytes = 0;
        DI_HIP(hipMalloc(&p, n ? n : 16));
        bytes = n;
    }
    template <class T>
    T *as() const {
        return static_cast<T *>(p);
    }
};

// Per-kernel timing with HIP events recorded on the launching stream.
struct Timer {
    struct Pending {
        std::string name;
        hipEvent_t a, b;
    };
    std::vector<Pending> pending;
    std::map<std::string, std::pair<double, int64_t>> acc;
    std::vector<hipEvent_t> pool;

    hipEvent_t ev() {
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        hipEvent_t e;
        DI_HIP(hipEventCreate(&e));
        return e;
    }
    void begin(bool on, const char *name, hipStream_t s, hipEvent_t *a) {
        if (!on) return;
        *a = ev();
        DI_HIP(hipEventRecord(*a, s));
        pending.push_back({name, *a, nullptr});
    }
    void end(bool on, hipStream_t s) {
        if (!on) return;
        hipEvent_t b = ev();
        DI_HIP(hipEventRecord(b, s));
        pending.back().b = b;
    }
    // call after the stream has been synchronised
    void resolve() {
        for (auto &p : pending) {
            float ms = 0.f;
            DI_HIP(hipEventElapsedTime(&ms, p.a, p.b));
            auto &e = acc[p.name];
            e.first += ms;
            e.second += 1;
            pool.push_back(p.a);
            pool.push_back(p.b);
        }
        pending.clear();
    }
    void get(const char *name, di_timing *out, bool reset) {
        auto it = acc.find(name);
        out->ms = it == acc.end() ? 0.0 : it->second.first;
        out->launches = it == acc.end() ? 0 : it->second.second;
        if (reset) acc.clear();
    }
    ~Timer() {
        for (auto &p : pending) {
            (void)hipEventDestroy(p.a);
            if (p.b) (void)hipEventDestroy(p.b);
        }
        for (auto e : pool) (void)hipEventDestroy(e);
    }
};

// RAII timing scope around one kernel launch.
struct TimedLaunch {
    Timer &t;
    bool on;
    hipStream_t s;
    TimedLaunch(Timer &t_, bool on_, const char *name, hipStream_t s_) : t(t_), on(on_), s(s_) {
        hipEvent_t a;
        t.begin(on, name, s, &a);
    }
    ~TimedLaunch() noexcept(false) { t.end(on, s); }
};

inline void check_launch(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("launch of %s failed: %s", what, hipGetErrorString(e));
        throw Error{DI_EHIP};
    }
}

// Copy `bytes` from a host or device pointer into a device buffer on stream s.
inline const void *stage_in(const void *src, size_t bytes, bool device_ptrs, DevBuf &buf,
                            hipStream_t s) {
    if (device_ptrs || bytes == 0) return src;
    buf.reserve(bytes);
    DI_HIP(hipMemcpyAsync(buf.p, src, bytes, hipMemcpyHostToDevice, s));
    return buf.p;
}

}  // namespace di
