// Device plumbing for the engine: HIP error handling, a caching device allocator (buffers are
// reused across runs so repeated checks pay no hipMalloc), and the HBM visited-set view.
#pragma once
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

namespace sr {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define SR_HIP(expr)                                                                              \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess)                                                                     \
            throw ::sr::Error(-2, std::string(#expr) + ": " + hipGetErrorString(e_) + " at " +   \
                                      __FILE__ + ":" + std::to_string(__LINE__));                 \
    } while (0)

// The host waits until every launch enqueued on `s` has finished: a spin on hipStreamQuery for up
// to ~0.5 ms, then a blocking wait. A blocking hipStreamSynchronize returned ~30 us after the last
// kernel had ended (measured at the end of a 2pc N=9 check), and a check's host path has a few
// such waits on short device work (votes, counters, the last level).
// A query that answered "not ready" may leave hipErrorNotReady as the thread's last error: cleared
// here (only that one) so that a later hipGetLastError after a launch does not report it.
inline void clear_not_ready() {
    if (hipPeekAtLastError() == hipErrorNotReady) (void)hipGetLastError();
}
inline hipError_t stream_sync(hipStream_t s) {
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned spin = 1;; ++spin) {
        const hipError_t e = hipStreamQuery(s);
        if (e != hipErrorNotReady) {
            if (spin > 1) clear_not_ready();
            return e;
        }
        if ((spin & 255) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(500))
            return clear_not_ready(), hipStreamSynchronize(s);
        __builtin_ia32_pause();
    }
}

// Streams this library created per device (the pooled contexts' streams, never destroyed), and the
// hardware queues the HIP runtime gives this process per device (GPU_MAX_HW_QUEUES, read by the
// runtime at its initialisation; HIP's default is 4). The runtime gives each stream a queue of its
// own while there are enough, and makes later streams SHARE queues: a kernel that spins on the
// device (the direct exchange's wait) can then sit in front of the kernel it waits for.
struct StreamCensus {
    static StreamCensus& get() {
        static StreamCensus c;
        return c;
    }
    void created(int dev) {
        std::lock_guard<std::mutex> g(mu_);
        ++n_[dev];
    }
    void destroyed(int dev) {
        std::lock_guard<std::mutex> g(mu_);
        --n_[dev];
    }
    int on(int dev) {
        std::lock_guard<std::mutex> g(mu_);
        return n_[dev];
    }
    static int hw_queues() {
        const char* e = std::getenv("GPU_MAX_HW_QUEUES");
        return e && std::atoi(e) > 0 ? std::atoi(e) : 4;
    }
    std::mutex mu_;
    std::map<int, int> n_;
};
inline hipError_t create_stream(hipStream_t* s, int dev) {
    const hipError_t e = hipStreamCreateWithFlags(s, hipStreamNonBlocking);
    if (e == hipSuccess) StreamCensus::get().created(dev);
    return e;
}

// Process-wide caching allocator: freed blocks go to a per-(device, size) free list. Sizes are
// rounded up to 2 MiB (or a power of two below that) so that a run with a slightly different
// frontier reuses the same blocks.
class DevicePool {
  public:
    static DevicePool& get() {
        static DevicePool p;
        return p;
    }
    // kind 0: ordinary (coarse-grained) device memory; kind 1: fine-grained device memory
    // (hipDeviceMallocFinegrained), which a system-scope acquire makes coherent with stores that
    // ANOTHER device issued over xGMI while a kernel runs (the direct exchange's flags and receive
    // buffers: its owner's L2 must not serve a line it cached before a peer's store); kind 2:
    // uncached device memory (hipDeviceMallocUncached: no line of it is held dirty in an L2).
    void* alloc(int dev, size_t bytes, int kind = 0) {
        bytes = round(bytes);
        {
            std::lock_guard<std::mutex> g(mu_);
            auto& fl = free_[{dev, bytes, kind}];
            if (!fl.empty()) {
                void* p = fl.back();
                fl.pop_back();
                return p;
            }
            if (kind == 0)
                if (void* p = take_zeroed_locked(dev, bytes)) return p;
        }
        void* p = nullptr;
        auto raw = [&]() {
            return kind == 1   ? hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained)
                   : kind == 2 ? hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached)
                               : hipMalloc(&p, bytes);
        };
        const auto t0 = std::chrono::steady_clock::now();
        hipError_t e = raw();
        const bool retried = e != hipSuccess;
        if (retried) {
            release_all(dev);  // retry once with the cache emptied
            (void)hipGetLastError();
            SR_HIP(raw());
        }
        if (trace())
            std::fprintf(stderr, "[pool] device %d: %zu bytes (kind %d) fresh%s in %.3f ms\n", dev, bytes, kind,
                         retried ? " after emptying the cache" : "",
                         std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        return p;
    }
    void free(int dev, void* p, size_t bytes, int kind = 0) {
        if (!p) return;
        std::lock_guard<std::mutex> g(mu_);
        free_[{dev, round(bytes), kind}].push_back(p);
    }
    // Blocks handed back while the work that zeroes them is still in flight: `ready` is recorded
    // behind that work. A check returns its visited set this way as soon as its last level is
    // done, and the clear then runs while the host finishes that check and sets up the next one.
    void free_zeroed(int dev, void* p, size_t bytes, hipEvent_t ready, int kind = 0) {
        std::lock_guard<std::mutex> g(mu_);
        zeroed_[{dev, round(bytes), kind}].push_back({p, ready});
    }
    // A zeroed block of this size if one is pooled, with `s` ordered after its clear on the device
    // (the host does not wait), else nullptr. A block whose clear has finished is preferred.
    void* alloc_zeroed(int dev, size_t bytes, hipStream_t s, int kind = 0) {
        Zeroed z{nullptr, nullptr};
        {
            std::lock_guard<std::mutex> g(mu_);
            auto& fl = zeroed_[{dev, round(bytes), kind}];
            if (fl.empty()) return nullptr;
            size_t pick = 0;
            for (size_t i = 0; i < fl.size(); ++i)
                if (hipEventQuery(fl[i].ready) == hipSuccess) {
                    pick = i;
                    break;
                }
            clear_not_ready();
            z = fl[pick];
            fl.erase(fl.begin() + (long)pick);
        }
        const hipError_t e = hipStreamWaitEvent(s, z.ready, 0);
        if (e != hipSuccess) {
            (void)hipEventSynchronize(z.ready);
            (void)hipEventDestroy(z.ready);
            free(dev, z.p, bytes, kind);  // not known to be ordered for this stream: an ordinary block
            return nullptr;
        }
        (void)hipEventDestroy(z.ready);  // the wait holds what it needs
        return z.p;
    }
    void release_all(int dev) {
        std::lock_guard<std::mutex> g(mu_);
        ++epoch_[dev];  // blocks may come back at the same addresses: peers' IPC mappings are stale
        for (auto& [k, v] : free_)
            if (std::get<0>(k) == dev) {
                for (void* p : v) (void)hipFree(p);
                v.clear();
            }
        for (auto& [k, v] : zeroed_)
            if (std::get<0>(k) == dev) {
                for (auto& z : v) {
                    (void)hipEventSynchronize(z.ready);
                    (void)hipEventDestroy(z.ready);
                    (void)hipFree(z.p);
                }
                v.clear();
            }
    }
    // SR_POOL_TRACE=1: every fresh device allocation on stderr (size, whether the cache had to be
    // emptied first, and its duration).
    static bool trace() {
        static const bool on = std::getenv("SR_POOL_TRACE") && std::atoi(std::getenv("SR_POOL_TRACE")) != 0;
        return on;
    }
    static size_t round(size_t b) {
        if (b < 256) return 256;
        if (b >= (2u << 20)) return (b + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
        size_t r = 256;
        while (r < b) r <<= 1;
        return r;
    }

    // Incremented whenever blocks of `dev` are returned to the driver (direct exchange: PeerBlob).
    uint64_t epoch(int dev) {
        std::lock_guard<std::mutex> g(mu_);
        return epoch_[dev];
    }

  private:
    struct Zeroed {
        void* p;
        hipEvent_t ready;
    };
    // An ordinary allocation may take a pooled zeroed block of its size class whose clear has
    // finished (the clear is then simply wasted): a table size that no later check asks for again
    // would otherwise hold its memory until an out-of-memory retry flushes the whole pool. A block
    // whose clear is still in flight is left for the check it was released for (alloc() has no
    // stream to order after it).
    void* take_zeroed_locked(int dev, size_t bytes) {
        auto it = zeroed_.find({dev, bytes, 0});
        if (it == zeroed_.end()) return nullptr;
        auto& fl = it->second;
        for (size_t i = 0; i < fl.size(); ++i) {
            if (hipEventQuery(fl[i].ready) != hipSuccess) continue;
            Zeroed z = fl[i];
            fl.erase(fl.begin() + (long)i);
            (void)hipEventDestroy(z.ready);
            clear_not_ready();
            return z.p;
        }
        clear_not_ready();
        return nullptr;
    }
    std::mutex mu_;
    std::map<std::tuple<int, size_t, int>, std::vector<void*>> free_;
    std::map<std::tuple<int, size_t, int>, std::vector<Zeroed>> zeroed_;
    std::map<int, uint64_t> epoch_;
};

// RAII device buffer backed by the pool.
template <class T>
struct DBuf {
    T* p = nullptr;
    size_t n = 0;
    int dev = 0;
    int kind = 0;  // DevicePool memory kind (1: fine-grained)
    DBuf() = default;
    DBuf(const DBuf&) = delete;
    DBuf& operator=(const DBuf&) = delete;
    DBuf(DBuf&& o) noexcept { swap(o); }
    ~DBuf() { reset(); }
    void reset() {
        if (p) DevicePool::get().free(dev, p, n * sizeof(T), kind);
        p = nullptr;
        n = 0;
        kind = 0;
    }
    void alloc(int d, size_t count, int k = 0) {
        reset();
        dev = d;
        n = count ? count : 1;
        kind = k;
        p = static_cast<T*>(DevicePool::get().alloc(d, n * sizeof(T), k));
    }
    // All-zero bytes, ordered before the work enqueued on `s` afterwards: a pooled zeroed block,
    // or a fresh one cleared on `s`.
    void alloc_zero(int d, size_t count, hipStream_t s, int k = 0) {
        reset();
        dev = d;
        n = count ? count : 1;
        kind = k;
        p = static_cast<T*>(DevicePool::get().alloc_zeroed(d, n * sizeof(T), s, k));
        if (p) return;
        p = static_cast<T*>(DevicePool::get().alloc(d, n * sizeof(T), k));
        SR_HIP(hipMemsetAsync(p, 0, n * sizeof(T), s));
    }
    // Hands the block back to be zeroed on `s` behind the work enqueued there so far (alloc_zero
    // takes it without a clear at its start). Falls back to an ordinary free on any error.
    void release_zero(hipStream_t s) noexcept {
        if (!p) return;
        hipEvent_t ready = nullptr;
        if (hipEventCreateWithFlags(&ready, hipEventDisableTiming) == hipSuccess) {
            if (hipMemsetAsync(p, 0, n * sizeof(T), s) == hipSuccess && hipEventRecord(ready, s) == hipSuccess) {
                DevicePool::get().free_zeroed(dev, p, n * sizeof(T), ready, kind);
                p = nullptr;
                n = 0;
                kind = 0;
                return;
            }
            (void)hipEventDestroy(ready);
        }
        (void)hipStreamSynchronize(s);  // no writer of the block may still be in flight
        (void)hipGetLastError();
        reset();
    }
    void swap(DBuf& o) {
        std::swap(p, o.p);
        std::swap(n, o.n);
        std::swap(dev, o.dev);
        std::swap(kind, o.kind);
    }
};

// A per-device execution context, created once and reused by every check on that device: the
// stream, the device counters, the pinned host mirror they are published to, and a pool of HIP
// events for per-launch timing. Contexts are pooled (a context is used by one check at a time).
template <class Counters, class HostMirror>
struct DeviceContext {
    int dev = 0;
    hipStream_t stream = nullptr;
    Counters* lc = nullptr;        // device
    HostMirror* hc = nullptr;      // pinned, host pointer
    HostMirror* hc_dev = nullptr;  // the same memory, device pointer
    uint32_t seq = 0;
    std::vector<hipEvent_t> events;
    hipEvent_t done = nullptr;  // marks a point of the stream the host waits for (no timing)

    void init(int d) {
        dev = d;
        SR_HIP(hipSetDevice(d));
        SR_HIP(create_stream(&stream, d));
        SR_HIP(hipEventCreateWithFlags(&done, hipEventDisableTiming));
        SR_HIP(hipMalloc(&lc, sizeof(Counters)));
        // two mirrors: launch `seq` publishes to slot seq & 1, so a launch may run while the host
        // still reads the previous one's snapshot
        SR_HIP(hipHostMalloc(&hc, 2 * sizeof(HostMirror), hipHostMallocCoherent | hipHostMallocMapped));
        SR_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&hc_dev), hc, 0));
        std::memset(hc, 0, 2 * sizeof(HostMirror));
    }
    hipEvent_t event(size_t i) {
        while (events.size() <= i) {
            hipEvent_t e;
            SR_HIP(hipEventCreate(&e));
            events.push_back(e);
        }
        return events[i];
    }
};

template <class Ctx>
class ContextPool {
  public:
    static ContextPool& get() {
        static ContextPool p;
        return p;
    }
    Ctx* acquire(int dev) {
        {
            std::lock_guard<std::mutex> g(mu_);
            auto& fl = free_[dev];
            if (!fl.empty()) {
                Ctx* c = fl.back();
                fl.pop_back();
                return c;
            }
        }
        auto* c = new Ctx();
        c->init(dev);
        return c;
    }
    void release(Ctx* c) {
        if (!c) return;
        std::lock_guard<std::mutex> g(mu_);
        free_[c->dev].push_back(c);
    }

  private:
    std::mutex mu_;
    std::map<int, std::vector<Ctx*>> free_;
};

}  // namespace sr
