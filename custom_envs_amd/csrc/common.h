// Shared host-side plumbing for the C ABI: thread-local error text and the
// HIP-call check used by every entry point (nothing throws across the ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstring>
#include <mutex>
#include <string>

#include "../../include/custom_envs_amd.h"

namespace ce {

// Sticky HIP errors found pending when an entry point starts.  Such an error
// was left by an earlier failed operation that is not this call's (a
// caller's aborted stream capture, another library's failed launch) and must
// not be reported as the failure of the launches that follow, so the entry
// point clears it -- but it is kept: counted, and its text noted, for
// ce_stale_error_count / ce_stale_error_note (the Python side warns once).
struct StaleErrors {
    std::atomic<long long> count{0};
    std::mutex mu;
    std::string note;
};
inline StaleErrors &stale_errors() {
    static StaleErrors s;
    return s;
}
inline void note_stale(int code, const char *text, const char *where) {
    StaleErrors &s = stale_errors();
    s.count.fetch_add(1);
    std::lock_guard<std::mutex> lock(s.mu);
    s.note = std::string("HIP error ") + std::to_string(code) + " (" + (text ? text : "?") +
             ") was pending at " + (where ? where : "?") + " and was cleared";
}

}  // namespace ce

#define CE_CLEAR_STALE_ERROR()                                              \
    do {                                                                    \
        const hipError_t stale_ = hipGetLastError();                        \
        if (stale_ != hipSuccess)                                           \
            ce::note_stale(static_cast<int>(stale_), hipGetErrorString(stale_), __func__); \
    } while (0)

#define CE_HIP(call)                                                              \
    do {                                                                          \
        hipError_t err_ = (call);                                                 \
        if (err_ != hipSuccess)                                                   \
            return ce::fail(CE_EHIP, std::string(#call " failed: ") +             \
                                         hipGetErrorString(err_));                \
    } while (0)

namespace ce {

inline std::string &last_error() {
    static thread_local std::string msg;
    return msg;
}

inline int fail(int code, const std::string &msg) {
    last_error() = msg;
    return code;
}

inline size_t align16(size_t v) { return (v + 15) & ~static_cast<size_t>(15); }

// Everything the launches of a captured k-step graph bake in.
struct GraphKey {
    int k = 0;
    int parity = 0;                  // engines with ping-pong state (multinn)
    const void *act = nullptr;
    int64_t stride = 0;
    hipStream_t stream = nullptr;
    unsigned char out[64] = {0};     // the caller's output pointer struct
    bool operator==(const GraphKey &o) const {
        return k == o.k && parity == o.parity && act == o.act && stride == o.stride &&
               stream == o.stream && std::memcmp(out, o.out, sizeof(out)) == 0;
    }
};

template <typename Outputs>
GraphKey graph_key(int k, int parity, const void *act, int64_t stride, hipStream_t stream,
                   const Outputs &o) {
    static_assert(sizeof(Outputs) <= sizeof(GraphKey::out), "output struct too large");
    GraphKey key;
    key.k = k;
    key.parity = parity;
    key.act = act;
    key.stride = stride;
    key.stream = stream;
    std::memcpy(key.out, &o, sizeof(Outputs));
    return key;
}

// Instantiated hipGraphs of k back-to-back step launches (ce_*_step_many),
// least-recently-used eviction.  Several stay live so a caller alternating
// k (a warm-up and a timed region, a tail of a long run) never re-captures
// inside its timed loop; ce_*_step_many_prepare instantiates and uploads
// one without launching it.
struct GraphCache {
    static constexpr int kSlots = 4;
    struct Slot {
        hipGraphExec_t exec = nullptr;
        GraphKey key;
        unsigned long long used = 0;
    };
    Slot slots[kSlots];
    unsigned long long clock = 0;

    void release() {
        for (auto &s : slots)
            if (s.exec) {
                (void)hipGraphExecDestroy(s.exec);
                s.exec = nullptr;
            }
    }

    // `capture()` issues the k launches on key.stream while it is captured.
    template <typename Capture>
    int get(const GraphKey &key, Capture &&capture, hipGraphExec_t *out) {
        for (auto &s : slots)
            if (s.exec && s.key == key) {
                s.used = ++clock;
                *out = s.exec;
                return CE_OK;
            }
        Slot *victim = &slots[0];
        for (auto &s : slots)
            if (!s.exec || s.used < victim->used) victim = &s;
        if (victim->exec) {
            CE_HIP(hipGraphExecDestroy(victim->exec));
            victim->exec = nullptr;
        }
        hipGraph_t g;
        CE_HIP(hipStreamBeginCapture(key.stream, hipStreamCaptureModeThreadLocal));
        capture();
        CE_HIP(hipStreamEndCapture(key.stream, &g));
        hipError_t err = hipGraphInstantiate(&victim->exec, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        if (err != hipSuccess) {
            victim->exec = nullptr;
            return fail(CE_EHIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(err));
        }
        CE_HIP(hipGraphUpload(victim->exec, key.stream));
        victim->key = key;
        victim->used = ++clock;
        *out = victim->exec;
        return CE_OK;
    }
};

}  // namespace ce
