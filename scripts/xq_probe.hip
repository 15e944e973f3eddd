// Cross-queue step probe: can a chain of dependent step launches run faster
// when consecutive steps go to two HIP streams (two hardware queues) and each
// workgroup waits in the kernel for ITS predecessor workgroup (an epoch flag
// per block) instead of the queue's barrier between whole kernels?
//   hipcc --offload-arch=gfx950 -O3 scripts/xq_probe.hip -o scripts/bin/xq_probe
// The step kernel: 256 workgroups x 256 threads; each block reads and writes
// a 16 KB state slice (write-through stores), then runs a dependent f64 FMA
// chain of `work` iterations per thread.  Every wait is bounded (20 ms of
// s_memrealtime): a block that times out records it and runs on, so every
// launch drains.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

constexpr int kBlocks = 256, kThreads = 256, kSlice = 2048;   // doubles per block

__device__ __forceinline__ unsigned long long rt() { return __builtin_amdgcn_s_memrealtime(); }

// wait: 0 none; 1 acquire per poll, release fence in every thread; 2 relaxed
// polls + one acquire fence, one release by thread 0 after the barrier; 3 no
// agent-scope fences: relaxed agent-scope polls, state loads and stores
__global__ __launch_bounds__(kThreads) void step(double *state, unsigned *flags, unsigned *err,
                                                 unsigned epoch, int work, int wait) {
    const int b = blockIdx.x, t = threadIdx.x;
    if (wait) {
        if (t == 0) {
            const unsigned long long t0 = rt();
            if (wait == 1) {
                while (__hip_atomic_load(flags + b, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < epoch) {
                    if (rt() - t0 > 2000000ull) {
                        err[0] = 1u;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            } else {
                while (__hip_atomic_load(flags + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < epoch) {
                    if (rt() - t0 > 2000000ull) {
                        err[0] = 1u;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                if (wait == 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            }
        }
        __syncthreads();
    }
    double *s = state + static_cast<size_t>(b) * kSlice;
    double v[kSlice / kThreads];
#pragma unroll
    for (int i = 0; i < kSlice / kThreads; ++i)
        v[i] = wait == 3 ? __hip_atomic_load(s + t + i * kThreads, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                         : s[t + i * kThreads];
    double acc = v[0] + v[1] + v[2] + v[3] + v[4] + v[5] + v[6] + v[7];
    for (int i = 0; i < work; ++i) acc = fma(acc, 0.999999999, 1e-9);
#pragma unroll
    for (int i = 0; i < kSlice / kThreads; ++i)
        __hip_atomic_store(s + t + i * kThreads, v[i] + acc * 1e-30, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    if (wait == 1) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __syncthreads();
        if (t == 0) __hip_atomic_store(flags + b, epoch + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else if (wait) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __syncthreads();
        if (t == 0)
            __hip_atomic_store(flags + b, epoch + 1, wait == 2 ? __ATOMIC_RELEASE : __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main(int argc, char **argv) {
    const int work = argc > 1 ? atoi(argv[1]) : 600;
    double *state;
    unsigned *flags, *err;
    CK(hipMalloc(&state, sizeof(double) * kBlocks * kSlice));
    CK(hipMalloc(&flags, sizeof(unsigned) * kBlocks));
    CK(hipMalloc(&err, sizeof(unsigned)));
    CK(hipMemset(state, 0, sizeof(double) * kBlocks * kSlice));
    CK(hipMemset(err, 0, sizeof(unsigned)));
    hipStream_t s[3];
    for (auto &x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    struct Variant { const char *name; int nstreams, wait; } variants[] = {
        {"one_stream_plain", 1, 0}, {"one_stream_flags", 1, 1}, {"two_streams_flags", 2, 1},
        {"one_stream_once", 1, 2}, {"two_streams_once", 2, 2},
        {"one_stream_relaxed", 1, 3}, {"two_streams_relaxed", 2, 3}};
    for (int K : {20, 400}) {
        for (auto var : variants) {
            for (int rep = 0; rep < 4; ++rep) {
                CK(hipMemset(flags, 0, sizeof(unsigned) * kBlocks));
                CK(hipDeviceSynchronize());
                for (int k = 0; k < 5; ++k)   // warm-up on one stream, flags 0 -> 5
                    hipLaunchKernelGGL(step, dim3(kBlocks), dim3(kThreads), 0, s[0], state, flags, err,
                                       k, work, var.wait);
                CK(hipDeviceSynchronize());
                const auto t0 = std::chrono::steady_clock::now();
                for (int k = 0; k < K; ++k)
                    hipLaunchKernelGGL(step, dim3(kBlocks), dim3(kThreads), 0, s[k % var.nstreams], state,
                                       flags, err, 5 + k, work, var.wait);
                CK(hipDeviceSynchronize());
                const double us = std::chrono::duration<double, std::micro>(
                                      std::chrono::steady_clock::now() - t0).count();
                unsigned h_err = 0;
                CK(hipMemcpy(&h_err, err, sizeof(unsigned), hipMemcpyDeviceToHost));
                printf("{\"variant\": \"%s\", \"steps\": %d, \"work\": %d, \"rep\": %d, \"us_per_step\": %.3f, "
                       "\"timeouts\": %u}\n", var.name, K, work, rep, us / K, h_err);
                fflush(stdout);
                if (h_err) return 2;
            }
        }
    }
    return 0;
}
