// Does hipFree wait for work on other streams?  (the r3w teardown fault.)
//
// A 200 ms spin kernel (wall clock + s_sleep, no memory access) is queued on a non-blocking stream; the host then
// frees device buffers and times each call.  If hipFree returned at once while the stream was still busy, a library
// object destroyed while another stream's kernels still read its buffers would free memory under them -- the
// use-after-free that the destroy paths now close by draining the whole device first.  Nothing here reads freed
// memory: the spin kernel touches no buffer, so the experiment cannot fault.
//   case A: hipFree of a buffer allocated before the spin was queued
//   case B: hipMalloc + hipFree of a fresh buffer while the spin runs
//   case C: hipDeviceSynchronize (reference: the full wait)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void k_spin(unsigned long long ticks) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(32);
}

static double ms_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main() {
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 2;
    const unsigned long long ticks = 200ull * 100000ull;   // wall_clock64 runs at 100 MHz on gfx950
    double a = 0, b = 0, c = 0;
    for (int rep = 0; rep < 2; ++rep) {
        void* p = nullptr;
        if (hipMalloc(&p, 64 << 20) != hipSuccess) return 2;
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, ticks);
        auto t = std::chrono::steady_clock::now();
        if (hipFree(p) != hipSuccess) return 3;
        a = ms_since(t);
        void* q = nullptr;
        t = std::chrono::steady_clock::now();
        if (hipMalloc(&q, 64 << 20) != hipSuccess || hipFree(q) != hipSuccess) return 3;
        b = ms_since(t);
        t = std::chrono::steady_clock::now();
        if (hipDeviceSynchronize() != hipSuccess) return 3;
        c = ms_since(t);
    }
    std::printf("{\"spin_ms\": 200, \"free_old_buffer_ms\": %.3f, \"malloc_free_new_ms\": %.3f, \"device_sync_after_ms\": %.3f, "
                "\"hipFree_waits_for_other_streams\": %s}\n",
                a, b, c, a > 100.0 ? "true" : "false");
    (void)hipStreamDestroy(s);
    return 0;
}
