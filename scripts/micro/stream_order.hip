// Diagnostics: which HIP upload / event calls are ordered before later work on a NON-BLOCKING stream?
//
// The extractor's configure() used to zero its per-cell FAST counts with hipMemset (null stream) and upload its
// geometry tables with hipMemcpy (pageable, null stream), then return; the first call's FAST then ran on the
// extractor's non-blocking side stream.  Each case below delays the null stream (or a producer stream) with a spin
// kernel and checks whether work launched afterwards on a non-blocking stream sees the upload / the producer.
//
//   A  hipMemset(d, 0) on the null stream, then k_set(d, 1) on a non-blocking stream          (expected race)
//   B  hipMemcpy(d, &7, pageable H2D) on the null stream, then k_copy(d -> out) non-blocking
//   C  hipMemsetAsync(d, 0, s_up) + hipStreamSynchronize(s_up), then k_set(d, 1) non-blocking (the fix: ordered)
//   D  event recorded on A after spin+k_set(flag,1); B waits the event; the event is then RE-RECORDED on an idle
//      stream; B copies flag.  Stream-ordered semantics: B's wait captured the first record, so out = 1.
//
// hipcc -O2 --offload-arch=gfx950 scripts/micro/stream_order.hip -o build/stream_order && build/stream_order
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            std::exit(2);                                                                      \
        }                                                                                      \
    } while (0)

// bounded spin: one lane waits `ticks` of the 100 MHz constant clock (wall_clock64), then returns
__global__ void k_spin(unsigned long long ticks) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(64);
}
__global__ void k_set(int* d, int v) { if (threadIdx.x == 0) d[0] = v; }
__global__ void k_copy(const int* src, int* dst) { if (threadIdx.x == 0) dst[0] = src[0]; }

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    const unsigned long long spin = 100ull * 1000 * 100;   // 100 ms at 100 MHz
    int *d, *out;
    CK(hipMalloc(&d, 4));
    CK(hipMalloc(&out, 4));
    hipStream_t nb, up, a, b, idle;
    CK(hipStreamCreateWithFlags(&nb, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&up, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&idle, hipStreamNonBlocking));
    int h = 0;
    int fails = 0;

    // A: hipMemset on the null stream behind a spin
    CK(hipMemset(d, 0x55, 4));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, (hipStream_t)0, spin);
    double t0 = now_ms();
    CK(hipMemset(d, 0, 4));
    double t1 = now_ms();
    hipLaunchKernelGGL(k_set, dim3(1), dim3(64), 0, nb, d, 1);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost));
    std::printf("A hipMemset(null stream) returned after %.3f ms; later non-blocking k_set(1) -> d = %d (%s)\n", t1 - t0, h,
                h == 1 ? "ordered" : "RACE: the memset landed after the later kernel");
    const bool memset_races = h != 1;

    // B: pageable hipMemcpy H2D on the null stream behind a spin
    int seven = 7;
    CK(hipMemset(d, 0, 4));
    CK(hipMemset(out, 0, 4));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, (hipStream_t)0, spin);
    t0 = now_ms();
    CK(hipMemcpy(d, &seven, 4, hipMemcpyHostToDevice));
    t1 = now_ms();
    hipLaunchKernelGGL(k_copy, dim3(1), dim3(64), 0, nb, d, out);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(&h, out, 4, hipMemcpyDeviceToHost));
    std::printf("B hipMemcpy(pageable H2D, null stream) returned after %.3f ms; later non-blocking read -> %d (%s)\n", t1 - t0,
                h, h == 7 ? "ordered" : "RACE: the kernel read the old value");
    const bool memcpy_races = h != 7;

    // C: the fix -- the upload on a stream of our own, synchronised before returning
    CK(hipMemset(d, 0x55, 4));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, up, spin);
    t0 = now_ms();
    CK(hipMemsetAsync(d, 0, 4, up));
    CK(hipStreamSynchronize(up));
    t1 = now_ms();
    hipLaunchKernelGGL(k_set, dim3(1), dim3(64), 0, nb, d, 1);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost));
    std::printf("C hipMemsetAsync(own stream)+hipStreamSynchronize took %.3f ms; later k_set(1) -> d = %d (%s)\n", t1 - t0, h,
                h == 1 ? "ordered" : "RACE");
    fails += h != 1;

    // D: re-recording an event while another stream's wait on its previous record is pending
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipMemset(d, 0, 4));
        CK(hipMemset(out, 0, 4));
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, a, spin);
        hipLaunchKernelGGL(k_set, dim3(1), dim3(64), 0, a, d, 1);
        CK(hipEventRecord(ev, a));
        CK(hipStreamWaitEvent(b, ev, 0));
        CK(hipEventRecord(ev, idle));   // re-record at once, on an idle stream
        hipLaunchKernelGGL(k_copy, dim3(1), dim3(64), 0, b, d, out);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(&h, out, 4, hipMemcpyDeviceToHost));
        std::printf("D rep %d: wait then immediate re-record -> waiter read %d (%s)\n", rep, h,
                    h == 1 ? "ordered: the wait kept the first record" : "RE-RECORD BROKE THE WAIT");
        fails += h != 1;
    }
    std::printf("summary: null-stream hipMemset %s, pageable hipMemcpy %s; own-stream upload + sync %s; event re-record %s\n",
                memset_races ? "RACES with non-blocking streams" : "ordered",
                memcpy_races ? "RACES with non-blocking streams" : "ordered", fails ? "FAILED" : "ordered",
                fails ? "see above" : "safe");
    return fails ? 1 : 0;
}
