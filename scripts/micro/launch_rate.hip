// Micro-benchmark: how fast does the dispatcher launch short waves?  Empty-ish kernels over large grids.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty(int* out, int n) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && n < 0) out[0] = 1;
}
__global__ void k_work(int* out, int iters) {
    int v = threadIdx.x;
    for (int i = 0; i < iters; ++i) v = v * 1664525 + 1013904223;
    if (v == 0x7fffffff) out[0] = v;
}

__global__ void k_lds(int* out, int n) {
    extern __shared__ int sm[];
    sm[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (sm[(threadIdx.x + 1) & 255] == n) out[0] = 1;
}

int main() {
    int* d;
    (void)hipMalloc(&d, 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int bs : {64, 256, 1024}) {
        for (int waves : {65536, 262144, 1048576}) {
            const int blocks = waves * 64 / bs;
            for (int rep = 0; rep < 2; ++rep) {
                (void)hipEventRecord(a);
                hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(bs), 0, 0, d, 1);
                (void)hipEventRecord(b);
                (void)hipEventSynchronize(b);
            }
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            printf("empty bs=%4d waves=%8d : %8.3f ms  %.3f waves/ns\n", bs, waves, ms, waves / (ms * 1e6));
        }
    }
    for (int lds : {0, 8192, 22528, 40960}) {
        const int blocks = 150000;
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipEventRecord(a);
            hipLaunchKernelGGL(k_lds, dim3(blocks), dim3(256), lds + 1024, 0, d, -5);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
        }
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        printf("lds+barrier bs=256 blocks=%d lds=%d : %.3f ms\n", blocks, lds + 1024, ms);
    }
    for (int iters : {100, 1000}) {
        const int waves = 262144;
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k_work, dim3(waves / 4), dim3(256), 0, 0, d, iters);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        printf("work iters=%d waves=%d : %.3f ms\n", iters, waves, ms);
    }
    return 0;
}
