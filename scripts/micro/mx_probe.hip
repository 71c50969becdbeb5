// Diagnostics: the two hardware facts the blur-at-the-samples describe (k_describe_sb) relies on, checked on the GPU.
//
//   1. A 32-bit LDS read at a 2-byte-aligned address returns the 4 bytes that start there (ds_read_b32 and the two
//      dwords of ds_read2_b32 offset1:1), so a u16 pair (H[r], H[r+1]) is one read whatever the parity of r.
//   2. v_mfma_i32_16x16x64_i8 pairs element e of lane group g = lane >> 4 of A with element e of lane group g of B
//      (A[row lane & 15], B[col lane & 15]), so a k labelling chosen by the kernel is free as long as A and B share
//      it; the result is read in the documented C map (col = lane & 15, row = 4 (lane >> 4) + reg).
//   3. Cycles per MFMA of 16x16x64_i8 and the CDNA3-form 16x16x32_i8, back to back on one wave (s_memtime).
//
// hipcc -O2 --offload-arch=gfx950 scripts/micro/mx_probe.hip -o build/mx_probe && build/mx_probe
#include <hip/hip_runtime.h>

#include <cstdint>
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

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void k_lds_unaligned(uint32_t* out) {
    __shared__ __attribute__((aligned(16))) uint8_t s[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) s[i] = (uint8_t)(i * 7 + 3);
    __syncthreads();
    const uint32_t a = (uint32_t)(uintptr_t)(s + 2 + 6 * threadIdx.x);   // 2 mod 4 for even lanes, 0 mod 4 for odd
    uint32_t r0, r1, r2;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r0) : "v"(a) : "memory");
    asm volatile("ds_read2_b32 %0, %1 offset0:0 offset1:1\n\ts_waitcnt lgkmcnt(0)" : "=v"(*(uint64_t*)&r1) : "v"(a) : "memory");
    (void)r2;
    out[3 * threadIdx.x + 0] = r0;
    uint64_t p;
    asm volatile("ds_read2_b32 %0, %1 offset0:0 offset1:1\n\ts_waitcnt lgkmcnt(0)" : "=v"(p) : "v"(a) : "memory");
    out[3 * threadIdx.x + 1] = (uint32_t)p;
    out[3 * threadIdx.x + 2] = (uint32_t)(p >> 32);
}

__global__ void k_mfma(const int8_t* A, const int8_t* B, int* C) {   // A 16 x 64 row-major, B 64 x 16 row-major
    const int l = threadIdx.x, g = l >> 4, r = l & 15;
    v4i a, b;
    int8_t* pa = (int8_t*)&a;
    int8_t* pb = (int8_t*)&b;
    for (int e = 0; e < 16; ++e) {
        pa[e] = A[r * 64 + 16 * g + e];
        pb[e] = B[(16 * g + e) * 16 + r];
    }
    v4i c = {1000, 1000, 1000, 1000};
    c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
    for (int j = 0; j < 4; ++j) C[(4 * g + j) * 16 + r] = c[j];
}

template <int kForm>
__global__ void k_mfma_rate(int* out, long long* cyc, int n) {
    v4i a = {(int)threadIdx.x, 3, 5, 7}, b = {11, (int)threadIdx.x, 13, 17};
    v4i c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
        if constexpr (kForm == 64) {
            c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c3, 0, 0, 0);
        } else {
            const long la = ((long)a.y << 32) | (unsigned)a.x, lb = ((long)b.y << 32) | (unsigned)b.x;
            c0 = __builtin_amdgcn_mfma_i32_16x16x32_i8(la, lb, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_i32_16x16x32_i8(la, lb, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_i32_16x16x32_i8(la, lb, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_i32_16x16x32_i8(la, lb, c3, 0, 0, 0);
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = c0.x + c1.y + c2.z + c3.w;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
    int bad = 0;
    {
        uint32_t* d;
        CK(hipMalloc(&d, 64 * 3 * 4));
        k_lds_unaligned<<<1, 64>>>(d);
        CK(hipDeviceSynchronize());
        uint32_t h[64 * 3];
        CK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
        int nbad = 0;
        for (int l = 0; l < 64; ++l) {
            const int a = 2 + 6 * l;
            auto word = [&](int o) {
                uint32_t w = 0;
                for (int b = 0; b < 4; ++b) w |= (uint32_t)(uint8_t)((o + b) * 7 + 3) << (8 * b);
                return w;
            };
            if (h[3 * l] != word(a) || h[3 * l + 1] != word(a) || h[3 * l + 2] != word(a + 4)) {
                if (nbad++ < 4)
                    std::printf("  lane %d addr %d: b32 %08x read2 %08x %08x expected %08x %08x\n", l, a, h[3 * l],
                                h[3 * l + 1], h[3 * l + 2], word(a), word(a + 4));
            }
        }
        std::printf("lds_unaligned_b32: %s (%d of 64 lanes differ)\n", nbad ? "FAIL" : "ok", nbad);
        bad += nbad != 0;
        CK(hipFree(d));
    }
    {
        int8_t hA[16 * 64], hB[64 * 16];
        srand(7);
        for (auto& v : hA) v = (int8_t)(rand() % 256 - 128);
        for (auto& v : hB) v = (int8_t)(rand() % 256 - 128);
        int8_t *dA, *dB;
        int* dC;
        CK(hipMalloc(&dA, sizeof(hA)));
        CK(hipMalloc(&dB, sizeof(hB)));
        CK(hipMalloc(&dC, 256 * 4));
        CK(hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice));
        CK(hipMemcpy(dB, hB, sizeof(hB), hipMemcpyHostToDevice));
        k_mfma<<<1, 64>>>(dA, dB, dC);
        CK(hipDeviceSynchronize());
        int hC[256];
        CK(hipMemcpy(hC, dC, sizeof(hC), hipMemcpyDeviceToHost));
        int nbad = 0;
        for (int m = 0; m < 16; ++m)
            for (int n = 0; n < 16; ++n) {
                int s = 1000;
                for (int k = 0; k < 64; ++k) s += hA[m * 64 + k] * hB[k * 16 + n];
                if (s != hC[m * 16 + n] && nbad++ < 4) std::printf("  C[%d][%d] = %d expected %d\n", m, n, hC[m * 16 + n], s);
            }
        std::printf("mfma_i32_16x16x64_i8 symmetric A/B map + C map: %s (%d of 256 differ)\n", nbad ? "FAIL" : "ok", nbad);
        bad += nbad != 0;
    }
    {
        int* dout;
        long long* dc;
        CK(hipMalloc(&dout, 64 * 4));
        CK(hipMalloc(&dc, 8));
        for (int form : {64, 32}) {
            long long best = 1LL << 60;
            for (int rep = 0; rep < 5; ++rep) {
                if (form == 64) k_mfma_rate<64><<<1, 64>>>(dout, dc, 1000);
                else k_mfma_rate<32><<<1, 64>>>(dout, dc, 1000);
                CK(hipDeviceSynchronize());
                long long c;
                CK(hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost));
                best = c < best ? c : best;
            }
            std::printf("mfma_i32_16x16x%d_i8: %.1f cycles per MFMA (one wave, 4 accumulators)\n", form, best / 4000.0);
        }
    }
    return bad ? 1 : 0;
}
