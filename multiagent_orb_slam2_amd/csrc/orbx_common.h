// Shared helpers for the orbx HIP sources (gfx950 / CDNA4, wave64).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <mutex>
#include <string>

#include "../../include/orbx.h"

namespace orbx {

// An object's own stream (the queue of its host-API entry points), created on first use: an object driven only
// through the device API (caller's streams) never creates one, so it holds no hardware queue -- streams beyond
// GPU_MAX_HW_QUEUES share queues, and two busy streams on one queue serialise.
// A non-blocking stream that may not use every compute unit: cu_exclude > 0 leaves that many CUs (every k-th of the
// device's CU enumeration, so the excluded ones spread over the shader engines) out of its CU mask, so that work on
// streams without the mask (the keyframe path's chain of small kernels) finds free CUs while the front end fills the
// rest.  CU masks carry no priority; cu_exclude <= 0 gives a plain stream of the given priority.
inline hipError_t create_stream_masked(hipStream_t* s, int priority, int cu_exclude) {
    if (cu_exclude == 0 || cu_exclude < -4096) return hipStreamCreateWithPriority(s, hipStreamNonBlocking, priority);
    int dev = 0, n = 0;
    hipError_t he = hipGetDevice(&dev);
    if (he == hipSuccess) he = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    if (he != hipSuccess) return he;
    uint32_t mask[32] = {};
    const int words = (n + 31) / 32;
    if (words > 32) return hipErrorInvalidValue;
    if (cu_exclude < 0) {                              // keep -cu_exclude CUs, every (n / keep)-th one
        const int keep = -cu_exclude;
        if (keep >= n) return hipStreamCreateWithPriority(s, hipStreamNonBlocking, priority);
        const int k = n / keep;
        int kept = 0;
        for (int i = 0; i < n && kept < keep; ++i)
            if (i % k == 0) { mask[i >> 5] |= 1u << (i & 31); ++kept; }
        return hipExtStreamCreateWithCUMask(s, (uint32_t)words, mask);
    }
    if (cu_exclude >= n) return hipErrorInvalidValue;
    const int k = n / cu_exclude;
    int dropped = 0;
    for (int i = 0; i < n; ++i) {
        const bool drop = dropped < cu_exclude && (i % k) == k - 1;
        dropped += drop ? 1 : 0;
        if (!drop) mask[i >> 5] |= 1u << (i & 31);
    }
    return hipExtStreamCreateWithCUMask(s, (uint32_t)words, mask);
}

// Device-memory initialisation (hipMalloc'd tables and counters filled with hipMemset / hipMemcpy on the null stream)
// is complete only after this returns.  hipMemset returns before the device has done it, and the null stream does not
// order the non-blocking streams every kernel of this library runs on (scripts/micro/stream_order.hip, case A): the
// first kernel after an initialisation could otherwise run before it, or have its results overwritten by it.
inline hipError_t init_done() { return hipStreamSynchronize(nullptr); }

// Diagnostics: a kernel that occupies `stream` for about `ms` milliseconds (bounded spin on the 100 MHz constant
// clock), used by tests to delay one stream and expose a missing ordering edge deterministically.
hipError_t debug_spin(hipStream_t stream, double ms);

// Host-graph captures and the library's device-wide / legacy-stream operations, process-wide.  An extractor captures
// its host call on its first call per configuration (orbx_extract); a hipDeviceSynchronize, a hipFree or a
// synchronous hipMemset / hipMemcpy from another thread meanwhile (a second extractor configuring itself on the
// first frame, Frame.cc:78-81) fails with "operation would make the legacy stream depend on a capturing blocking
// stream" and invalidates the capture.  Both hold this lock, innermost: no other lock is taken while it is held.
inline std::recursive_mutex& legacy_mutex() {
    static std::recursive_mutex m;
    return m;
}
struct LegacyLock {
    std::lock_guard<std::recursive_mutex> g{legacy_mutex()};
};
inline hipError_t device_sync() {
    LegacyLock l;
    return hipDeviceSynchronize();
}

inline hipStream_t lazy_stream(hipStream_t& s, std::once_flag& once, int device) {
    std::call_once(once, [&] {
        int cur = 0;
        (void)hipGetDevice(&cur);
        (void)hipSetDevice(device);
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) s = nullptr;
        (void)hipSetDevice(cur);
    });
    return s;
}

// ---------------------------------------------------------------------------------------------
// Error reporting: every C-ABI entry returns a status and leaves a message for orbx_last_error().
// ---------------------------------------------------------------------------------------------
void set_error(const char* fmt, ...);

// Matcher internals shared with orbx_proj.hip (defined in orbx_match.hip): the device a matcher is bound to,
// and its growable scratch buffer + own stream for the host-form entry points.
int matcher_device(const orbx_matcher* m);
int matcher_scratch(orbx_matcher* m, size_t bytes, void** base, void** stream);
// One call's hold on a matcher's scratch / own stream: the matcher's lock for the call's duration, and (used = true)
// the call's stream recorded as the last scratch user, which the next call's stream waits for (Matcher::reserve_on).
void matcher_acquire(orbx_matcher* m);
void matcher_release(orbx_matcher* m, hipStream_t s, bool used);
// Internal entry points across the library's files (not in include/orbx.h): the halves of an extractor's host call and
// where its device outputs are (orbx_extract.hip), for orbx_stereo_frame (orbx_match.hip).
extern "C" {
int orbx_internal_extract_begin(orbx_extractor* e, const uint8_t* image, int rows, int cols, size_t step);
int orbx_internal_extract_end(orbx_extractor* e, orbx_keypoint* kps, uint8_t* desc, int capacity, int* n_out);
int orbx_internal_host_outputs(orbx_extractor* e, const orbx_keypoint** kps, const uint8_t** desc, const int32_t** count,
                               int* capacity, void** stream);
}

struct MatcherLease {
    orbx_matcher* m;
    hipStream_t s = nullptr;
    bool used = false;   // set once s is the stream the call's scratch work runs on
    MatcherLease(orbx_matcher* mm, hipStream_t st) : m(mm), s(st), used(true) { matcher_acquire(m); }
    explicit MatcherLease(orbx_matcher* mm) : m(mm) { matcher_acquire(m); }
    void on(hipStream_t st) { s = st; used = true; }
    ~MatcherLease() { matcher_release(m, s, used); }
    MatcherLease(const MatcherLease&) = delete;
    MatcherLease& operator=(const MatcherLease&) = delete;
};

#define ORBX_HIP(call)                                                                          \
    do {                                                                                        \
        hipError_t e_ = (call);                                                                 \
        if (e_ != hipSuccess) {                                                                 \
            ::orbx::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
            return ORBX_ERR_HIP;                                                                \
        }                                                                                       \
    } while (0)

#define ORBX_REQUIRE(cond, code, ...)      \
    do {                                   \
        if (!(cond)) {                     \
            ::orbx::set_error(__VA_ARGS__); \
            return (code);                 \
        }                                  \
    } while (0)

// ---------------------------------------------------------------------------------------------
// Device helpers
// ---------------------------------------------------------------------------------------------
constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0)); }

// number of set bits of 'mask' in lanes below this lane
__device__ __forceinline__ int lanes_below(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
}

// Wave-uniform minimum: DPP inside each 16-lane row (quad xor 1, xor 2, half-row mirror, row mirror -- all
// VALU, no LDS), then the four row results read into scalars.  Every lane must be active.
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0xB1, 0xF, 0xF, false));    // quad_perm 1,0,3,2
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x4E, 0xF, 0xF, false));    // quad_perm 2,3,0,1
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x141, 0xF, 0xF, false));   // row_half_mirror
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x140, 0xF, 0xF, false));   // row_mirror
    const uint32_t r0 = __builtin_amdgcn_readlane(v, 0), r1 = __builtin_amdgcn_readlane(v, 16);
    const uint32_t r2 = __builtin_amdgcn_readlane(v, 32), r3 = __builtin_amdgcn_readlane(v, 48);
    return min(min(r0, r1), min(r2, r3));
}

// Wave-uniform sum by DPP inside each 16-lane row (no LDS traffic), then the four row sums as scalars.
// Every lane must be active.
__device__ __forceinline__ int wave_sum_dpp(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);     // quad_perm 1,0,3,2
    v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);     // quad_perm 2,3,0,1
    v += __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false);    // row_half_mirror
    v += __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false);    // row_mirror
    return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
           __builtin_amdgcn_readlane(v, 48);
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

__device__ __forceinline__ int wave_incl_scan(int v) {
    const int l = lane_id();
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        int t = __shfl_up(v, o, kWave);
        if (l >= o) v += t;
    }
    return v;
}

// Block-wide exclusive scan of one int per thread.  'tmp' = LDS scratch of >= (blockDim/64 + 1) ints.
// Returns the exclusive prefix; *total receives the block sum.  Contains two barriers.
__device__ __forceinline__ int block_excl_scan(int v, int* tmp, int* total) {
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int inc = wave_incl_scan(v);
    if (lane_id() == kWave - 1) tmp[w] = inc;
    __syncthreads();
    int off = 0, tot = 0;
    for (int i = 0; i < nw; ++i) {
        const int t = tmp[i];
        off += (i < w) ? t : 0;
        tot += t;
    }
    __syncthreads();
    *total = tot;
    return off + inc - v;
}

// Exclusive scan over n items held in 'a' (LDS), in place, using the whole block: each thread owns a
// contiguous chunk.  Returns the total.  'tmp' as above.
__device__ __forceinline__ int block_scan_array(int* a, int n, int* tmp) {
    const int T = blockDim.x;
    const int per = (n + T - 1) / T;
    const int b = threadIdx.x * per, e = min(b + per, n);
    int s = 0;
    for (int i = b; i < e; ++i) s += a[i];
    int total;
    int off = block_excl_scan(s, tmp, &total);
    for (int i = b; i < e; ++i) {
        const int t = a[i];
        a[i] = off;
        off += t;
    }
    __syncthreads();
    return total;
}

// Bitonic sort (ascending) of P2 (a power of two) 64-bit keys in LDS by the whole block (blockDim a multiple of 64).
// Thread t takes compare pairs p = t, t + T, ...: pair p of stage j is (i, i | j) with i = p with a zero bit inserted at
// log2(j), so the 64 pairs of a wave span 128 consecutive keys and every stage with j <= 64 stays inside one wave: those
// stages need only a wave-level fence; only the stages with j >= 128 (10 of 66 at P2 = 2048) take a block barrier.
// Every thread must call it; it ends with a block barrier.
__device__ __forceinline__ void block_bitonic_u64(unsigned long long* a, int P2) {
    const int half = P2 >> 1;
    for (int k = 2; k <= P2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int p = threadIdx.x; p < half; p += blockDim.x) {
                const int i = ((p & ~(j - 1)) << 1) | (p & (j - 1)), ixj = i | j;
                const unsigned long long x = a[i], y = a[ixj];
                if ((x > y) == ((i & k) == 0)) { a[i] = y; a[ixj] = x; }
            }
            const int nj = j > 1 ? j >> 1 : k;                   // the next stage's j
            if (j >= 128 || nj >= 128) {
                __syncthreads();
            } else {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
    __syncthreads();
}

// XCD-aware block -> work-item mapping.  Workgroups are dealt round-robin to the 8 XCDs (blocks b and
// b + 8 share one XCD and its 4 MiB L2; MI355X_MICROARCH.md, workgroup dispatch), so with a 1-D grid of
// 8 * chunk blocks XCD x gets the contiguous items [x * chunk, (x + 1) * chunk) in dispatch order:
// neighbouring items (adjacent cells, keypoints of one image) share one L2 instead of being fetched by
// all eight.  Placement is used for speed only; correctness never depends on it.
constexpr int kXcds = 8;
__host__ __device__ __forceinline__ int xcd_chunk(int total) { return (total + kXcds - 1) / kXcds; }
__device__ __forceinline__ int xcd_item(int chunk) {
    const int b = (int)blockIdx.x;
    return (b % kXcds) * chunk + b / kXcds;
}

__device__ __forceinline__ int popc32(uint32_t v) { return __builtin_popcount(v); }

// 256-bit Hamming distance (ORBmatcher::DescriptorDistance, src/ORBmatcher.cc:1649-1665): the
// reference's SWAR popcount of 8 XORed 32-bit words equals the bit count, here v_bcnt_u32_b32.
__device__ __forceinline__ int hamming256(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1) {
    return popc32(a0.x ^ b0.x) + popc32(a0.y ^ b0.y) + popc32(a0.z ^ b0.z) + popc32(a0.w ^ b0.w) +
           popc32(a1.x ^ b1.x) + popc32(a1.y ^ b1.y) + popc32(a1.z ^ b1.z) + popc32(a1.w ^ b1.w);
}

}  // namespace orbx
