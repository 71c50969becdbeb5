// =====================================================================================================
// orbx_match.hip — MI355X (gfx950) 256-bit Hamming matchers behind include/orbx.h.
//
//   k_hamming_pairs     ORBmatcher::DescriptorDistance over n row pairs        (src/ORBmatcher.cc:1649-1665)
//   k_bf_mfma           all-pairs match on the matrix cores (default): popcount(q & t) as an i8 dot product of
//                        the unpacked bits, v_mfma_i32_16x16x64_i8, best / second as keys.
//   k_bf_tile/k_bf_merge the VALU form (ORBX_BF_MFMA=0): 64 queries per workgroup (one per lane, descriptor in
//                        8 VGPRs), train descriptors staged through LDS in 256-row blocks and read as
//                        wave-uniform broadcasts; v_xor + v_bcnt_u32_b32; per-(query, train-chunk)
//                        partial best/second merged by a second launch.
//   k_stereo_rows/k_stereo_blk  Frame::ComputeStereoMatches descriptor search (src/Frame.cc:466-552): both
//                        images' keypoints bucketed by row, then one workgroup per (pair, 8 left rows) with the
//                        reachable right buckets staged in LDS, band/octave/disparity mask, packed (dist, index) min;
//                        k_stereo (one wave per left keypoint) for the host API's single frame.
//   k_bow_kfkf / k_bow_kff / k_triangulate   BoW-bucketed matchers (src/ORBmatcher.cc:161-290, 524-657,
//                        659-825): one wave per FeatureVector node of the first view; the greedy
//                        "already matched" state is node-local (a feature belongs to one node), so the
//                        wave walks the node's queries in order with lanes over the candidates.
//   k_rot_filter        rotation-consistency histogram + ComputeThreeMaxima (src/ORBmatcher.cc:1603-1644).
// =====================================================================================================
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "orbx_common.h"

namespace orbx {

constexpr int kThHigh = 100, kThLow = 50, kHisto = 30;   // src/ORBmatcher.cc:37-39

__device__ __forceinline__ void load_desc(const uint8_t* p, uint4& a, uint4& b) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    a = q[0];
    b = q[1];
}

__global__ __launch_bounds__(256) void k_hamming_pairs(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b, int n,
                                                       int32_t* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint4 a0, a1, b0, b1;
    load_desc(a + 32 * (size_t)i, a0, a1);
    load_desc(b + 32 * (size_t)i, b0, b1);
    out[i] = hamming256(a0, a1, b0, b1);
}

// ---------------------------------------------------------------------------------------------
// all-pairs brute force
// ---------------------------------------------------------------------------------------------
constexpr int kBfQ = 256;      // queries per workgroup (4 waves, one query per lane)
constexpr int kBfStage = 256;  // train rows staged in LDS per step (8 KB)

// partial record: best (dist << 20 | train idx), second dist.  blockIdx.z = problem: query set z at q + z*q_stride,
// train set z at t + z*t_stride (bytes), partials at z * nchunks * nq.
// (A one-launch form whose last-arriving chunk workgroup folded the partials measured 17.6 us against 11.65 for tile +
// merge; removed in round 6.)
__global__ __launch_bounds__(256) void k_bf_tile(const uint8_t* __restrict__ q, int nq, size_t q_stride, const uint8_t* __restrict__ t,
                                                 int nt, size_t t_stride, int chunk, uint32_t* __restrict__ pbest,
                                                 int32_t* __restrict__ psecond) {
    __shared__ uint4 tile[kBfStage * 2];
    const int qi = blockIdx.x * kBfQ + threadIdx.x;
    const int c = blockIdx.y, z = blockIdx.z, nch = gridDim.y;
    q += (size_t)z * q_stride;
    t += (size_t)z * t_stride;
    const int t0 = c * chunk, t1 = min(nt, t0 + chunk);
    uint4 a0 = make_uint4(0, 0, 0, 0), a1 = a0;
    if (qi < nq) load_desc(q + 32 * (size_t)qi, a0, a1);
    uint32_t best = 256u << 20;   // a distance of 256 never updates (init 256, strict <)
    int second = 256;
    for (int s = t0; s < t1; s += kBfStage) {
        const int cnt = min(kBfStage, t1 - s);
        __syncthreads();
        for (int r = threadIdx.x; r < cnt * 2; r += blockDim.x)
            tile[r] = reinterpret_cast<const uint4*>(t + 32 * (size_t)s)[r];
        __syncthreads();
#pragma unroll 4
        for (int j = 0; j < cnt; ++j) {
            const int d = hamming256(a0, a1, tile[2 * j], tile[2 * j + 1]);
            const uint32_t key = ((uint32_t)d << 20) | (uint32_t)(s + j);
            // reference update: d < best -> (second = best, best = d); else d < second -> second = d
            const uint32_t bd = best >> 20;
            if (key < best) {          // same as d < bd, since indices grow
                second = (int)bd;
                best = key;
            } else if (d < second) {
                second = d;
            }
        }
    }
    if (qi < nq) {
        const size_t o = ((size_t)z * nch + c) * nq + qi;
        pbest[o] = best;
        psecond[o] = second;
    }
}

__global__ __launch_bounds__(256) void k_bf_merge(const uint32_t* __restrict__ pbest, const int32_t* __restrict__ psecond,
                                                  int nq, int nchunks, int32_t* __restrict__ best_idx,
                                                  int32_t* __restrict__ best_dist, int32_t* __restrict__ second_dist) {
    const int qi = blockIdx.x * blockDim.x + threadIdx.x, z = blockIdx.y;
    if (qi >= nq) return;
    pbest += (size_t)z * nchunks * nq;
    psecond += (size_t)z * nchunks * nq;
    uint32_t best = 256u << 20;
    int second = 256;
    for (int c = 0; c < nchunks; ++c) {   // chunks in ascending train order: same rule as a sequential scan
        const uint32_t b = pbest[(size_t)c * nq + qi];
        const int s = psecond[(size_t)c * nq + qi];
        const int bd = (int)(best >> 20), cd = (int)(b >> 20);
        if (cd < bd) {
            second = min(bd, s);
            best = b;
        } else {
            second = min(second, cd);   // the chunk's best is a non-improving value: d >= best
            second = min(second, s);
        }
    }
    const int bd = (int)(best >> 20);
    const size_t o = (size_t)z * nq + qi;
    best_dist[o] = bd;
    best_idx[o] = bd < 256 ? (int)(best & 0xfffff) : -1;
    second_dist[o] = second;
}

// k_bf_merge with the chunk walk split over 8 lanes per query (32 queries per workgroup): the (best key, second
// distance) pair of a chunk range is a top-2 reduction -- best = the smallest (distance, index) key, second = the
// second order statistic of the distances -- so partial pairs combine in any order: (k1, s1) + (k2, s2) =
// k1 < k2 ? (k1, min(s1, d2)) : (k2, min(s2, d1)).  Each lane walks every 8th chunk (independent, coalesced
// loads), the 8 partials meet in LDS.  Same results as the sequential chunk order of k_bf_merge.
#ifndef ORBX_BF_MERGE_G
#define ORBX_BF_MERGE_G 16
#endif
constexpr int kBfMergeG = ORBX_BF_MERGE_G;   // lanes per query (8: 7.4 us merge for one 2000x2000 problem)
__global__ __launch_bounds__(256) void k_bf_merge_g(const uint32_t* __restrict__ pbest, const int32_t* __restrict__ psecond,
                                                    int nq, int nchunks, int32_t* __restrict__ best_idx,
                                                    int32_t* __restrict__ best_dist, int32_t* __restrict__ second_dist) {
    constexpr int kQ = 256 / kBfMergeG;
    __shared__ uint32_t sb[kBfMergeG][kQ];
    __shared__ int32_t ss[kBfMergeG][kQ];
    const int ql = threadIdx.x % kQ, g = threadIdx.x / kQ;
    const int qi = blockIdx.x * kQ + ql, z = blockIdx.y;
    uint32_t best = 256u << 20;
    int second = 256;
    if (qi < nq) {
        const uint32_t* pb = pbest + (size_t)z * nchunks * nq + qi;
        const int32_t* pss = psecond + (size_t)z * nchunks * nq + qi;
#pragma unroll 4
        for (int c = g; c < nchunks; c += kBfMergeG) {
            const uint32_t b = pb[(size_t)c * nq];
            const int sc = pss[(size_t)c * nq];
            if (b < best) {
                second = min(sc, (int)(best >> 20));
                best = b;
            } else {
                second = min(second, (int)(b >> 20));
            }
        }
    }
    sb[g][ql] = best;
    ss[g][ql] = second;
    __syncthreads();
    if (g != 0 || qi >= nq) return;
#pragma unroll
    for (int h = 1; h < kBfMergeG; ++h) {
        const uint32_t b = sb[h][ql];
        const int sc = ss[h][ql];
        if (b < best) {
            second = min(sc, (int)(best >> 20));
            best = b;
        } else {
            second = min(second, (int)(b >> 20));
        }
    }
    const int bd = (int)(best >> 20);
    const size_t o = (size_t)z * nq + qi;
    best_dist[o] = bd;
    best_idx[o] = bd < 256 ? (int)(best & 0xfffff) : -1;
    second_dist[o] = second;
}

// No train rows: every query keeps the reference's initial state (no match, distances 256).
__global__ __launch_bounds__(256) void k_bf_empty(int n, int32_t* __restrict__ best_idx, int32_t* __restrict__ best_dist,
                                                  int32_t* __restrict__ second_dist) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    best_idx[i] = -1;
    best_dist[i] = 256;
    second_dist[i] = 256;
}

// ---------------------------------------------------------------------------------------------
// all-pairs brute force on the matrix cores (the default; ORBX_BF_MFMA=0: k_bf_tile)
// ---------------------------------------------------------------------------------------------
// popcount(q ^ t) = |q| + |t| - 2 popcount(q & t), and popcount(q & t) is the dot product of the two descriptors' bits
// unpacked to 0 / 1 bytes: a 16 x 16 tile of (query, train) pairs is 4 v_mfma_i32_16x16x64_i8 over K = 256 bits.  A
// workgroup takes 64 kMxQt queries (16 kMxQt per wave, unpacked once into the A operands) against a chunk of the train set, staged
// 64 rows at a time: the 256 threads unpack the rows' bits into LDS (256 B per row, padded to kMxStride so the 16
// lanes of a B read sit on distinct banks) with |t| + 256 beside them.  Lane (g, n) of a tile holds train row n and
// query rows 4 g .. 4 g + 3 (the C map); per pair e = |t| + 256 - 2 acc = d - |q| + 256 (|q| is constant per query,
// so e orders the pairs of a query as d does) and the key ((1024 - e) << 20 | 0xfffff - train index) runs through the
// best / second rule as k_bf_tile's, as maxima (best = max key; second = max over the keys that are not the best: its
// distance is the second order statistic).  At the end the 16 lanes of a row group merge their pairs by shuffles, and the keys go back
// to distances with |q|: the chunk partials of k_bf_merge, or the outputs directly when the train set is one chunk.
// A wave holds kMxQt query tiles, so each B fragment it reads from LDS feeds kMxQt MFMAs (the LDS reads and the
// unpack stores per pair were the limit at one tile per wave: 64 queries per workgroup, 112 us for 64 problems).
// Bits are labelled alike on both operands: element e of lane group g of K-step s is bit 64 s + 16 g + e.
#ifndef ORBX_MX_QT
#define ORBX_MX_QT 2
#endif
constexpr int kMxQt = ORBX_MX_QT;                 // 16-query tiles per wave: each B fragment read feeds kMxQt MFMAs
constexpr int kMxQ = 64 * kMxQt, kMxRows = 64, kMxStride = 272;
typedef int mx_v4i __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t mx_nibble(uint32_t v, int j) {   // bits 4 j .. 4 j + 3 of v as four 0 / 1 bytes
    return (((v >> (4 * j)) & 15u) * 0x00204081u) & 0x01010101u;
}
__global__ __launch_bounds__(256) void k_bf_mfma(const uint8_t* __restrict__ q, int nq, size_t q_stride,
                                                 const uint8_t* __restrict__ t, int nt, size_t t_stride, int chunk,
                                                 uint32_t* __restrict__ pbest, int32_t* __restrict__ psecond,
                                                 int32_t* __restrict__ best_idx, int32_t* __restrict__ best_dist,
                                                 int32_t* __restrict__ second_dist) {
    __shared__ __attribute__((aligned(16))) uint8_t tb[kMxRows * kMxStride];
    __shared__ int tsum[kMxRows];
    const int w = threadIdx.x >> 6, l = lane_id(), g = l >> 4, n = l & 15;
    const int c = blockIdx.y, z = blockIdx.z, nch = gridDim.y;
    q += (size_t)z * q_stride;
    t += (size_t)z * t_stride;
    const int qb = blockIdx.x * kMxQ + 16 * kMxQt * w;          // the wave's kMxQt x 16 queries
    const int t0 = c * chunk, t1 = min(nt, t0 + chunk);
    mx_v4i a[kMxQt][4];
#pragma unroll
    for (int u = 0; u < kMxQt; ++u) {
        uint4 d0 = make_uint4(0, 0, 0, 0), d1 = d0;
        const int qi = qb + 16 * u + n;
        if (qi < nq) load_desc(q + 32 * (size_t)qi, d0, d1);
        const uint32_t dw[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
#pragma unroll
        for (int s = 0; s < 4; ++s) {                           // bits 64 s + 16 g .. + 15: half g & 1 of dword 2 s + g / 2
            const uint32_t word = (g >> 1) ? dw[2 * s + 1] : dw[2 * s];
            const uint32_t h = (g & 1) ? word >> 16 : word & 0xffffu;
            a[u][s] = mx_v4i{(int)mx_nibble(h, 0), (int)mx_nibble(h, 1), (int)mx_nibble(h, 2), (int)mx_nibble(h, 3)};
        }
    }
    // keys run as maxima: key = ((1024 - e) << 20) | (0xfffff - index), e = |t| + 256 - 2 acc, so the largest key is the
    // smallest distance with the lowest index; 0 = none (a real key is >= 1 << 20)
    uint32_t best[kMxQt][4], second[kMxQt][4];
#pragma unroll
    for (int u = 0; u < kMxQt; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) best[u][j] = second[u][j] = 0u;
    // thread -> (row r, quarter qq) of a stage: descriptor bytes 8 qq .. 8 qq + 7 -> unpacked bytes 64 qq .. 64 qq + 63.
    // The next stage's bytes are loaded while this stage's tiles run.
    const int r = threadIdx.x >> 2, qq = threadIdx.x & 3;
    uint2 nx = make_uint2(0, 0);
    if (t0 + r < t1) nx = *reinterpret_cast<const uint2*>(t + 32 * (size_t)(t0 + r) + 8 * qq);
    for (int s0 = t0; s0 < t1; s0 += kMxRows) {
        const int cnt = min(kMxRows, t1 - s0);
        const uint32_t v0 = nx.x, v1 = nx.y;
        nx = make_uint2(0, 0);                                   // rows past the chunk unpack to zeros
        if (s0 + kMxRows + r < t1) nx = *reinterpret_cast<const uint2*>(t + 32 * (size_t)(s0 + kMxRows + r) + 8 * qq);
        __syncthreads();
        {
            int pc = popc32(v0) + popc32(v1);
            pc += __builtin_amdgcn_update_dpp(0, pc, 0xB1, 0xF, 0xF, false);    // quad_perm 1,0,3,2
            pc += __builtin_amdgcn_update_dpp(0, pc, 0x4E, 0xF, 0xF, false);    // quad_perm 2,3,0,1
            uint4* dst = reinterpret_cast<uint4*>(tb + r * kMxStride + 64 * qq);
            dst[0] = make_uint4(mx_nibble(v0, 0), mx_nibble(v0, 1), mx_nibble(v0, 2), mx_nibble(v0, 3));
            dst[1] = make_uint4(mx_nibble(v0, 4), mx_nibble(v0, 5), mx_nibble(v0, 6), mx_nibble(v0, 7));
            dst[2] = make_uint4(mx_nibble(v1, 0), mx_nibble(v1, 1), mx_nibble(v1, 2), mx_nibble(v1, 3));
            dst[3] = make_uint4(mx_nibble(v1, 4), mx_nibble(v1, 5), mx_nibble(v1, 6), mx_nibble(v1, 7));
            // rows past the chunk: e = 1023 > any real e (<= 512), never a best; as a second it clamps to 256 below
            if (qq == 0) tsum[r] = r < cnt ? pc + 256 : 1023;
        }
        __syncthreads();
        for (int tt = 0; tt < kMxRows / 16; ++tt) {
            if (16 * tt >= cnt) break;                           // workgroup-uniform
            const int row = 16 * tt + n;
            mx_v4i b[4];
#pragma unroll
            for (int s = 0; s < 4; ++s) b[s] = *reinterpret_cast<const mx_v4i*>(tb + row * kMxStride + 64 * s + 16 * g);
            // key = acc * 2^21 + k0 with k0 = ((1024 - |t| - 256) << 20) | (0xfffff - index): one v_mad_u32_u24 per pair
            // (acc <= 256; emitted by the compiler, which also pads the MFMA -> VALU read of acc)
            const uint32_t k0 = ((uint32_t)(1024 - tsum[row]) << 20) | (uint32_t)(0xfffff - (s0 + row));
#pragma unroll
            for (int u = 0; u < kMxQt; ++u) {
                mx_v4i acc = {0, 0, 0, 0};
#pragma unroll
                for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[u][s], b[s], acc, 0, 0, 0);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t key = __umul24((uint32_t)acc[j], 1u << 21) + k0;
                    // best >= second always, so max(second, min(best, key)) is the median of the three (asm: the
                    // compiler does not form v_med3_u32 from variables; its operands are VALU results, no MFMA hazard)
                    uint32_t m3;
                    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(m3) : "v"(best[u][j]), "v"(key), "v"(second[u][j]));
                    second[u][j] = m3;
                    best[u][j] = max(best[u][j], key);
                }
            }
        }
    }
    // the 16 lanes of a row group (one train column each) merge: (b1, s1) + (b2, s2) = (max b, max(s1, s2, min b))
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
#pragma unroll
        for (int u = 0; u < kMxQt; ++u)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t ob = (uint32_t)__shfl_xor((int)best[u][j], o, 16);
                const uint32_t os = (uint32_t)__shfl_xor((int)second[u][j], o, 16);
                second[u][j] = max(max(second[u][j], os), min(best[u][j], ob));
                best[u][j] = max(best[u][j], ob);
            }
    }
    if (n >= 4 * kMxQt) return;
    const int u = n >> 2, j = n & 3, qi = qb + 16 * u + 4 * g + j;   // lane n < 4 kMxQt of row group g: tile u, row 4 g + j
    if (qi >= nq) return;
    uint32_t bk = best[0][0], sk = second[0][0];
#pragma unroll
    for (int uu = 0; uu < kMxQt; ++uu)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const bool me = u == uu && j == k;
            bk = me ? best[uu][k] : bk;
            sk = me ? second[uu][k] : sk;
        }
    uint4 d0, d1;
    load_desc(q + 32 * (size_t)qi, d0, d1);
    const int nq1 = popc32(d0.x) + popc32(d0.y) + popc32(d0.z) + popc32(d0.w) + popc32(d1.x) + popc32(d1.y) +
                    popc32(d1.z) + popc32(d1.w);
    // back to distances (d = e - 256 + |q| = 768 - (key >> 20) + |q|, index = 0xfffff - low bits); the reference's
    // initial (256, 256) with strict < : a best needs d < 256, distances clamp at 256
    const int db = bk == 0u ? 256 : 768 - (int)(bk >> 20) + nq1;
    const int ds = sk == 0u ? 256 : min(256, 768 - (int)(sk >> 20) + nq1);
    const bool found = db < 256;
    const uint32_t bidx = 0xfffffu - (bk & 0xfffffu);
    if (pbest) {
        const size_t o = ((size_t)z * nch + c) * nq + qi;
        pbest[o] = found ? ((uint32_t)db << 20) | bidx : (256u << 20);
        psecond[o] = found ? ds : 256;
    } else {
        const size_t o = (size_t)z * nq + qi;
        best_dist[o] = found ? db : 256;
        best_idx[o] = found ? (int)bidx : -1;
        second_dist[o] = found ? ds : 256;
    }
}

// ---------------------------------------------------------------------------------------------
// stereo band match
// ---------------------------------------------------------------------------------------------
struct StereoArgs {
    const orbx_keypoint* kl; const uint8_t* dl; const int32_t* nl;
    const orbx_keypoint* kr; const uint8_t* dr; const int32_t* nr;
    int capacity;           // per-image stride of the batched layout
    int nl_fixed, nr_fixed; // used when nl/nr are null
    float scale[32];
    int nlevels, rows;
    int band;               // rows a right keypoint's band can reach: ceil(2 * max scale) + 2
    float maxD;             // bf / b (Frame.cc:496-498)
    int32_t* row_start;     // [batch][rows + 1]  right keypoints bucketed by floor(y)
    int32_t* row_idx;       // [batch][capacity]
    int32_t* lrow_start;    // [batch][rows + 1]  left keypoints bucketed by vRowIndices row (int)y (k_stereo_blk)
    int32_t* lrow_idx;      // [batch][capacity]
    int32_t* best_idx; int32_t* best_dist;
    int batch, nbx;         // images; k_stereo: workgroups per image (XCD-aware 1-D grid)
};

// Counting sort of one image pair's right keypoints by row (the row table of Frame.cc:476-493, kept as
// a bucket per floor(y) instead of one list per covered row); order inside a bucket is irrelevant
// because the search below reduces with a (distance, index) minimum.  blockIdx.y = 1: the left keypoints'
// buckets, in a workgroup of their own.
#ifndef ORBX_STEREO_ROWS_T
#define ORBX_STEREO_ROWS_T 256
#endif
constexpr int kStereoRowsThreads = ORBX_STEREO_ROWS_T;
__global__ __launch_bounds__(kStereoRowsThreads) void k_stereo_rows(StereoArgs A) {
    extern __shared__ int cnt[];   // rows + 1
    __shared__ int tmp[40];
    const int img = blockIdx.x, tid = threadIdx.x;
    const size_t ob = (size_t)img * A.capacity;
    if (blockIdx.y == 1) {
        if (!A.lrow_start) return;
        // the left keypoints by their own row (vRowIndices index (int)y, :511); rows outside the image go to the last
        // bucket and find nothing (the search re-checks the row)
        const int nl = A.nl ? A.nl[img] : A.nl_fixed;
        for (int r = tid; r <= A.rows; r += blockDim.x) cnt[r] = 0;
        __syncthreads();
        for (int i = tid; i < nl; i += blockDim.x) atomicAdd(&cnt[min(max((int)A.kl[ob + i].y, 0), A.rows - 1)], 1);
        __syncthreads();
        block_scan_array(cnt, A.rows + 1, tmp);
        int32_t* ls = A.lrow_start + (size_t)img * (A.rows + 1);
        for (int r = tid; r <= A.rows; r += blockDim.x) ls[r] = cnt[r];
        __syncthreads();
        for (int i = tid; i < nl; i += blockDim.x)
            A.lrow_idx[ob + atomicAdd(&cnt[min(max((int)A.kl[ob + i].y, 0), A.rows - 1)], 1)] = i;
        return;
    }
    const int nr = A.nr ? A.nr[img] : A.nr_fixed;
    for (int r = tid; r <= A.rows; r += blockDim.x) cnt[r] = 0;
    __syncthreads();
    for (int i = tid; i < nr; i += blockDim.x) {
        const int r = min(max((int)floorf(A.kr[ob + i].y), 0), A.rows - 1);
        atomicAdd(&cnt[r], 1);
    }
    __syncthreads();
    block_scan_array(cnt, A.rows + 1, tmp);
    int32_t* rs = A.row_start + (size_t)img * (A.rows + 1);
    for (int r = tid; r <= A.rows; r += blockDim.x) rs[r] = cnt[r];
    __syncthreads();
    for (int i = tid; i < nr; i += blockDim.x) {
        const int r = min(max((int)floorf(A.kr[ob + i].y), 0), A.rows - 1);
        A.row_idx[ob + atomicAdd(&cnt[r], 1)] = i;
    }
}

// Row-block form of the search: one workgroup per (image pair, kStereoRows rows of left keypoints).  The right
// keypoints of every bucket the block's rows can reach ([r0 - band, r1 - 1 + band], a superset of each left
// keypoint's own [vrow - band, vrow + band]) are staged in LDS once -- descriptor, x, the octave and the row band
// [floor(y - 2s), ceil(y + 2s)] of :487-492 -- and each wave takes left keypoints of the block with lanes over the
// staged candidates.  The per-candidate tests are the reference's (row band, octave +-1, disparity window), so the
// candidate set and the (distance, index) minimum are exactly the per-keypoint search's; a candidate outside a left
// keypoint's own bucket window never passes its row test.  Replaces ~8 dependent HBM round trips per left keypoint by one staged
// load per block.
constexpr int kStereoRows = 8, kStereoRC = 256, kStereoLC = 64;
__global__ __launch_bounds__(256) void k_stereo_blk(StereoArgs A, int nblk) {
    __shared__ uint4 rd[2 * kStereoRC];
    __shared__ float rx[kStereoRC];
    __shared__ int rband[kStereoRC];     // minr (low 16, signed) | maxr (high 16, signed)
    __shared__ int rmeta[kStereoRC];     // index << 8 | octave
    __shared__ uint4 ldsc[2 * kStereoLC];
    __shared__ float lx[kStereoLC];
    __shared__ int lmeta[kStereoLC];     // vrow << 8 | octave (vrow clamped to 16 bits)
    __shared__ int lidx[kStereoLC];
    __shared__ uint32_t lbest[kStereoLC];
    const int item = xcd_item(xcd_chunk(nblk * A.batch));   // row blocks of one pair on one XCD
    if (item >= nblk * A.batch) return;
    const int img = item / nblk, blk = item - img * nblk;
    const int tid = threadIdx.x, w = tid >> 6, ln = lane_id();
    const size_t ob = (size_t)img * A.capacity;
    const int r0 = blk * kStereoRows, r1 = min(r0 + kStereoRows, A.rows);
    const int32_t* lrs = A.lrow_start + (size_t)img * (A.rows + 1);
    const int32_t* rrs = A.row_start + (size_t)img * (A.rows + 1);
    const int ls = lrs[r0], le = lrs[r1];
    const int rs0 = rrs[max(r0 - A.band, 0)], rs1 = rrs[min(r1 - 1 + A.band, A.rows - 1) + 1];
    for (int lc = ls; lc < le; lc += kStereoLC) {
        const int nL = min(kStereoLC, le - lc);
        __syncthreads();
        for (int t = tid; t < nL; t += 256) {
            const int iL = A.lrow_idx[ob + lc + t];
            const orbx_keypoint k = A.kl[ob + iL];
            const int vrow = (int)k.y;
            lx[t] = k.x;
            lmeta[t] = (min(max(vrow, -32768), 32767) << 8) | (k.octave & 0xff);
            lidx[t] = iL;
            lbest[t] = 0xffffffffu;
            load_desc(A.dl + 32 * (ob + iL), ldsc[2 * t], ldsc[2 * t + 1]);
        }
        for (int rc = rs0; rc < rs1; rc += kStereoRC) {
            const int nR = min(kStereoRC, rs1 - rc);
            __syncthreads();
            for (int t = tid; t < nR; t += 256) {
                const int iR = A.row_idx[ob + rc + t];
                const orbx_keypoint k = A.kr[ob + iR];
                const float r = 2.0f * A.scale[k.octave];                               // :487
                const int maxr = (int)ceilf(k.y + r), minr = (int)floorf(k.y - r);
                rx[t] = k.x;
                rband[t] = (min(max(minr, -32768), 32767) & 0xffff) | (min(max(maxr, -32768), 32767) << 16);
                rmeta[t] = (iR << 8) | (k.octave & 0xff);
                load_desc(A.dr + 32 * (ob + iR), rd[2 * t], rd[2 * t + 1]);
            }
            __syncthreads();
            for (int j = w; j < nL; j += 4) {
                const int lm = lmeta[j];
                const int vrow = lm >> 8, octL = (int)(signed char)(lm & 0xff);
                const float uL = lx[j];
                const float minU = uL - A.maxD, maxU = uL - 0.0f;
                if (vrow < 0 || vrow >= A.rows || maxU < 0) continue;                 // wave-uniform
                const uint4 a0 = ldsc[2 * j], a1 = ldsc[2 * j + 1];
                uint32_t best = 0xffffffffu;
                for (int c = ln; c < nR; c += kWave) {
                    const int rb = rband[c];
                    const int minr = (int)(short)(rb & 0xffff), maxr = rb >> 16;
                    if (vrow < minr || vrow > maxr) continue;                          // row band (:491-492)
                    const int rm = rmeta[c];
                    const int octR = (int)(signed char)(rm & 0xff);
                    if (octR < octL - 1 || octR > octL + 1) continue;                  // :533
                    const float xr = rx[c];
                    if (!(xr >= minU && xr <= maxU)) continue;                         // :538
                    const uint32_t key = ((uint32_t)hamming256(a0, a1, rd[2 * c], rd[2 * c + 1]) << 20) | (uint32_t)(rm >> 8);
                    best = min(best, key);
                }
                best = wave_min_u32(best);
                if (ln == 0) lbest[j] = min(lbest[j], best);
            }
        }
        __syncthreads();
        for (int t = tid; t < nL; t += 256) {
            const uint32_t best = lbest[t];
            int d = (best == 0xffffffffu) ? kThHigh : (int)(best >> 20);
            d = min(d, kThHigh);                                                        // init TH_HIGH, strict <
            const int thOrb = (kThHigh + kThLow) / 2;                                   // :471
            A.best_dist[ob + lidx[t]] = d;
            A.best_idx[ob + lidx[t]] = (d < thOrb) ? (int)(best & 0xfffff) : -1;        // :552
        }
    }
}

// Per-keypoint form of the same search (one wave per left keypoint, lanes over the right buckets its band reaches, the
// same tests and (distance, index) minimum): the host API's single stereo frame (orbx_compute_stereo_matches), where
// the row-block form's 47 staged workgroups per frame cost more latency than ~2,000 independent waves (r6zn: the host
// call's stereo 0.060 -> 0.077 ms with the row-block form).
__global__ __launch_bounds__(256) void k_stereo(StereoArgs A) {
    const int item = xcd_item(xcd_chunk(A.nbx * A.batch));   // left keypoints of one pair on one XCD
    if (item >= A.nbx * A.batch) return;
    const int img = item / A.nbx;
    const int iL = ((item - img * A.nbx) * blockDim.x + threadIdx.x) >> 6;
    const int ln = lane_id();
    const int nl = A.nl ? A.nl[img] : A.nl_fixed;
    if (iL >= nl) return;
    const size_t ob = (size_t)img * A.capacity;
    const orbx_keypoint kL = A.kl[ob + iL];
    const int vrow = (int)kL.y;                      // vRowIndices[vL] (:511)
    const float uL = kL.x;
    const float minU = uL - A.maxD, maxU = uL - 0.0f;
    uint32_t best = 0xffffffffu;
    if (vrow >= 0 && vrow < A.rows && !(maxU < 0)) {
        uint4 a0, a1;
        load_desc(A.dl + 32 * (ob + iL), a0, a1);
        const int32_t* rs = A.row_start + (size_t)img * (A.rows + 1);
        const int c0 = rs[max(vrow - A.band, 0)], c1 = rs[min(vrow + A.band, A.rows - 1) + 1];
        for (int c = c0 + ln; c < c1; c += kWave) {
            const int iR = A.row_idx[ob + c];
            const orbx_keypoint kR = A.kr[ob + iR];
            const float r = 2.0f * A.scale[kR.octave];                       // :487
            const int maxr = (int)ceilf(kR.y + r), minr = (int)floorf(kR.y - r);
            if (vrow < minr || vrow > maxr) continue;                        // row band (:491-492)
            if (kR.octave < kL.octave - 1 || kR.octave > kL.octave + 1) continue;   // :533
            if (!(kR.x >= minU && kR.x <= maxU)) continue;                   // :538
            uint4 b0, b1;
            load_desc(A.dr + 32 * (ob + iR), b0, b1);
            const uint32_t key = ((uint32_t)hamming256(a0, a1, b0, b1) << 20) | (uint32_t)iR;
            best = min(best, key);
        }
    }
    best = wave_min_u32(best);
    if (ln == 0) {
        int d = (best == 0xffffffffu) ? kThHigh : (int)(best >> 20);
        d = min(d, kThHigh);                                                // init TH_HIGH, strict < (:522-547)
        const int thOrb = (kThHigh + kThLow) / 2;                           // :471
        A.best_dist[ob + iL] = d;
        A.best_idx[ob + iL] = (d < thOrb) ? (int)(best & 0xfffff) : -1;    // :552
    }
}

// ---------------------------------------------------------------------------------------------
// BoW-bucketed matchers
// ---------------------------------------------------------------------------------------------
struct FvDev { const uint32_t* node; const int32_t* off; int n; const int32_t* idx; };

__device__ __forceinline__ int fv_lower_bound(const FvDev& f, uint32_t id) {
    int lo = 0, hi = f.n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (f.node[mid] < id) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ int rot_bin(float a1, float a2) {   // src/ORBmatcher.cc:609-614
    float rot = __fsub_rn(a1, a2);
    if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
    int bin = (int)roundf(__fmul_rn(rot, 1.0f / kHisto));
    if (bin == kHisto) bin = 0;
    return bin;
}

// best (lowest position on ties) and multiset-second over one wave's candidates; values 256 = none
// best distance, its (first) position, and the second-best distance of one value per lane, with the
// reference's sequential update rule (ties for the best count as second).  Wave-uniform results.
__device__ __forceinline__ void wave_best2(int d, int pos, int& b1, int& bpos, int& b2) {
    const uint32_t key = ((uint32_t)d << 20) | (uint32_t)pos;
    const uint32_t m = wave_min_u32(key);
    b1 = (int)(m >> 20);
    bpos = (int)(m & 0xfffff);
    b2 = (int)wave_min_u32((key == m) ? 256u : (uint32_t)d);
}

struct BowArgs {
    // view 1 (queries) and view 2 (candidates); angles read with a float stride (1 for a plain array,
    // 7 for orbx_keypoint records, where angle is field 3)
    const uint8_t* d1; const float* a1; int as1; const uint8_t* v1; FvDev f1;
    const uint8_t* d2; const float* a2; int as2; const uint8_t* v2; FvDev f2;
    float nnratio;
    int checkOri;
    int kff;               // 0: KF-KF (TH_LOW strict, greedy on view-2 index, result indexed by view 1)
                           // 1: KF-F  (TH_LOW inclusive, greedy on frame index, result indexed by frame)
    int32_t* match;        // KF-KF: [n1] -> idx2; KF-F: [n2] -> idx1
    int32_t* bin;          // rotation bin per result index
    int32_t* hist;         // [30]
    int32_t* nmatch;
};

// One FeatureVector node of view 1 against the same node of view 2 (merge-join of :547-634 by binary
// search): queries in node order, lanes over the candidates.  Candidate descriptors of the first kBowRegChunks
// 64-wide chunks stay in registers for the whole node, so the sequential (greedy) query loop only loads the
// wave-uniform query descriptor; the "already matched" flags (vbMatched2 / vpMapPointMatches, node-local
// because a feature belongs to exactly one node) are one bit per (lane, chunk) in a register.
constexpr int kBowRegChunks = 2;

// Position of node id in a FeatureVector's ascending node list, or -1: 64 ids per load round and a ballot
// instead of a chain of dependent binary-search loads.
__device__ __forceinline__ int fv_find_wave(const FvDev& f, uint32_t id) {
    for (int base = 0; base < f.n; base += kWave) {
        const int k = base + lane_id();
        const uint32_t v = k < f.n ? f.node[k] : 0xffffffffu;
        const uint64_t hit = __ballot(v == id);
        if (hit) return base + (int)__builtin_ctzll(hit);
        if (__builtin_amdgcn_readlane((int)(v >= id), kWave - 1)) return -1;   // ids ascending: passed it
    }
    return -1;
}

__device__ void bow_node(const BowArgs& A, int a) {
    const int ln = lane_id();
    const uint32_t id = A.f1.node[a];
    const int b = fv_find_wave(A.f2, id);
    if (b < 0) return;
    const int q0 = A.f1.off[a], q1 = A.f1.off[a + 1];
    const int c0 = A.f2.off[b], c1 = A.f2.off[b + 1];
    const int nc = min(c1 - c0, 4096);
    const int nch = (nc + kWave - 1) / kWave;
    uint4 r0[kBowRegChunks], r1[kBowRegChunks];
    bool rok[kBowRegChunks];
#pragma unroll
    for (int c = 0; c < kBowRegChunks; ++c) {
        const int j = c * kWave + ln;
        rok[c] = false;
        r0[c] = r1[c] = make_uint4(0, 0, 0, 0);
        if (j < nc) {
            const int i2 = A.f2.idx[c0 + j];
            rok[c] = A.kff ? true : (A.v2[i2] != 0);
            if (rok[c]) load_desc(A.d2 + 32 * (size_t)i2, r0[c], r1[c]);
        }
    }
    int local = 0;
    if (nc <= kWave) {
        // Small node (the common case): lanes = 64 queries compute their best / second-best over ALL candidates at
        // once (candidate descriptors broadcast by v_readlane), then the greedy loop walks the queries in order with
        // the "already matched" set as one scalar bit mask over candidate positions.  A query's precomputed result is
        // the exact one unless its best position bp or a position j2 (!= bp) holding its second-best value has been
        // taken: without them removed the minimum and its first position are unchanged, and the second-best over
        // the remaining positions is still reached at j2.  Only then is the query redone over the untaken candidates.
        const uint64_t rokm = __ballot(rok[0]);
        uint64_t taken = 0;
        for (int qb = q0; qb < q1; qb += kWave) {
            const int nq = min(kWave, q1 - qb);
            int qi = 0, qv = 0;
            uint4 qx0 = make_uint4(0, 0, 0, 0), qx1 = qx0;
            if (ln < nq) {
                qi = A.f1.idx[qb + ln];
                qv = A.v1[qi] != 0;
                if (qv) load_desc(A.d1 + 32 * (size_t)qi, qx0, qx1);
            }
            int b1 = 256, bp = -1, b2 = 256, j2 = -1;          // the reference's sequential rule, candidate order
            for (int j = 0; j < nc; ++j) {
                if (!((rokm >> j) & 1)) continue;
                uint4 y0, y1;
                y0.x = __builtin_amdgcn_readlane(r0[0].x, j); y0.y = __builtin_amdgcn_readlane(r0[0].y, j);
                y0.z = __builtin_amdgcn_readlane(r0[0].z, j); y0.w = __builtin_amdgcn_readlane(r0[0].w, j);
                y1.x = __builtin_amdgcn_readlane(r1[0].x, j); y1.y = __builtin_amdgcn_readlane(r1[0].y, j);
                y1.z = __builtin_amdgcn_readlane(r1[0].z, j); y1.w = __builtin_amdgcn_readlane(r1[0].w, j);
                const int d = hamming256(qx0, qx1, y0, y1);
                if (d < b1) { b2 = b1; j2 = bp; b1 = d; bp = j; }
                else if (d < b2) { b2 = d; j2 = j; }
            }
            for (int k = 0; k < nq; ++k) {
                if (!__builtin_amdgcn_readlane(qv, k)) continue;
                int kb1 = __builtin_amdgcn_readlane(b1, k), kbp = __builtin_amdgcn_readlane(bp, k);
                int kb2 = __builtin_amdgcn_readlane(b2, k);
                const int kj2 = __builtin_amdgcn_readlane(j2, k);
                if ((kbp >= 0 && ((taken >> kbp) & 1)) || (kj2 >= 0 && ((taken >> kj2) & 1))) {
                    uint4 x0, x1;
                    x0.x = __builtin_amdgcn_readlane(qx0.x, k); x0.y = __builtin_amdgcn_readlane(qx0.y, k);
                    x0.z = __builtin_amdgcn_readlane(qx0.z, k); x0.w = __builtin_amdgcn_readlane(qx0.w, k);
                    x1.x = __builtin_amdgcn_readlane(qx1.x, k); x1.y = __builtin_amdgcn_readlane(qx1.y, k);
                    x1.z = __builtin_amdgcn_readlane(qx1.z, k); x1.w = __builtin_amdgcn_readlane(qx1.w, k);
                    const int d = (rok[0] && !((taken >> ln) & 1)) ? hamming256(x0, x1, r0[0], r1[0]) : 256;
                    wave_best2(d, ln < nc ? ln : 0xfffff, kb1, kbp, kb2);
                }
                const bool pass = A.kff ? (kb1 <= kThLow) : (kb1 < kThLow);      // :230 vs :600
                if (pass && (float)kb1 < A.nnratio * (float)kb2) {
                    taken |= 1ull << kbp;
                    if (ln == 0) {
                        const int i1 = __builtin_amdgcn_readlane(qi, k);
                        const int i2 = A.f2.idx[c0 + kbp];
                        const int ridx = A.kff ? i2 : i1;
                        A.match[ridx] = A.kff ? i1 : i2;
                        if (A.checkOri) {
                            const int bn = rot_bin(A.a1[(size_t)i1 * A.as1], A.a2[(size_t)i2 * A.as2]);
                            A.bin[ridx] = bn;
                            atomicAdd(&A.hist[bn], 1);
                        }
                    }
                    ++local;
                }
            }
        }
        if (ln == 0 && local) atomicAdd(A.nmatch, local);
        return;
    }
    uint64_t taken = 0;   // bit c: candidate c*64 + lane already matched
    for (int qb = q0; qb < q1; qb += kWave) {
        // 64 queries at a time: lane k holds query qb+k (index, MapPoint flag, descriptor); the sequential
        // greedy loop below reads them with v_readlane, so it issues no memory loads of its own
        const int nq = min(kWave, q1 - qb);
        int qi = 0, qv = 0;
        uint4 qx0 = make_uint4(0, 0, 0, 0), qx1 = qx0;
        if (ln < nq) {
            qi = A.f1.idx[qb + ln];
            qv = A.v1[qi] != 0;
            if (qv) load_desc(A.d1 + 32 * (size_t)qi, qx0, qx1);
        }
        for (int k = 0; k < nq; ++k) {
            if (!__builtin_amdgcn_readlane(qv, k)) continue;
            const int i1 = __builtin_amdgcn_readlane(qi, k);
            uint4 x0, x1;
            x0.x = __builtin_amdgcn_readlane(qx0.x, k); x0.y = __builtin_amdgcn_readlane(qx0.y, k);
            x0.z = __builtin_amdgcn_readlane(qx0.z, k); x0.w = __builtin_amdgcn_readlane(qx0.w, k);
            x1.x = __builtin_amdgcn_readlane(qx1.x, k); x1.y = __builtin_amdgcn_readlane(qx1.y, k);
            x1.z = __builtin_amdgcn_readlane(qx1.z, k); x1.w = __builtin_amdgcn_readlane(qx1.w, k);
            int b1 = 256, bp = 0xfffff, b2 = 256;
            auto merge = [&](int d, int j) {   // chunks in candidate order
                int cb1, cbp, cb2;
                wave_best2(d, j < nc ? j : 0xfffff, cb1, cbp, cb2);
                if (cb1 < b1) { b2 = min(b1, cb2); b1 = cb1; bp = cbp; }
                else { b2 = min(b2, min(cb1, cb2)); }
            };
#pragma unroll
            for (int c = 0; c < kBowRegChunks; ++c) {
                if (c < nch) {
                    const int j = c * kWave + ln;
                    const int d = (rok[c] && !((taken >> c) & 1)) ? hamming256(x0, x1, r0[c], r1[c]) : 256;
                    merge(d, j);
                }
            }
            for (int c = kBowRegChunks; c < nch; ++c) {   // large nodes: the remaining chunks from memory
                const int j = c * kWave + ln;
                int d = 256;
                if (j < nc && !((taken >> c) & 1)) {
                    const int i2 = A.f2.idx[c0 + j];
                    if (A.kff || A.v2[i2]) {
                        uint4 y0, y1;
                        load_desc(A.d2 + 32 * (size_t)i2, y0, y1);
                        d = hamming256(x0, x1, y0, y1);
                    }
                }
                merge(d, j);
            }
            const bool pass = A.kff ? (b1 <= kThLow) : (b1 < kThLow);          // :230 vs :600
            if (pass && (float)b1 < A.nnratio * (float)b2) {
                if (ln == (bp & (kWave - 1))) taken |= 1ull << (bp / kWave);
                if (ln == 0) {
                    const int i2 = A.f2.idx[c0 + bp];
                    const int ridx = A.kff ? i2 : i1;
                    A.match[ridx] = A.kff ? i1 : i2;
                    if (A.checkOri) {
                        const int bn = rot_bin(A.a1[(size_t)i1 * A.as1], A.a2[(size_t)i2 * A.as2]);
                        A.bin[ridx] = bn;
                        atomicAdd(&A.hist[bn], 1);
                    }
                }
                ++local;
            }
        }
    }
    if (ln == 0 && local) atomicAdd(A.nmatch, local);
}

// one wave per node of view 1
__global__ __launch_bounds__(64) void k_bow(BowArgs A) {
    if ((int)blockIdx.x >= A.f1.n) return;
    bow_node(A, blockIdx.x);
}

template <typename T>
__device__ __forceinline__ const T* slot_ptr(const T* base, size_t stride, int k) {
    return reinterpret_cast<const T*>(reinterpret_cast<const uint8_t*>(base) + (size_t)k * stride);
}

__device__ __forceinline__ FvDev store_fv(const orbx_kf_store& S, int k) {
    FvDev f;
    f.node = slot_ptr(S.fv_nodes, S.fv_nodes_stride, k);
    f.off = slot_ptr(S.fv_offsets, S.fv_offsets_stride, k);
    f.idx = slot_ptr(S.fv_indices, S.fv_indices_stride, k);
    f.n = *slot_ptr(S.n_fv, S.n_fv_stride, k);
    return f;
}

__global__ __launch_bounds__(64) void k_bow_pairs(orbx_kf_store S, const int32_t* __restrict__ pairs, float nnratio, int checkOri,
                                                  int32_t* match, int32_t* bin, int32_t* hist, int32_t* nmatch) {
    const int pr = blockIdx.y;
    const int k1 = pairs[2 * pr], k2 = pairs[2 * pr + 1];
    if (k1 < 0 || k2 < 0) return;                       // padding pair: no matches
    BowArgs A;
    A.f1 = store_fv(S, k1);
    if ((int)blockIdx.x >= A.f1.n) return;
    A.f2 = store_fv(S, k2);
    A.d1 = slot_ptr(S.desc, S.desc_stride, k1); A.d2 = slot_ptr(S.desc, S.desc_stride, k2);
    A.a1 = &slot_ptr(S.kps, S.kps_stride, k1)->angle; A.a2 = &slot_ptr(S.kps, S.kps_stride, k2)->angle; A.as1 = A.as2 = 7;
    A.v1 = slot_ptr(S.valid, S.valid_stride, k1); A.v2 = slot_ptr(S.valid, S.valid_stride, k2);
    A.nnratio = nnratio; A.checkOri = checkOri; A.kff = 0;
    A.match = match + (size_t)pr * S.capacity; A.bin = bin + (size_t)pr * S.capacity;
    A.hist = hist + (size_t)pr * 32; A.nmatch = nmatch + pr;
    for (int a = blockIdx.x; a < A.f1.n; a += gridDim.x) bow_node(A, a);   // grid.x is only a width hint
}

struct TriArgs {
    const uint8_t* d1; const orbx_keypoint* k1; const uint8_t* mp1; const float* ur1; FvDev f1;
    const uint8_t* d2; const orbx_keypoint* k2; const uint8_t* mp2; const float* ur2; FvDev f2;
    float F[9];
    float sigma2[32], scale2[32];
    float ex, ey;
    int onlyStereo, checkOri;
    int32_t* match; int32_t* bin; int32_t* hist; int32_t* nmatch;
};

// SearchForTriangulation: no greedy coupling between queries (vbMatched2 is never set, :679,727), so
// the result of a query is the LAST candidate (in node order) among those with the minimum distance
// that pass the epipole and epipolar tests (dist <= TH_LOW, ties replace: :740).
// One wave per node: up to 64 queries and 64 candidates of the node are staged in lanes at once (all loads issued
// together), then each query is broadcast to the wave with v_readlane and tested against every candidate lane,
// so the inner loop touches no memory.  s_sig2 / s_sc2: KF2's level tables in LDS.
__device__ __forceinline__ void tri_node(const TriArgs& A, const float* s_sig2, const float* s_sc2, int a) {
    const int ln = lane_id();
    const uint32_t id = A.f1.node[a];
    const int b = fv_lower_bound(A.f2, id);
    if (b >= A.f2.n || A.f2.node[b] != id) return;
    const int q0 = A.f1.off[a], q1 = A.f1.off[a + 1];
    const int c0 = A.f2.off[b], c1 = A.f2.off[b + 1];
    int local = 0;
    for (int qb = q0; qb < q1; qb += kWave) {
        // this lane's query (node position qb + ln)
        const bool qin = qb + ln < q1;
        const int i1 = qin ? A.f1.idx[qb + ln] : 0;
        bool qok = qin && !A.mp1[i1];
        const bool st1 = qok && A.ur1[i1] >= 0;
        if (A.onlyStereo && !st1) qok = false;
        uint4 x0 = make_uint4(0, 0, 0, 0), x1 = x0;
        float la = 0.0f, lb = 0.0f, lc = 0.0f;
        if (qok) {
            const orbx_keypoint kp1 = A.k1[i1];
            load_desc(A.d1 + 32 * (size_t)i1, x0, x1);
            // CheckDistEpipolarLine (:142-159) line coefficients
            la = __fadd_rn(__fadd_rn(__fmul_rn(kp1.x, A.F[0]), __fmul_rn(kp1.y, A.F[3])), A.F[6]);
            lb = __fadd_rn(__fadd_rn(__fmul_rn(kp1.x, A.F[1]), __fmul_rn(kp1.y, A.F[4])), A.F[7]);
            lc = __fadd_rn(__fadd_rn(__fmul_rn(kp1.x, A.F[2]), __fmul_rn(kp1.y, A.F[5])), A.F[8]);
        }
        const float den = __fadd_rn(__fmul_rn(la, la), __fmul_rn(lb, lb));
        const uint64_t qmask = __ballot(qok);
        if (!qmask) continue;
        uint32_t mybest = 0;    // ((256 - d) << 20 | pos): max -> min distance, last position
        for (int cb = c0; cb < c1; cb += kWave) {
            // this lane's candidate (node position cb + ln)
            const bool cin = cb + ln < c1;
            const int i2 = cin ? A.f2.idx[cb + ln] : 0;
            bool cok = cin && !A.mp2[i2];
            const bool st2 = cok && A.ur2[i2] >= 0;
            if (A.onlyStereo && !st2) cok = false;
            uint4 y0 = make_uint4(0, 0, 0, 0), y1 = y0;
            float x2 = 0.0f, y2 = 0.0f, sig2 = 0.0f;
            bool near_epi = false;
            if (cok) {
                const orbx_keypoint kp2 = A.k2[i2];
                load_desc(A.d2 + 32 * (size_t)i2, y0, y1);
                x2 = kp2.x; y2 = kp2.y;
                sig2 = s_sig2[kp2.octave];
                const float dx = __fsub_rn(A.ex, kp2.x), dy = __fsub_rn(A.ey, kp2.y);
                near_epi = __fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)) < __fmul_rn(100.0f, s_sc2[kp2.octave]);
            }
            if (!__ballot(cok)) continue;
            const uint32_t pos = (uint32_t)(cb + ln - c0);
            for (uint64_t mq = qmask; mq; mq &= mq - 1) {
                const int k = __builtin_ctzll(mq);
                uint4 q0v, q1v;
                q0v.x = __builtin_amdgcn_readlane(x0.x, k); q0v.y = __builtin_amdgcn_readlane(x0.y, k);
                q0v.z = __builtin_amdgcn_readlane(x0.z, k); q0v.w = __builtin_amdgcn_readlane(x0.w, k);
                q1v.x = __builtin_amdgcn_readlane(x1.x, k); q1v.y = __builtin_amdgcn_readlane(x1.y, k);
                q1v.z = __builtin_amdgcn_readlane(x1.z, k); q1v.w = __builtin_amdgcn_readlane(x1.w, k);
                const float qa = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, la), k));
                const float qb_ = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, lb), k));
                const float qc = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, lc), k));
                const float qd = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, den), k));
                const bool qst = __builtin_amdgcn_readlane((int)st1, k) != 0;
                uint32_t key = 0;
                if (cok) {
                    const int d = hamming256(q0v, q1v, y0, y1);
                    bool pass = d <= kThLow && !(!qst && !st2 && near_epi) && qd != 0.0f;
                    if (pass) {
                        const float num = __fadd_rn(__fadd_rn(__fmul_rn(qa, x2), __fmul_rn(qb_, y2)), qc);
                        const float dsqr = __fdiv_rn(__fmul_rn(num, num), qd);
                        pass = (double)dsqr < 3.84 * (double)sig2;
                    }
                    if (pass) key = ((uint32_t)(256 - d) << 20) | pos;
                }
                const uint32_t best = ~wave_min_u32(~key);
                if (ln == k) mybest = max(mybest, best);
            }
        }
        const bool hit = mybest != 0;
        if (hit) {
            const int j2 = A.f2.idx[c0 + (int)(mybest & 0xfffff)];
            A.match[i1] = j2;
            if (A.checkOri) {
                const int bn = rot_bin(A.k1[i1].angle, A.k2[j2].angle);
                A.bin[i1] = bn;
                atomicAdd(&A.hist[bn], 1);
            }
        }
        local += __builtin_popcountll(__ballot(hit));
    }
    if (ln == 0 && local) atomicAdd(A.nmatch, local);
}

// KF2's level tables into LDS (byval kernel-argument arrays indexed with constants only)
__device__ __forceinline__ void tri_tables(const float (&sig2)[32], const float (&sc2)[32], float* s_sig2, float* s_sc2) {
#pragma unroll
    for (int l = 0; l < 32; ++l)
        if (lane_id() == l) { s_sig2[l] = sig2[l]; s_sc2[l] = sc2[l]; }
    __syncthreads();
}

__global__ __launch_bounds__(64) void k_triangulate(TriArgs A) {
    __shared__ float s_sig2[32], s_sc2[32];
    if ((int)blockIdx.x >= A.f1.n) return;
    tri_tables(A.sigma2, A.scale2, s_sig2, s_sc2);
    tri_node(A, s_sig2, s_sc2, blockIdx.x);
}

// SearchForTriangulation over (kf1, kf2) slot pairs of a device keyframe store (LocalMapping::CreateNewMapPoints'
// loop over the new keyframe's neighbours, LocalMapping.cc:243-274): MapPoint flags = the store's valid field,
// uright per slot (optional), F12 and the epipole per pair, the level tables of KF2 shared (one extractor).
struct TriTables { float sigma2[32], scale2[32]; };

__global__ __launch_bounds__(64) void k_triangulate_pairs(orbx_kf_store S, const uint8_t* __restrict__ has_mp, size_t mp_stride,
                                                          const float* __restrict__ uright, size_t ur_stride,
                                                          const int32_t* __restrict__ pairs, const orbx_tri_geom* __restrict__ geom,
                                                          TriTables T, int onlyStereo, int checkOri, const float* __restrict__ no_ur,
                                                          int32_t* match, int32_t* bin, int32_t* hist, int32_t* nmatch) {
    __shared__ float s_sig2[32], s_sc2[32];
    const int pr = blockIdx.y;
    const int k1 = pairs[2 * pr], k2 = pairs[2 * pr + 1];
    if (k1 < 0 || k2 < 0) return;                       // padding pair: no matches
    TriArgs A;
    A.f1 = store_fv(S, k1);
    if ((int)blockIdx.x >= A.f1.n) return;
    A.f2 = store_fv(S, k2);
    A.d1 = slot_ptr(S.desc, S.desc_stride, k1); A.d2 = slot_ptr(S.desc, S.desc_stride, k2);
    A.k1 = slot_ptr(S.kps, S.kps_stride, k1); A.k2 = slot_ptr(S.kps, S.kps_stride, k2);
    A.mp1 = has_mp ? slot_ptr(has_mp, mp_stride, k1) : slot_ptr(S.valid, S.valid_stride, k1);
    A.mp2 = has_mp ? slot_ptr(has_mp, mp_stride, k2) : slot_ptr(S.valid, S.valid_stride, k2);
    A.ur1 = uright ? slot_ptr(uright, ur_stride, k1) : no_ur;
    A.ur2 = uright ? slot_ptr(uright, ur_stride, k2) : no_ur;
    const orbx_tri_geom g = geom[pr];
#pragma unroll
    for (int i = 0; i < 9; ++i) A.F[i] = g.F12[i];
    A.ex = g.ex; A.ey = g.ey; A.onlyStereo = onlyStereo; A.checkOri = checkOri;
    A.match = match + (size_t)pr * S.capacity; A.bin = bin + (size_t)pr * S.capacity;
    A.hist = hist + (size_t)pr * 32; A.nmatch = nmatch + pr;
    tri_tables(T.sigma2, T.scale2, s_sig2, s_sc2);
    for (int a = blockIdx.x; a < A.f1.n; a += gridDim.x) tri_node(A, s_sig2, s_sc2, a);   // grid.x: a width hint
}

// rotation-consistency filter: keep matches whose bin is one of the three largest bins
// (ComputeThreeMaxima, :1603-1644, with the 10 % rule); single workgroup.
__global__ __launch_bounds__(256) void k_rot_filter(int32_t* match, const int32_t* bin, int n, const int32_t* hist,
                                                    int32_t* nmatch, int stride) {
    __shared__ int keep[3];
    __shared__ int removed;
    match += (size_t)blockIdx.x * stride;
    bin += (size_t)blockIdx.x * stride;
    hist += (size_t)blockIdx.x * 32;
    nmatch += blockIdx.x;
    if (threadIdx.x == 0) {
        int m1 = 0, m2 = 0, m3 = 0, i1 = -1, i2 = -1, i3 = -1;
        for (int i = 0; i < kHisto; ++i) {
            const int s = hist[i];
            if (s > m1) { m3 = m2; m2 = m1; m1 = s; i3 = i2; i2 = i1; i1 = i; }
            else if (s > m2) { m3 = m2; m2 = s; i3 = i2; i2 = i; }
            else if (s > m3) { m3 = s; i3 = i; }
        }
        if (m2 < 0.1f * (float)m1) { i2 = -1; i3 = -1; }
        else if (m3 < 0.1f * (float)m1) { i3 = -1; }
        keep[0] = i1; keep[1] = i2; keep[2] = i3;
        removed = 0;
    }
    __syncthreads();
    int r = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        if (match[i] < 0) continue;
        const int b = bin[i];
        if (b == keep[0] || b == keep[1] || b == keep[2]) continue;
        match[i] = -1;
        ++r;
    }
    r = wave_sum(r);
    if (lane_id() == 0 && r) atomicAdd(&removed, r);
    __syncthreads();
    if (threadIdx.x == 0) nmatch[0] -= removed;
}

// ---------------------------------------------------------------------------------------------
// stereo sub-pixel refinement (src/Frame.cc:554-639)
// ---------------------------------------------------------------------------------------------
struct RefineArgs {
    const orbx_keypoint* kl; const int32_t* nl; int nl_fixed;
    const orbx_keypoint* kr; const int32_t* best_idx;
    int capacity;
    orbx_pyramid L, R;
    int left_first, right_first;
    float bf, maxD;
    float* uright; float* depth; int32_t* sad;
    int batch, nbx;         // k_stereo_sad_rows: pairs, workgroups per pair (XCD-aware 1-D grid)
};

__device__ __forceinline__ const uint8_t* pyr_level(const orbx_pyramid& P, int img, int l, int& step) {
    if (l == 0) {
        step = (int)P.level0_step;
        return P.level0 + (size_t)img * P.level0_image_stride;
    }
    step = P.cols[l];
    return P.levels + (size_t)img * P.image_stride + P.offset[l];
}

// Row-parallel form: lane (keypoint k of 5 per wave, window row y of 11) loads its row of the left 11 x 11 window
// (11 bytes) and of the right strip that every shift touches (21 bytes: columns iuR0 - 10 .. iuR0 + 10), once, and
// computes its row's share of all 11 SADs -- |(L - cL) - (R - cR(inc))| = |(L + 512 - d) - (R + 512)| with
// d = cL - cR(inc), two pixels per v_sad_u16 -- instead of one lane per (keypoint, shift) re-reading 242 single
// bytes (the first form, one lane per (keypoint, shift); removed in round 6).  Row shares are summed through LDS; each
// keypoint's shift-(-5) lane then runs the reference's sequential tail (first minimum, parabola, disparity test) in
// float with the same operation order.  Every value is a small integer, so the reference's float Mats and
// cv::norm(NORM_L1) give exactly these integer SADs.
constexpr int kSadKpWave = 5;
__device__ __forceinline__ uint32_t pair16(uint32_t lo4, uint32_t hi4, int b) {   // bytes b, b+1 of (hi4:lo4) as u16x2
    return __builtin_amdgcn_perm(hi4, lo4, 0x0c000c00u | (uint32_t)b | ((uint32_t)(b + 1) << 16));
}
__global__ __launch_bounds__(256) void k_stereo_sad_rows(RefineArgs A) {
    constexpr int w = 5, W = 2 * w + 1, Ls = 5, KP = 4 * kSadKpWave;
    __shared__ int part[KP][W][W + 1];      // [keypoint][shift][row]
    __shared__ int dist[KP][W];
    const int item = xcd_item(xcd_chunk(A.nbx * A.batch));
    if (item >= A.nbx * A.batch) return;
    const int img = item / A.nbx, t = threadIdx.x, wv = t >> 6, ln = lane_id();
    const int kq = ln / W, y = ln - kq * W;                    // lanes 55..63: kq = 5 (idle)
    const int q = wv * kSadKpWave + kq;                        // keypoint of the workgroup
    const int l = (item - img * A.nbx) * KP + q;
    const bool lane_kp = kq < kSadKpWave && l < A.capacity;
    const int nl = A.nl ? A.nl[img] : A.nl_fixed;
    const size_t o = (size_t)img * A.capacity + (lane_kp ? l : 0);
    const int bi = (lane_kp && l < nl) ? A.best_idx[o] : -1;
    int oct = 0, ivL = 0, iuL = 0;
    float suR0 = 0.f, uL = 0.f;
    bool ok = bi >= 0;
    int iuR0 = 0;
    if (ok) {
        const orbx_keypoint kp = A.kl[o];
        oct = kp.octave;
        uL = kp.x;
        const float sf = A.L.inv_scale[oct];
        const float uR0 = A.kr[(size_t)img * A.capacity + bi].x;
        const float suL = __builtin_roundf(__fmul_rn(kp.x, sf)), svL = __builtin_roundf(__fmul_rn(kp.y, sf));
        suR0 = __builtin_roundf(__fmul_rn(uR0, sf));
        iuL = (int)suL; ivL = (int)svL; iuR0 = (int)suR0;
        ok = !(ivL - w < 0 || ivL + w >= A.L.rows[oct] || iuL - w < 0 || iuL + w >= A.L.cols[oct] ||
               ivL + w >= A.R.rows[oct] || iuR0 - Ls - w < 0);
        const float endu = suR0 + (float)(Ls + w + 1);
        ok = ok && !(suR0 < 0.f || endu >= (float)A.R.cols[oct]);   // iniu = scaleduR0 + L - w
    }
    uint32_t lw[3] = {0, 0, 0}, rw[6] = {0, 0, 0, 0, 0, 0};
    if (ok) {
        int sl, sr;
        const uint8_t* IL = pyr_level(A.L, A.left_first + img, oct, sl) + (size_t)(ivL - w + y) * sl + (iuL - w);
        const uint8_t* IR = pyr_level(A.R, A.right_first + img, oct, sr) + (size_t)(ivL - w + y) * sr + (iuR0 - Ls - w);
        __builtin_memcpy(lw, IL, 11);                          // exact widths: never past the window
        __builtin_memcpy(rw, IR, 21);
    }
    // centre values from row 5's lane of the keypoint: cL = L[5][5], cR(inc) = strip[5][10 + inc]
    const int src = kq * W + w;
    const uint32_t cl1 = __shfl(lw[1], src, kWave);
    const uint32_t cr1 = __shfl(rw[1], src, kWave), cr2 = __shfl(rw[2], src, kWave), cr3 = __shfl(rw[3], src, kWave);
    const int cL = (int)((cl1 >> 8) & 0xff);                   // byte 5
    // left pixels as u16 pairs (x, x+1), x = 0, 2, .., 10 (the last pair's high half is masked off below)
    uint32_t Lp[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const int b = 2 * i;
        Lp[i] = pair16(b < 4 ? lw[0] : (b < 8 ? lw[1] : lw[2]), b < 4 ? lw[1] : (b < 8 ? lw[2] : 0u), b & 3);
    }
    Lp[5] &= 0xffffu;                                          // x = 11 does not exist
    int acc[W];
#pragma unroll
    for (int k = 0; k < W; ++k) {                              // shift inc = k - 5: strip columns x + k, x = 0..10
        const int cb = 5 + k;                                   // strip byte of cR(inc)
        const uint32_t cw = cb < 8 ? cr1 : (cb < 12 ? cr2 : cr3);
        const int cR = (int)((cw >> (8 * (cb & 3))) & 0xff);
        const uint32_t off = (uint32_t)(512 - (cL - cR)) * 0x00010001u;
        uint32_t a = 0;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const int b = k + 2 * i;                            // strip bytes b, b+1
            const uint32_t lo4 = rw[b >> 2], hi4 = (b >> 2) + 1 < 6 ? rw[(b >> 2) + 1] : 0u;
            uint32_t rp = pair16(lo4, hi4, b & 3) + 0x02000200u;   // R + 512
            uint32_t lp = Lp[i] + off;                          // L + 512 - d
            if (i == 5) { rp &= 0xffffu; lp &= 0xffffu; }       // (x = 11)
            a = __builtin_amdgcn_sad_u16(lp, rp, a);
        }
        acc[k] = (int)a;
    }
    if (kq < kSadKpWave) {
#pragma unroll
        for (int k = 0; k < W; ++k) part[q][k][y] = acc[k];
    }
    __syncthreads();
    if (kq < kSadKpWave && y < W) {                            // lane (keypoint, shift = y - 5): sum the 11 rows
        int d = 0;
#pragma unroll
        for (int r = 0; r < W; ++r) d += part[q][y][r];
        dist[q][y] = d;
    }
    __syncthreads();
    if (!lane_kp || y != 0) return;
    float ur = -1.0f, dp = -1.0f;
    int sd = -1;
    if (ok) {
        int best = 0x7fffffff, binc = 0;
        for (int k = -Ls; k <= Ls; ++k) {
            const int d = dist[q][k + Ls];
            if ((float)d < (float)best) { best = d; binc = k; }
        }
        if (binc != -Ls && binc != Ls) {
            const float d1 = (float)dist[q][Ls + binc - 1], d2 = (float)dist[q][Ls + binc], d3 = (float)dist[q][Ls + binc + 1];
            const float den = __fmul_rn(2.0f, __fsub_rn(__fadd_rn(d1, d3), __fmul_rn(2.0f, d2)));
            const float deltaR = __fdiv_rn(__fsub_rn(d1, d3), den);
            if (!(deltaR < -1.f || deltaR > 1.f)) {
                float bestuR = __fmul_rn(A.L.scale[oct], __fadd_rn(__fadd_rn(suR0, (float)binc), deltaR));
                float disparity = __fsub_rn(uL, bestuR);
                if (disparity >= 0.f && disparity < A.maxD) {
                    if (disparity <= 0.f) {
                        disparity = 0.01f;
                        bestuR = (float)((double)uL - 0.01);
                    }
                    dp = __fdiv_rn(A.bf, disparity);
                    ur = bestuR;
                    sd = best;
                }
            }
        }
    }
    A.uright[o] = ur;
    A.depth[o] = dp;
    A.sad[o] = sd;
}

// Median-SAD outlier rejection of one stereo pair (src/Frame.cc:627-639): sort the accepted SAD values,
// median = element n/2, reject every match with SAD >= 1.5*1.4*median (the reference's backward loop
// stops at the first value below the threshold of an ascending list).
__global__ __launch_bounds__(1024) void k_stereo_median(RefineArgs A) {
    // element n/2 of the ascending accepted SADs (0 <= SAD <= 121 * 510 < 2^16) by a two-digit radix select: a
    // histogram of the high bytes finds the bin holding rank n/2, a histogram of the low bytes inside that bin finds
    // the value (two passes over the pair's keypoints, no sort)
    __shared__ int hist[256];
    __shared__ int sel[4];                 // n, high byte, rank left inside the bin, low byte
    const int img = blockIdx.x, tid = threadIdx.x;
    const int nl = min(A.nl ? A.nl[img] : A.nl_fixed, A.capacity);
    const size_t o = (size_t)img * A.capacity;
    if (tid < 256) hist[tid] = 0;
    if (tid < 4) sel[tid] = 0;
    __syncthreads();
    int c = 0;
    for (int i = tid; i < nl; i += blockDim.x) {
        const int v = A.sad[o + i];
        if (v >= 0) { atomicAdd(&hist[(v >> 8) & 0xff], 1); ++c; }
    }
    c = wave_sum(c);
    if (lane_id() == 0 && c) atomicAdd(&sel[0], c);
    __syncthreads();
    const int n = sel[0];
    if (n == 0) return;
    const int k = n / 2;
    if (tid < kWave) {                     // wave 0: inclusive scan of the 256 bins, 4 per lane
        const int b0 = 4 * tid;
        const int h0 = hist[b0], h1 = hist[b0 + 1], h2 = hist[b0 + 2], h3 = hist[b0 + 3];
        const int inc = wave_incl_scan(h0 + h1 + h2 + h3);
        int before = inc - (h0 + h1 + h2 + h3);
        const int hh[4] = {h0, h1, h2, h3};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (before <= k && k < before + hh[j]) { sel[1] = b0 + j; sel[2] = k - before; }
            before += hh[j];
        }
    }
    __syncthreads();
    const int hb = sel[1], kk = sel[2];
    if (tid < 256) hist[tid] = 0;
    __syncthreads();
    for (int i = tid; i < nl; i += blockDim.x) {
        const int v = A.sad[o + i];
        if (v >= 0 && ((v >> 8) & 0xff) == hb) atomicAdd(&hist[v & 0xff], 1);
    }
    __syncthreads();
    if (tid < kWave) {
        const int b0 = 4 * tid;
        const int h0 = hist[b0], h1 = hist[b0 + 1], h2 = hist[b0 + 2], h3 = hist[b0 + 3];
        const int inc = wave_incl_scan(h0 + h1 + h2 + h3);
        int before = inc - (h0 + h1 + h2 + h3);
        const int hh[4] = {h0, h1, h2, h3};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (before <= kk && kk < before + hh[j]) sel[3] = b0 + j;
            before += hh[j];
        }
    }
    __syncthreads();
    const float median = (float)((hb << 8) | sel[3]);
    const float thDist = __fmul_rn(__fmul_rn(1.5f, 1.4f), median);
    for (int i = tid; i < nl; i += blockDim.x) {
        const int v = A.sad[o + i];
        if (v >= 0 && !((float)v < thDist)) {
            A.uright[o + i] = -1.0f;
            A.depth[o + i] = -1.0f;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:246-311), batched over MapPoints
// ---------------------------------------------------------------------------------------------
// The reference fills the N x N distance table, sorts each row and takes element (size_t)(0.5*(N-1)) =
// (N-1)/2 as the row's median, keeping the first row with the strictly smallest median.  Here one wave per
// MapPoint, lane = row: the median of row i is the smallest v with #{j : d(i, j) <= v} >= (N-1)/2 + 1 (d(i, i) = 0
// included, as in the table), found by a 9-step binary search over v in [0, 256] -- each step counts the row
// against every descriptor of the MapPoint, broadcast from registers (v_readlane), so nothing is sorted and
// nothing goes through LDS.  (median << 20 | row) wave minimum = first row with the smallest median.
struct DistinctArgs {
    const uint8_t* desc;      // flat observation descriptors [total][32] (store == 0)
    const int32_t* obs;       // (slot, keypoint index) per observation (store == 1)
    orbx_kf_store S;
    int store;
    const int32_t* off;       // [M + 1]
    int M;
    int32_t* best;            // [M] index in the MapPoint's observation list, -1 when it has none
    uint8_t* out;             // [M][32] the chosen descriptor (mDescriptor; zeros without observations), or NULL
    int nbx;
};

__device__ __forceinline__ const uint8_t* obs_desc(const DistinctArgs& A, int o) {
    if (!A.store) return A.desc + 32 * (size_t)o;
    const int slot = A.obs[2 * (size_t)o], idx = A.obs[2 * (size_t)o + 1];
    return A.S.desc + (size_t)slot * A.S.desc_stride + 32 * (size_t)idx;
}

__global__ __launch_bounds__(256) void k_distinctive(DistinctArgs A) {
    const int item = xcd_item(xcd_chunk(A.nbx));
    if (item >= A.nbx) return;
    const int mp = item * 4 + (int)(threadIdx.x >> 6);
    if (mp >= A.M) return;
    const int ln = lane_id();
    const int o0 = A.off[mp], N = A.off[mp + 1] - o0;
    if (N <= 0) {                                          // no observation: best -1, a zero descriptor row
        if (ln == 0) A.best[mp] = -1;
        if (A.out && ln < 8) reinterpret_cast<uint32_t*>(A.out + 32 * (size_t)mp)[ln] = 0u;
        return;
    }
    const int need = (N - 1) / 2 + 1;          // rank of vDists[(size_t)(0.5 * (N - 1))], 1-based
    uint32_t bestkey = 0xffffffffu;
    for (int rc = 0; rc < N; rc += kWave) {
        const int i = rc + ln;
        uint4 a0 = make_uint4(0, 0, 0, 0), a1 = a0;
        if (i < N) load_desc(obs_desc(A, o0 + i), a0, a1);
        int lo = 0, hi = 256;
#pragma unroll 1
        for (int it = 0; it < 9; ++it) {
            const int mid = (lo + hi) >> 1;
            int cnt = 0;
            for (int cc = 0; cc < N; cc += kWave) {
                const int j = cc + ln;
                uint4 b0 = make_uint4(0, 0, 0, 0), b1 = b0;
                if (j < N) load_desc(obs_desc(A, o0 + j), b0, b1);
                const int nc = min(kWave, N - cc);
                for (int t = 0; t < nc; ++t) {
                    uint4 x0, x1;
                    x0.x = __builtin_amdgcn_readlane(b0.x, t); x0.y = __builtin_amdgcn_readlane(b0.y, t);
                    x0.z = __builtin_amdgcn_readlane(b0.z, t); x0.w = __builtin_amdgcn_readlane(b0.w, t);
                    x1.x = __builtin_amdgcn_readlane(b1.x, t); x1.y = __builtin_amdgcn_readlane(b1.y, t);
                    x1.z = __builtin_amdgcn_readlane(b1.z, t); x1.w = __builtin_amdgcn_readlane(b1.w, t);
                    cnt += hamming256(a0, a1, x0, x1) <= mid;
                }
            }
            if (cnt >= need) hi = mid; else lo = mid + 1;
        }
        const uint32_t key = (i < N) ? (((uint32_t)lo << 20) | (uint32_t)i) : 0xffffffffu;
        bestkey = min(bestkey, wave_min_u32(key));
    }
    const int bi = (int)(bestkey & 0xfffff);
    if (ln == 0) A.best[mp] = bi;
    if (A.out && ln < 8) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(obs_desc(A, o0 + bi));
        reinterpret_cast<uint32_t*>(A.out + 32 * (size_t)mp)[ln] = src[ln];
    }
}

// The MapPoints of new keyframes, read straight from CreateNewMapPoints' match tables (no CSR built).  In the reference
// a keypoint of the new keyframe becomes a MapPoint at most once, from the first neighbour whose match triangulates
// (LocalMapping.cc:244-448: later neighbours' searches skip keypoints that already hold a MapPoint); the new MapPoint
// has exactly two observations, the neighbour's keypoint and the new keyframe's (:440-441), and
// ComputeDistinctiveDescriptors over two descriptors takes row 0: both rows' medians are vDists[0] = 0
// (MapPoint.cc:293-306), so the descriptor is that of the first observation in mObservations order -- a map keyed by
// KeyFrame*, pinned to creation order (the neighbour, the older keyframe, first; the same pin as the quadtree's
// heap-address tie).  Here the triangulation itself (pose checks, SVD) runs on the map side, so the first
// neighbour with a match stands for the first that triangulates.  MapPoint (j, i): list [(neighbour k*, match),
// (new keyframe, i)] with k* the first neighbour in order with a match; no match -> no MapPoint (best = -1, nothing
// written).  multiagent.neighbour_observations builds the same lists as a CSR.  One wave per MapPoint.
struct DistinctNbArgs {
    orbx_kf_store S;
    const int32_t* new_slots;   // [n]
    const int32_t* nb;          // [n][nn] neighbour slots, -1 = none
    const int32_t* m12;         // [n][nn][capacity]
    int n, nn, M;
    int32_t* best;              // [M] list index (0), -1 without a MapPoint
    uint8_t* out;               // [M][32] or NULL
    int nbx;
};

__global__ __launch_bounds__(256) void k_distinctive_nb(DistinctNbArgs A) {
    const int item = xcd_item(xcd_chunk(A.nbx));
    if (item >= A.nbx) return;
    const int mp = item * 4 + (int)(threadIdx.x >> 6);
    if (mp >= A.M) return;
    const int ln = lane_id(), cap = A.S.capacity;
    const int j = mp / cap, i = mp - j * cap;
    int slot = -1, kp = -1;
    if (ln < A.nn) {                                       // lane k: neighbour k
        const int nbk = A.nb[j * A.nn + ln];
        if (nbk >= 0) {
            const int m = A.m12[((size_t)j * A.nn + ln) * cap + i];
            if (m >= 0) { slot = nbk; kp = m; }
        }
    }
    const uint64_t mask = __ballot(kp >= 0);
    if (!mask) {                                           // no MapPoint: best -1, a zero descriptor row
        if (ln == 0) A.best[mp] = -1;
        if (A.out && ln < 8) reinterpret_cast<uint32_t*>(A.out + 32 * (size_t)mp)[ln] = 0u;
        return;
    }
    const int first = __builtin_ctzll(mask);               // the first neighbour with a match
    const int wslot = __builtin_amdgcn_readlane(slot, first), wkp = __builtin_amdgcn_readlane(kp, first);
    if (ln == 0) A.best[mp] = 0;                           // list row 0: the neighbour's observation
    if (A.out && ln < 8) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(A.S.desc + (size_t)wslot * A.S.desc_stride + 32 * (size_t)wkp);
        reinterpret_cast<uint32_t*>(A.out + 32 * (size_t)mp)[ln] = src[ln];
    }
}

// =============================================================================================
// host side
// =============================================================================================
struct Matcher {
    float nnratio;
    int checkOri;
    int device;
    hipStream_t stream = nullptr;      // lazy: own() on first host-API use
    std::once_flag stream_once;
    hipStream_t own() { return lazy_stream(stream, stream_once, device); }
    // growable device scratch.  Contract: one call at a time holds the matcher ('mtx', MatcherLease), and a call's
    // stream is ordered after the previous scratch user before its own kernels touch the scratch -- device calls on
    // different streams are ordered, not racing on one buffer.  A matcher used from one stream only (the common case:
    // the reference builds an ORBmatcher per call site) needs nothing beyond stream order, so nothing is enqueued for
    // it: the first call from a second stream drains the device once, and from then on ('multi') every call records
    // 'last_op' on its stream and the next call on another stream waits for it (the per-call event wait
    // and record cost ~3 us per launch).
    void* scratch = nullptr;
    size_t scratch_bytes = 0;
    std::recursive_mutex mtx;
    hipEvent_t last_op = nullptr;
    hipEvent_t frame_ev[2] = {nullptr, nullptr};   // orbx_stereo_frame: the two extractions' ends (lazy)
    bool last_op_set = false;            // last_op recorded after the previous call (multi-stream mode)
    bool have_last = false, multi = false;
    hipStream_t last_stream = nullptr;   // the previous call's stream
    // pinned host staging of the host API (one H2D and one D2H copy per call instead of one pageable copy per array;
    // host calls end synchronised, so the next call may reuse it)
    uint8_t* h_stage = nullptr;
    size_t h_stage_bytes = 0;
    int stage_host(size_t bytes) {
        if (bytes <= h_stage_bytes) return ORBX_OK;
        const size_t nb = std::max(bytes, h_stage_bytes * 2);     // geometric growth over the old size
        ::orbx::LegacyLock legacy_;
        if (h_stage) (void)hipHostFree(h_stage);
        h_stage = nullptr;
        h_stage_bytes = 0;
        ORBX_HIP(hipHostMalloc((void**)&h_stage, nb, hipHostMallocDefault));
        h_stage_bytes = nb;
        return ORBX_OK;
    }
    int reserve(size_t bytes) { return reserve_on(bytes, own()); }
    // order 'on' after the previous scratch user; grow the buffer (after every user has finished) if needed
    int reserve_on(size_t bytes, hipStream_t on) {
        if (have_last && last_stream != on) {
            if (!multi) {
                ORBX_HIP(::orbx::device_sync());
                multi = true;
            } else if (last_op_set) {
                ORBX_HIP(hipStreamWaitEvent(on, last_op, 0));
            }
        }
        if (bytes <= scratch_bytes) return ORBX_OK;
        ::orbx::LegacyLock legacy_;
        if (scratch) {
            ORBX_HIP(::orbx::device_sync());   // earlier users on any stream done before the buffer goes away
            (void)hipFree(scratch);
            scratch = nullptr;
        }
        size_t nb = std::max(bytes, scratch_bytes * 2);
        ORBX_HIP(hipMalloc(&scratch, nb));
        scratch_bytes = nb;
        return ORBX_OK;
    }
};

// bump allocator over the scratch buffer (256-B aligned pieces)
struct Bump {
    uint8_t* base; size_t off = 0;
    template <typename T> T* take(size_t n) {
        T* p = (T*)(base + off);
        off += (n * sizeof(T) + 255) & ~(size_t)255;
        return p;
    }
};
static size_t a256(size_t b) { return (b + 255) & ~(size_t)255; }

// Grid: 256 queries per workgroup x train chunks x problems.  The train set of a problem is split into chunks so that
// the whole launch has >= ~2048 workgroups when the problems are few (a single 2000 x 2000 match is 8 query blocks:
// 64 chunks of 32 rows fill the chip; at many problems one chunk per problem suffices).
static int bf_target_wgs() { return 2048; }   // workgroups the train chunking aims for
static int bf_chunks(int nq, int nt, int nprob) {
    const int qb = (nq + kBfQ - 1) / kBfQ;
    const int want = (bf_target_wgs() + qb * nprob - 1) / (qb * nprob);
    return std::max(1, std::min(want, (nt + 31) / 32));
}
// k_bf_mfma: 64 queries per workgroup, chunks of >= 64 train rows (one LDS stage)
static int bf_chunks_mx(int nq, int nt, int nprob) {
    const int qb = (nq + kMxQ - 1) / kMxQ;
    const int want = (bf_target_wgs() + qb * nprob - 1) / (qb * nprob);
    return std::max(1, std::min(want, (nt + kMxRows - 1) / kMxRows));
}
static size_t bf_scratch(int nq, int nt, int nprob) {
    const int nch = std::max(bf_chunks(nq, nt, nprob), bf_chunks_mx(nq, nt, nprob));
    return 2 * a256((size_t)nch * nq * nprob * 4) + 256;
}
// The matrix-core form is the default (r6h, 64 problems of 2000 x 2000 per launch: 108.5 us against 171.0 for k_bf_tile
// + merge; one problem: 11.4-12.0 against 11.8-11.9, launch-bound); ORBX_BF_MFMA=0 selects the tile form (read per call:
// the tests run both).
static bool bf_mfma() {
    const char* e = std::getenv("ORBX_BF_MFMA");
    return !e || std::atoi(e) != 0;
}
static int bf_launch(Matcher* m, const uint8_t* dq, int nq, size_t qs, const uint8_t* dt, int nt, size_t ts, int nprob, int32_t* bi,
                     int32_t* bd, int32_t* sd, hipStream_t s, void* scratch) {
    if (nt == 0) {
        hipLaunchKernelGGL(k_bf_empty, dim3(((size_t)nq * nprob + 255) / 256), dim3(256), 0, s, nq * nprob, bi, bd, sd);
        ORBX_HIP(hipGetLastError());
        return ORBX_OK;
    }
    if (bf_mfma()) {
        const int qb = (nq + kMxQ - 1) / kMxQ;
        int nch = bf_chunks_mx(nq, nt, nprob);
        const int chunk = (nt + nch - 1) / nch;
        nch = (nt + chunk - 1) / chunk;
        uint32_t* pb = (uint32_t*)scratch;
        int32_t* ps = (int32_t*)((uint8_t*)scratch + a256((size_t)nch * nq * nprob * 4));
        if (nch == 1) {                                            // one chunk: the outputs directly, no merge launch
            hipLaunchKernelGGL(k_bf_mfma, dim3(qb, 1, nprob), dim3(256), 0, s, dq, nq, qs, dt, nt, ts, chunk, nullptr, nullptr,
                               bi, bd, sd);
        } else {
            hipLaunchKernelGGL(k_bf_mfma, dim3(qb, nch, nprob), dim3(256), 0, s, dq, nq, qs, dt, nt, ts, chunk, pb, ps,
                               nullptr, nullptr, nullptr);
            if (nch >= 2 * kBfMergeG)
                hipLaunchKernelGGL(k_bf_merge_g, dim3((nq + 256 / kBfMergeG - 1) / (256 / kBfMergeG), nprob), dim3(256), 0, s,
                                   pb, ps, nq, nch, bi, bd, sd);
            else
                hipLaunchKernelGGL(k_bf_merge, dim3((nq + 255) / 256, nprob), dim3(256), 0, s, pb, ps, nq, nch, bi, bd, sd);
        }
        ORBX_HIP(hipGetLastError());
        return ORBX_OK;
    }
    const int qb = (nq + kBfQ - 1) / kBfQ;
    int nch = bf_chunks(nq, nt, nprob);
    const int chunk = (nt + nch - 1) / nch;
    nch = (nt + chunk - 1) / chunk;
    uint32_t* pb = (uint32_t*)scratch;
    int32_t* ps = (int32_t*)((uint8_t*)scratch + a256((size_t)nch * nq * nprob * 4));
    hipLaunchKernelGGL(k_bf_tile, dim3(qb, nch, nprob), dim3(256), 0, s, dq, nq, qs, dt, nt, ts, chunk, pb, ps);
    if (nch >= 2 * kBfMergeG)   // a long chunk walk: split it over 8 lanes per query
        hipLaunchKernelGGL(k_bf_merge_g, dim3((nq + 256 / kBfMergeG - 1) / (256 / kBfMergeG), nprob), dim3(256), 0, s, pb, ps,
                           nq, nch, bi, bd, sd);
    else
        hipLaunchKernelGGL(k_bf_merge, dim3((nq + 255) / 256, nprob), dim3(256), 0, s, pb, ps, nq, nch, bi, bd, sd);
    ORBX_HIP(hipGetLastError());
    return ORBX_OK;
}

}  // namespace orbx

using namespace orbx;
struct orbx_matcher : public orbx::Matcher {};

int orbx::matcher_device(const orbx_matcher* m) { return m->device; }
void orbx::matcher_acquire(orbx_matcher* m) { m->mtx.lock(); }
void orbx::matcher_release(orbx_matcher* m, hipStream_t s, bool used) {
    if (used) {
        if (m->multi && m->last_op) m->last_op_set = hipEventRecord(m->last_op, s) == hipSuccess;
        m->last_stream = s;
        m->have_last = true;
    }
    m->mtx.unlock();
}
int orbx::matcher_scratch(orbx_matcher* m, size_t bytes, void** base, void** stream) {
    int st = m->reserve(bytes);   // (the caller holds a MatcherLease)
    if (st) return st;
    *base = m->scratch;
    *stream = (void*)m->own();
    return ORBX_OK;
}

extern "C" {

int orbx_th_high(void) { return kThHigh; }
int orbx_th_low(void) { return kThLow; }
int orbx_histo_length(void) { return kHisto; }

int orbx_matcher_create(float nnratio, int checkOri, int device, orbx_matcher** out) {
    ORBX_REQUIRE(out, ORBX_ERR_ARG, "out is NULL");
    *out = nullptr;
    int ndev = 0;
    ORBX_HIP(hipGetDeviceCount(&ndev));
    ORBX_REQUIRE(device >= 0 && device < ndev, ORBX_ERR_ARG, "device %d out of range (%d devices)", device, ndev);
    orbx_matcher* m = new orbx_matcher();
    m->nnratio = nnratio;
    m->checkOri = checkOri;
    m->device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&m->last_op, hipEventDisableTiming);
    if (e != hipSuccess) {
        set_error("stream create: %s", hipGetErrorString(e));
        delete m;
        return ORBX_ERR_HIP;
    }
    *out = m;
    return ORBX_OK;
}

int orbx_matcher_destroy(orbx_matcher* m) {
    if (!m) return ORBX_OK;
    (void)hipSetDevice(m->device);
    (void)::orbx::device_sync();                                // device calls on callers' streams use the scratch
    if (m->last_op) (void)hipEventDestroy(m->last_op);
    for (hipEvent_t ev : m->frame_ev)
        if (ev) (void)hipEventDestroy(ev);
    ::orbx::LegacyLock legacy_;
    if (m->scratch) (void)hipFree(m->scratch);
    if (m->h_stage) (void)hipHostFree(m->h_stage);
    if (m->stream) (void)hipStreamDestroy(m->stream);
    delete m;
    return ORBX_OK;
}

int orbx_descriptor_distance_device(orbx_matcher* m, const uint8_t* a, const uint8_t* b, int n, int32_t* d, void* stream) {
    ORBX_REQUIRE(m && a && b && d && n >= 0, ORBX_ERR_ARG, "bad argument");
    if (n == 0) return ORBX_OK;
    ORBX_HIP(hipSetDevice(m->device));
    hipStream_t s = (hipStream_t)stream;   // NULL = the HIP null stream
    hipLaunchKernelGGL(k_hamming_pairs, dim3((n + 255) / 256), dim3(256), 0, s, a, b, n, d);
    ORBX_HIP(hipGetLastError());
    return ORBX_OK;
}

int orbx_bf_match_device(orbx_matcher* m, const uint8_t* dq, int nq, const uint8_t* dt, int nt, int32_t* bi, int32_t* bd,
                         int32_t* sd, void* stream) {
    return orbx_bf_match_batch_device(m, dq, nq, 0, dt, nt, 0, 1, bi, bd, sd, stream);
}

int orbx_bf_match_batch_device(orbx_matcher* m, const uint8_t* dq, int nq, size_t query_stride, const uint8_t* dt, int nt,
                               size_t train_stride, int n_problems, int32_t* bi, int32_t* bd, int32_t* sd, void* stream) {
    ORBX_REQUIRE(m && nq >= 0 && nt >= 0 && n_problems >= 0, ORBX_ERR_ARG, "bad argument");
    ORBX_REQUIRE(nt < (1 << 20), ORBX_ERR_UNSUPPORTED, "train set too large (%d)", nt);
    ORBX_REQUIRE(n_problems <= 65535, ORBX_ERR_UNSUPPORTED, "too many problems (%d)", n_problems);
    if (nq == 0 || n_problems == 0) return ORBX_OK;
    ORBX_REQUIRE(dq && bi && bd && sd && (nt == 0 || dt), ORBX_ERR_ARG, "null pointer");
    ORBX_REQUIRE(n_problems == 1 || ((query_stride % 16) == 0 && (train_stride % 16) == 0), ORBX_ERR_ARG,
                 "problem strides must be multiples of 16 bytes");
    ORBX_HIP(hipSetDevice(m->device));
    hipStream_t s = (hipStream_t)stream;   // NULL = the HIP null stream
    MatcherLease lease_(m, s);
    int st = m->reserve_on(bf_scratch(nq, std::max(nt, 1), n_problems), s);
    if (st) return st;
    return bf_launch(m, dq, nq, query_stride, dt, nt, train_stride, n_problems, bi, bd, sd, s, m->scratch);
}

int orbx_bf_match(orbx_matcher* m, const uint8_t* q, int nq, const uint8_t* t, int nt, int32_t* bi, int32_t* bd, int32_t* sd) {
    ORBX_REQUIRE(m && nq >= 0 && nt >= 0, ORBX_ERR_ARG, "bad argument");
    if (nq == 0) return ORBX_OK;
    ORBX_REQUIRE(q && bi && bd && sd && (nt == 0 || t), ORBX_ERR_ARG, "null pointer");
    ORBX_REQUIRE(nt < (1 << 20), ORBX_ERR_UNSUPPORTED, "train set too large (%d)", nt);
    ORBX_HIP(hipSetDevice(m->device));
    const size_t io = a256((size_t)nq * 32) + a256((size_t)std::max(nt, 1) * 32) + 3 * a256((size_t)nq * 4);
    MatcherLease lease_(m, m->own());
    int st = m->reserve(io + bf_scratch(nq, std::max(nt, 1), 1));
    if (st) return st;
    Bump bp{(uint8_t*)m->scratch};
    uint8_t* dq = bp.take<uint8_t>((size_t)nq * 32);
    uint8_t* dt = bp.take<uint8_t>((size_t)std::max(nt, 1) * 32);
    int32_t* dbi = bp.take<int32_t>(nq);
    int32_t* dbd = bp.take<int32_t>(nq);
    int32_t* dsd = bp.take<int32_t>(nq);
    hipStream_t s = m->own();
    ORBX_HIP(hipMemcpyAsync(dq, q, (size_t)nq * 32, hipMemcpyHostToDevice, s));
    if (nt > 0) {
        ORBX_HIP(hipMemcpyAsync(dt, t, (size_t)nt * 32, hipMemcpyHostToDevice, s));
        st = bf_launch(m, dq, nq, 0, dt, nt, 0, 1, dbi, dbd, dsd, s, (uint8_t*)m->scratch + bp.off);
        if (st) return st;
        ORBX_HIP(hipMemcpyAsync(bi, dbi, 4 * (size_t)nq, hipMemcpyDeviceToHost, s));
        ORBX_HIP(hipMemcpyAsync(bd, dbd, 4 * (size_t)nq, hipMemcpyDeviceToHost, s));
        ORBX_HIP(hipMemcpyAsync(sd, dsd, 4 * (size_t)nq, hipMemcpyDeviceToHost, s));
        ORBX_HIP(hipStreamSynchronize(s));
    } else {
        for (int i = 0; i < nq; ++i) { bi[i] = -1; bd[i] = 256; sd[i] = 256; }
    }
    return ORBX_OK;
}

static int stereo_common(orbx_matcher* m, StereoArgs& A, const float* scale, int nlevels, int rows, float bf, float b) {
    ORBX_REQUIRE(nlevels >= 1 && nlevels <= 32 && scale, ORBX_ERR_ARG, "bad level table");
    ORBX_REQUIRE(b != 0.0f, ORBX_ERR_ARG, "baseline is zero");
    ORBX_REQUIRE(rows > 0 && rows <= 16384, ORBX_ERR_ARG, "bad row count %d", rows);
    float smax = 0.f;
    for (int l = 0; l < nlevels; ++l) { A.scale[l] = scale[l]; smax = std::max(smax, scale[l]); }
    A.nlevels = nlevels;
    A.rows = rows;
    A.band = (int)std::ceil(2.0f * smax) + 2;
    A.maxD = bf / b;   // minZ = mb, maxD = mbf/minZ (Frame.cc:496-498)
    (void)m;
    return ORBX_OK;
}

static int stereo_launch(StereoArgs& A, int batch, int nl_max, hipStream_t s) {
    // with left-row buckets (lrow_*): the row-block search (batches: ~8 dependent HBM round trips per keypoint fewer);
    // without: one wave per left keypoint (the host API's single frame, where latency rules)
    ORBX_REQUIRE(A.row_start && A.row_idx && (!A.lrow_start) == (!A.lrow_idx), ORBX_ERR_ARG, "stereo search without row buckets");
    hipLaunchKernelGGL(k_stereo_rows, dim3(batch, A.lrow_start ? 2 : 1), dim3(kStereoRowsThreads),
                       (size_t)(A.rows + 1) * sizeof(int), s, A);
    A.batch = batch;
    if (A.lrow_start) {
        const int nblk = (A.rows + kStereoRows - 1) / kStereoRows;
        hipLaunchKernelGGL(k_stereo_blk, dim3(kXcds * xcd_chunk(nblk * batch)), dim3(256), 0, s, A, nblk);
    } else {
        A.nbx = (nl_max * 64 + 255) / 256;
        hipLaunchKernelGGL(k_stereo, dim3(kXcds * xcd_chunk(A.nbx * batch)), dim3(256), 0, s, A);
    }
    ORBX_HIP(hipGetLastError());
    return ORBX_OK;
}

static size_t stereo_scratch(int batch, int rows, int capacity) {
    return 2 * (a256((size_t)batch * (rows + 1) * 4) + a256((size_t)batch * capacity * 4));
}

int orbx_stereo_match_batch_device(orbx_matcher* m, const orbx_keypoint* kl, const uint8_t* dl, const int32_t* nl,
                                   const orbx_keypoint* kr, const uint8_t* dr, const int32_t* nr, int batch, int capacity,
                                   const float* scale, int nlevels, int rows, float bf, float b, int32_t* bi, int32_t* bd,
                                   void* stream) {
    ORBX_REQUIRE(m && kl && dl && nl && kr && dr && nr && bi && bd && batch > 0 && capacity > 0, ORBX_ERR_ARG, "bad argument");
    ORBX_REQUIRE(capacity < (1 << 20), ORBX_ERR_UNSUPPORTED, "capacity too large");
    StereoArgs A{};
    int st = stereo_common(m, A, scale, nlevels, rows, bf, b);
    if (st) return st;
    ORBX_HIP(hipSetDevice(m->device));
    hipStream_t s = (hipStream_t)stream;   // NULL = the HIP null stream
    MatcherLease lease_(m, s);
    if ((st = m->reserve_on(stereo_scratch(batch, rows, capacity), s))) return st;
    Bump bp{(uint8_t*)m->scratch};
    A.row_start = bp.take<int32_t>((size_t)batch * (rows + 1));
    A.row_idx = bp.take<int32_t>((size_t)batch * capacity);
    A.lrow_start = bp.take<int32_t>((size_t)batch * (rows + 1));
    A.lrow_idx = bp.take<int32_t>((size_t)batch * capacity);
    A.kl = kl; A.dl = dl; A.nl = nl; A.kr = kr; A.dr = dr; A.nr = nr; A.capacity = capacity;
    A.best_idx = bi; A.best_dist = bd;
    return stereo_launch(A, batch, capacity, s);
}

int orbx_stereo_match(orbx_matcher* m, const orbx_keypoint* kpl, const uint8_t* desc_l, int nl, const orbx_keypoint* kpr,
                      const uint8_t* desc_r, int nr, const float* scale, int nlevels, int rows, float bf, float b,
                      int32_t* best_idx, int32_t* best_dist, int* n_matched) {
    ORBX_REQUIRE(m && n_matched && nl >= 0 && nr >= 0, ORBX_ERR_ARG, "bad argument");
    *n_matched = 0;
    if (nl == 0) return ORBX_OK;
    ORBX_REQUIRE(kpl && desc_l && best_idx && best_dist && (nr == 0 || (kpr && desc_r)), ORBX_ERR_ARG, "null pointer");
    ORBX_REQUIRE(nr < (1 << 20) && nl < (1 << 20), ORBX_ERR_UNSUPPORTED, "too many keypoints");
    StereoArgs A{};
    int st = stereo_common(m, A, scale, nlevels, rows, bf, b);
    if (st) return st;
    ORBX_HIP(hipSetDevice(m->device));
    const int cap = std::max(nl, std::max(nr, 1));
    const size_t bytes = a256(28 * (size_t)cap) * 2 + a256(32 * (size_t)cap) * 2 + 2 * a256(4 * (size_t)cap) +
                         stereo_scratch(1, rows, cap);
    MatcherLease lease_(m, m->own());
    if ((st = m->reserve(bytes))) return st;
    Bump bp{(uint8_t*)m->scratch};
    orbx_keypoint* dkl = bp.take<orbx_keypoint>(cap);
    uint8_t* ddl = bp.take<uint8_t>(32 * (size_t)cap);
    orbx_keypoint* dkr = bp.take<orbx_keypoint>(cap);
    uint8_t* ddr = bp.take<uint8_t>(32 * (size_t)cap);
    int32_t* dbi = bp.take<int32_t>(cap);
    int32_t* dbd = bp.take<int32_t>(cap);
    A.row_start = bp.take<int32_t>((size_t)rows + 1);
    A.row_idx = bp.take<int32_t>(cap);
    A.lrow_start = bp.take<int32_t>((size_t)rows + 1);
    A.lrow_idx = bp.take<int32_t>(cap);
    hipStream_t s = m->own();
    // the four inputs into pinned staging laid out as the scratch (keypoints / descriptors of both sides are
    // contiguous there), one H2D copy; the two outputs come back the same way
    const size_t in_bytes = (size_t)((uint8_t*)dbi - (uint8_t*)dkl), out_off = in_bytes;
    const size_t out_bytes = (size_t)((uint8_t*)dbd - (uint8_t*)dbi) + 4 * (size_t)nl;
    if ((st = m->stage_host(std::max(in_bytes, out_off + out_bytes)))) return st;
    uint8_t* hs = m->h_stage;
    std::memcpy(hs, kpl, 28 * (size_t)nl);
    std::memcpy(hs + ((uint8_t*)ddl - (uint8_t*)dkl), desc_l, 32 * (size_t)nl);
    if (nr > 0) {
        std::memcpy(hs + ((uint8_t*)dkr - (uint8_t*)dkl), kpr, 28 * (size_t)nr);
        std::memcpy(hs + ((uint8_t*)ddr - (uint8_t*)dkl), desc_r, 32 * (size_t)nr);
    }
    ORBX_HIP(hipMemcpyAsync(dkl, hs, in_bytes, hipMemcpyHostToDevice, s));
    A.kl = dkl; A.dl = ddl; A.kr = dkr; A.dr = ddr; A.nl = nullptr; A.nr = nullptr;
    A.nl_fixed = nl; A.nr_fixed = nr; A.capacity = cap;
    A.best_idx = dbi; A.best_dist = dbd;
    if ((st = stereo_launch(A, 1, nl, s))) return st;
    ORBX_HIP(hipMemcpyAsync(hs + out_off, dbi, out_bytes, hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipStreamSynchronize(s));
    std::memcpy(best_idx, hs + out_off, 4 * (size_t)nl);
    std::memcpy(best_dist, hs + out_off + ((uint8_t*)dbd - (uint8_t*)dbi), 4 * (size_t)nl);
    int n = 0;
    for (int i = 0; i < nl; ++i) n += best_idx[i] >= 0;
    *n_matched = n;
    return ORBX_OK;
}

static int refine_launch(RefineArgs& A, int batch, hipStream_t s) {
    A.batch = batch;
    A.nbx = (A.capacity + 4 * kSadKpWave - 1) / (4 * kSadKpWave);
    hipLaunchKernelGGL(k_stereo_sad_rows, dim3(kXcds * xcd_chunk(A.nbx * batch)), dim3(256), 0, s, A);
    hipLaunchKernelGGL(k_stereo_median, dim3(batch), dim3(1024), 0, s, A);
    ORBX_HIP(hipGetLastError());
    return ORBX_OK;
}

static int check_pyramid(const orbx_pyramid* P, int first, int batch, const char* which) {
    ORBX_REQUIRE(P && P->level0 && P->nlevels >= 1 && P->nlevels <= ORBX_MAX_LEVELS, ORBX_ERR_ARG, "bad %s pyramid", which);
    ORBX_REQUIRE(first >= 0 && first + batch <= P->batch, ORBX_ERR_ARG, "%s images [%d, %d) outside the pyramid batch %d",
                 which, first, first + batch, P->batch);
    ORBX_REQUIRE(P->nlevels == 1 || P->levels, ORBX_ERR_ARG, "bad %s pyramid", which);
    return ORBX_OK;
}

int orbx_stereo_refine_batch_device(orbx_matcher* m, const orbx_keypoint* kl, const int32_t* nl, const orbx_keypoint* kr,
                                    const int32_t* best_idx, int batch, int capacity, const orbx_pyramid* left, int left_first,
                                    const orbx_pyramid* right, int right_first, float bf, float b, float* uright, float* depth,
                                    void* stream) {
    ORBX_REQUIRE(m && kl && nl && kr && best_idx && uright && depth && batch > 0 && capacity > 0, ORBX_ERR_ARG, "bad argument");
    ORBX_REQUIRE(capacity <= 4096, ORBX_ERR_UNSUPPORTED, "capacity %d > 4096", capacity);
    ORBX_REQUIRE(b != 0.0f, ORBX_ERR_ARG, "baseline is zero");
    int st;
    if ((st = check_pyramid(left, left_first, batch, "left"))) return st;
    if ((st = check_pyramid(right, right_first, batch, "right"))) return st;
    ORBX_REQUIRE(left->nlevels == right->nlevels, ORBX_ERR_ARG, "left/right pyramids differ in levels");
    ORBX_HIP(hipSetDevice(m->device));
    hipStream_t s = (hipStream_t)stream;
    MatcherLease lease_(m, s);
    if ((st = m->reserve_on(a256((size_t)batch * capacity * 4), s))) return st;
    RefineArgs A{};
    A.kl = kl; A.nl = nl; A.kr = kr; A.best_idx = best_idx; A.capacity = capacity;
    A.L = *left; A.R = *right; A.left_first = left_first; A.right_first = right_first;
    A.bf = bf; A.maxD = bf / b;
    A.uright = uright; A.depth = depth; A.sad = (int32_t*)m->scratch;
    return refine_launch(A, batch, s);
}

int orbx_stereo_frame(orbx_matcher* m, orbx_extractor* left, orbx_extractor* right, const uint8_t* image_left,
                      size_t step_left, const uint8_t* image_right, size_t step_right, int rows, int cols,
                      orbx_keypoint* kps_left, uint8_t* desc_left, int capacity_left, int* n_left, orbx_keypoint* kps_right,
                      uint8_t* desc_right, int capacity_right, int* n_right, float bf, float b, float* uright, float* depth,
                      int* n_stereo) {
    ORBX_REQUIRE(m && left && right && left != right && n_left && n_right && n_stereo, ORBX_ERR_ARG,
                 "a matcher, two distinct extractors and the three counts are required");
    *n_left = *n_right = *n_stereo = 0;
    if (!image_left || !image_right || rows <= 0 || cols <= 0) {
        // an empty side: the extractions as orbx_extract_pair gives them, no stereo (ComputeStereoMatches finds nothing)
        return orbx_extract_pair(left, right, image_left, step_left, image_right, step_right, rows, cols, kps_left, desc_left,
                                 capacity_left, n_left, kps_right, desc_right, capacity_right, n_right);
    }
    int st;
    if ((st = orbx_internal_extract_begin(left, image_left, rows, cols, step_left))) return st;
    // Until both extract_end calls below have run, an early return still finishes the extractions in flight (their
    // streams synchronised, results dropped): the next call on an extractor packs its image into the pinned staging
    // this call's upload may still be reading.
    struct Finish {
        orbx_extractor* e[2];
        ~Finish() {
            if (!e[0] && !e[1]) return;
            const std::string why = orbx_last_error();                // the error being returned, not the drop's
            for (orbx_extractor* x : e)
                if (x) { int n = 0; (void)orbx_internal_extract_end(x, nullptr, nullptr, 1 << 30, &n); }
            set_error("%s", why.c_str());
        }
    } pending{{left, nullptr}};
    if ((st = orbx_internal_extract_begin(right, image_right, rows, cols, step_right))) return st;
    pending.e[1] = right;
    const orbx_keypoint *dkl = nullptr, *dkr = nullptr;
    const uint8_t *ddl = nullptr, *ddr = nullptr;
    const int32_t *dcl = nullptr, *dcr = nullptr;
    int capl = 0, capr = 0;
    void *sl = nullptr, *sr = nullptr;
    orbx_pyramid PL, PR;
    StereoArgs A{};
    st = orbx_internal_host_outputs(left, &dkl, &ddl, &dcl, &capl, &sl);
    if (!st) st = orbx_internal_host_outputs(right, &dkr, &ddr, &dcr, &capr, &sr);
    if (!st) st = orbx_extractor_pyramid_device(left, &PL);
    if (!st) st = orbx_extractor_pyramid_device(right, &PR);
    if (!st && (PL.nlevels != PR.nlevels || capl != capr || capl > 4096)) {
        set_error("left/right extractors differ (levels %d / %d, capacity %d / %d) or capacity > 4096", PL.nlevels, PR.nlevels,
                  capl, capr);
        st = ORBX_ERR_ARG;
    }
    if (!st) st = stereo_common(m, A, PL.scale, PL.nlevels, PL.rows[0], bf, b);
    if (st) return st;
    // the stereo search on the matcher's stream once both extractions are done, straight on their device outputs (the
    // two-call form copies them to the host and back): one wait per side, one result copy, one synchronisation
    ORBX_HIP(hipSetDevice(m->device));
    hipStream_t s = m->own();
    for (hipEvent_t& ev : m->frame_ev)
        if (!ev) ORBX_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    ORBX_HIP(hipEventRecord(m->frame_ev[0], (hipStream_t)sl));
    ORBX_HIP(hipEventRecord(m->frame_ev[1], (hipStream_t)sr));
    ORBX_HIP(hipStreamWaitEvent(s, m->frame_ev[0], 0));
    ORBX_HIP(hipStreamWaitEvent(s, m->frame_ev[1], 0));
    const int cap = capl;
    const size_t bytes = 2 * a256(4 * (size_t)cap) + stereo_scratch(1, PL.rows[0], cap) + 3 * a256(4 * (size_t)cap);
    {
        MatcherLease lease_(m, s);
        if ((st = m->reserve(bytes))) return st;
        Bump bp{(uint8_t*)m->scratch};
        int32_t* dbi = bp.take<int32_t>(cap);
        int32_t* dbd = bp.take<int32_t>(cap);
        A.row_start = bp.take<int32_t>((size_t)PL.rows[0] + 1);
        A.row_idx = bp.take<int32_t>(cap);
        (void)bp.take<int32_t>((size_t)PL.rows[0] + 1);      // the batch form's left-row buckets: unused (per-keypoint search)
        (void)bp.take<int32_t>(cap);
        float* dur = bp.take<float>(cap);
        float* ddp = bp.take<float>(cap);
        int32_t* dsad = bp.take<int32_t>(cap);
        A.kl = dkl; A.dl = ddl; A.kr = dkr; A.dr = ddr; A.nl = dcl; A.nr = dcr; A.capacity = cap;
        A.best_idx = dbi; A.best_dist = dbd;
        if ((st = stereo_launch(A, 1, cap, s))) return st;
        RefineArgs R{};
        R.kl = dkl; R.nl = dcl; R.kr = dkr; R.best_idx = dbi; R.capacity = cap;
        R.L = PL; R.R = PR; R.left_first = 0; R.right_first = 0;
        R.bf = bf; R.maxD = bf / b;
        R.uright = dur; R.depth = ddp; R.sad = dsad;
        if ((st = refine_launch(R, 1, s))) return st;
        const size_t out_bytes = (size_t)((uint8_t*)ddp - (uint8_t*)dur) + 4 * (size_t)cap;
        if ((st = m->stage_host(out_bytes))) return st;
        ORBX_HIP(hipMemcpyAsync(m->h_stage, dur, out_bytes, hipMemcpyDeviceToHost, s));
        // the extractions' results (their streams were synchronised by extract_end); the stereo copy runs meanwhile
        pending.e[0] = pending.e[1] = nullptr;
        const int stl = orbx_internal_extract_end(left, kps_left, desc_left, capacity_left, n_left);
        const int str = orbx_internal_extract_end(right, kps_right, desc_right, capacity_right, n_right);
        ORBX_HIP(hipStreamSynchronize(s));
        if (stl) return stl;
        if (str) return str;
        ORBX_REQUIRE((uright && depth) || *n_left == 0, ORBX_ERR_ARG, "null uright / depth");
        const int nl = *n_left;
        std::memcpy(uright, m->h_stage, 4 * (size_t)nl);
        std::memcpy(depth, m->h_stage + ((uint8_t*)ddp - (uint8_t*)dur), 4 * (size_t)nl);
        int n = 0;
        for (int i = 0; i < nl; ++i) n += depth[i] > 0;
        *n_stereo = n;
    }
    return ORBX_OK;
}

int orbx_compute_stereo_matches(orbx_matcher* m, const orbx_extractor* left, const orbx_extractor* right, const orbx_keypoint* kpl,
                                const uint8_t* desc_l, int nl, const orbx_keypoint* kpr, const uint8_t* desc_r, int nr, float bf,
                                float b, float* uright, float* depth, int* n_stereo) {
    ORBX_REQUIRE(m && left && right && n_stereo && nl >= 0 && nr >= 0, ORBX_ERR_ARG, "bad argument");
    *n_stereo = 0;
    if (nl == 0) return ORBX_OK;
    ORBX_REQUIRE(kpl && desc_l && uright && depth && (nr == 0 || (kpr && desc_r)), ORBX_ERR_ARG, "null pointer");
    ORBX_REQUIRE(nl <= 4096 && nr < (1 << 20), ORBX_ERR_UNSUPPORTED, "too many keypoints");
    orbx_pyramid PL, PR;
    int st;
    if ((st = orbx_extractor_pyramid_device(left, &PL))) return st;
    if ((st = orbx_extractor_pyramid_device(right, &PR))) return st;
    ORBX_REQUIRE(PL.nlevels == PR.nlevels, ORBX_ERR_ARG, "left/right extractors differ in levels");
    StereoArgs A{};
    if ((st = stereo_common(m, A, PL.scale, PL.nlevels, PL.rows[0], bf, b))) return st;
    ORBX_HIP(hipSetDevice(m->device));
    const int cap = std::max(nl, std::max(nr, 1));
    const size_t bytes = a256(28 * (size_t)cap) * 2 + a256(32 * (size_t)cap) * 2 + 2 * a256(4 * (size_t)cap) +
                         stereo_scratch(1, PL.rows[0], cap) + 3 * a256(4 * (size_t)cap);
    MatcherLease lease_(m, m->own());
    if ((st = m->reserve(bytes))) return st;
    Bump bp{(uint8_t*)m->scratch};
    orbx_keypoint* dkl = bp.take<orbx_keypoint>(cap);
    uint8_t* ddl = bp.take<uint8_t>(32 * (size_t)cap);
    orbx_keypoint* dkr = bp.take<orbx_keypoint>(cap);
    uint8_t* ddr = bp.take<uint8_t>(32 * (size_t)cap);
    int32_t* dbi = bp.take<int32_t>(cap);
    int32_t* dbd = bp.take<int32_t>(cap);
    A.row_start = bp.take<int32_t>((size_t)PL.rows[0] + 1);
    A.row_idx = bp.take<int32_t>(cap);
    (void)bp.take<int32_t>((size_t)PL.rows[0] + 1);      // (the scratch layout keeps the batch form's left-row buckets;
    (void)bp.take<int32_t>(cap);                          // this single-frame path searches per keypoint: none needed)
    float* dur = bp.take<float>(cap);
    float* ddp = bp.take<float>(cap);
    int32_t* dsad = bp.take<int32_t>(cap);
    hipStream_t s = m->own();
    // the four inputs into pinned staging laid out as the scratch (keypoints / descriptors of both sides are
    // contiguous there), one H2D copy; the two outputs come back the same way
    const size_t in_bytes = (size_t)((uint8_t*)dbi - (uint8_t*)dkl), out_off = (size_t)((uint8_t*)dur - (uint8_t*)dkl);
    const size_t out_bytes = (size_t)((uint8_t*)ddp - (uint8_t*)dur) + 4 * (size_t)nl;
    if ((st = m->stage_host(std::max(in_bytes, out_off + out_bytes)))) return st;
    uint8_t* hs = m->h_stage;
    std::memcpy(hs, kpl, 28 * (size_t)nl);
    std::memcpy(hs + ((uint8_t*)ddl - (uint8_t*)dkl), desc_l, 32 * (size_t)nl);
    if (nr > 0) {
        std::memcpy(hs + ((uint8_t*)dkr - (uint8_t*)dkl), kpr, 28 * (size_t)nr);
        std::memcpy(hs + ((uint8_t*)ddr - (uint8_t*)dkl), desc_r, 32 * (size_t)nr);
    }
    ORBX_HIP(hipMemcpyAsync(dkl, hs, in_bytes, hipMemcpyHostToDevice, s));
    A.kl = dkl; A.dl = ddl; A.kr = dkr; A.dr = ddr; A.nl = nullptr; A.nr = nullptr;
    A.nl_fixed = nl; A.nr_fixed = nr; A.capacity = cap;
    A.best_idx = dbi; A.best_dist = dbd;
    if ((st = stereo_launch(A, 1, nl, s))) return st;
    RefineArgs R{};
    R.kl = dkl; R.nl = nullptr; R.nl_fixed = nl; R.kr = dkr; R.best_idx = dbi; R.capacity = cap;
    R.L = PL; R.R = PR; R.left_first = 0; R.right_first = 0;
    R.bf = bf; R.maxD = bf / b;
    R.uright = dur; R.depth = ddp; R.sad = dsad;
    if ((st = refine_launch(R, 1, s))) return st;
    ORBX_HIP(hipMemcpyAsync(hs + out_off, dur, out_bytes, hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipStreamSynchronize(s));
    std::memcpy(uright, hs + out_off, 4 * (size_t)nl);
    std::memcpy(depth, hs + out_off + ((uint8_t*)ddp - (uint8_t*)dur), 4 * (size_t)nl);
    int n = 0;
    for (int i = 0; i < nl; ++i) n += depth[i] > 0;
    *n_stereo = n;
    return ORBX_OK;
}

// -------- host staging of a FeatureVector into the bump region
static FvDev stage_fv(Bump& bp, const orbx_featvec& f, int nfeat, hipStream_t s, int* st) {
    FvDev d{};
    d.n = f.n_nodes;
    uint32_t* node = bp.take<uint32_t>(std::max(f.n_nodes, 1));
    int32_t* off = bp.take<int32_t>((size_t)f.n_nodes + 1);
    const int nidx = f.n_nodes > 0 ? f.offsets[f.n_nodes] : 0;
    int32_t* idx = bp.take<int32_t>(std::max(nidx, 1));
    (void)nfeat;
    *st = ORBX_OK;
    if (f.n_nodes > 0) {
        if (hipMemcpyAsync(node, f.node_ids, 4 * (size_t)f.n_nodes, hipMemcpyHostToDevice, s) != hipSuccess ||
            hipMemcpyAsync(off, f.offsets, 4 * ((size_t)f.n_nodes + 1), hipMemcpyHostToDevice, s) != hipSuccess ||
            (nidx > 0 && hipMemcpyAsync(idx, f.indices, 4 * (size_t)nidx, hipMemcpyHostToDevice, s) != hipSuccess)) {
            set_error("featvec upload failed");
            *st = ORBX_ERR_HIP;
        }
    }
    d.node = node; d.off = off; d.idx = idx;
    return d;
}
static size_t fv_bytes(const orbx_featvec& f) {
    const int nidx = f.n_nodes > 0 ? f.offsets[f.n_nodes] : 0;
    return a256(4 * (size_t)std::max(f.n_nodes, 1)) + a256(4 * ((size_t)f.n_nodes + 1)) + a256(4 * (size_t)std::max(nidx, 1));
}
static int check_fv(const orbx_featvec& f, int nfeat) {
    ORBX_REQUIRE(f.n_nodes >= 0 && (f.n_nodes == 0 || (f.node_ids && f.offsets && f.indices)), ORBX_ERR_ARG, "bad featvec");
    for (int i = 0; i < f.n_nodes; ++i) {
        ORBX_REQUIRE(f.offsets[i + 1] >= f.offsets[i], ORBX_ERR_ARG, "featvec offsets not monotone");
        ORBX_REQUIRE(i == 0 || f.node_ids[i] > f.node_ids[i - 1], ORBX_ERR_ARG, "featvec node ids not ascending");
        ORBX_REQUIRE(f.offsets[i + 1] - f.offsets[i] <= 4096, ORBX_ERR_UNSUPPORTED, "node with > 4096 features");
    }
    const int nidx = f.n_nodes > 0 ? f.offsets[f.n_nodes] : 0;
    for (int i = 0; i < nidx; ++i) ORBX_REQUIRE(f.indices[i] >= 0 && f.indices[i] < nfeat, ORBX_ERR_ARG, "featvec index out of range");
    return ORBX_OK;
}

static int run_bow(orbx_matcher* m, int kff, const uint8_t* d1, const float* a1, const uint8_t* v1, int n1, orbx_featvec fv1,
                   const uint8_t* d2, const float* a2, const uint8_t* v2, int n2, orbx_featvec fv2, int32_t* match,
                   int nres, int* n_matches) {
    int st;
    if ((st = check_fv(fv1, n1)) || (st = check_fv(fv2, n2))) return st;
    ORBX_HIP(hipSetDevice(m->device));
    const size_t N1 = std::max(n1, 1), N2 = std::max(n2, 1), NR = std::max(nres, 1);
    const size_t bytes = a256(32 * N1) + a256(4 * N1) + a256(N1) + a256(32 * N2) + a256(4 * N2) + a256(N2) + fv_bytes(fv1) +
                         fv_bytes(fv2) + 2 * a256(4 * NR) + a256(4 * 32) + 256;
    MatcherLease lease_(m, m->own());
    if ((st = m->reserve(bytes))) return st;
    hipStream_t s = m->own();
    Bump bp{(uint8_t*)m->scratch};
    uint8_t* dd1 = bp.take<uint8_t>(32 * N1);
    float* da1 = bp.take<float>(N1);
    uint8_t* dv1 = bp.take<uint8_t>(N1);
    uint8_t* dd2 = bp.take<uint8_t>(32 * N2);
    float* da2 = bp.take<float>(N2);
    uint8_t* dv2 = bp.take<uint8_t>(N2);
    FvDev f1 = stage_fv(bp, fv1, n1, s, &st);
    if (st) return st;
    FvDev f2 = stage_fv(bp, fv2, n2, s, &st);
    if (st) return st;
    int32_t* dm = bp.take<int32_t>(NR);
    int32_t* db = bp.take<int32_t>(NR);
    int32_t* dh = bp.take<int32_t>(32);   // hist[30], nmatch at [31]
    if (n1) {
        ORBX_HIP(hipMemcpyAsync(dd1, d1, 32 * (size_t)n1, hipMemcpyHostToDevice, s));
        ORBX_HIP(hipMemcpyAsync(da1, a1, 4 * (size_t)n1, hipMemcpyHostToDevice, s));
        ORBX_HIP(hipMemcpyAsync(dv1, v1, (size_t)n1, hipMemcpyHostToDevice, s));
    }
    if (n2) {
        ORBX_HIP(hipMemcpyAsync(dd2, d2, 32 * (size_t)n2, hipMemcpyHostToDevice, s));
        ORBX_HIP(hipMemcpyAsync(da2, a2, 4 * (size_t)n2, hipMemcpyHostToDevice, s));
        if (v2) ORBX_HIP(hipMemcpyAsync(dv2, v2, (size_t)n2, hipMemcpyHostToDevice, s));
    }
    ORBX_HIP(hipMemsetAsync(dm, 0xff, 4 * NR, s));
    ORBX_HIP(hipMemsetAsync(dh, 0, 4 * 32, s));
    BowArgs A{};
    A.d1 = dd1; A.a1 = da1; A.as1 = 1; A.v1 = dv1; A.f1 = f1;
    A.d2 = dd2; A.a2 = da2; A.as2 = 1; A.v2 = dv2; A.f2 = f2;
    A.nnratio = m->nnratio; A.checkOri = m->checkOri; A.kff = kff;
    A.match = dm; A.bin = db; A.hist = dh; A.nmatch = dh + 31;
    if (fv1.n_nodes > 0) hipLaunchKernelGGL(k_bow, dim3(fv1.n_nodes), dim3(64), 0, s, A);
    if (m->checkOri) hipLaunchKernelGGL(k_rot_filter, dim3(1), dim3(256), 0, s, dm, db, nres, dh, dh + 31, 0);
    ORBX_HIP(hipGetLastError());
    int nm = 0;
    if (nres) ORBX_HIP(hipMemcpyAsync(match, dm, 4 * (size_t)nres, hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipMemcpyAsync(&nm, dh + 31, 4, hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipStreamSynchronize(s));
    *n_matches = nm;
    return ORBX_OK;
}

int orbx_search_by_bow_kfkf(orbx_matcher* m, const uint8_t* desc1, const float* angle1, const uint8_t* valid1, int n1,
                            orbx_featvec fv1, const uint8_t* desc2, const float* angle2, const uint8_t* valid2, int n2,
                            orbx_featvec fv2, int32_t* match12, int* n_matches) {
    ORBX_REQUIRE(m && n_matches && n1 >= 0 && n2 >= 0 && (n1 == 0 || (desc1 && angle1 && valid1 && match12)) &&
                     (n2 == 0 || (desc2 && angle2 && valid2)),
                 ORBX_ERR_ARG, "bad argument");
    *n_matches = 0;
    return run_bow(m, 0, desc1, angle1, valid1, n1, fv1, desc2, angle2, valid2, n2, fv2, match12, n1, n_matches);
}

int orbx_search_by_bow_kff(orbx_matcher* m, const uint8_t* desck, const float* anglek, const uint8_t* validk, int nk,
                           orbx_featvec fvk, const uint8_t* descf, const float* anglef, int nf, orbx_featvec fvf,
                           int32_t* matchf, int* n_matches) {
    ORBX_REQUIRE(m && n_matches && nk >= 0 && nf >= 0 && (nk == 0 || (desck && anglek && validk)) &&
                     (nf == 0 || (descf && anglef && matchf)),
                 ORBX_ERR_ARG, "bad argument");
    *n_matches = 0;
    return run_bow(m, 1, desck, anglek, validk, nk, fvk, descf, anglef, nullptr, nf, fvf, matchf, nf, n_matches);
}

int orbx_search_by_bow_kfkf_pairs_device(orbx_matcher* m, const orbx_kf_store* store, const int32_t* d_pairs, int n_pairs,
                                         int max_fv_nodes, int32_t* d_match12, int32_t* d_nmatches, void* stream) {
    ORBX_REQUIRE(m && store && d_pairs && d_match12 && d_nmatches && n_pairs >= 0 && max_fv_nodes >= 0, ORBX_ERR_ARG,
                 "bad argument");
    const orbx_kf_store& S = *store;
    ORBX_REQUIRE(S.desc && S.kps && S.valid && S.fv_nodes && S.fv_offsets && S.fv_indices && S.n_fv && S.capacity > 0,
                 ORBX_ERR_ARG, "incomplete keyframe store");
    ORBX_REQUIRE(((uintptr_t)S.desc % 16) == 0 && S.desc_stride % 16 == 0 && ((uintptr_t)S.kps % 4) == 0 &&
                     S.kps_stride % 4 == 0 && S.fv_nodes_stride % 4 == 0 && S.fv_offsets_stride % 4 == 0 &&
                     S.fv_indices_stride % 4 == 0 && S.n_fv_stride % 4 == 0,
                 ORBX_ERR_ARG, "misaligned keyframe store");
    ORBX_REQUIRE(S.desc_stride >= 32 * (size_t)S.capacity && S.kps_stride >= sizeof(orbx_keypoint) * (size_t)S.capacity,
                 ORBX_ERR_ARG, "keyframe store strides smaller than capacity");
    if (n_pairs == 0) return ORBX_OK;
    ORBX_HIP(hipSetDevice(m->device));
    hipStream_t s = (hipStream_t)stream;
    const size_t cap = (size_t)S.capacity;
    ORBX_HIP(hipMemsetAsync(d_match12, 0xff, (size_t)n_pairs * cap * 4, s));
    ORBX_HIP(hipMemsetAsync(d_nmatches, 0, (size_t)n_pairs * 4, s));
    MatcherLease lease_(m, s);
    int st = m->reserve_on(a256((size_t)n_pairs * cap * 4) + a256((size_t)n_pairs * 32 * 4), s);
    if (st) return st;
    int32_t* bin = (int32_t*)m->scratch;
    int32_t* hist = (int32_t*)((uint8_t*)m->scratch + a256((size_t)n_pairs * cap * 4));
    ORBX_HIP(hipMemsetAsync(hist, 0, (size_t)n_pairs * 32 * 4, s));
    hipLaunchKernelGGL(k_bow_pairs, dim3(std::max(1, std::min(max_fv_nodes, 4096)), n_pairs), dim3(64), 0, s, S, d_pairs, m->nnratio, m->checkOri, d_match12,
                       bin, hist, d_nmatches);
    if (m->checkOri)
        hipLaunchKernelGGL(k_rot_filter, dim3(n_pairs), dim3(256), 0, s, d_match12, bin, S.capacity, hist, d_nmatches, S.capacity);
    ORBX_HIP(hipGetLastError());
    return ORBX_OK;
}

int orbx_search_for_triangulation_pairs_device(orbx_matcher* m, const orbx_kf_store* store, const uint8_t* d_has_mp,
                                               size_t has_mp_stride, const float* d_uright, size_t uright_stride, const int32_t* d_pairs, const orbx_tri_geom* d_geom,
                                               int n_pairs, int max_fv_nodes, const float* sigma2_2, const float* scale_2,
                                               int nlevels, int only_stereo, int32_t* d_match12, int32_t* d_nmatches,
                                               void* stream) {
    ORBX_REQUIRE(m && store && d_pairs && d_geom && d_match12 && d_nmatches && n_pairs >= 0 && max_fv_nodes >= 0 && sigma2_2 &&
                     scale_2 && nlevels >= 1 && nlevels <= 32, ORBX_ERR_ARG, "bad argument");
    const orbx_kf_store& S = *store;
    ORBX_REQUIRE(S.desc && S.kps && S.valid && S.fv_nodes && S.fv_offsets && S.fv_indices && S.n_fv && S.capacity > 0,
                 ORBX_ERR_ARG, "incomplete keyframe store");
    ORBX_REQUIRE(((uintptr_t)S.desc % 16) == 0 && S.desc_stride % 16 == 0 && ((uintptr_t)S.kps % 4) == 0 &&
                     S.kps_stride % 4 == 0 && S.fv_nodes_stride % 4 == 0 && S.fv_offsets_stride % 4 == 0 &&
                     S.fv_indices_stride % 4 == 0 && S.n_fv_stride % 4 == 0 && (!d_uright || uright_stride % 4 == 0),
                 ORBX_ERR_ARG, "misaligned keyframe store");
    if (n_pairs == 0) return ORBX_OK;
    ORBX_REQUIRE(n_pairs <= 65535, ORBX_ERR_UNSUPPORTED, "too many pairs (%d)", n_pairs);
    ORBX_HIP(hipSetDevice(m->device));
    hipStream_t s = (hipStream_t)stream;
    const size_t cap = (size_t)S.capacity;
    ORBX_HIP(hipMemsetAsync(d_match12, 0xff, (size_t)n_pairs * cap * 4, s));
    ORBX_HIP(hipMemsetAsync(d_nmatches, 0, (size_t)n_pairs * 4, s));
    MatcherLease lease_(m, s);
    // scratch: bins, histograms, and (no uright given) one row of -1 = "no stereo keypoint"
    int st = m->reserve_on(a256((size_t)n_pairs * cap * 4) + a256((size_t)n_pairs * 32 * 4) + a256(cap * 4), s);
    if (st) return st;
    int32_t* bin = (int32_t*)m->scratch;
    int32_t* hist = (int32_t*)((uint8_t*)m->scratch + a256((size_t)n_pairs * cap * 4));
    float* no_ur = (float*)((uint8_t*)hist + a256((size_t)n_pairs * 32 * 4));
    ORBX_HIP(hipMemsetAsync(hist, 0, (size_t)n_pairs * 32 * 4, s));
    if (!d_uright) ORBX_HIP(hipMemsetAsync(no_ur, 0xff, cap * 4, s));   // 0xffffffff = NaN: "ur >= 0" false
    TriTables T{};
    for (int l = 0; l < nlevels; ++l) { T.sigma2[l] = sigma2_2[l]; T.scale2[l] = scale_2[l]; }
    hipLaunchKernelGGL(k_triangulate_pairs, dim3(std::max(1, std::min(max_fv_nodes, 4096)), n_pairs), dim3(64), 0, s, S, d_has_mp, has_mp_stride, d_uright,
                       uright_stride, d_pairs, d_geom, T, only_stereo, m->checkOri, no_ur, d_match12, bin, hist, d_nmatches);
    if (m->checkOri)
        hipLaunchKernelGGL(k_rot_filter, dim3(n_pairs), dim3(256), 0, s, d_match12, bin, S.capacity, hist, d_nmatches, S.capacity);
    ORBX_HIP(hipGetLastError());
    return ORBX_OK;
}

static int distinct_launch(DistinctArgs& A, hipStream_t s) {
    if (A.M == 0) return ORBX_OK;
    A.nbx = (A.M + 3) / 4;
    hipLaunchKernelGGL(k_distinctive, dim3(kXcds * xcd_chunk(A.nbx)), dim3(256), 0, s, A);
    ORBX_HIP(hipGetLastError());
    return ORBX_OK;
}

int orbx_distinctive_descriptors_device(orbx_matcher* m, const uint8_t* d_desc, const int32_t* d_offsets, int n_mappoints,
                                        int32_t* d_best, uint8_t* d_out_desc, void* stream) {
    ORBX_REQUIRE(m && n_mappoints >= 0 && (n_mappoints == 0 || (d_desc && d_offsets && d_best)), ORBX_ERR_ARG, "bad argument");
    ORBX_HIP(hipSetDevice(m->device));
    DistinctArgs A{};
    A.desc = d_desc; A.store = 0; A.off = d_offsets; A.M = n_mappoints; A.best = d_best; A.out = d_out_desc;
    return distinct_launch(A, (hipStream_t)stream);
}

int orbx_distinctive_descriptors_store_device(orbx_matcher* m, const orbx_kf_store* store, const int32_t* d_obs,
                                              const int32_t* d_offsets, int n_mappoints, int32_t* d_best, uint8_t* d_out_desc,
                                              void* stream) {
    ORBX_REQUIRE(m && store && n_mappoints >= 0 && (n_mappoints == 0 || (d_obs && d_offsets && d_best)), ORBX_ERR_ARG,
                 "bad argument");
    ORBX_REQUIRE(store->desc && ((uintptr_t)store->desc % 16) == 0 && store->desc_stride % 16 == 0, ORBX_ERR_ARG,
                 "misaligned keyframe store");
    ORBX_HIP(hipSetDevice(m->device));
    DistinctArgs A{};
    A.obs = d_obs; A.S = *store; A.store = 1; A.off = d_offsets; A.M = n_mappoints; A.best = d_best; A.out = d_out_desc;
    return distinct_launch(A, (hipStream_t)stream);
}

int orbx_distinctive_descriptors_neighbours_device(orbx_matcher* m, const orbx_kf_store* store, const int32_t* d_new_slots,
                                                   const int32_t* d_neighbours, int n_new, int n_neighbours,
                                                   const int32_t* d_match12, int32_t* d_best, uint8_t* d_out_desc,
                                                   void* stream) {
    ORBX_REQUIRE(m && store && n_new >= 0 && n_neighbours >= 0 && n_neighbours <= kWave &&
                     (n_new == 0 || (d_new_slots && d_best && (n_neighbours == 0 || (d_neighbours && d_match12)))),
                 ORBX_ERR_ARG, "bad argument");
    ORBX_REQUIRE(store->desc && ((uintptr_t)store->desc % 16) == 0 && store->desc_stride % 16 == 0 && store->capacity > 0,
                 ORBX_ERR_ARG, "misaligned keyframe store");
    ORBX_REQUIRE((size_t)n_new * store->capacity < (1u << 31), ORBX_ERR_UNSUPPORTED, "too many MapPoints");
    if (n_new == 0) return ORBX_OK;
    ORBX_HIP(hipSetDevice(m->device));
    DistinctNbArgs A{};
    A.S = *store; A.new_slots = d_new_slots; A.nb = d_neighbours; A.m12 = d_match12; A.n = n_new; A.nn = n_neighbours;
    A.M = n_new * store->capacity; A.best = d_best; A.out = d_out_desc; A.nbx = (A.M + 3) / 4;
    hipLaunchKernelGGL(k_distinctive_nb, dim3(kXcds * xcd_chunk(A.nbx)), dim3(256), 0, (hipStream_t)stream, A);
    ORBX_HIP(hipGetLastError());
    return ORBX_OK;
}

int orbx_distinctive_descriptors(orbx_matcher* m, const uint8_t* desc, const int32_t* offsets, int n_mappoints, int32_t* best,
                                 uint8_t* out_desc) {
    ORBX_REQUIRE(m && n_mappoints >= 0 && (n_mappoints == 0 || (offsets && best)), ORBX_ERR_ARG, "bad argument");
    if (n_mappoints == 0) return ORBX_OK;
    ORBX_REQUIRE(offsets[0] == 0, ORBX_ERR_ARG, "offsets[0] must be 0");
    for (int i = 0; i < n_mappoints; ++i)
        ORBX_REQUIRE(offsets[i + 1] >= offsets[i], ORBX_ERR_ARG, "offsets not monotone at %d", i);
    const int total = offsets[n_mappoints];
    ORBX_REQUIRE(total == 0 || desc, ORBX_ERR_ARG, "null descriptors");
    ORBX_REQUIRE(total < (1 << 30) / 32, ORBX_ERR_UNSUPPORTED, "too many observations");
    ORBX_HIP(hipSetDevice(m->device));
    const size_t M = (size_t)n_mappoints;
    MatcherLease lease_(m, m->own());
    int st = m->reserve(a256(32 * (size_t)std::max(total, 1)) + a256(4 * (M + 1)) + a256(4 * M) + a256(32 * M));
    if (st) return st;
    Bump bp{(uint8_t*)m->scratch};
    uint8_t* dd = bp.take<uint8_t>(32 * (size_t)std::max(total, 1));
    int32_t* doff = bp.take<int32_t>(M + 1);
    int32_t* dbest = bp.take<int32_t>(M);
    uint8_t* dout = bp.take<uint8_t>(32 * M);
    hipStream_t s = m->own();
    if (total) ORBX_HIP(hipMemcpyAsync(dd, desc, 32 * (size_t)total, hipMemcpyHostToDevice, s));
    ORBX_HIP(hipMemcpyAsync(doff, offsets, 4 * (M + 1), hipMemcpyHostToDevice, s));
    DistinctArgs A{};
    A.desc = dd; A.store = 0; A.off = doff; A.M = n_mappoints; A.best = dbest; A.out = out_desc ? dout : nullptr;
    if ((st = distinct_launch(A, s))) return st;
    ORBX_HIP(hipMemcpyAsync(best, dbest, 4 * M, hipMemcpyDeviceToHost, s));
    if (out_desc) ORBX_HIP(hipMemcpyAsync(out_desc, dout, 32 * M, hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipStreamSynchronize(s));
    return ORBX_OK;
}

int orbx_search_for_triangulation(orbx_matcher* m, const uint8_t* desc1, const orbx_keypoint* kp1, const uint8_t* has_mp1,
                                  const float* uright1, int n1, orbx_featvec fv1, const uint8_t* desc2, const orbx_keypoint* kp2,
                                  const uint8_t* has_mp2, const float* uright2, int n2, orbx_featvec fv2, const float* F12,
                                  const float* sigma2_2, const float* scale_2, int nlevels, float ex, float ey, int only_stereo,
                                  int32_t* match12, int* n_matches) {
    ORBX_REQUIRE(m && n_matches && F12 && sigma2_2 && scale_2 && nlevels >= 1 && nlevels <= 32 && n1 >= 0 && n2 >= 0,
                 ORBX_ERR_ARG, "bad argument");
    ORBX_REQUIRE((n1 == 0 || (desc1 && kp1 && has_mp1 && uright1 && match12)) && (n2 == 0 || (desc2 && kp2 && has_mp2 && uright2)),
                 ORBX_ERR_ARG, "null pointer");
    *n_matches = 0;
    int st;
    if ((st = check_fv(fv1, n1)) || (st = check_fv(fv2, n2))) return st;
    ORBX_HIP(hipSetDevice(m->device));
    const size_t N1 = std::max(n1, 1), N2 = std::max(n2, 1);
    const size_t bytes = a256(32 * N1) + a256(28 * N1) + a256(N1) + a256(4 * N1) + a256(32 * N2) + a256(28 * N2) + a256(N2) +
                         a256(4 * N2) + fv_bytes(fv1) + fv_bytes(fv2) + 2 * a256(4 * N1) + a256(4 * 32) + 256;
    MatcherLease lease_(m, m->own());
    if ((st = m->reserve(bytes))) return st;
    hipStream_t s = m->own();
    Bump bp{(uint8_t*)m->scratch};
    uint8_t* dd1 = bp.take<uint8_t>(32 * N1);
    orbx_keypoint* dk1 = bp.take<orbx_keypoint>(N1);
    uint8_t* dm1 = bp.take<uint8_t>(N1);
    float* du1 = bp.take<float>(N1);
    uint8_t* dd2 = bp.take<uint8_t>(32 * N2);
    orbx_keypoint* dk2 = bp.take<orbx_keypoint>(N2);
    uint8_t* dm2 = bp.take<uint8_t>(N2);
    float* du2 = bp.take<float>(N2);
    FvDev f1 = stage_fv(bp, fv1, n1, s, &st);
    if (st) return st;
    FvDev f2 = stage_fv(bp, fv2, n2, s, &st);
    if (st) return st;
    int32_t* dm = bp.take<int32_t>(N1);
    int32_t* db = bp.take<int32_t>(N1);
    int32_t* dh = bp.take<int32_t>(32);
    if (n1) {
        ORBX_HIP(hipMemcpyAsync(dd1, desc1, 32 * (size_t)n1, hipMemcpyHostToDevice, s));
        ORBX_HIP(hipMemcpyAsync(dk1, kp1, 28 * (size_t)n1, hipMemcpyHostToDevice, s));
        ORBX_HIP(hipMemcpyAsync(dm1, has_mp1, (size_t)n1, hipMemcpyHostToDevice, s));
        ORBX_HIP(hipMemcpyAsync(du1, uright1, 4 * (size_t)n1, hipMemcpyHostToDevice, s));
    }
    if (n2) {
        ORBX_HIP(hipMemcpyAsync(dd2, desc2, 32 * (size_t)n2, hipMemcpyHostToDevice, s));
        ORBX_HIP(hipMemcpyAsync(dk2, kp2, 28 * (size_t)n2, hipMemcpyHostToDevice, s));
        ORBX_HIP(hipMemcpyAsync(dm2, has_mp2, (size_t)n2, hipMemcpyHostToDevice, s));
        ORBX_HIP(hipMemcpyAsync(du2, uright2, 4 * (size_t)n2, hipMemcpyHostToDevice, s));
    }
    ORBX_HIP(hipMemsetAsync(dm, 0xff, 4 * N1, s));
    ORBX_HIP(hipMemsetAsync(dh, 0, 4 * 32, s));
    TriArgs A{};
    A.d1 = dd1; A.k1 = dk1; A.mp1 = dm1; A.ur1 = du1; A.f1 = f1;
    A.d2 = dd2; A.k2 = dk2; A.mp2 = dm2; A.ur2 = du2; A.f2 = f2;
    for (int i = 0; i < 9; ++i) A.F[i] = F12[i];
    for (int l = 0; l < nlevels; ++l) { A.sigma2[l] = sigma2_2[l]; A.scale2[l] = scale_2[l]; }
    A.ex = ex; A.ey = ey; A.onlyStereo = only_stereo; A.checkOri = m->checkOri;
    A.match = dm; A.bin = db; A.hist = dh; A.nmatch = dh + 31;
    if (fv1.n_nodes > 0) hipLaunchKernelGGL(k_triangulate, dim3(fv1.n_nodes), dim3(64), 0, s, A);
    if (m->checkOri) hipLaunchKernelGGL(k_rot_filter, dim3(1), dim3(256), 0, s, dm, db, n1, dh, dh + 31, 0);
    ORBX_HIP(hipGetLastError());
    int nm = 0;
    if (n1) ORBX_HIP(hipMemcpyAsync(match12, dm, 4 * (size_t)n1, hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipMemcpyAsync(&nm, dh + 31, 4, hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipStreamSynchronize(s));
    *n_matches = nm;
    return ORBX_OK;
}

}  // extern "C"
