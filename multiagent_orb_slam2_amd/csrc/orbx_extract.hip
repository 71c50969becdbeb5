// =====================================================================================================
// orbx_extract.hip — MI355X (gfx950) ORB extractor: the hot path of ORBextractor::operator()
// (reference src/ORBextractor.cc:1043-1105) as batched HIP kernels behind the C-ABI of include/orbx.h.
//
// Per device call over a batch of B images (all rows x cols), two streams (run_batch; §7 of DESIGN.md):
//   (level 0 is read in place from the caller's images: no copy)   (ComputePyramid :1127)
//   k_resize4       level l-1 -> level l, l = 1..L-1 (chained, launch stream)      (ComputePyramid :1120)
//   k_fast_wave     one wave per (cell, image): the cell ROI as an f16-biased u16 pair image in the wave's LDS
//                   slice, compass pre-test in quads, closed-form FAST scores of the survivors, strict 3x3 NMS at
//                   iniThFAST / minThFAST, per-cell fallback, row-major slots by wave ballots (no barrier)
//                   (level 0 on the side stream, levels 1..L-1 on the launch stream)   (:789-829)
//   k_blur7         7x7 sigma-2 Gaussian on every level (REFLECT_101), register-streaming, side stream (:1085-1086)
//   k_quadtree      one workgroup per (level, image): DistributeOctTree's list/quadtree as data-parallel
//                   passes over LDS node arrays                     (:539-763, :834-847)
//   k_describe_m    two keypoints per wave: IC angle on the level, steered BRIEF on the blurred level,
//                   level-major output with coordinates scaled to level 0 (on the caller's output stream with
//                   the split entry point)                            (:77-147, :851-852, :1075-1104)
// Cross-call reuse of every buffer is ordered by events from a pool of per-call sets (Extractor::CallEvents).
// Pinned arithmetic (identical to oracle/orb_oracle.cpp): fixed-point resize and blur,
// round-half-even, no FMA contraction (-ffp-contract=off + explicit __f*_rn), correctly rounded
// float cos/sin of the BRIEF angle, quadtree phase-2 ties in creation order.
// =====================================================================================================
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "orbx_common.h"
#include "orbx_pattern.h"
#include "orbx_sincos.h"

namespace orbx {

// ---------------------------------------------------------------------------------------------
// error plumbing (shared by every translation unit of liborbx)
// ---------------------------------------------------------------------------------------------
static thread_local std::string g_err;

void set_error(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
}

constexpr int kEdge = 19;          // EDGE_THRESHOLD (src/ORBextractor.cc:74)
constexpr int kHalfPatch = 15;     // HALF_PATCH_SIZE (:73)
constexpr int kMaxRoi = 72;        // cell ROI side bound: wCell < 60 (+6)
#ifndef ORBX_QT_THREADS
#define ORBX_QT_THREADS 256
#endif
constexpr int kQtThreads = ORBX_QT_THREADS;
constexpr int kMaxLevels = 32;

// ---------------------------------------------------------------------------------------------
// device-side geometry records
// ---------------------------------------------------------------------------------------------
struct LevelDev {
    int w, h;            // level size
    int pyr_off;         // offset of the level inside one image's pyramid
    int cell_begin, cell_end;
    int cand_off;        // candidate slot region (per image) of the level
    int cand_cap;
    int out_off;         // quadtree output slot region (per image)
    int out_cap;
    int N;               // mnFeaturesPerLevel
    int nIni;
    float hX;
    int win_w, win_h;    // maxBorder - minBorder
    float scale;         // mvScaleFactor
    int patch;           // (int)(PATCH_SIZE * scale)
};

struct CellDev {
    int level;
    int x0, y0;          // ROI origin in level coords (iniX, iniY)
    int W, H;            // ROI size (maxX - iniX, maxY - iniY)
    int slot_off;        // candidate slot offset (per image)
    int slot_cap;
    int pad;
};

// Level 0 is the caller's image itself (no copy): base pointer, row step and image stride.
struct Src0 {
    const uint8_t* p;
    size_t step, istride;
};

__device__ __forceinline__ const uint8_t* level_pixels(const uint8_t* pyr, size_t pyr_stride, const LevelDev& L,
                                                       int lvl, int img, const Src0& s0, int& stride) {
    if (lvl == 0) {
        stride = (int)s0.step;
        return s0.p + img * s0.istride;
    }
    stride = L.w;
    return pyr + img * pyr_stride + L.pyr_off;
}

struct ResizeTab {       // per level >= 1, device arrays
    int* x0; int* x1; int* a0; int* a1;   // [w]
    int* y0; int* y1; int* b0; int* b1;   // [h]
};

// The rBRIEF tests laid out per describe lane: with kLp lanes per keypoint, lane lk runs tests g * kLp + lk (g < 256 /
// kLp), and its words sit contiguously at [lk * (256 / kLp) + g], so a lane fetches them with 16-byte loads from one
// base address instead of one dword load and one 64-bit address per test.
constexpr signed char kPatternInit[ORBX_PATTERN_TESTS * 4] = ORBX_PATTERN_INIT;
template <int kLp>
struct PatternByLane { uint32_t w[ORBX_PATTERN_TESTS]; };
template <int kLp>
constexpr PatternByLane<kLp> make_pattern_by_lane() {
    PatternByLane<kLp> t{};
    constexpr int nt = ORBX_PATTERN_TESTS / kLp;
    for (int lk = 0; lk < kLp; ++lk)
        for (int g = 0; g < nt; ++g) {
            const int s = 4 * (g * kLp + lk);
            t.w[lk * nt + g] = (uint32_t)(uint8_t)kPatternInit[s] | ((uint32_t)(uint8_t)kPatternInit[s + 1] << 8) |
                               ((uint32_t)(uint8_t)kPatternInit[s + 2] << 16) | ((uint32_t)(uint8_t)kPatternInit[s + 3] << 24);
        }
    return t;
}
// Initialised in their declarations: the tables are part of the code object, so every device the module is loaded on
// holds them (an uninitialised __constant__ filled by hipMemcpyToSymbol is written on the current device only).
__constant__ __attribute__((aligned(16))) PatternByLane<32> c_pattern_l32 = make_pattern_by_lane<32>();
__constant__ __attribute__((aligned(16))) PatternByLane<16> c_pattern_l16 = make_pattern_by_lane<16>();
// umax for HALF_PATCH_SIZE = 15 (ORBextractor ctor :454-469); the host recomputes it and checks equality
constexpr int kUmax[16] = {15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3};


// =============================================================================================
// kernels
// =============================================================================================

// resize INTER_LINEAR 8U, fixed point (pinned OpenCV 3.2 generic path): horizontal taps a0/a1 (x2048)
// with clamped source columns, vertical (r0*b0 + r1*b1 + 2^21) >> 22 saturated.
__global__ __launch_bounds__(256) void k_resize(uint8_t* __restrict__ pyr, size_t pyr_stride, const uint8_t* __restrict__ src,
                                                size_t src_step, size_t src_istride, int dst_off, int dw, int dh, ResizeTab t) {
    const int img = blockIdx.z, y = blockIdx.y;
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= dw || y >= dh) return;
    const uint8_t* S = src + img * src_istride;
    const uint8_t* r0 = S + (size_t)t.y0[y] * src_step;
    const uint8_t* r1 = S + (size_t)t.y1[y] * src_step;
    const int xa = t.x0[x], xb = t.x1[x], a0 = t.a0[x], a1 = t.a1[x];
    const int h0 = (int)r0[xa] * a0 + (int)r0[xb] * a1;
    const int h1 = (int)r1[xa] * a0 + (int)r1[xb] * a1;
    int v = (h0 * t.b0[y] + h1 * t.b1[y] + (1 << 21)) >> 22;
    v = min(max(v, 0), 255);
    pyr[img * pyr_stride + dst_off + (size_t)y * dw + x] = (uint8_t)v;
}

// Vectorised form of the same arithmetic: one wave per (image, 8-row band, 256-column strip); lane l owns
// the 4 output columns of group g = strip*64 + l.  The source bytes of a group's 8 taps lie in an 8-byte
// window at column xb[g] (the host checks the span), so per source row a lane issues one 8-byte load, and
// per column one v_perm_b32 (selector sel[g][k] = left and right tap offsets, as u16 lanes) and one
// v_dot2_u32_u16 with the packed taps (a0 | a1 << 16) give the horizontal value exactly.  The row's
// vertical taps are wave-uniform (scalar loads); the 4 output bytes leave as one dword store.
#ifndef ORBX_RESIZE_BAND
#define ORBX_RESIZE_BAND 8      // output rows per wave (r2z A/B: 4 is 1 % slower, 16 is 29 % slower)
#endif
constexpr int kResizeBand = ORBX_RESIZE_BAND, kResizeStrip = 256;
struct ResizeVec {       // per level >= 1 with every group's span <= 8 bytes
    const int* xb;       // [groups] (host copy; the kernel recomputes it from sxs, resize_xb)
    const uint4* sel;    // [groups] perm selectors of the 4 columns
    const uint4* coef;   // [groups] a0 | a1 << 16 of the 4 columns
    const int4* yrow;    // [h] y0, y1, b0, b1
    int groups;
    double sxs;          // source / destination width, as the host tables use it
};

// A group's window column, hx0[4 g] of the host tables (the OpenCV 3.2 fixed-point INTER_LINEAR x map: fx = (float)((x +
// 0.5) * sxs - 0.5), floor, clamped to [0, sw - 1]) recomputed in the lane with the same IEEE operations: the window
// loads then need no table load in front of them (one dependent memory round trip less per wave).
__device__ __forceinline__ int resize_xb(int g, double sxs, int sw) {
    const float fx = __double2float_rn(__dsub_rn(__dmul_rn(__dadd_rn((double)(4 * g), 0.5), sxs), 0.5));
    return min(max((int)floorf(fx), 0), sw - 1);
}
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void resize_window(const uint8_t* __restrict__ row, int xb, int sw, bool fast, uint32_t& lo,
                                              uint32_t& hi) {
    if (fast) {
        uint32_t v[2];
        __builtin_memcpy(v, row + xb, 8);
        lo = v[0]; hi = v[1];
    } else {                      // window reaches past the row end: only bytes inside the row are ever selected
        uint32_t v[2] = {0, 0};
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (xb + i < sw) v[i >> 2] |= (uint32_t)row[xb + i] << (8 * (i & 3));
        lo = v[0]; hi = v[1];
    }
}

// Branch-free form for rows of >= 8 bytes: one 8-byte load clamped inside the row, shifted so that byte i is column
// xb + i (columns past the row end read as 0 and are never selected).  Every lane loads, so a wave's loads for
// several rows issue back to back instead of one divergent branch (and one wait) per row.
__device__ __forceinline__ void resize_window8(const uint8_t* __restrict__ row, int xb, int sw, uint32_t& lo, uint32_t& hi) {
    const int xc = min(xb, sw - 8);
    uint64_t v;
    __builtin_memcpy(&v, row + xc, 8);
    v >>= 8 * (xb - xc);
    lo = (uint32_t)v; hi = (uint32_t)(v >> 32);
}

// Vertical step of one output pixel, exact under the table conditions the host checks for the vectorised form (every
// tap >= 0, a0 + a1 <= 2049, b0 + b1 <= 2049): hv <= 255 * 2049 < 2^24, so both products are 24-bit multiplies
// (v_mad_u32_u24, full rate; the u32 form is a quarter-rate v_mul_lo_u32), and with b scaled by 4
// acc = 4 * (hv0 * b0 + hv1 * b1 + 2^21) < 2^32, whose byte 3 is (hv0 * b0 + hv1 * b1 + 2^21) >> 22 <= 255 (the
// saturation of the generic path cannot bite).
__device__ __forceinline__ uint32_t resize_acc(uint32_t hv0, uint32_t hv1, int b0, int b1) {
    return __umul24(hv0, (uint32_t)b0 << 2) + __umul24(hv1, (uint32_t)b1 << 2) + (1u << 23);
}
// byte 3 of four accumulators -> the 4 output bytes (two v_perm_b32 and an OR)
__device__ __forceinline__ uint32_t resize_pack(const uint32_t* acc) {
    return __builtin_amdgcn_perm(acc[1], acc[0], 0x0c0c0703u) | __builtin_amdgcn_perm(acc[3], acc[2], 0x07030c0cu);
}

// One wave's work item of the vectorised resize: (256-column strip, 8-row band) of one image's level.
__device__ __forceinline__ void resize4_item(uint8_t* __restrict__ pyr, size_t pyr_stride, const uint8_t* __restrict__ src,
                                             size_t src_step, size_t src_istride, int sw, int dst_off, int dw, int dh,
                                             const ResizeVec& t, int strip, int band, int img) {
    const int g = strip * (kResizeStrip / 4) + lane_id();
    if (g >= t.groups) return;
    const int xb = resize_xb(g, t.sxs, sw);
    const uint4 sel = t.sel[g], coef = t.coef[g];
    const bool fast = xb + 8 <= sw;
    const int x = 4 * g;
    const bool full = x + 4 <= dw;
    const uint8_t* S = src + img * src_istride;
    uint8_t* D = pyr + img * pyr_stride + dst_off;
    const int y0 = band * kResizeBand, y1 = min(y0 + kResizeBand, dh);
    if (sw >= 8) {
        // every source window of the band's rows first (one memory round trip per wave), then the arithmetic
        const int ny = y1 - y0;
        int4 yr[kResizeBand];
        uint32_t lo[2 * kResizeBand], hi[2 * kResizeBand];
#pragma unroll
        for (int r = 0; r < kResizeBand; ++r) yr[r] = t.yrow[y0 + min(r, ny - 1)];
#pragma unroll
        for (int r = 0; r < kResizeBand; ++r) {
            resize_window8(S + (size_t)yr[r].x * src_step, xb, sw, lo[2 * r], hi[2 * r]);
            resize_window8(S + (size_t)yr[r].y * src_step, xb, sw, lo[2 * r + 1], hi[2 * r + 1]);
        }
        const uint32_t sl[4] = {sel.x, sel.y, sel.z, sel.w}, cf[4] = {coef.x, coef.y, coef.z, coef.w};
#pragma unroll
        for (int r = 0; r < kResizeBand; ++r) {
            if (r >= ny) break;
            uint32_t acc[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const u16x2 c = __builtin_bit_cast(u16x2, cf[k]);
                const uint32_t hv0 = __builtin_amdgcn_udot2(
                    __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(hi[2 * r], lo[2 * r], sl[k])), c, 0u, false);
                const uint32_t hv1 = __builtin_amdgcn_udot2(
                    __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(hi[2 * r + 1], lo[2 * r + 1], sl[k])), c, 0u, false);
                acc[k] = resize_acc(hv0, hv1, yr[r].z, yr[r].w);
            }
            const uint32_t packed = resize_pack(acc);
            uint8_t* o = D + (size_t)(y0 + r) * dw + x;
            if (full) {
                __builtin_memcpy(o, &packed, 4);
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (x + k < dw) o[k] = (uint8_t)(packed >> (8 * k));
            }
        }
        return;
    }
    for (int y = y0; y < y1; ++y) {          // source rows narrower than 8 bytes
        const int4 yr = t.yrow[y];
        uint32_t l0, h0, l1, h1;
        resize_window(S + (size_t)yr.x * src_step, xb, sw, fast, l0, h0);
        resize_window(S + (size_t)yr.y * src_step, xb, sw, fast, l1, h1);
        const uint32_t sl[4] = {sel.x, sel.y, sel.z, sel.w}, cf[4] = {coef.x, coef.y, coef.z, coef.w};
        uint32_t acc[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u16x2 c = __builtin_bit_cast(u16x2, cf[k]);
            const uint32_t hv0 = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, __builtin_amdgcn_perm(h0, l0, sl[k])), c, 0u, false);
            const uint32_t hv1 = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, __builtin_amdgcn_perm(h1, l1, sl[k])), c, 0u, false);
            acc[k] = resize_acc(hv0, hv1, yr.z, yr.w);
        }
        const uint32_t packed = resize_pack(acc);
        uint8_t* o = D + (size_t)y * dw + x;
        if (full) {
            __builtin_memcpy(o, &packed, 4);
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (x + k < dw) o[k] = (uint8_t)(packed >> (8 * k));
        }
    }
}

__global__ __launch_bounds__(256) void k_resize4(uint8_t* __restrict__ pyr, size_t pyr_stride, const uint8_t* __restrict__ src,
                                                 size_t src_step, size_t src_istride, int sw, int dst_off, int dw, int dh,
                                                 ResizeVec t, int nstrips, int nbands, int batch) {
    const int nwaves = nstrips * nbands * batch;
    const int nwg = (nwaves + 3) / 4;
    const int wg = xcd_item(xcd_chunk(nwg));
    const int wv = wg * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (wg >= nwg || wv >= nwaves) return;
    const int img = wv / (nstrips * nbands);
    const int rem = wv - img * nstrips * nbands;
    const int band = rem / nstrips, strip = rem - band * nstrips;
    resize4_item(pyr, pyr_stride, src, src_step, src_istride, sw, dst_off, dw, dh, t, strip, band, img);
}

// The small levels of the chain in one launch: one 256-thread workgroup per image, no LDS, computes
// levels l0 .. n-1 in order from the pyramid in memory -- its 4 waves walk level l's (strip, band) items as k_resize4's
// waves do, then a workgroup barrier (the level's rows, written through to L2 by this CU, are read by the next level's
// waves of the same workgroup) -- so the chain's upper levels are one launch instead of n - l0 dependent ones.
struct TailLevel { ResizeVec t; int sw, src_off, dst_off, dw, dh, nstrips, nbands; };
constexpr int kTailMax = 6;
struct TailArgs { TailLevel lv[kTailMax]; int n; };
__global__ __launch_bounds__(256) void k_resize_tail(uint8_t* __restrict__ pyr, size_t pyr_stride, TailArgs A, int batch) {
    const int img = blockIdx.x;
    if (img >= batch) return;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    for (int k = 0; k < A.n; ++k) {
        const TailLevel& L = A.lv[k];
        const int items = L.nstrips * L.nbands;
        for (int it = w; it < items; it += 4) {
            const int band = it / L.nstrips, strip = it - band * L.nstrips;
            resize4_item(pyr, pyr_stride, pyr + L.src_off, (size_t)L.sw, pyr_stride, L.sw, L.dst_off, L.dw, L.dh, L.t, strip,
                         band, img);
        }
        __syncthreads();
    }
}

// FAST-9/16 corner score in closed form.  For pixel value v and circle values p_k (Bresenham r=3,
// OpenCV order), with d_k = v - p_k:  m_dark = max over the 16 arcs of 9 of min d, m_bright = max
// over arcs of min(-d).  OpenCV's cornerScore<16> returns max(t, m_dark, m_bright) - 1 and the pixel
// is a corner at threshold t iff max(m_dark, m_bright) > t; hence s = max(m_dark, m_bright) - 1 is
// threshold independent and "corner at t" <=> s >= t.  Computed for two horizontally
// adjacent pixels at once in packed 16-bit lanes.
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ s16x2 as_s2(uint32_t v) { return __builtin_bit_cast(s16x2, v); }
__device__ __forceinline__ s16x2 pmax(s16x2 a, s16x2 b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ uint32_t align16(uint32_t hi, uint32_t lo) { return __builtin_amdgcn_alignbit(hi, lo, 16); }

// The cell ROI lives in LDS as an f16-biased pair image E of 2 x u16 per dword: E[r][i] = (roi[r][2i], roi[r][2i+1]),
// every u16 lane holding the f16 value 1024 + pixel (bits 0x6400 | pixel), so tap differences are exact f16
// subtractions and the arc minima / maxima use gfx950's 3-input packed f16 min / max.  The pair starting at an odd
// column, (roi[2i+1], roi[2i+2]), is v_alignbit(E[i+1], E[i], 16) of two aligned reads.  Scores below 0 are raised to
// -1 (never a corner, never blocks a neighbour in the NMS -- the same keypoints); the result is i16.
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ h16x2 as_h2(uint32_t v) { return __builtin_bit_cast(h16x2, v); }
__device__ __forceinline__ h16x2 hmin(h16x2 a, h16x2 b) { return __builtin_elementwise_min(a, b); }
__device__ __forceinline__ h16x2 hmax(h16x2 a, h16x2 b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ h16x2 hmin3(h16x2 a, h16x2 b, h16x2 c) {
    uint32_t r;
    asm("v_pk_minimum3_f16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return as_h2(r);
}
__device__ __forceinline__ h16x2 hmax3(h16x2 a, h16x2 b, h16x2 c) {
    uint32_t r;
    asm("v_pk_maximum3_f16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return as_h2(r);
}
// LDS-typed element types (address space 3): indexing through them is 32-bit address arithmetic
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) int16_t lds_i16;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
typedef __attribute__((address_space(3))) s16x2 lds_s16x2;
// Pair-image row r of k_fast_wave starts at dword kS * r + kC * (r / 4).  The padded form (kS = 19, kC = 4) is laid
// out for the compass pre-test's ds_read_b32 loads: a 32-lane half reads 8 rows x 4 quads (QR = 4) at base(row) + 4u
// + o; with kS odd, rows r .. r+3 of a group of four start in distinct residues mod 4, and rows r and r + 4 start
// 4 kS + kC = 80 = 16 (mod 32) dwords apart, so the half's 32 dwords sit in 32 distinct banks.  (A plain stride of 24
// put every row at a multiple of 8 dwords: 8 banks, 4-way conflicts on every pre-test load.)
template <int kS, int kC>
__device__ __forceinline__ int fastw_row(int r) { return __mul24(r, kS) + kC * (r >> 2); }   // v_mad_u32_u24, not a 64-bit mad
__host__ __device__ constexpr int fastw_image_words(int rows, int s, int c) { return s * rows + c * ((rows - 1) >> 2); }

// the 16 circle taps + centre of a pixel pair on the f16-biased pair image (pair words; odd offsets by v_alignbit)
template <int kS, int kC>
__device__ __forceinline__ void fast_taps_f16(const lds_u32* __restrict__ E, int y, int j, uint32_t (&r)[17]) {
    const int r0 = y - 3, m = r0 & 3;
    const lds_u32* eb = E + fastw_row<kS, kC>(r0) + j;
    // row r0 + d starts kS * d + kC * ((m + d) / 4) dwords after row r0
#define ORBX_TAP_W(dy, w) eb[((dy) + 3) * kS + (kC ? kC * ((m + (dy) + 3) >> 2) : 0) + (w)]
#define ORBX_TAP(k, dx, dy) \
    r[k] = ((dx) & 1) ? ORBX_TAP_W(dy, (3 + (dx)) / 2) : align16(ORBX_TAP_W(dy, 2 + (dx) / 2), ORBX_TAP_W(dy, 1 + (dx) / 2))
    ORBX_TAP(16, 0, 0);
    ORBX_TAP(0, 0, 3);    ORBX_TAP(1, 1, 3);    ORBX_TAP(2, 2, 2);    ORBX_TAP(3, 3, 1);
    ORBX_TAP(4, 3, 0);    ORBX_TAP(5, 3, -1);   ORBX_TAP(6, 2, -2);   ORBX_TAP(7, 1, -3);
    ORBX_TAP(8, 0, -3);   ORBX_TAP(9, -1, -3);  ORBX_TAP(10, -2, -2); ORBX_TAP(11, -3, -1);
    ORBX_TAP(12, -3, 0);  ORBX_TAP(13, -3, 1);  ORBX_TAP(14, -2, 2);  ORBX_TAP(15, -1, 3);
#undef ORBX_TAP
#undef ORBX_TAP_W
}
__device__ __forceinline__ s16x2 fast_score_from_taps_f16(const uint32_t (&r)[17]) {
    const h16x2 v = as_h2(r[16]);
    h16x2 d[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) d[k] = v - as_h2(r[k]);
    h16x2 a2[8], b2[8], a4[8], b4[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) { a2[m] = hmin(d[2 * m + 1], d[(2 * m + 2) & 15]); b2[m] = hmax(d[2 * m + 1], d[(2 * m + 2) & 15]); }
#pragma unroll
    for (int m = 0; m < 8; ++m) { a4[m] = hmin(a2[m], a2[(m + 1) & 7]); b4[m] = hmax(b2[m], b2[(m + 1) & 7]); }
    h16x2 dk[8], br[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        const h16x2 e0 = d[2 * m], e9 = d[(2 * m + 9) & 15];
        dk[m] = hmin3(a4[m], a4[(m + 2) & 7], hmax(e0, e9));
        br[m] = hmax3(b4[m], b4[(m + 2) & 7], hmin(e0, e9));
    }
    // (the 2-input steps as 3-input asm too: a builtin max of asm results canonicalises its inputs first)
    const h16x2 dmax = hmax3(hmax3(dk[0], dk[1], dk[2]), hmax3(dk[3], dk[4], dk[5]), hmax3(dk[6], dk[7], dk[7]));
    const h16x2 bmin = hmin3(hmin3(br[0], br[1], br[2]), hmin3(br[3], br[4], br[5]), hmin3(br[6], br[7], br[7]));
    const h16x2 zero = {(_Float16)0, (_Float16)0}, bias = {(_Float16)1024, (_Float16)1024};
    const h16x2 m = hmax3(dmax, -bmin, zero) + bias;                // 1024 + max(m, 0): bits 0x6400 + value
    return as_s2(__builtin_bit_cast(uint32_t, m)) - (s16x2){0x6401, 0x6401};
}

// OpenCV's NMS keeps a corner (s >= t) iff s > every neighbour's buffer value (s_n if s_n >= t, else
// 0).  For s >= max(t, 1) a neighbour with s_n < t never blocks (s_n < t <= s, and 0 < s), so the rule
// is: s >= max(t, 1) and s > max of the 8 raw neighbour scores -- one maximum serves both thresholds.
// For a pixel pair the 8 neighbour pairs come from 3 aligned dwords per row (v_alignbit for the odd
// shifts) and 7 v_pk_max_i16.

__device__ __forceinline__ int nms_pair(const lds_i16* __restrict__ sc, int SW, int rr, int j, int T1, int T2,
                                        bool second) {
    const lds_u32* r0 = (const lds_u32*)(sc + rr * SW + 2 * j);
    const lds_u32* r1 = r0 + (SW >> 1);
    const lds_u32* r2 = r1 + (SW >> 1);
    const uint32_t a0 = r0[0], a1 = r0[1], a2 = r0[2];
    const uint32_t b0 = r1[0], b1 = r1[1], b2 = r1[2];
    const uint32_t c0 = r2[0], c1 = r2[1], c2 = r2[2];
    s16x2 m = pmax(as_s2(align16(a1, a0)), as_s2(a1));
    m = pmax(m, as_s2(align16(a2, a1)));
    m = pmax(m, as_s2(align16(b1, b0)));
    m = pmax(m, as_s2(align16(b2, b1)));
    m = pmax(m, as_s2(align16(c1, c0)));
    m = pmax(m, as_s2(c1));
    m = pmax(m, as_s2(align16(c2, c1)));
    const s16x2 sv = as_s2(b1);
    const int g0 = sv.x > m.x, g1 = second && (sv.y > m.y);
    return (g0 & (sv.x >= T1)) | ((g1 & (sv.y >= T1)) << 1) | ((g0 & (sv.x >= T2)) << 2) | ((g1 & (sv.y >= T2)) << 3);
}

// ---------------------------------------------------------------------------------------------
// k_fast_wave: one WAVE per (image, cell) -- ComputeKeyPointsOctTree's per-cell FAST (:789-829) with no workgroup
// barrier.  OpenCV's FAST runs on the cell ROI, so a cell is self-contained: its ROI (detection window + 3) goes into the
// wave's own LDS slice as the f16-biased pair image, the compass pre-test runs in quads (4 pixel pairs per
// lane), the survivors are compacted in row-major order by wave ballots (no atomics), scored in closed form, and the
// strict 3x3 NMS at iniThFAST and minThFAST appends the kept pixels to two key lists by ballot rank -- so the lists are
// already in OpenCV's row-major output order and a kept pixel's slot is its list index (no rank pass).  The cell's
// count selects the iniTh list, or the minTh list when nothing was kept at iniTh (:812-816).  Phases of one wave are
// ordered by the in-order LDS queue (wavefront fences keep the compiler from reordering across them); the waves of a
// workgroup never wait for each other.
// ---------------------------------------------------------------------------------------------
struct WaveLds {               // per-wave slice of k_fast_wave's dynamic LDS (byte offsets inside the slice)
    int o_sc, o_list, bytes;   // E pair image at 0 (the NMS key lists reuse it), score map, survivor list; slice size
};

// rows: max ROI rows; scrow: score-map row bytes; np: max pixel pairs; iw: pair-image dwords (fastw_image_words)
__host__ __device__ __forceinline__ WaveLds wave_lds(int rows, int scrow, int np, int iw) {
    WaveLds b;
    int o = (iw * 4 + 15) & ~15;
    b.o_sc = o;   o += ((rows - 4) * scrow + 15) & ~15;
    b.o_list = o; o += (np * 2 + 15) & ~15;
    b.bytes = o;
    return b;
}

// Compass pre-test of quad (rr, u) of a cell (pairs 4u .. 4u+3 of detection row rr) at threshold t; also writes the
// quad's score-map words (0, or -1 for the missing second pixel of an odd-width row).  A lane reads the 7 E words of
// row y and the 5 of rows y-3 / y+3 of its 4 pixel pairs (17 dwords, 9 ds_read2_b32 / ds_read_b32 per 4 pairs, not 32);
// the padded row layout (fastw_row) keeps each 32-lane half of those reads on 32 distinct banks.
struct QuadTaps { uint32_t A[7], U[6], D[6]; };   // E words of rows y (7), y-3 and y+3 (5 each) of one quad

template <int kS, int kC>
__device__ __forceinline__ QuadTaps fastw_quad_load(const lds_u32* __restrict__ E, int rr, int u) {
    const lds_u32* e0 = E + fastw_row<kS, kC>(rr) + 4 * u;          // row y-3
    const lds_u32* e1 = E + fastw_row<kS, kC>(rr + 3) + 4 * u;      // row y
    const lds_u32* e2 = E + fastw_row<kS, kC>(rr + 6) + 4 * u;      // row y+3
    QuadTaps q;
#pragma unroll
    for (int k = 0; k < 7; ++k) q.A[k] = e1[k];
    q.U[0] = 0; q.D[0] = 0;
#pragma unroll
    for (int k = 1; k < 6; ++k) { q.U[k] = e0[k]; q.D[k] = e2[k]; }
    return q;
}

// Test of a loaded quad at threshold t: bit 8k + 7 is set iff pair 4u+k lies in the detection window's pairs (4u + k <
// PR) and one of its pixels has a compass value above t.  f16 form of the compass test (the pair image is f16-biased:
// differences are exact): per pair 4 packed differences, dk / br by packed min / max, m = max(dk, -br); the two pixels
// of a pair are merged by one packed max over two pairs' re-paired halves (v_perm), and z = max - (t + 1) has its sign
// bit set iff both pixels have m <= t; one more v_perm gathers the four sign bytes.  The second pixel of an odd-width
// row's last pair (column Wd) is not masked: it can only add that pair to the survivor list, where the score store and
// the NMS take the pair's second pixel only when 2j + 1 < Wd, and a pixel that failed the pre-test scores <= t, below
// every threshold it is kept at, and never blocks a kept neighbour.
__device__ __forceinline__ uint32_t fastw_quad_test(const QuadTaps& q, int u, int t, int PR) {
    const uint32_t *A = q.A, *U = q.U, *D = q.D;
    const h16x2 tq = {(_Float16)(t + 1), (_Float16)(t + 1)};
    uint32_t mk[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const h16x2 v = as_h2(align16(A[k + 2], A[k + 1]));             // pixels of pair 4u+k
        const h16x2 d0 = v - as_h2(align16(D[k + 2], D[k + 1]));        // ( 0,  3)
        const h16x2 d4 = v - as_h2(A[k + 3]);                           // ( 3,  0)
        const h16x2 d8 = v - as_h2(align16(U[k + 2], U[k + 1]));        // ( 0, -3)
        const h16x2 d12 = v - as_h2(A[k]);                              // (-3,  0)
        // on the 4-cycle 0-4-8-12 the largest adjacent minimum equals the smaller of the two opposite maxima (lattice
        // identity: the taps at or below any level must cover every edge, i.e. contain {0, 8} or {4, 12}), so
        // max(min(d0,d4), min(d4,d8), min(d8,d12), min(d12,d0)) = min(max(d0,d8), max(d4,d12)), and dually for br:
        // the same values as the 6-op forms in 3 ops each
        const h16x2 dk = hmin(hmax(d0, d8), hmax(d4, d12));
        const h16x2 br = hmax(hmin(d0, d8), hmin(d4, d12));
        mk[k] = __builtin_bit_cast(uint32_t, hmax(dk, -br));
    }
    // {max over pair 2i, max over pair 2i+1}: the low halves of two pairs against their high halves (asm: as a builtin
    // the compiler canonicalises both v_perm results first, two more packed maxes per call)
    auto pairmax = [](uint32_t a, uint32_t b) {
        uint32_t r;
        asm("v_pk_max_f16 %0, %1, %2" : "=v"(r) : "v"(__builtin_amdgcn_perm(b, a, 0x05040100u)), "v"(__builtin_amdgcn_perm(b, a, 0x07060302u)));
        return as_h2(r);
    };
    const uint32_t z01 = __builtin_bit_cast(uint32_t, pairmax(mk[0], mk[1]) - tq);
    const uint32_t z23 = __builtin_bit_cast(uint32_t, pairmax(mk[2], mk[3]) - tq);
    const uint32_t fail = __builtin_amdgcn_perm(z23, z01, 0x07050301u);   // sign byte of pair k at byte k
    const int sh = min(max(32 * u + 32 - 8 * PR, 0), 24);               // 8 x (4 - pairs of the quad in the window)
    return ~fail & (0x80808080u >> sh);
}

__device__ __forceinline__ void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); }
// Bitonic sort (ascending) of 64 * R 64-bit keys in LDS by ONE wave, in registers: element e = lane * R + r, stages
// with j < R swap registers of a lane, the others exchange with lane ^ (j / R) by a cross-lane shuffle -- no LDS traffic
// or fence inside the network, no block barrier.
template <int R>
__device__ __forceinline__ void wave_bitonic_u64(unsigned long long* a, int ln) {
    unsigned long long v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = a[ln * R + r];
#pragma unroll
    for (int k = 2; k <= 64 * R; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j >= R) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int e = ln * R + r;
                    const unsigned long long o = __shfl_xor(v[r], j / R, kWave);
                    const bool keep_min = ((e & k) == 0) == ((e & j) == 0);
                    v[r] = keep_min ? (v[r] < o ? v[r] : o) : (v[r] < o ? o : v[r]);
                }
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if (r & j) continue;
                    const int e = ln * R + r;
                    const unsigned long long x = v[r], y = v[r | j];
                    if ((x > y) == ((e & k) == 0)) { v[r] = y; v[r | j] = x; }
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) a[ln * R + r] = v[r];
}

// exclusive prefix sums of a[0, n) in place by one wave (lane ln); returns the total
__device__ __forceinline__ int wave_excl_scan_lds(int* a, int n, int ln) {
    int carry = 0;
    for (int b = 0; b < n; b += kWave) {
        const int i = b + ln;
        const int x = i < n ? a[i] : 0;
        const int inc = wave_incl_scan(x);
        if (i < n) a[i] = carry + inc - x;
        carry += __builtin_amdgcn_readlane(inc, kWave - 1);
    }
    return carry;
}
// acc + number of set bits of b below this lane: v_mbcnt_lo + v_mbcnt_hi (the compiler turns popcount(b & below) into
// two ANDs and two v_bcnt)
__device__ __forceinline__ int rank_below(uint64_t b, int acc = 0) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, (uint32_t)acc));
}

// score-map row stride (int16) per pair stride: >= (Wd + 5) & ~1 for every cell the pair stride admits.  The padded
// layout's 36 (18 dwords) is that minimum for its 38-column ROIs; the bank model put 20 dwords at 1.6 extra cycles per
// NMS access against 1.8 for 22 (scripts/micro/lds_banks.py), but the smaller map is what lets more waves in.
#ifndef ORBX_FAST_SW19
#define ORBX_FAST_SW19 36   // r5b: 36 (18 dwords, the minimum for 32-column detection windows) -> 5 / 6 FAST workgroups per
                            // CU at levels >= 1 / level 0 instead of 4 / 5: serial FAST 1.153 -> 1.060 ms, step +0.9 %
#endif
__host__ __device__ constexpr int fastw_sw(int ps) { return ps == 19 ? ORBX_FAST_SW19 : 76; }
__host__ __device__ constexpr int fastw_scrow(int ps) { return 2 * fastw_sw(ps); }

__device__ __forceinline__ void sc_store(lds_u8* __restrict__ scb, int SWB, int rr, int j, s16x2 v, bool second) {
    *(lds_s16x2*)(scb + (rr + 1) * SWB + 4 + 4 * j) = second ? v : (s16x2){v.x, (short)-1};
}

// ORBX_FAST_ATTR (diagnostics builds only, `make variant`; wrong keypoints): bit 0 reads the score taps, bit 1 the NMS
// neighbourhoods at one row and columns ln & 15 of the cell instead of the survivor's -- the same LDS instructions on
// addresses a 32-lane half reads without bank conflicts -- so a PMC pass attributes SQ_LDS_BANK_CONFLICT to them.
#ifndef ORBX_FAST_ATTR
#define ORBX_FAST_ATTR 0
#endif
// The part of a cell after its ROI is in LDS: pre-test, scores, NMS at both thresholds, the cell's candidate slots.
template <int kPS, int kPC>
__device__ __forceinline__ void fastw_body(lds_u32* __restrict__ E, lds_u8* __restrict__ scb, lds_u16* __restrict__ list,
                                           const CellDev& cd, int img, int* __restrict__ cnt_out, int Wd, int Hd, int T1,
                                           int T2, int tp, uint32_t* __restrict__ cand_xy, uint8_t* __restrict__ cand_s,
                                           int cand_stride, int kcap, int two_pass, int ln) {
    constexpr int SWB = fastw_scrow(kPS);                             // score-map row bytes
    wave_fence();
    // 2. compass pre-test at min(iniTh, minTh) in quads; survivors compacted in row-major order
    const int PR = (Wd + 1) >> 1, QR = (PR + 3) >> 2, NQ4 = Hd * QR;
    // With minThFAST < iniThFAST the cell runs at iniThFAST first (fewer survivors to score); only a cell that kept
    // nothing there -- a wave-uniform branch, no barrier -- runs again at minThFAST over all its pairs (:812-816).  The
    // second pass finds every minTh survivor (a superset of the first pass's, whose scores it rewrites with the same
    // values) and starts its list afresh.  Otherwise one pass at min(iniTh, minTh) keeps both thresholds' pixels.
    const bool two = two_pass && T2 < T1;
    lds_u16* k1 = (lds_u16*)E;                  // key lists over the pair image (dead after scoring)
    lds_u16* k2 = k1 + kcap;
    int n1 = 0, n2 = 0;                                               // wave-uniform
    for (int pass = 0; pass < 2; ++pass) {
    const int tpre = two ? (pass == 0 ? T1 : T2) : tp;
    const int fmask = two ? (pass == 0 ? 3 : 12) : 15;
    int ns = 0;                                                       // wave-uniform
    {
        // 2. compass pre-test in quads: quad q -> (row q / QR, column q % QR), walked incrementally; two quads per lane
        // per round (q, q + 64), both read before either is tested.  Survivors are appended in quad order (row-major).
        const int dr = kWave / QR, du = kWave - dr * QR;
        int rr = ln / QR, u = ln - rr * QR;
        auto step = [&](int& r0, int& u0) { r0 += dr; u0 += du; if (u0 >= QR) { u0 -= QR; ++r0; } };
        auto emit = [&](uint32_t mq, int r0, int u0) {                 // mq: bit 8k + 7 = pair 4 u0 + k survives
            const int cq = __builtin_popcount(mq);
            const uint64_t b0 = __ballot(cq & 1), b1 = __ballot(cq & 2), b2 = __ballot(cq & 4);
            int pos = rank_below(b0, ns) + 2 * rank_below(b1) + 4 * rank_below(b2);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if ((mq >> (8 * k + 7)) & 1u) list[pos++] = (uint16_t)((r0 << 8) | (4 * u0 + k));
            ns += __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
        };
        for (int q0 = 0; q0 < NQ4; q0 += 2 * kWave) {
            const int qa = q0 + ln, qb = qa + kWave;
            const int ra = rr, ua = u;
            step(rr, u);
            const int rb = rr, ub = u;
            step(rr, u);
            const bool va = qa < NQ4, vb = qb < NQ4;
            const QuadTaps ta = fastw_quad_load<kPS, kPC>(E, va ? ra : 0, va ? ua : 0);
            const QuadTaps tb = fastw_quad_load<kPS, kPC>(E, vb ? rb : 0, vb ? ub : 0);
            const uint32_t ma = va ? fastw_quad_test(ta, ua, tpre, PR) : 0u;
            const uint32_t mb = vb ? fastw_quad_test(tb, ub, tpre, PR) : 0u;
            emit(ma, ra, ua);
            emit(mb, rb, ub);
        }
    }
    wave_fence();
    // 3. closed-form scores of the survivors, two per lane per round (both tap sets read before either is scored); a
    //    round with at most 64 survivors left (two cells in three at iniThFAST) scores one per lane
    for (int i0 = 0; i0 < ns; i0 += 2 * kWave) {
        const int i = i0 + ln;
        if (i0 + kWave < ns) {                                        // wave-uniform
            const int i2 = i + kWave;
            if (i < ns) {
                const uint32_t e1 = list[i], e2 = i2 < ns ? list[i2] : e1;
                const int rr1 = e1 >> 8, j1 = e1 & 0xff, rr2 = e2 >> 8, j2 = e2 & 0xff;
                uint32_t t1[17], t2[17];
                if constexpr (ORBX_FAST_ATTR & 1) {
                    fast_taps_f16<kPS, kPC>(E, 3, ln & 15, t1);
                    fast_taps_f16<kPS, kPC>(E, 3, (ln & 15) ^ 1, t2);
                } else {
                    fast_taps_f16<kPS, kPC>(E, rr1 + 3, j1, t1);
                    fast_taps_f16<kPS, kPC>(E, rr2 + 3, j2, t2);
                }
                const s16x2 s1 = fast_score_from_taps_f16(t1), s2 = fast_score_from_taps_f16(t2);
                sc_store(scb, SWB, rr1, j1, s1, 2 * j1 + 1 < Wd);
                if (i2 < ns) sc_store(scb, SWB, rr2, j2, s2, 2 * j2 + 1 < Wd);
            }
        } else if (i < ns) {
            const uint32_t e1 = list[i];
            const int rr1 = e1 >> 8, j1 = e1 & 0xff;
            uint32_t t1[17];
            if constexpr (ORBX_FAST_ATTR & 1) fast_taps_f16<kPS, kPC>(E, 3, ln & 15, t1);
            else fast_taps_f16<kPS, kPC>(E, rr1 + 3, j1, t1);
            const s16x2 s1 = fast_score_from_taps_f16(t1);
            sc_store(scb, SWB, rr1, j1, s1, 2 * j1 + 1 < Wd);
        }
    }
    wave_fence();
    // 4. strict 3x3 NMS at iniTh (bits 0, 1) and minTh (bits 2, 3); kept pixels appended in list order (= row-major)
    //    to the two key lists, which take over the pair image's LDS (key = row * 128 + column in the detection window)
    for (int i0 = 0; i0 < ns; i0 += kWave) {
        const int i = i0 + ln;
        int f = 0, key = 0;
        if (i < ns) {
            const int rr = list[i] >> 8, j = list[i] & 0xff;
            if constexpr (ORBX_FAST_ATTR & 2) f = nms_pair((const lds_i16*)scb, SWB / 2, 0, ln & 15, T1, T2, 2 * j + 1 < Wd) & fmask;
            else f = nms_pair((const lds_i16*)scb, SWB / 2, rr, j, T1, T2, 2 * j + 1 < Wd) & fmask;
            key = rr * 128 + 2 * j;
        }
        const uint64_t a0 = __ballot(f & 1), a1 = __ballot(f & 2), c0 = __ballot(f & 4), c1 = __ballot(f & 8);
        int p1 = rank_below(a1, rank_below(a0, n1));
        int p2 = rank_below(c1, rank_below(c0, n2));
        if (f & 1) { if (p1 < kcap) k1[p1] = (uint16_t)key; ++p1; }
        if ((f & 2) && p1 < kcap) k1[p1] = (uint16_t)(key + 1);
        if (f & 4) { if (p2 < kcap) k2[p2] = (uint16_t)key; ++p2; }
        if ((f & 8) && p2 < kcap) k2[p2] = (uint16_t)(key + 1);
        n1 += __popcll(a0) + __popcll(a1);
        n2 += __popcll(c0) + __popcll(c1);
    }
    wave_fence();
    if (!two || n1 > 0) break;                                        // wave-uniform
    }
    // 5. the cell's list (iniTh, or minTh when iniTh kept nothing: :812-816) -> its candidate slots, coalesced
    const lds_u16* ks = n1 > 0 ? k1 : k2;
    const int n = min(n1 > 0 ? n1 : n2, min(kcap, cd.slot_cap));
    uint32_t* oxy = cand_xy + (size_t)img * cand_stride + cd.slot_off;
    uint8_t* os = cand_s + (size_t)img * cand_stride + cd.slot_off;
    for (int i = ln; i < n; i += kWave) {
        const int k = ks[i], rr = k >> 7, x = k & 127;
        oxy[i] = (uint32_t)(cd.x0 + 3 + x) | ((uint32_t)(cd.y0 + rr + 3) << 16);
        os[i] = (uint8_t)((const lds_i16*)scb)[(rr + 1) * (SWB / 2) + 2 + x];
    }
    if (ln == 0) *cnt_out = n;
}

template <int kPS, int kPC, int kWpg>
__global__ __launch_bounds__(64 * kWpg) void k_fast_wave(const uint8_t* __restrict__ pyr, size_t pyr_stride,
                                                         const LevelDev* __restrict__ levels, const CellDev* __restrict__ cells,
                                                         int cell0, int ncell, int iniTh, int minTh,
                                                         uint32_t* __restrict__ cand_xy, uint8_t* __restrict__ cand_s,
                                                         int cand_stride, int* __restrict__ cell_cnt, int ncells, int batch,
                                                         Src0 s0, WaveLds lay, int kcap, int two_pass) {
    extern __shared__ __attribute__((aligned(16))) uint32_t fsm[];
    const int w = threadIdx.x >> 6, ln = lane_id();
    const int total = ncell * batch, nwg = (total + kWpg - 1) / kWpg;
    const int wg = xcd_item(xcd_chunk(nwg));                        // cells of one image on one XCD
    const int item = __builtin_amdgcn_readfirstlane(wg * kWpg + w);
    if (wg >= nwg || item >= total) return;                         // whole wave (no barrier in this kernel)
    const int img = item / ncell, c = cell0 + (item - img * ncell);
    // typed LDS pointers: every address below is 32-bit arithmetic (through generic pointers the compiler formed them
    // with 64-bit multiply-adds)
    lds_u8* lds = (lds_u8*)fsm + w * lay.bytes;
    lds_u32* E = (lds_u32*)lds;
    lds_u8* scb = lds + lay.o_sc;
    lds_u16* list = (lds_u16*)(lds + lay.o_list);
    const CellDev cd = cells[c];
    const int W = cd.W, H = cd.H, Wd = W - 6, Hd = H - 6;
    int* cnt_out = cell_cnt + (size_t)img * ncells + c;
    if (Wd <= 0 || Hd <= 0) {
        if (ln == 0) *cnt_out = 0;
        return;
    }
    const int T1 = max(min(max(iniTh, 0), 255), 1), T2 = max(min(max(minTh, 0), 255), 1);
    const int tp = min(T1, T2);
    constexpr int SWB = fastw_scrow(kPS);
    // a pair word is (1024 + p1, 1024 + p0) as f16: bytes (p0, 0x64, p1, 0x64), one v_perm_b32 from a source dword and
    // this constant (selectors 4-7 pick its bytes) instead of a perm and an OR
    constexpr uint32_t kBias8 = 0x64646464u;
    {
        // 1. cell ROI -> f16-biased pair image: lane items (row, 8-column chunk), one 8-byte load each, all of a round
        //    issued before the first use.  Columns past the ROI's width (the last chunk's tail, real level pixels) are
        //    staged as they are: no pre-test, score or NMS of a detection-window pixel reads past column W - 1 (its taps
        //    reach 3 + 3 columns right of the window's last column Wd - 1 + 3); only the outside second pixel of an
        //    odd-width row's last pair reads column W, and its result is never kept (fastw_quad_test).
        const LevelDev& L = levels[cd.level];
        int lstride;
        const uint8_t* base = level_pixels(pyr, pyr_stride, L, cd.level, img, s0, lstride);
        const uint8_t* src0 = base + (size_t)cd.y0 * lstride + cd.x0;
        if constexpr (kPC == 0) {
            // 16-byte chunks (8 pair words each), rows 16-byte aligned: one round of <= 2 loads per lane for a 38 x 38
            // ROI.  The bytes past the ROI's width (< 16, inside the level row: the ROI ends >= 16 px before the level's
            // edge) only reach pixels outside the detection window, which are masked.
            const int cpr = (W + 15) >> 4, NQ = H * cpr;
            const int dr = kWave / cpr, dc = kWave - dr * cpr;      // item q -> q + 64 (no division per item)
            int r = ln / cpr, cc = ln - r * cpr;
            constexpr int kPf = 2;
            for (int q0 = 0; q0 < NQ; q0 += kPf * kWave) {
                uint4 pf[kPf];
                int rs[kPf], cs[kPf];
#pragma unroll
                for (int k = 0; k < kPf; ++k) {
                    rs[k] = r; cs[k] = cc;
                    r += dr; cc += dc;
                    if (cc >= cpr) { cc -= cpr; ++r; }
                    // every lane loads (an item past the ROI re-reads its last row and stores nothing), so a round's loads
                    // issue back to back from the wave-uniform ROI base plus a 32-bit offset
                    __builtin_memcpy(&pf[k], src0 + (uint32_t)(__mul24(min(rs[k], H - 1), lstride) + 16 * cs[k]), 16);
                }
                asm volatile("" : "+v"(pf[0].x), "+v"(pf[0].y), "+v"(pf[0].z), "+v"(pf[0].w));   // (as in the padded form)
#pragma unroll
                for (int k = 0; k < kPf; ++k) {
                    if (q0 + ln + k * kWave < NQ) {
                        const uint4 a = pf[k];
                        const u32x4 e0 = {__builtin_amdgcn_perm(kBias8, a.x, 0x04010400u), __builtin_amdgcn_perm(kBias8, a.x, 0x04030402u),
                                          __builtin_amdgcn_perm(kBias8, a.y, 0x04010400u), __builtin_amdgcn_perm(kBias8, a.y, 0x04030402u)};
                        const u32x4 e1 = {__builtin_amdgcn_perm(kBias8, a.z, 0x04010400u), __builtin_amdgcn_perm(kBias8, a.z, 0x04030402u),
                                          __builtin_amdgcn_perm(kBias8, a.w, 0x04010400u), __builtin_amdgcn_perm(kBias8, a.w, 0x04030402u)};
                        lds_u32x4* dst = (lds_u32x4*)(E + fastw_row<kPS, kPC>(rs[k]) + 8 * cs[k]);
                        dst[0] = e0;
                        dst[1] = e1;
                    }
                }
            }
        } else {
            // padded rows (4-byte aligned, exactly kPS = 19 words for the widest ROI, 38 columns): 8-byte chunks, four
            // ds_write_b32 per chunk without a per-word test.  Only word 3 of a row's last chunk can fall past the row:
            // on the next row's word 0 (or the pad after every fourth row, or after the last row on the score map, which
            // is cleared after the staging).  It is stored first, behind a compiler barrier, so that the next row's own
            // word 0 -- item q + 1, in the same round or a later one, never an earlier -- is written after it (one
            // wave's LDS stores complete in issue order).
            const int cpr = (W + 7) >> 3, NQ = H * cpr;
            const int dr = kWave / cpr, dc = kWave - dr * cpr;          // item q -> q + 64 (no division per item)
            int r = ln / cpr, cc = ln - r * cpr;
            constexpr int kPf = 4;                                      // 256 items: a 40 x 48 ROI in one round
            for (int q0 = 0; q0 < NQ; q0 += kPf * kWave) {
                uint32_t pf[2 * kPf];
                int rs[kPf], cs[kPf];
#pragma unroll
                for (int k = 0; k < kPf; ++k) {
                    rs[k] = r; cs[k] = cc;
                    r += dr; cc += dc;
                    if (cc >= cpr) { cc -= cpr; ++r; }
                    // every lane loads (an item past the ROI re-reads its last row and stores nothing), so a round's loads
                    // issue back to back from the wave-uniform ROI base plus a 32-bit offset
                    __builtin_memcpy(&pf[2 * k], src0 + (uint32_t)(__mul24(min(rs[k], H - 1), lstride) + 8 * cs[k]), 8);
                }
                // the first item's bytes pass through an empty asm on every path: otherwise the compiler sinks its load
                // into its store branch, issued after the others, and the first store waits for all four
                asm volatile("" : "+v"(pf[0]), "+v"(pf[1]));
#pragma unroll
                for (int k = 0; k < kPf; ++k) {
                    if (q0 + ln + k * kWave < NQ) {
                        const uint32_t lo = pf[2 * k], hi = pf[2 * k + 1];
                        lds_u32* dst = E + fastw_row<kPS, kPC>(rs[k]) + 4 * cs[k];
                        dst[3] = __builtin_amdgcn_perm(kBias8, hi, 0x04030402u);
                        asm volatile("" ::: "memory");
                        dst[2] = __builtin_amdgcn_perm(kBias8, hi, 0x04010400u);
                        dst[1] = __builtin_amdgcn_perm(kBias8, lo, 0x04030402u);
                        dst[0] = __builtin_amdgcn_perm(kBias8, lo, 0x04010400u);
                        asm volatile("" ::: "memory");
                    }
                }
        }
        }
        // score map cleared to 0: pixels that fail the pre-test and the pad ring (a 0 never blocks a kept score >= 1)
        const int n16 = ((Hd + 2) * SWB + 15) >> 4;
        for (int i = ln; i < n16; i += kWave) ((lds_u32x4*)scb)[i] = (u32x4){0u, 0u, 0u, 0u};
    }
    fastw_body<kPS, kPC>(E, scb, list, cd, img, cnt_out, Wd, Hd, T1, T2, tp, cand_xy, cand_s, cand_stride, kcap, two_pass, ln);
}

// GaussianBlur 7x7 sigma 2, BORDER_REFLECT_101, integer separable path: taps {18,34,49,55,49,34,18},
// column pass (acc + 2^15) >> 16 saturated.  Tiles (level, strip, band) of all levels in one grid.
struct BlurTile { int level, tx, ty, pad; };

__device__ __forceinline__ int refl101(int i, int n) {
    if (n == 1) return 0;
    while (i < 0 || i >= n) i = (i < 0) ? -i : 2 * n - 2 - i;
    return i;
}

// Register-streaming form: one wave per (level, 256-column strip, ORBX_BLUR_BAND-row band, 32 rows).  Lane l owns
// the 4 output columns x0 = strip*256 + 4l .. x0+3, walks down the band's 38 input rows once, and keeps the
// last 4 row pairs of horizontal sums in registers (a ring unrolled by 4, so no moves); no LDS, no
// divisions.  Reflection only at the level borders (scalar for rows, byte selectors for edge lanes).
// Per input row a lane issues one 12-byte load (x0-4 .. x0+7; global loads need no alignment on gfx950);
// a horizontal row sum is at most 255 * 257 = 65535, exact in u16.  The 4 output bytes leave as one dword store.
#ifndef ORBX_BLUR_BAND
#define ORBX_BLUR_BAND 32     // rows per wave (r4ax/r4ay with scalar tiles at 6 waves per SIMD: step 3.53-3.56 ms at 16, 3.49-3.50 at 24, 3.48 at 32, 3.49 at 48)
#endif
constexpr int kBlurBand = ORBX_BLUR_BAND, kBlurStrip = 256;

struct BlurWin { uint32_t w0, w1, w2; };   // 12 input bytes x0-4 .. x0+7 of one row

// Row window loads.  kMode 0: interior lane, one 12-byte load.  kMode 2: a level under 12 columns, per-byte loads
// with REFLECT_101 columns.  (A lane within 8 columns of the edge of a wider level uses blur_load_sel below.)
template <int kMode>
__device__ __forceinline__ BlurWin blur_load(const uint8_t* __restrict__ row, int x0, int w) {
    BlurWin o;
    if (kMode == 0) {
        uint32_t v[3];
        __builtin_memcpy(v, row + x0 - 4, 12);
        o.w0 = v[0]; o.w1 = v[1]; o.w2 = v[2];
    } else {
        uint32_t v[3] = {0, 0, 0};
#pragma unroll
        for (int i = 1; i < 11; ++i) v[i >> 2] |= (uint32_t)row[refl101(x0 - 4 + i, w)] << (8 * (i & 3));
        o.w0 = v[0]; o.w1 = v[1]; o.w2 = v[2];
    }
    return o;
}

// Vertical-pair form: two input rows at a time.  V_m = (row a byte m, row b byte m) as u16x2 (one
// v_perm each), so the horizontal sums of 4 columns come out vertically packed -- H_c = (row a sum, row b sum) -- and
// the column pass of an output pixel is 4 v_dot2_u32_u16 over 4 such pairs (weights (18,34), (49,55), (49,34), (18,0)
// for an output row aligned with a pair start, (0,18), (34,49), (55,49), (34,18) for the next row) with the rounding
// constant 2^15 as the first accumulator: no unpacking of u16 halves.  Same integers as the separable
// integer path (horizontal sums, then (column sum + 2^15) >> 16 saturated).
struct BlurPair { u16x2 h[4]; };   // columns x0 .. x0+3: (row a, row b) horizontal sums

template <int m>
__device__ __forceinline__ u16x2 vpair(const BlurWin& a, const BlurWin& b) {
    constexpr int q = m / 4, r = m % 4;
    const uint32_t lo = q == 0 ? a.w0 : (q == 1 ? a.w1 : a.w2);
    const uint32_t hi = q == 0 ? b.w0 : (q == 1 ? b.w1 : b.w2);
    constexpr uint32_t sel = 0x0c000c00u | (uint32_t)r | ((uint32_t)(r + 4) << 16);
    return __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(hi, lo, sel));
}

__device__ __forceinline__ BlurPair blur_hpair(const BlurWin& a, const BlurWin& b) {
    // window byte m = pixel x0 - 4 + m; output column x0 + c uses bytes c+1 .. c+7
    const u16x2 V1 = vpair<1>(a, b), V2 = vpair<2>(a, b), V3 = vpair<3>(a, b), V4 = vpair<4>(a, b), V5 = vpair<5>(a, b);
    const u16x2 V6 = vpair<6>(a, b), V7 = vpair<7>(a, b), V8 = vpair<8>(a, b), V9 = vpair<9>(a, b), V10 = vpair<10>(a, b);
    const u16x2 k18 = {18, 18}, k34 = {34, 34}, k49 = {49, 49}, k55 = {55, 55};
    BlurPair o;
    o.h[0] = (V1 + V7) * k18 + (V2 + V6) * k34 + (V3 + V5) * k49 + V4 * k55;
    o.h[1] = (V2 + V8) * k18 + (V3 + V7) * k34 + (V4 + V6) * k49 + V5 * k55;
    o.h[2] = (V3 + V9) * k18 + (V4 + V8) * k34 + (V5 + V7) * k49 + V6 * k55;
    o.h[3] = (V4 + V10) * k18 + (V5 + V9) * k34 + (V6 + V8) * k49 + V7 * k55;
    return o;
}

// output rows y (pairs a..d = rows y-3 .. y+4) and y+1, 4 columns each, packed bytes
__device__ __forceinline__ void blur_emit2(const BlurPair& a, const BlurPair& b, const BlurPair& c, const BlurPair& d,
                                           uint32_t& oe, uint32_t& oo) {
    const u16x2 e0 = {18, 34}, e1 = {49, 55}, e2 = {49, 34}, e3 = {18, 0};
    const u16x2 o0 = {0, 18}, o1 = {34, 49}, o2 = {55, 49}, o3 = {34, 18};
    // acc < 2^25, so (acc + 2^15) >> 16 is the u16 in bytes 2-3 of acc: one v_perm_b32 gathers it for two columns as
    // u16x2, one v_pk_min_u16 saturates both, one more v_perm_b32 packs four columns (5 VALU per 4 pixels instead of a
    // shift, a min and an OR per pixel)
    uint32_t ae[4], ao[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        ae[k] = __builtin_amdgcn_udot2(d.h[k], e3, 1u << 15, false);
        ae[k] = __builtin_amdgcn_udot2(c.h[k], e2, ae[k], false);
        ae[k] = __builtin_amdgcn_udot2(b.h[k], e1, ae[k], false);
        ae[k] = __builtin_amdgcn_udot2(a.h[k], e0, ae[k], false);
        ao[k] = __builtin_amdgcn_udot2(d.h[k], o3, 1u << 15, false);
        ao[k] = __builtin_amdgcn_udot2(c.h[k], o2, ao[k], false);
        ao[k] = __builtin_amdgcn_udot2(b.h[k], o1, ao[k], false);
        ao[k] = __builtin_amdgcn_udot2(a.h[k], o0, ao[k], false);
    }
    const u16x2 k255 = {255, 255};
    auto pack4 = [&](const uint32_t* v) {
        const u16x2 lo = __builtin_elementwise_min(__builtin_bit_cast(u16x2, __builtin_amdgcn_perm(v[1], v[0], 0x07060302u)), k255);
        const u16x2 hi = __builtin_elementwise_min(__builtin_bit_cast(u16x2, __builtin_amdgcn_perm(v[3], v[2], 0x07060302u)), k255);
        return __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, hi), __builtin_bit_cast(uint32_t, lo), 0x06040200u);
    };
    oe = pack4(ae);
    oo = pack4(ao);
}

// Edge-strip window of blur_load<1> as byte selectors: which byte of the clamped 12-byte load each window byte
// 1..10 takes depends on the lane's column only, so the REFLECT_101 picks are computed once per band and every row
// then costs two v_perm_b32 and one OR per window dword (the per-byte loop of blur_load<1> was ~80 VALU per row).
struct ReflSel { uint32_t a[3], b[3]; int xs; };
__device__ __forceinline__ ReflSel refl_sel(int x0, int w) {
    ReflSel s;
    s.xs = min(max(x0 - 4, 0), w - 12);
#pragma unroll
    for (int j = 0; j < 3; ++j) { s.a[j] = 0x0c0c0c0cu; s.b[j] = 0x0c0c0c0cu; }   // 0x0c selects a zero byte
#pragma unroll
    for (int i = 1; i < 11; ++i) {
        const int x = x0 - 4 + i;
        const int k = (x < 0 ? -x : (x >= w ? 2 * w - 2 - x : x)) - s.xs;          // 0 <= k < 12
        const int sh = 8 * (i & 3);
        const uint32_t clr = ~(0xffu << sh);
        if (k < 8) s.a[i >> 2] = (s.a[i >> 2] & clr) | ((uint32_t)k << sh);        // byte k of {v1:v0}
        else s.b[i >> 2] = (s.b[i >> 2] & clr) | ((uint32_t)(k - 8) << sh);       // byte k-8 of v2
    }
    return s;
}
__device__ __forceinline__ BlurWin blur_load_sel(const uint8_t* __restrict__ row, const ReflSel& s) {
    uint32_t v[3];
    __builtin_memcpy(v, row + s.xs, 12);
    BlurWin o;
    o.w0 = __builtin_amdgcn_perm(v[1], v[0], s.a[0]) | __builtin_amdgcn_perm(v[2], v[2], s.b[0]);
    o.w1 = __builtin_amdgcn_perm(v[1], v[0], s.a[1]) | __builtin_amdgcn_perm(v[2], v[2], s.b[1]);
    o.w2 = __builtin_amdgcn_perm(v[1], v[0], s.a[2]) | __builtin_amdgcn_perm(v[2], v[2], s.b[2]);
    return o;
}

template <int kMode>
__device__ __forceinline__ void blur_band2(const uint8_t* __restrict__ S, int sstride, uint8_t* __restrict__ D,
                                           const LevelDev& L, int x0, int y0, int y1) {
    const int h = L.h, w = L.w;
    auto row_ptr = [&](int yy) {
        const int r = h >= 16 ? (yy < 0 ? -yy : (yy >= h ? 2 * h - 2 - yy : yy)) : refl101(yy, h);
        return S + (size_t)r * sstride;
    };
    ReflSel rs;
    if constexpr (kMode == 1) rs = refl_sel(x0, w);
    auto load = [&](const uint8_t* row) { return kMode == 1 ? blur_load_sel(row, rs) : blur_load<kMode>(row, x0, w); };
    const bool full = x0 + 4 <= w;
    auto store = [&](int y, uint32_t packed) {
        uint8_t* o = D + (size_t)y * w + x0;
        if (kMode == 0 || full) {
            __builtin_memcpy(o, &packed, 4);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (x0 + j < w) o[j] = (uint8_t)(packed >> (8 * j));
        }
    };
    BlurPair q0, q1, q2, q3;
    {
        BlurWin p[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) p[k] = load(row_ptr(y0 - 3 + k));
        q0 = blur_hpair(p[0], p[1]); q1 = blur_hpair(p[2], p[3]); q2 = blur_hpair(p[4], p[5]);
    }
    // ring of 4 row pairs; 8 output rows per iteration.  Interior and edge strips load the iteration's 8 input rows at
    // once; tiny levels (per-byte loads, more registers) 4 at a time (8 spilled at 128 VGPRs)
    for (int y = y0; y < y1; y += 8) {
        constexpr int kB = kMode <= 1 ? 8 : 4;
        BlurWin p[kB];
        uint32_t oe, oo;
#pragma unroll
        for (int k = 0; k < kB; ++k) p[k] = load(row_ptr(y + 3 + k));
        q3 = blur_hpair(p[0], p[1]); blur_emit2(q0, q1, q2, q3, oe, oo);
        store(y, oe); if (y + 1 >= y1) break; store(y + 1, oo); if (y + 2 >= y1) break;
        q0 = blur_hpair(p[2], p[3]); blur_emit2(q1, q2, q3, q0, oe, oo);
        store(y + 2, oe); if (y + 3 >= y1) break; store(y + 3, oo); if (y + 4 >= y1) break;
        if constexpr (kB == 4) {
#pragma unroll
            for (int k = 0; k < 4; ++k) p[k] = load(row_ptr(y + 7 + k));
        }
        q1 = blur_hpair(p[kB - 4], p[kB - 3]); blur_emit2(q2, q3, q0, q1, oe, oo);
        store(y + 4, oe); if (y + 5 >= y1) break; store(y + 5, oo); if (y + 6 >= y1) break;
        q2 = blur_hpair(p[kB - 2], p[kB - 1]); blur_emit2(q3, q0, q1, q2, oe, oo);
        store(y + 6, oe); if (y + 7 >= y1) break; store(y + 7, oo);
    }
}

#ifndef ORBX_BLUR_WPE
#define ORBX_BLUR_WPE 5     // 82 VGPRs, no spills: 5 waves per SIMD.  r5ae: serial blur 0.550 -> 0.561 ms, but the step
                            // +1.6 % (72.6k -> 73.8k frames/s, 4 ties 5, two rounds): fewer blur waves beside FAST and the
                            // describe.  (6 per SIMD at 80 VGPRs was r4ak's choice by the serial time: 0.588 -> 0.571 ms.)
#endif
// one wave's blur tile (level, 256-column strip, ORBX_BLUR_BAND-row band) of image img
__device__ __forceinline__ void blur_tile(const uint8_t* __restrict__ pyr, uint8_t* __restrict__ blur, size_t pyr_stride,
                                          const LevelDev* __restrict__ levels, const BlurTile& bt, int img, const Src0& s0) {
    const LevelDev L = levels[bt.level];
    int sstride;
    const uint8_t* S = level_pixels(pyr, pyr_stride, L, bt.level, img, s0, sstride);
    uint8_t* D = blur + img * pyr_stride + L.pyr_off;
    const int y0 = bt.ty * kBlurBand, y1 = min(y0 + kBlurBand, L.h);
    const int x0 = bt.tx * kBlurStrip + 4 * lane_id();
    if (x0 >= L.w) return;
    const bool interior = (x0 - 4 >= 0) && (x0 + 8 <= L.w);
    // wave-uniform choice of the load form (strips touching a level's left/right edge pick reflected bytes)
    if (__builtin_amdgcn_read_exec() == __ballot(interior))
        blur_band2<0>(S, sstride, D, L, x0, y0, y1);
    else if (L.w >= 12)
        blur_band2<1>(S, sstride, D, L, x0, y0, y1);
    else
        blur_band2<2>(S, sstride, D, L, x0, y0, y1);
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ORBX_BLUR_WPE))) void k_blur7(
    const uint8_t* __restrict__ pyr, uint8_t* __restrict__ blur, size_t pyr_stride, const LevelDev* __restrict__ levels,
    const BlurTile* __restrict__ tiles, int ntiles, int batch, Src0 s0, int tile0) {
    // tiles [tile0, tile0 + ntiles) of every image (a level range: tiles are level-major)
    const int nbx = (ntiles + 3) / 4;                         // 4 tiles (waves) per workgroup
    const int item = xcd_item(xcd_chunk(nbx * batch));       // bands of one image on one XCD
    if (item >= nbx * batch) return;
    const int img = item / nbx;
    // the tile index is wave-uniform: as an SGPR the tile and its level load by scalar loads and every row address
    // and reflection is scalar work
    const int tl = __builtin_amdgcn_readfirstlane((item - img * nbx) * (blockDim.x >> 6) + (threadIdx.x >> 6));
    if (tl >= ntiles) return;
    blur_tile(pyr, blur, pyr_stride, levels, tiles[tile0 + tl], img, s0);
}

// ---------------------------------------------------------------------------------------------
// Quadtree: DistributeOctTree (:539-763) as data-parallel passes.
//
// The reference keeps a std::list of nodes.  One phase-1 pass splits every node holding >1 key and
// pushes the non-empty children (n1,n2,n3,n4) to the list FRONT, so after a pass the list reads:
// [children of the last split node (n4..n1), ..., children of the first split node, unsplit nodes in
// their previous order].  A phase-2 pass sorts the expandable nodes by (size, creation order),
// splits from the largest down and stops as soon as the list holds >= N nodes.  Both are positional
// permutations computable with prefix sums: node arrays live in LDS (double-buffered, list order),
// each key carries the list position of its node (key_node), child counts come from LDS atomics.
// ---------------------------------------------------------------------------------------------
// bits of the extractor's device error word (orbx_extractor_status)
constexpr int kErrQtCap = 1, kErrStale = 4;

struct QtScratch {
    uint32_t* key_xy;    // window-relative (x | y << 16), reference order
    uint8_t* key_r;      // FAST response
    int16_t* key_node;   // list position of the key's node
};

__device__ __forceinline__ void child_rect(int x0, int x1, int y0, int y1, int q, int& cx0, int& cx1, int& cy0,
                                           int& cy1) {
    // ExtractorNode::DivideNode (:483-509): halfX = ceil((float)(UR.x-UL.x)/2)
    const int hx = (int)ceilf(__fdiv_rn((float)(x1 - x0), 2.0f));
    const int hy = (int)ceilf(__fdiv_rn((float)(y1 - y0), 2.0f));
    const int mx = x0 + hx, my = y0 + hy;
    cx0 = (q & 1) ? mx : x0;
    cx1 = (q & 1) ? x1 : mx;
    cy0 = (q & 2) ? my : y0;
    cy1 = (q & 2) ? y1 : my;
}

__device__ __forceinline__ int quadrant(uint32_t xy, int x0, int x1, int y0, int y1) {
    const int hx = (int)ceilf(__fdiv_rn((float)(x1 - x0), 2.0f));
    const int hy = (int)ceilf(__fdiv_rn((float)(y1 - y0), 2.0f));
    const int x = (int)(xy & 0xffff), y = (int)(xy >> 16);
    return (x < x0 + hx ? 0 : 1) + (y < y0 + hy ? 0 : 2);   // (:515-525)
}

// number of non-empty children with quadrant index > q (children are pushed n1..n4 to the front, so
// the group reads n4, n3, n2, n1)
__device__ __forceinline__ int rank_desc(const int* cc, int q) {
    int r = 0;
#pragma unroll
    for (int k = 3; k >= 0; --k) r += (k > q && cc[k] > 0) ? 1 : 0;
    return r;
}
__device__ __forceinline__ int rank_asc(const int* cc, int q) {
    int r = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) r += (k < q && cc[k] > 0) ? 1 : 0;
    return r;
}

#ifdef ORBX_QT_PROF
// Diagnostics build only (make qtprof): wall-clock stamps of thread 0 of the (first level, image 0) workgroup at the
// stage boundaries of k_quadtree, read back by orbx_debug_qt_prof.
__device__ unsigned long long g_qtprof[2][64];
#define QTP(tag)                                                                                                     \
    do {                                                                                                             \
        if (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0 && qtp_n < 32) {                                 \
            g_qtprof[lvl0 ? 1 : 0][2 * qtp_n] = wall_clock64();                                                      \
            g_qtprof[lvl0 ? 1 : 0][2 * qtp_n + 1] = (tag);                                                           \
        }                                                                                                            \
        ++qtp_n;                                                                                                     \
    } while (0)
#else
#define QTP(tag) do {} while (0)
#endif


// split point of a node, packed (x0 + ceil((x1-x0)/2)) | (y0 + ceil((y1-y0)/2)) << 16 (DivideNode :483-509; the float
// halving of an integer width is exact, so its ceiling is (w + 1) >> 1); a key's quadrant is (x >= mx) + 2 (y >= my)
__device__ __forceinline__ int node_mid(int x0, int x1, int y0, int y1) {
    return (x0 + ((x1 - x0 + 1) >> 1)) | ((y0 + ((y1 - y0 + 1) >> 1)) << 16);
}
__device__ __forceinline__ int mid_quadrant(uint32_t xy, int mid) {
    return ((int)(xy & 0xffff) >= (mid & 0xffff) ? 1 : 0) + ((int)(xy >> 16) >= (mid >> 16) ? 2 : 0);
}

struct QtState {         // one workgroup's LDS arrays (k_quadtree)
    int *A_xr, *A_yr, *A_cnt, *A_seq, *A_mid, *B_xr, *B_yr, *B_cnt, *B_seq, *B_mid;
    int *cc, *cc2, *base, *sa, *sb, *tmp, *misc;
    unsigned long long* sk;
};

// Everything after the level's key count is known, for keys in LDS (PXY / PN address-space-3 pointers: ds_ loads) or
// in the HBM scratch (plain pointers).
template <typename PXY, typename PN, typename PR>
__device__ __forceinline__ void qt_level(QtState S, const LevelDev& L, int lvl, int img, int K, int ncl, PXY kxy, PN kn,
                                         PR kr, const uint32_t* __restrict__ cand_xy,
                                         const uint8_t* __restrict__ cand_s, int cand_stride,
                                         uint32_t* __restrict__ out_xy, uint8_t* __restrict__ out_r, int out_stride,
                                         int* __restrict__ level_cnt, int nlevels, int cap, int* __restrict__ err,
                                         unsigned seq) {
    const int tid = threadIdx.x, T = blockDim.x;
#ifdef ORBX_QT_PROF
    int qtp_n = 1;
    const int lvl0 = lvl;      // QTP stamps the blockIdx.x == 0 workgroup, whose level is the launch's first
#endif
    int *A_xr = S.A_xr, *A_yr = S.A_yr, *A_cnt = S.A_cnt, *A_seq = S.A_seq, *A_mid = S.A_mid;
    int *B_xr = S.B_xr, *B_yr = S.B_yr, *B_cnt = S.B_cnt, *B_seq = S.B_seq, *B_mid = S.B_mid;
    int *cc = S.cc, *cc2 = S.cc2, *base = S.base, *sa = S.sa, *sb = S.sb, *misc = S.misc;
    unsigned long long* sk = S.sk;
    const int minB = kEdge - 3;
    // ---- 2. root nodes (:543-585), laid out before the gather so that the gather also assigns every key to its root
    //    and counts the root's quadrants (the first pass's child counts)
    const int nIni = L.nIni;
    const float hX = L.hX;
    for (int i = tid; i < nIni; i += T) {
        const int x0 = (int)__fmul_rn(hX, (float)i), x1 = (int)__fmul_rn(hX, (float)(i + 1));
        A_xr[i] = (x0 & 0xffff) | (x1 << 16);
        A_yr[i] = 0 | (L.win_h << 16);
        A_mid[i] = node_mid(x0, x1, 0, L.win_h);
        A_cnt[i] = 0;
        A_seq[i] = i;
    }
    for (int i = tid; i < 4 * nIni; i += T) cc2[i] = 0;
    // owner cell of every key (LDS / scratch writes only), then one flat gather over the keys with every load
    // independent, each key assigned to its root and counted in the root's quadrant on the way (a walk cell by cell
    // chains three dependent HBM loads per cell: ~150 us at level 0; G threads per cell walking its slots: 19.4 against
    // 15.3 us to here, r4q)
    for (int c = tid; c < ncl; c += T) {
        const int b = sa[c], e = (c + 1 < ncl) ? sa[c + 1] : K;
        for (int k = b; k < e; ++k) kn[k] = (int16_t)c;
    }
    __syncthreads();
    {
        const size_t io = (size_t)img * cand_stride;
        constexpr int U = 4;
        for (int k0 = tid; k0 < K; k0 += U * T) {
            uint32_t xy[U];
            uint8_t r[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int k = k0 + u * T;
                if (k < K) {
                    const int c = kn[k];
                    const int sbc = sb[c];
                    const size_t src = io + (size_t)sbc + (k - sa[c]);
                    xy[u] = cand_xy[src];
                    r[u] = cand_s[src];
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int k = k0 + u * T;
                if (k < K) {
                    const uint32_t w = ((xy[u] & 0xffff) - minB) | (((xy[u] >> 16) - minB) << 16);
                    kxy[k] = w;
                    kr[k] = r[u];
                    const int x = (int)(w & 0xffff);
                    const int rt = min((int)__fdiv_rn((float)x, hX), nIni - 1);
                    kn[k] = (int16_t)rt;
                    atomicAdd(&A_cnt[rt], 1);
                    atomicAdd(&cc2[4 * rt + mid_quadrant(w, A_mid[rt])], 1);
                }
            }
        }
    }
    __syncthreads();
    QTP(1);
    // drop empty roots (order preserved), on wave 0: the list, its child counts, and the root -> position map in sb
    // that the first key move reads
    const bool w0 = tid < kWave;
    const int ln = tid & (kWave - 1);
    if (w0) {
        int carry = 0;
        for (int b0 = 0; b0 < nIni; b0 += kWave) {
            const int i = b0 + ln;
            const bool keep = i < nIni && A_cnt[i] > 0;
            const uint64_t m = __ballot(keep);
            const int p = carry + lanes_below(m);
            if (keep) {
                B_xr[p] = A_xr[i]; B_yr[p] = A_yr[i]; B_cnt[p] = A_cnt[i]; B_seq[p] = A_seq[i]; B_mid[p] = A_mid[i];
                reinterpret_cast<int4*>(cc)[p] = reinterpret_cast<const int4*>(cc2)[i];
            }
            if (i < nIni) sb[i] = keep ? p : -1;
            carry += __popcll(m);
        }
        if (ln == 0) misc[7] = carry;
    }
    __syncthreads();
    int n = misc[7];
    {
        int* t;
        t = A_xr; A_xr = B_xr; B_xr = t;
        t = A_yr; A_yr = B_yr; B_yr = t;
        t = A_cnt; A_cnt = B_cnt; B_cnt = t;
        t = A_seq; A_seq = B_seq; B_seq = t;
        t = A_mid; A_mid = B_mid; B_mid = t;
    }
    bool remap = true;                                     // kn holds root indices until the first key move

    const int N = L.N;
    // A = the node list of the current pass, B = the list it builds; after a pass the two swap roles
    auto swap_nodes = [&]() {
        int* t;
        t = cc; cc = cc2; cc2 = t;
        t = A_xr; A_xr = B_xr; B_xr = t;
        t = A_yr; A_yr = B_yr; B_yr = t;
        t = A_cnt; A_cnt = B_cnt; B_cnt = t;
        t = A_seq; A_seq = B_seq; B_seq = t;
        t = A_mid; A_mid = B_mid; B_mid = t;
    };
    // A split node's children (quadrant q) go to the new list from group base gb on, in the reference's order (n4 .. n1,
    // empty children dropped: gb + rank_desc), with their rectangle, count, creation order and split point;
    // base[i] = the new position of a node that stays, or -2 - gb for a split node.
    auto write_children = [&](int i, int gb, int cre) {
        const int x0 = A_xr[i] & 0xffff, x1 = A_xr[i] >> 16, y0 = A_yr[i] & 0xffff, y1 = A_yr[i] >> 16;
        const int mid = A_mid[i], mx = mid & 0xffff, my = mid >> 16;
        const int* c4 = cc + 4 * i;
        for (int q = 0; q < 4; ++q) {
            if (c4[q] == 0) continue;
            const int cx0 = (q & 1) ? mx : x0, cx1 = (q & 1) ? x1 : mx, cy0 = (q & 2) ? my : y0, cy1 = (q & 2) ? y1 : my;
            const int p = gb + rank_desc(c4, q);
            B_xr[p] = (cx0 & 0xffff) | (cx1 << 16);
            B_yr[p] = (cy0 & 0xffff) | (cy1 << 16);
            B_cnt[p] = c4[q];
            B_seq[p] = cre + rank_asc(c4, q);
            B_mid[p] = node_mid(cx0, cx1, cy0, cy1);
            reinterpret_cast<int4*>(cc2)[p] = make_int4(0, 0, 0, 0);
        }
        base[i] = -2 - gb;
    };
    auto keep_node = [&](int i, int p) {
        base[i] = p;
        B_xr[p] = A_xr[i]; B_yr[p] = A_yr[i]; B_cnt[p] = A_cnt[i]; B_seq[p] = A_seq[i]; B_mid[p] = A_mid[i];
        reinterpret_cast<int4*>(cc2)[p] = make_int4(0, 0, 0, 0);
    };
    // every key to its node of the new list; the new list's child counts taken on the way (the next pass's cc)
    auto move_keys = [&]() {
        for (int k = tid; k < K; k += T) {
            const int i = remap ? sb[kn[k]] : kn[k];
            const uint32_t xy = kxy[k];
            const int b = base[i];
            int p = b;
            if (b < 0) {                                     // split: one 16-byte read of the node's child counts
                const int4 c = reinterpret_cast<const int4*>(cc)[i];
                const int c4[4] = {c.x, c.y, c.z, c.w};
                p = -2 - b + rank_desc(c4, mid_quadrant(xy, A_mid[i]));
            }
            kn[k] = (int16_t)p;
            if (B_cnt[p] > 1) atomicAdd(&cc2[4 * p + mid_quadrant(xy, B_mid[p])], 1);
        }
    };
    bool phase2 = false, finished = false;
    // The node-list bookkeeping of a pass (flags, prefix sums, the new list, the phase decisions) is O(nodes <= cap)
    // and runs on wave 0 alone with wave-level scans and fences; the other waves wait at one barrier, then every thread
    // moves the keys.  Two block barriers per pass (phase 2: plus the sort's), where block-wide scans took ~7.
    QTP(2);
    while (!finished) {
        const int prev = n;
        QTP(10 + phase2);
        QTP(20);
        if (!phase2) {
            // ---------------- phase 1 pass (:606-665), bookkeeping on wave 0
            // per node: children (split) or 1 survivor, packed as children << 16 | survivor so that ONE scan gives both
            // prefixes (children before node i in the high half, survivors before it in the low half; totals < 2^15);
            // base = the node's children count; nodes of >1 key to expand next (nexp)
            if (w0) {
                int nexp = 0;
                for (int i = ln; i < n; i += kWave) {
                    const int* c4 = cc + 4 * i;
                    const bool split = A_cnt[i] > 1;
                    const int nch = split ? (c4[0] > 0) + (c4[1] > 0) + (c4[2] > 0) + (c4[3] > 0) : 0;
                    sa[i] = split ? (nch << 16) : 1;
                    base[i] = nch;
                    if (split) nexp += (c4[0] > 1) + (c4[1] > 1) + (c4[2] > 1) + (c4[3] > 1);
                }
                nexp = wave_sum(nexp);
                wave_fence();
                const int CU = wave_excl_scan_lds(sa, n, ln);
                wave_fence();
                const int C = CU >> 16, U = CU & 0xffff;
                const int nn = C + U;
                if (nn > cap) {
                    if (ln == 0) { atomicOr(err, kErrQtCap); misc[2] = -1; }
                } else {
                    for (int i = ln; i < n; i += kWave) {
                        if (A_cnt[i] > 1) write_children(i, C - (sa[i] >> 16) - base[i], sa[i] >> 16);
                        else keep_node(i, C + (sa[i] & 0xffff));
                    }
                    if (ln == 0) {
                        // :669-673, decided here for every thread: 1 finished, 2 on to phase 2
                        misc[2] = (nn >= N || nn == prev) ? 1 : (nn + nexp * 3 > N) ? 2 : 0;
                        misc[3] = nn;
                    }
                }
            }
            __syncthreads();
            QTP(30);
            const int dec = misc[2];
            if (dec < 0) { finished = true; break; }
            const int nn = misc[3];
            move_keys();
            __syncthreads();
            remap = false;
            swap_nodes();                                        // the new list becomes A (no copy, no barrier)
            n = nn;
            QTP(50);
            if (dec == 1) finished = true;
            else if (dec == 2) phase2 = true;
        } else {
            // ---------------- phase 2 pass (:676-737)
            // expandable nodes -> sort keys (size, creation order, node), on wave 0; up to 512 of them wave 0 sorts in
            // registers too and goes straight on to the bookkeeping (one block barrier for the pass's list work)
            int nV = 0, P2 = 1;
            const bool wsort = n <= 512;                       // workgroup-uniform: nV <= n
            if (w0) {
                for (int i = ln; i < n; i += kWave) sa[i] = A_cnt[i] > 1 ? 1 : 0;
                wave_fence();
                nV = wave_excl_scan_lds(sa, n, ln);
                wave_fence();
                while (P2 < nV) P2 <<= 1;
                const int PW = wsort ? max(P2, kWave) : P2;      // the wave sort pads to at least 64 keys
                for (int i = ln; i < PW; i += kWave) sk[i] = ~0ull;
                wave_fence();
                for (int i = ln; i < n; i += kWave)
                    if (A_cnt[i] > 1)
                        sk[sa[i]] = ((unsigned long long)A_cnt[i] << 40) | ((unsigned long long)A_seq[i] << 20) | (unsigned long long)i;
                wave_fence();
                if (wsort) {
                    if (PW <= kWave) wave_bitonic_u64<1>(sk, ln);
                    else if (PW <= 2 * kWave) wave_bitonic_u64<2>(sk, ln);
                    else if (PW <= 4 * kWave) wave_bitonic_u64<4>(sk, ln);
                    else wave_bitonic_u64<8>(sk, ln);
                    wave_fence();
                }
                if (ln == 0) { misc[4] = nV; misc[5] = P2; }
            }
            if (!wsort) {
                // larger lists: every wave sorts (stages inside a wave's 128 keys need only a wave-level fence,
                // block_bitonic_u64).  (Ranking each key by counting the smaller ones measured slower, r3am.)
                __syncthreads();
                nV = misc[4];
                P2 = misc[5];
                if (P2 >= 2) block_bitonic_u64(sk, P2);
            }
            auto key_at = [&](int p) { return sk[nV - 1 - p]; };     // processing order: descending keys
            QTP(31);
            if (w0) {
                // children of the p-th processed node (sb), the first p at which the list reaches N (:713-720): the
                // list grows by children - 1 per processed node, so n + inclusive prefix of the deltas is nondecreasing;
                // the children before p (the new nodes' creation prefix, sa) = the deltas' exclusive prefix + p
                int brk = nV, acc = 0, inc_brk = 0;
                for (int b0 = 0; b0 < nV; b0 += kWave) {
                    const int p = b0 + ln;
                    int d = 0;
                    if (p < nV) {
                        const int i = (int)(key_at(p) & 0xfffff);
                        const int4 c = reinterpret_cast<const int4*>(cc)[i];
                        const int ch = (c.x > 0) + (c.y > 0) + (c.z > 0) + (c.w > 0);
                        sb[p] = ch;
                        d = ch - 1;
                    }
                    const int inc = acc + wave_incl_scan(d);
                    if (p < nV) sa[p] = inc - d + p;
                    const uint64_t hit = __ballot(p < nV && n + inc >= N);
                    if (brk == nV && hit) {
                        brk = b0 + (int)__builtin_ctzll(hit);
                        inc_brk = __builtin_amdgcn_readlane(inc, brk - b0);
                    }
                    acc = __builtin_amdgcn_readlane(inc, kWave - 1);
                }
                const int nproc = min(brk + 1, nV);
                const int Cn = (brk < nV ? inc_brk : acc) + nproc;   // children of the processed nodes
                for (int i = ln; i < n; i += kWave) base[i] = 0;
                wave_fence();
                // processed nodes: their group base (kept in base as -2 - gb) and creation prefix (in A_seq: the node is
                // erased anyway); the survivors are ranked after the groups
                for (int p = ln; p < nproc; p += kWave) {
                    const int i = (int)(key_at(p) & 0xfffff);
                    base[i] = -2 - (Cn - sa[p] - sb[p]);
                    A_seq[i] = -1 - sa[p];
                }
                wave_fence();
                // survivors' ranks (base >= 0) into sb
                int U = 0;
                for (int b0 = 0; b0 < n; b0 += kWave) {
                    const int i = b0 + ln;
                    const bool sv = i < n && base[i] >= 0;
                    const uint64_t m = __ballot(sv);
                    if (i < n) sb[i] = U + lanes_below(m);
                    U += __popcll(m);
                }
                wave_fence();
                const int nn = Cn + U;
                if (nn > cap) {
                    if (ln == 0) { atomicOr(err, kErrQtCap); misc[2] = -1; }
                } else {
                    for (int i = ln; i < n; i += kWave) {
                        const int b = base[i];
                        if (b < 0) write_children(i, -2 - b, -1 - A_seq[i]);
                        else keep_node(i, Cn + sb[i]);
                    }
                    if (ln == 0) { misc[2] = (nn >= N || nn == prev) ? 1 : 0; misc[3] = nn; }   // :734-735
                }
            }
            __syncthreads();
            QTP(32);
            const int dec = misc[2];
            if (dec < 0) { finished = true; break; }
            const int nn = misc[3];
            move_keys();
            __syncthreads();
            remap = false;
            swap_nodes();
            n = nn;
            QTP(51);
            if (dec == 1) finished = true;
        }
    }
    if (remap) {                                             // no pass ran: the keys still name their roots
        for (int k = tid; k < K; k += T) kn[k] = (int16_t)sb[kn[k]];
        __syncthreads();
    }

    QTP(80);
    // ---- retain the first maximum-response key of every node (:742-760)
    for (int i = tid; i < n; i += T) sk[i] = 0ull;
    __syncthreads();
    for (int k = tid; k < K; k += T) {
        const unsigned long long v = ((unsigned long long)kr[k] << 32) | (unsigned long long)(0xffffffffu - (uint32_t)k);
        atomicMax(&sk[kn[k]], v);
    }
    __syncthreads();
    uint32_t* oxy = out_xy + (size_t)img * out_stride + L.out_off;
    uint8_t* orr = out_r + (size_t)img * out_stride + L.out_off;
    const int nout = min(n, L.out_cap);
    for (int i = tid; i < nout; i += T) {
        const uint32_t k = 0xffffffffu - (uint32_t)(sk[i] & 0xffffffffu);
        const uint32_t xy = kxy[k];
        oxy[i] = ((xy & 0xffff) + minB) | (((xy >> 16) + minB) << 16);
        orr[i] = kr[k];
    }
    // count | call sequence number << 16: the describe that reads this level checks the stamp (ordering canary)
    if (tid == 0) level_cnt[img * nlevels + lvl] = nout | (int)((seq & 0x7fffu) << 16);
    QTP(90);
}

__global__ __launch_bounds__(kQtThreads) void k_quadtree(const LevelDev* __restrict__ levels, const CellDev* __restrict__ cells,
                                                         const uint32_t* __restrict__ cand_xy, const uint8_t* __restrict__ cand_s,
                                                         int cand_stride, const int* __restrict__ cell_cnt, int ncells,
                                                         QtScratch qs, uint32_t* __restrict__ out_xy, uint8_t* __restrict__ out_r,
                                                         int out_stride, int* __restrict__ level_cnt, int nlevels, int cap,
                                                         int scan_cap, int* __restrict__ err, int lvl0, int key_lds_off,
                                                         int key_lds_cap, unsigned seq) {
    extern __shared__ __attribute__((aligned(16))) int smem[];
    const int lvl = lvl0 + (int)blockIdx.x, img = blockIdx.y, tid = threadIdx.x, T = blockDim.x;
#ifdef ORBX_QT_PROF
    int qtp_n = 0;
#endif
    QTP(0);
    const LevelDev L = levels[lvl];
    // LDS layout
    QtState S;
    const int cs = (cap + 3) & ~3;     // array stride (16-byte aligned int4 rows below)
    S.A_xr = smem;               // x0 | x1 << 16
    S.A_yr = S.A_xr + cs;       // y0 | y1 << 16
    S.A_cnt = S.A_yr + cs;
    S.A_seq = S.A_cnt + cs;
    S.A_mid = S.A_seq + cs;     // split point (node_mid)
    S.B_xr = S.A_mid + cs;
    S.B_yr = S.B_xr + cs;
    S.B_cnt = S.B_yr + cs;
    S.B_seq = S.B_cnt + cs;
    S.B_mid = S.B_seq + cs;
    S.cc = S.B_mid + cs;        // [cap][4] child counts of the current list 
    S.cc2 = S.cc + 4 * cs;      // [cap][4] child counts of the list being built (counted while keys move)
    S.base = S.cc2 + 4 * cs;    // new list position of a node that stays, -2 - group base: split
    S.sa = S.base + cs;         // scan array [scan_cap]
    S.sb = S.sa + scan_cap;      // scan array [scan_cap]
    S.tmp = S.sb + scan_cap;     // 32 ints
    S.misc = S.tmp + 32;         // 16 ints
    S.sk = (unsigned long long*)(S.misc + 16 + ((S.misc + 16 - smem) & 1));  // [pow2 >= cap]
    const int ncl = L.cell_end - L.cell_begin;
    int* sa = S.sa;
    int* sb = S.sb;

    // ---- 1. compact the level's cell candidates into reference order (cell row-major, then FAST order)
    // (per cell: count -> sa, slot offset -> sb; all loads independent)
    for (int i = tid; i < ncl; i += T) {
        const int cw = cell_cnt[(size_t)img * ncells + L.cell_begin + i];
        sa[i] = cw;
        sb[i] = cells[L.cell_begin + i].slot_off;
    }
    __syncthreads();
    const int K = block_scan_array(sa, ncl, S.tmp);
    // Every pass walks all K keys: they live in LDS when the level's keys fit the launch's key region (the common case:
    // ~2-4k keys at level 0 of a KITTI frame) -- then every key access is an LDS instruction -- and in the HBM scratch
    // otherwise.
    if (K <= key_lds_cap) {
        lds_u32* kxy = (lds_u32*)(reinterpret_cast<char*>(smem) + key_lds_off);
        lds_i16* kn = (lds_i16*)(kxy + key_lds_cap);
        lds_u8* kr = (lds_u8*)(kn + key_lds_cap);
        qt_level(S, L, lvl, img, K, ncl, kxy, kn, kr, cand_xy, cand_s, cand_stride, out_xy, out_r, out_stride, level_cnt,
                 nlevels, cap, err, seq);
    } else {
        uint32_t* kxy = qs.key_xy + (size_t)img * cand_stride + L.cand_off;
        int16_t* kn = qs.key_node + (size_t)img * cand_stride + L.cand_off;
        uint8_t* kr = qs.key_r + (size_t)img * cand_stride + L.cand_off;
        qt_level(S, L, lvl, img, K, ncl, kxy, kn, kr, cand_xy, cand_s, cand_stride, out_xy, out_r, out_stride, level_cnt,
                 nlevels, cap, err, seq);
    }
}

// ---------------------------------------------------------------------------------------------
// IC angle + steered BRIEF + output assembly (k_describe_m).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float fast_atan2_deg(float y, float x) {   // OpenCV fastAtan2 (pinned, :103)
    const float k = (float)(180.0 / M_PI);
    const float p1 = __fmul_rn(0.9997878412794807f, k), p3 = __fmul_rn(-0.3258083974640975f, k);
    const float p5 = __fmul_rn(0.1555786518463281f, k), p7 = __fmul_rn(-0.04432655554792128f, k);
    const float eps = (float)2.2204460492503131e-016;
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = __fdiv_rn(ay, __fadd_rn(ax, eps));
        c2 = __fmul_rn(c, c);
        a = __fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(p7, c2), p5), c2), p3), c2), p1), c);
    } else {
        c = __fdiv_rn(ax, __fadd_rn(ay, eps));
        c2 = __fmul_rn(c, c);
        a = __fsub_rn(90.f, __fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(p7, c2), p5), c2), p3), c2), p1), c));
    }
    if (x < 0) a = __fsub_rn(180.f, a);
    if (y < 0) a = __fsub_rn(360.f, a);
    return a;
}

struct SlotTable { int out_off[kMaxLevels]; };   // LevelDev::out_off per level, as a kernel argument

// Ordering canary.  k_quadtree stamps each level count with the low 15 bits of the call's sequence number; the
// describe of that call finds another call's stamp only if some edge that orders the kept-keypoint buffers across
// calls is missing, and then raises kErrStale in the extractor's error word instead of returning wrong keypoints.
__device__ __forceinline__ bool lvl_stale(int packed, unsigned seq) {
    return (((unsigned)packed >> 16) & 0x7fffu) != (seq & 0x7fffu);
}
constexpr int kBriefR = 18;                      // max |rotated pattern offset|: round(hypot(-13, -13)) = 18
constexpr int kBriefRow = 40;                    // LDS bytes per window row (5 x 8-byte chunks)
constexpr int kBriefWin = (2 * kBriefR + 1) * kBriefRow;
#ifndef ORBX_BRIEF_BATCH
#define ORBX_BRIEF_BATCH 4
#endif
constexpr int kBriefBatch = ORBX_BRIEF_BATCH;                 // BRIEF test groups whose LDS reads are issued together

// Sum of v over the kLp-lane group of each lane (groups of 16, 32 or 64 lanes), in every lane of the group.
template <int kLp>
__device__ __forceinline__ int group_sum(int v, int sub) {
    // old = 0, the sum's identity: the compiler folds each move into its add as a DPP operand (one v_add_u32_dpp
    // instead of a copy, a v_mov_b32_dpp and an add); same rule in orbx_common.h's reductions
    v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);     // quad_perm 1,0,3,2
    v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);     // quad_perm 2,3,0,1
    v += __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false);    // row_half_mirror
    v += __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false);    // row_mirror: row sum in every lane of the row
    if (kLp == 16) return v;
    const int r0 = __builtin_amdgcn_readlane(v, 0), r1 = __builtin_amdgcn_readlane(v, 16);
    const int r2 = __builtin_amdgcn_readlane(v, 32), r3 = __builtin_amdgcn_readlane(v, 48);
    if (kLp == 32) return sub == 0 ? r0 + r1 : r2 + r3;
    return r0 + r1 + r2 + r3;
}

// Disc masks of the IC box chunks for 32 lanes per keypoint (the shipped kKpw = 2): chunk q = lane + 32 k covers row
// q / 4 - kHalfPatch, columns 8 (q % 4) - kHalfPatch .. +7; byte b is inside the disc iff |u| <= umax[|v|]
// (ORBextractor.cc:84-99).  Built at compile time from kUmax: the per-lane bounds, shifts and 64-bit masks are then one
// constant load per chunk instead of ~20 VALU.
struct IcMaskTab { unsigned long long m[4][32]; };
constexpr IcMaskTab make_ic_masks() {
    IcMaskTab t{};
    for (int k = 0; k < 4; ++k)
        for (int lk = 0; lk < 32; ++lk) {
            const int q = lk + 32 * k;
            unsigned long long m = 0;
            if (q < 4 * (2 * kHalfPatch + 1)) {
                const int v = (q >> 2) - kHalfPatch, av = v < 0 ? -v : v;
                const int um = kUmax[av > 15 ? 15 : av], u0 = 8 * (q & 3) - kHalfPatch;
                for (int b = 0; b < 8; ++b) {
                    const int u = u0 + b;
                    if (u >= -um && u <= um) m |= 0xffull << (8 * b);
                }
            }
            t.m[k][lk] = m;
        }
    return t;
}
__constant__ IcMaskTab c_ic_mask = make_ic_masks();

// IC angle + steered BRIEF + output assembly, kKpw keypoints per wave (kLp = 64 / kKpw lanes each; the shipped form is
// 2 -- one keypoint per wave measured 449 vs 444 us serial, 4 no faster): the wave-uniform part of a keypoint (level
// lookup, moment reductions, fastAtan2, the double sin/cos, the keypoint record) is paid once per kKpw keypoints,
// and each lane loads kKpw times as many window chunks and runs kKpw times as many BRIEF tests.  The keypoints of a
// wave can straddle a level boundary, so the level is per lane.
//   The blurred 37 x 37 window the BRIEF tests can touch (|rotated offset| <= 18) is loaded beside the IC_Angle loads
// into the keypoint's LDS slice (rows of kBriefRow bytes): the tests then read LDS, so the angle -> BRIEF dependency
// costs no second memory round trip.  Keypoints lie >= 19 px inside the level (FAST window :789-797), so rows
// cy-18 .. cy+18 exist; a row's bytes past cx+18 are never read.  IC_Angle (:77-104): the 31 x 32 box around the
// disc as 124 (row, 8-byte chunk) items; per chunk the bytes outside the disc (|u| > umax[|v|]) are masked off, then
// sum (u+16)*I and sum I come from v_dot4_u32_u8 against packed weights: m10 += that - 16 * sum I, m01 += v * sum I.
template <int kKpw>
__global__ __launch_bounds__(256) void k_describe_m(const uint8_t* __restrict__ pyr, const uint8_t* __restrict__ blur,
                                                    size_t pyr_stride, const LevelDev* __restrict__ levels, int nlevels,
                                                    const uint32_t* __restrict__ lvl_xy, const uint8_t* __restrict__ lvl_r,
                                                    int out_stride, const int* __restrict__ level_cnt,
                                                    orbx_keypoint* __restrict__ kps, uint8_t* __restrict__ desc,
                                                    int32_t* __restrict__ counts, int capacity, int slot0, int nslots,
                                                    int write_count, int batch, Src0 s0, SlotTable tab, unsigned seq,
                                                    int* __restrict__ err) {
    constexpr int kLp = kWave / kKpw;
    constexpr int kWinItems = 5 * (2 * kBriefR + 1);             // 37 rows x 5 chunks of 8 bytes
    constexpr int kNW = (kWinItems + kLp - 1) / kLp;             // window chunks per lane
    constexpr int kIcItems = 4 * (2 * kHalfPatch + 1);           // 31 rows x 4 chunks (124)
    constexpr int kNI = (kIcItems + kLp - 1) / kLp;              // IC chunks per lane
    constexpr int kNT = 256 / kLp;                               // BRIEF tests per lane
    static_assert(kKpw == 2 || kKpw == 4, "2 or 4 keypoints per wave");
    __shared__ __attribute__((aligned(16))) uint8_t brief_lds[4 * kKpw * kBriefWin];
    const int per_wg = 4 * kKpw;
    const int nbx = (nslots + per_wg - 1) / per_wg;
    const int item = xcd_item(xcd_chunk(nbx * batch));
    if (item >= nbx * batch) return;
    const int img = item / nbx;
    const int wrel = __builtin_amdgcn_readfirstlane(((item - img * nbx) * blockDim.x + threadIdx.x) >> 6);
    if (wrel * kKpw >= nslots) return;                           // whole wave
    const int ln = lane_id();
    const int sub = ln / kLp, lk = ln - sub * kLp;
    const int rel = wrel * kKpw + sub;
    const int slot = slot0 + rel;
    int lvl = 0;                                                 // a uniform loop over the levels in use (the unrolled
    for (int l = 1; l < nlevels; ++l) lvl += slot >= tab.out_off[l] ? 1 : 0;   // kMaxLevels form was 62 VALU)
    const int* lcs = level_cnt + img * nlevels;
    int off = 0, total = 0;
    for (int l = 0; l < nlevels; ++l) {
        const int c = lcs[l] & 0xffff;
        off += l < lvl ? c : 0;
        total += c;
    }
    const int craw = lcs[lvl], ci = craw & 0xffff;
    // the level this lane reads must carry this call's stamp (lanes past the launch's slots read nothing)
    if (__ballot(rel < nslots && lvl_stale(craw, seq)) && ln == 0) atomicOr(err, kErrStale);
    if (write_count && wrel == 0 && ln == 0) counts[img] = min(total, capacity);
    const LevelDev& L = levels[lvl];
    const int lw = L.w, lpo = L.pyr_off, loo = L.out_off;
    const int i = slot - loo;
    const int o = off + i;
    const bool valid = rel < nslots && i < ci && o < capacity;
    if (__ballot(valid) == 0) return;                            // whole wave

    const uint32_t xy = valid ? lvl_xy[(size_t)img * out_stride + loo + i] : 0u;
    const int cx = (int)(xy & 0xffff), cy = (int)(xy >> 16);
    const uint8_t* B = blur + img * pyr_stride + lpo;
    uint8_t* win = brief_lds + ((threadIdx.x >> 6) * kKpw + sub) * kBriefWin;
    uint64_t wv[kNW];
    int woff[kNW];                                               // LDS offset of chunk q = lk + kLp * k (row q / 5, chunk q % 5)
    {
        int wr = lk / 5, wc = lk - 5 * wr;                       // one division; later chunks step by kLp = 5 A + B
#pragma unroll
        for (int k = 0; k < kNW; ++k) {
            woff[k] = __mul24(wr, kBriefRow) + 8 * wc;
            if (valid) __builtin_memcpy(&wv[k], B + (size_t)(cy - kBriefR + min(wr, 2 * kBriefR)) * lw + (cx - kBriefR + 8 * wc), 8);
            wc += kLp % 5; wr += kLp / 5;
            if (wc >= 5) { wc -= 5; ++wr; }
        }
    }
    int pstride;
    const uint8_t* P = lvl == 0 ? s0.p + img * s0.istride : pyr + img * pyr_stride + lpo;
    pstride = lvl == 0 ? (int)s0.step : lw;
    int m10 = 0, m01 = 0;
    {
        uint64_t ic[kNI];
        const uint8_t* p0 = P + (size_t)(cy - kHalfPatch) * pstride + (cx - kHalfPatch);
        if (valid) {
#pragma unroll
            for (int k = 0; k < kNI; ++k) {
                const int q = lk + kLp * k, r = min(q >> 2, 2 * kHalfPatch);
                __builtin_memcpy(&ic[k], p0 + (size_t)r * pstride + 8 * (q & 3), 8);
            }
        }
#pragma unroll
        for (int k = 0; k < kNI; ++k) {
            const int q = lk + kLp * k;
            const int v = (q >> 2) - kHalfPatch, av = v < 0 ? -v : v;
            const int u0 = 8 * (q & 3) - kHalfPatch;
            uint64_t m = 0;
            if constexpr (kLp == 32) {
                m = valid ? c_ic_mask.m[k][lk] : 0ull;
            } else {
                const int um = kUmax[av > 15 ? 15 : av];
                const int lo = max(0, -um - u0), hi = min(7, um - u0);
                if (valid && q < kIcItems && lo <= hi) m = (hi >= 7 ? ~0ull : ((1ull << (8 * hi + 8)) - 1ull)) & (~0ull << (8 * lo));
            }
            const uint64_t px = ic[k] & m;
            const uint32_t a = (uint32_t)px, b = (uint32_t)(px >> 32);
            const uint32_t wa = (uint32_t)(u0 + 16) * 0x01010101u + 0x03020100u, wb = wa + 0x04040404u;
            const int dot = (int)__builtin_amdgcn_udot4(b, wb, __builtin_amdgcn_udot4(a, wa, 0u, false), false);
            const int sum = (int)__builtin_amdgcn_udot4(b, 0x01010101u, __builtin_amdgcn_udot4(a, 0x01010101u, 0u, false), false);
            m10 += dot - 16 * sum;
            m01 += v * sum;
        }
    }
    if (valid) {
#pragma unroll
        for (int k = 0; k < kNW; ++k) {
            const int q = lk + kLp * k;
            if (q < kWinItems) *reinterpret_cast<uint64_t*>(win + woff[k]) = wv[k];
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    m10 = group_sum<kLp>(m10, sub);
    m01 = group_sum<kLp>(m01, sub);
    const float angle = fast_atan2_deg((float)m01, (float)m10);
    const float ang = __fmul_rn(angle, (float)(M_PI / 180.f));
    float a, b;
    orbx_sincos_brief(ang, &a, &b);
    const uint8_t* center = win + kBriefR * kBriefRow + kBriefR;
    // this lane's pattern words (tests g * kLp + lk), contiguous in the per-lane table
    uint32_t pat[kNT];
    {
        const uint32_t* pw = (kLp == 32 ? c_pattern_l32.w : c_pattern_l16.w) + lk * kNT;
#pragma unroll
        for (int g = 0; g < kNT; g += 4) __builtin_memcpy(&pat[g], pw + g, 16);
    }
    // The rotated offsets (computeOrbDescriptor :120-124): ry = fx b + fy a, rx = fx a - fy b, each product and sum
    // rounded separately (no fusion): two v_pk_mul_f32 ({b, a} and {a, -b}; the negated product is exact) and a
    // v_pk_add_f32.  cvRound (ties to even) by the magic constant M = 1.5 * 2^23: for |v| < 2^22 the float sum v + M is
    // an integer and its bits are 0x4B400000 + rint(v), so bits(ry + M) [low 24 bits, v_mad_i32_i24] * kBriefRow +
    // bits(rx + M) - kMagicOff is the window offset -- one packed add per point instead of two v_rndne_f32 and two
    // v_cvt_i32_f32.  Written as asm: the compiler's own pairing of the scalar form costs ~40 register moves per lane.
    // (The elements are copied to floats before their bits are taken: this compiler turns __builtin_bit_cast of an
    // ext_vector element .y into element .x.)
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    const f32x2 ab1 = {b, a}, ab2 = {a, -b}, magic = {12582912.0f, 12582912.0f};
    constexpr int kMagicOff = (int)(0x400000u * (unsigned)kBriefRow + 0x4B400000u);
    // kBriefBatch groups of tests at a time: their LDS offsets, then their reads back to back, then the comparisons
    // (no branch: a rotated offset is within kBriefR of the centre, inside the slice, for invalid lanes too, whose
    // moments are 0 and angle 0)
    uint32_t words[kNT];                                          // this lane's keypoint: tests g*kLp .. g*kLp+kLp-1
#pragma unroll
    for (int g0 = 0; g0 < kNT; g0 += kBriefBatch) {
        int toff[kBriefBatch][2], vals[kBriefBatch][2];
#pragma unroll
        for (int h = 0; h < kBriefBatch; ++h) {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const uint32_t w = pat[g0 + h];
                const float fx = (float)(int)(signed char)(w >> (16 * e)), fy = (float)(int)(signed char)(w >> (16 * e + 8));
                const f32x2 fxy = {fx, fy};
                f32x2 p, q, r;
                asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(p) : "v"(fxy), "v"(ab1));             // {fx b, fx a}
                asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]" : "=v"(q) : "v"(fxy), "v"(ab2)); // {fy a, -fy b}
                asm("v_pk_add_f32 %0, %1, %2" : "=v"(r) : "v"(p), "v"(q));                                 // {ry, rx}
                asm("v_pk_add_f32 %0, %1, %2" : "=v"(p) : "v"(r), "v"(magic));                             // + M
                const float ryM = p.x, rxM = p.y;
                int t;
                asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(t) : "v"(__float_as_int(ryM)), "n"(kBriefRow), "v"(__float_as_int(rxM)));
                toff[h][e] = t - kMagicOff;
            }
        }
#pragma unroll
        for (int h = 0; h < kBriefBatch; ++h) {
            vals[h][0] = center[toff[h][0]];
            vals[h][1] = center[toff[h][1]];
        }
#pragma unroll
        for (int h = 0; h < kBriefBatch; ++h) {
            const uint64_t bm = __ballot(vals[h][0] < vals[h][1]);
            words[g0 + h] = (uint32_t)(bm >> (sub * kLp)) & (uint32_t)((1ull << kLp) - 1ull);
        }
    }
    if (!valid) return;
    // descriptor dword j (j < 8) of this lane's keypoint, written by lane lk = j
    uint32_t dw = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t w = kLp == 32 ? words[j] : (words[2 * j] | (words[2 * j + 1] << 16));
        dw = lk == j ? w : dw;
    }
    if (lk < 8) reinterpret_cast<uint32_t*>(desc + ((size_t)img * capacity + o) * 32)[lk] = dw;
    if (lk == 0) {
        orbx_keypoint k;
        float x = (float)cx, y = (float)cy;
        if (lvl != 0) { x = __fmul_rn(x, L.scale); y = __fmul_rn(y, L.scale); }
        k.x = x; k.y = y;
        k.size = (float)L.patch;
        k.angle = angle;
        k.response = (float)lvl_r[(size_t)img * out_stride + loo + i];
        k.octave = lvl;
        k.class_id = -1;
        kps[(size_t)img * capacity + o] = k;
    }
}

// ---------------------------------------------------------------------------------------------
// k_describe_sb: IC angle + steered BRIEF with the Gaussian blur taken at the BRIEF sample points (no blurred pyramid)
// ---------------------------------------------------------------------------------------------
// The pinned GaussianBlur (7 x 7, sigma 2, taps {18,34,49,55,49,34,18}, REFLECT_101; ORBextractor.cc:1085-1086,
// DESIGN §2) is exact integer arithmetic rounded once: out = (sum_ij k_i k_j p + 2^15) >> 16, so its two passes can run
// in either order and the second one only where computeOrbDescriptor reads (:108-147, the 512 rotated sample points,
// |offset| <= kBriefR).  Per keypoint, the whole wave:
//   pass 1, matrix cores: H = R K over the raw 43 x 43 window (rows cy-21..cy+21, columns cx-21..cx+21; keypoints lie
//     >= 19 px inside the level, so the REFLECT_101 rows and columns are at most 2 px outside it).  H column c (0..36,
//     raw column cx-18+c) is the horizontal 7-tap sum over raw window columns c..c+6, H row h the raw row cy-21+h.  As
//     3 x 3 tiles of v_mfma_i32_16x16x64_i8: A = the raw bytes - 128 (the i8 range; lane groups 2 s, 2 s + 1 hold
//     keypoint s's raw columns 16 (nt + g % 2) .. +15 of tile column nt, zeros past the window's third chunk), B = the
//     tap band of keypoint s (constant; element e of group 2 s + h is tap 16 h + e - n, the other groups zero), C = 0;
//     adding 128 * 257 to each packed u16 half gives the exact horizontal sum (<= 255 * 257).  A and B share the k labelling and the C map is col = lane & 15, row = 4 (lane >> 4) + reg
//     (scripts/micro/mx_probe.hip).  H is stored column-major in the wave's LDS slice: kSbRows u16 per column.
//   pass 2, vector ALU: the blurred pixel at (ry, rx) is (sum_j k_j H[rx + 18][ry + 18 + j] + 2^15) >> 16 -- 7
//     consecutive u16 of one column: two ds_read2_b32 from the even row at or above, the u16 pairs realigned by
//     v_alignbit when the first row is odd, and four v_dot2_u32_u16 against the tap pairs, accumulated from 2^15.  The blurred value saturates at 255 (taps summing to 257: (S >> 16) reaches 257), so a test (a < b on the
//     rounded, saturated values) is S_a < min(S_b & ~0xffff, 255 << 16): an S_a of 256 << 16 or more fails it as its
//     saturated 255 must.
// The IC moments and the BRIEF tests run as in k_describe_m<2> (32 lanes per keypoint); the raw window loads of both
// keypoints share one A operand (lanes 32 s .. 32 s + 31 hold keypoint s's rows), and each keypoint has its own H slice.
constexpr int kSbRows = 44;                       // u16 rows per H column: rows 0..43 (a sample reads r0 .. r0 + 7)
constexpr int kSbCols = 2 * kBriefR + 1;          // 37 H columns
constexpr int kSbSlice = kSbCols * kSbRows * 2;   // 3,256 B of LDS per keypoint, two per wave
constexpr int kSbC0 = 128 * 257;                  // 128 * (sum of the taps): undoes the -128 of the i8 operand
#ifndef ORBX_SB_BATCH
#define ORBX_SB_BATCH 4
#endif
constexpr int kSbBatch = ORBX_SB_BATCH;           // BRIEF tests per lane whose sample reads are issued together (1, 2, 4)
struct BlurBandTab { uint32_t w[2 * 64 * 4]; };   // per keypoint s of a wave and lane: the 16 B operand of its tap band
constexpr BlurBandTab make_blur_band() {
    BlurBandTab t{};
    constexpr int taps[7] = {18, 34, 49, 55, 49, 34, 18};
    for (int s = 0; s < 2; ++s)
        for (int l = 0; l < 64; ++l)
            for (int e = 0; e < 16; ++e) {
                const int g = l >> 4, n = l & 15, i = 16 * (g & 1) + e - n;
                const uint32_t v = ((g >> 1) == s && i >= 0 && i < 7) ? (uint32_t)taps[i] : 0u;
                t.w[(s * 64 + l) * 4 + e / 4] |= v << (8 * (e & 3));
            }
    return t;
}
__constant__ __attribute__((aligned(16))) BlurBandTab c_blur_band = make_blur_band();

__global__ __launch_bounds__(256) void k_describe_sb(const uint8_t* __restrict__ pyr, size_t pyr_stride,
                                                     const LevelDev* __restrict__ levels, int nlevels,
                                                     const uint32_t* __restrict__ lvl_xy, const uint8_t* __restrict__ lvl_r,
                                                     int out_stride, const int* __restrict__ level_cnt,
                                                     orbx_keypoint* __restrict__ kps, uint8_t* __restrict__ desc,
                                                     int32_t* __restrict__ counts, int capacity, int slot0, int nslots,
                                                     int write_count, int batch, Src0 s0, SlotTable tab, unsigned seq,
                                                     int* __restrict__ err) {
    constexpr int kKpw = 2, kLp = 32;
    constexpr int kIcItems = 4 * (2 * kHalfPatch + 1);           // 31 rows x 4 chunks (124)
    constexpr int kNI = (kIcItems + kLp - 1) / kLp;              // IC chunks per lane
    typedef int v4i __attribute__((ext_vector_type(4)));
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    __shared__ __attribute__((aligned(16))) uint8_t hbuf[4 * kKpw * kSbSlice];
    const int per_wg = 4 * kKpw;
    const int nbx = (nslots + per_wg - 1) / per_wg;
    const int item = xcd_item(xcd_chunk(nbx * batch));
    if (item >= nbx * batch) return;
    const int img = item / nbx;
    const int wrel = __builtin_amdgcn_readfirstlane(((item - img * nbx) * blockDim.x + threadIdx.x) >> 6);
    if (wrel * kKpw >= nslots) return;                           // whole wave
    const int ln = lane_id();
    const int sub = ln / kLp, lk = ln - sub * kLp;
    const int rel = wrel * kKpw + sub;
    const int slot = slot0 + rel;
    int lvl = 0;
    for (int l = 1; l < nlevels; ++l) lvl += slot >= tab.out_off[l] ? 1 : 0;
    const int* lcs = level_cnt + img * nlevels;
    int off = 0, total = 0;
    for (int l = 0; l < nlevels; ++l) {
        const int c = lcs[l] & 0xffff;
        off += l < lvl ? c : 0;
        total += c;
    }
    const int craw = lcs[lvl], ci = craw & 0xffff;
    if (__ballot(rel < nslots && lvl_stale(craw, seq)) && ln == 0) atomicOr(err, kErrStale);
    if (write_count && wrel == 0 && ln == 0) counts[img] = min(total, capacity);
    const LevelDev& L = levels[lvl];
    const int lpo = L.pyr_off, loo = L.out_off;
    const int i = slot - loo;
    const int o = off + i;
    const bool valid = rel < nslots && i < ci && o < capacity;
    const uint64_t vmask = __ballot(valid);
    if (vmask == 0) return;                                      // whole wave

    const uint32_t xy = valid ? lvl_xy[(size_t)img * out_stride + loo + i] : 0u;
    const int cx = (int)(xy & 0xffff), cy = (int)(xy >> 16);
    const uint8_t* P = lvl == 0 ? s0.p + img * s0.istride : pyr + img * pyr_stride + lpo;
    const int pstride = lvl == 0 ? (int)s0.step : L.w;
    // IC_Angle (:77-104), as k_describe_m<2>
    int m10 = 0, m01 = 0;
    {
        uint64_t ic[kNI];
        const uint8_t* p0 = P + (size_t)(cy - kHalfPatch) * pstride + (cx - kHalfPatch);
        if (valid) {
#pragma unroll
            for (int k = 0; k < kNI; ++k) {
                const int q = lk + kLp * k, r = min(q >> 2, 2 * kHalfPatch);
                __builtin_memcpy(&ic[k], p0 + (size_t)r * pstride + 8 * (q & 3), 8);
            }
        }
#pragma unroll
        for (int k = 0; k < kNI; ++k) {
            const int q = lk + kLp * k;
            const int v = (q >> 2) - kHalfPatch;
            const int u0 = 8 * (q & 3) - kHalfPatch;
            const uint64_t m = valid ? c_ic_mask.m[k][lk] : 0ull;
            const uint64_t px = ic[k] & m;
            const uint32_t a = (uint32_t)px, b = (uint32_t)(px >> 32);
            const uint32_t wa = (uint32_t)(u0 + 16) * 0x01010101u + 0x03020100u, wb = wa + 0x04040404u;
            const int dot = (int)__builtin_amdgcn_udot4(b, wb, __builtin_amdgcn_udot4(a, wa, 0u, false), false);
            const int sum = (int)__builtin_amdgcn_udot4(b, 0x01010101u, __builtin_amdgcn_udot4(a, 0x01010101u, 0u, false), false);
            m10 += dot - 16 * sum;
            m01 += v * sum;
        }
    }
    m10 = group_sum<kLp>(m10, sub);
    m01 = group_sum<kLp>(m01, sub);
    const float angle = fast_atan2_deg((float)m01, (float)m10);
    const float ang = __fmul_rn(angle, (float)(M_PI / 180.f));
    float sa, sb;
    orbx_sincos_brief(ang, &sa, &sb);

    uint8_t* hb = hbuf + (threadIdx.x >> 6) * kKpw * kSbSlice;
    const int g = ln >> 4, n16 = ln & 15;
    // ---- pass 1 operands of BOTH keypoints, loaded once: lanes 32 sub + 16 gh + n (gh = g & 1) hold raw window row
    // 16 mt + n of keypoint sub, columns 16 (nt + gh) .. +15.  Keypoint s's product takes band s, whose taps sit in
    // lane groups 2 s, 2 s + 1 (the other keypoint's bytes meet zeros), so one A operand serves both.
    v4i a[3][3];
    {
        const int gh = g & 1;
        const int ws = L.w, hs = L.h;
        // chunks reach raw columns cx-21 .. cx+26; closer to a level edge every byte is placed by REFLECT_101
        const bool edge = cx < kBriefR + 3 || cx + 26 > ws - 1;
#pragma unroll
        for (int mt = 0; mt < 3; ++mt) {
            int y = cy - (kBriefR + 3) + min(16 * mt + n16, 2 * kBriefR + 6);
            y = y < 0 ? -y : (y > hs - 1 ? 2 * (hs - 1) - y : y);
            const uint8_t* rowp = P + (size_t)y * pstride;
#pragma unroll
            for (int nt = 0; nt < 3; ++nt) {
                const int cc = nt + gh;                           // 16-column chunk of the window
                a[mt][nt] = v4i{0, 0, 0, 0};
                if (valid && cc < 3) {
                    const int x0 = cx - (kBriefR + 3) + 16 * cc;
                    if (!edge) {
                        __builtin_memcpy(&a[mt][nt], rowp + x0, 16);
                    } else {
                        int wv[4];
#pragma unroll 1
                        for (int d = 0; d < 4; ++d) {
                            uint32_t v = 0;
                            for (int e = 0; e < 4; ++e) {
                                int x = x0 + 4 * d + e;
                                x = x < 0 ? -x : (x > ws - 1 ? 2 * (ws - 1) - x : x);
                                x = min(max(x, 0), ws - 1);           // columns past cx+21 have zero taps
                                v |= (uint32_t)rowp[x] << (8 * e);
                            }
                            wv[d] = (int)v;
                        }
                        a[mt][nt] = v4i{wv[0], wv[1], wv[2], wv[3]};
                    }
                    a[mt][nt] ^= (int)0x80808080;
                }
            }
        }
    }
    // ---- pass 1: H = R K on the matrix cores for both keypoints, each into its own LDS slice, column-major
#pragma unroll
    for (int mt = 0; mt < 3; ++mt) {
        const int r0 = 16 * mt + 4 * g;
#pragma unroll
        for (int nt = 0; nt < 3; ++nt) {
            const int c = 16 * nt + n16;
#pragma unroll
            for (int s = 0; s < kKpw; ++s) {
                const v4i band = *reinterpret_cast<const v4i*>(&c_blur_band.w[(s * 64 + ln) * 4]);
                // C = 0 (an inline operand): the tile is H - 128 * 257; the u16 halves get 128 * 257 back after packing
                const v4i acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[mt][nt], band, v4i{0, 0, 0, 0}, 0, 0, 0);
                if (c < kSbCols && r0 < kSbRows) {
                    const u16x2 off = {kSbC0, kSbC0};
                    const u16x2 lo = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm((uint32_t)acc.y, (uint32_t)acc.x, 0x05040100u)) + off;
                    const u16x2 hi = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm((uint32_t)acc.w, (uint32_t)acc.z, 0x05040100u)) + off;
                    *reinterpret_cast<uint2*>(hb + s * kSbSlice + c * (2 * kSbRows) + 2 * r0) =
                        make_uint2(__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi));
                }
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // ---- pass 2 + BRIEF, 32 lanes per keypoint (tests g * 32 + lk, as k_describe_m<2>): the vertical taps at the two
    // sample points of each test, read from the lane's keypoint's slice
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    const f32x2 ab1 = {sb, sa}, ab2 = {sa, -sb}, magic = {12582912.0f, 12582912.0f};
    // u16 H[rx + 18][ry + 18] from the magic-constant bits (see k_describe_m): the i24 product t is
    // (0x400000 + rx) * kSbRows + 0x4B400000 + ry, so t - kSbMagic is the element index; kSbMagic is even, so t's parity
    // is the row's, and the dword at or above it is at byte 2 (t & ~1) - 2 kSbMagic
    constexpr uint32_t kSbMagic = 0x400000u * (uint32_t)kSbRows + 0x4B400000u - (uint32_t)(kBriefR * kSbRows + kBriefR);
    static_assert((kSbMagic & 1u) == 0u, "row parity from t");
    // (an LDS-typed pointer: 32-bit offsets on the LDS address itself; a generic pointer cast to an integer would be
    // the flat address, whose aperture bits a 32-bit truncation loses)
    const lds_u8* hsl = (const lds_u8*)(hb + sub * kSbSlice);
    const u16x2 t01 = {18, 34}, t23 = {49, 55}, t45 = {49, 34}, t6 = {18, 0};
    constexpr int kNT = 256 / kLp;
    uint32_t pat[kNT];
    {
        const uint32_t* pw = c_pattern_l32.w + lk * kNT;
#pragma unroll
        for (int q = 0; q < kNT; q += 4) __builtin_memcpy(&pat[q], pw + q, 16);
    }
    uint32_t words[kNT];
#pragma unroll
    for (int q0 = 0; q0 < kNT; q0 += kSbBatch) {
        uint32_t S[kSbBatch][2];
#pragma unroll
        for (int qb = 0; qb < kSbBatch; ++qb) {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const uint32_t w = pat[q0 + qb];
                const float fx = (float)(int)(signed char)(w >> (16 * e)), fy = (float)(int)(signed char)(w >> (16 * e + 8));
                const f32x2 fxy = {fx, fy};
                f32x2 p, qq, r;
                asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(p) : "v"(fxy), "v"(ab1));              // {fx b, fx a}
                asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]" : "=v"(qq) : "v"(fxy), "v"(ab2)); // {fy a, -fy b}
                asm("v_pk_add_f32 %0, %1, %2" : "=v"(r) : "v"(p), "v"(qq));                                 // {ry, rx}
                asm("v_pk_add_f32 %0, %1, %2" : "=v"(p) : "v"(r), "v"(magic));                              // + M
                const float ryM = p.x, rxM = p.y;
                int t;
                asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(t) : "v"(__float_as_int(rxM)), "n"(kSbRows), "v"(__float_as_int(ryM)));
                // 4-byte-aligned reads from the even row at or above r0 (a 32-bit LDS read off its 4-byte alignment returns
                // the right bytes but is replayed: r6b, 3.5 ms against 0.67), then the u16 pairs realigned by 16 bits
                // when r0 is odd (v_alignbit reads the low 5 bits of the shift: t << 4 is 16 or 0)
                const lds_u32* hp = (const lds_u32*)(hsl + (2u * ((uint32_t)t & ~1u) - 2u * kSbMagic));
                const uint32_t d0 = hp[0], d1 = hp[1], d2 = hp[2], d3 = hp[3], sh = (uint32_t)t << 4;
                uint32_t acc = 0x8000u;
                acc = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, __builtin_amdgcn_alignbit(d1, d0, sh)), t01, acc, false);
                acc = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, __builtin_amdgcn_alignbit(d2, d1, sh)), t23, acc, false);
                acc = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, __builtin_amdgcn_alignbit(d3, d2, sh)), t45, acc, false);
                acc = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, __builtin_amdgcn_alignbit(d3, d3, sh)), t6, acc, false);
                S[qb][e] = acc;
            }
        }
#pragma unroll
        for (int qb = 0; qb < kSbBatch; ++qb) {
            const uint64_t bm = __ballot(S[qb][0] < min(S[qb][1] & 0xffff0000u, 0x00ff0000u));
            words[q0 + qb] = (uint32_t)(bm >> (sub * kLp));
        }
    }
    if (!valid) return;
    uint32_t dw = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) dw = lk == j ? words[j] : dw;
    if (lk < 8) reinterpret_cast<uint32_t*>(desc + ((size_t)img * capacity + o) * 32)[lk] = dw;
    if (lk == 0) {
        orbx_keypoint k;
        float x = (float)cx, y = (float)cy;
        if (lvl != 0) { x = __fmul_rn(x, L.scale); y = __fmul_rn(y, L.scale); }
        k.x = x; k.y = y;
        k.size = (float)L.patch;
        k.angle = angle;
        k.response = (float)lvl_r[(size_t)img * out_stride + loo + i];
        k.octave = lvl;
        k.class_id = -1;
        kps[(size_t)img * capacity + o] = k;
    }
}

// =============================================================================================
// host side
// =============================================================================================
__global__ void k_debug_spin(unsigned long long ticks) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(32);
}

hipError_t debug_spin(hipStream_t stream, double ms) {
    ms = std::min(std::max(ms, 0.0), 2000.0);
    hipLaunchKernelGGL(k_debug_spin, dim3(1), dim3(64), 0, stream, (unsigned long long)(ms * 1e5));
    return hipGetLastError();
}

static int round_even_f(float v) { return (int)std::nearbyintf(v); }
static int round_even_d(double v) { return (int)std::nearbyint(v); }

// Stage spans per call (HIP events on the stream each launch is issued on).  The *_busy entries are the union of a
// kernel family's two launches (level 0 on the side stream, levels >= 1 on the launch stream), which overlap each
// other: the wall time during which that kernel is running, <= the sum of the two spans.
enum Stage { ST_RESIZE = 0, ST_FAST, ST_BLUR, ST_QUADTREE, ST_DESCRIBE, ST_FAST_L0, ST_QUADTREE_L0, ST_FAST_BUSY,
             ST_QUADTREE_BUSY, ST_COUNT };
static const char* kStageNames[ST_COUNT] = {"resize", "fast_cells", "blur7", "quadtree", "describe", "fast_cells_l0",
                                            "quadtree_l0", "fast_busy", "quadtree_busy"};
constexpr int kSpanStages = ST_FAST_BUSY;   // stages [0, kSpanStages) are single event pairs

struct Extractor {
    // ORBextractor parameters and tables (:410-470)
    int nfeatures, nlevels, iniTh, minTh;
    double scaleFactor;
    std::vector<float> scale, invScale, sigma2, invSigma2;
    std::vector<int> nPerLevel;
    int umax[16];
    int device = 0;
    hipStream_t stream = nullptr;    // own stream of the host API, created on first use (lazy_stream)
    std::once_flag stream_once;
    hipStream_t own() { return lazy_stream(stream, stream_once, device); }
    bool own_stream = false;
    // Two-stream schedule (run_batch).  Level 0 of the pyramid is the caller's image, so FAST, DistributeOctTree
    // and the blur of level 0 need nothing from the resize chain: they run on a side stream while the launch stream
    // builds levels 1..7 (seven dependent, latency-bound resize launches) and runs FAST / DistributeOctTree on them.
    // The side stream then blurs levels 1..7 once the pyramid is done; k_describe joins both.
    hipStream_t side = nullptr;
    // Per-call events come from a pool (CallEvents below): an event is recorded again only 32 calls later, never
    // while a wait on its previous record may still be in flight.
    int pipeline = 1;         // ORBX_PIPELINE: 1 two streams (above), 0 every launch in order on the launch stream
    // Describe stream (orbx_extract_batch_device_split): k_describe runs on the caller's output stream, so the next
    // call's front half (resize chain, FAST) on the input stream overlaps this call's describe.  What the next call
    // overwrites that describe reads is ordered by events: the kept keypoints and the blurred pyramid (its quadtree
    // and blur wait for the previous call's describe) and its pyramid set (the resize chain waits for that set's last
    // describe).
    static constexpr int kCallEv = 32;
    struct CallEvents {
        hipEvent_t fork, pyr, join, front, desc, qt;      // fork from the caller, pyramid built, side join,
        bool used;                                         // launch-stream FAST / quadtree, describe done, levels
                                                           // 1..n-1 quadtree on the output stream (qt_out)
    };
    CallEvents cev[kCallEv] = {};
    unsigned long long cev_next = 0;
    unsigned call_seq = 0;                                 // per-call stamp of the ordering canary (lvl_stale)
    int dbg_skip_desc_wait = 0;   // ORBX_DEBUG_SKIP_DESC_WAIT=1 (tests only): drop the quadtree's wait for the previous
                                  // describe, i.e. remove an ordering edge on purpose so the canary must fire
    int slot_call[8] = {-1, -1, -1, -1, -1, -1, -1, -1};   // per pyramid set: pool index of its last describe
    // Host API (orbx_extract): the whole call -- H2D copy, run_batch's kernels on both streams, D2H copies -- is
    // captured once per configuration as a hipGraph and replayed, one launch per call instead of ~25 stream operations.
    // A replay is synchronised before orbx_extract returns, so it leaves no edge for later calls to wait on.
    hipGraph_t hgraph = nullptr;
    hipGraphExec_t hgexec = nullptr;
    bool capturing = false;       // run_batch inside the capture: no waits on earlier calls, no host synchronisation
    bool host_graph = true;       // ORBX_HOST_GRAPH=0: the host API issues its stream operations every call (A/B)
    // ORBX_HOST_SERIAL=0: the host API's one-image calls fork the level-0 branch onto the side stream like the batches.
    // Serial by default: two extractors called from two threads (Frame.cc:78-81) then use one hardware queue each
    // instead of sharing the process's 4 among four streams (r4haf: 0.370 -> 0.297 ms per stereo frame, median)
    bool host_serial = true;
    bool host_merged = true;      // ORBX_HOST_MERGED=0: serial host calls keep the level-0 / levels >= 1 launch split
    bool async_pending = false;   // a device-API call may still run: the next replay first waits for every describe
    uint8_t* hg_pyr = nullptr;    // the pyramid set the graph's kernels write
    void drop_graph() {
        if (hgexec) (void)hipGraphExecDestroy(hgexec);
        if (hgraph) (void)hipGraphDestroy(hgraph);
        hgexec = nullptr;
        hgraph = nullptr;
    }
    int last_call = -1;                                    // pool index of the previous call, -1 none
    int sync_calls() {                                     // every describe issued so far is done
        for (auto& c : cev)
            if (c.used) ORBX_HIP(hipEventSynchronize(c.desc));
        return ORBX_OK;
    }

    // geometry for the reserved size
    int rows = 0, cols = 0, max_batch = 0;
    std::vector<LevelDev> lv;
    std::vector<CellDev> cellv;
    std::vector<BlurTile> tilev;
    size_t pyr_size = 0;      // bytes per image pyramid
    int cand_stride = 0;      // candidate slots per image
    int out_stride = 0;       // quadtree output slots per image
    int node_cap = 0;
    // k_fast_wave: one wave per (cell, image), 4 waves per workgroup; launch 0 = level 0, launch 1 = levels >= 1, each
    // wave's LDS slice sized for its launch's largest cell
    struct WaveLaunch { int cell0, n, ps, pc, kcap; WaveLds lay; };   // ps / pc: pair-image row stride / pad (fastw_row)
    WaveLaunch wave_launch[3] = {};   // level 0, levels 1..n-1, all levels (the host API's one-launch-per-stage form)
#ifndef ORBX_FAST_WPG
#define ORBX_FAST_WPG 4
#endif
    static constexpr int kWaveWpg = ORBX_FAST_WPG;   // (1 or 2 waves per workgroup: faster alone, slower in the step)
    int wave_twopass = 1;     // iniTh first, minTh only for the cells left empty (0: one pass at min(iniTh, minTh))
    std::vector<int> tile_off;   // blur tiles of level l: [tile_off[l], tile_off[l + 1])
    int scan_cap = 0;         // scan arrays: >= nodes, cells of a level, roots
    size_t qt_lds = 0;        // k_quadtree dynamic LDS bytes of the node arrays (the key region follows at this offset)
    int qt_keys[2] = {0, 0};  // LDS-resident key capacity of the level-0 launch / the levels 1..n-1 launch
    int qt_prev = -1;         // call event set whose ce.qt the next FAST of levels >= 1 waits for (qt_out)
    int qt_out = 1;           // levels 1..n-1 quadtree on the output stream when it differs (ORBX_QT_OUT=0: the launch
                              // stream, the round-4 schedule)
    int out_capacity = 0;     // max keypoints per image

    // device buffers
    LevelDev* d_levels = nullptr;
    CellDev* d_cells = nullptr;
    BlurTile* d_tiles = nullptr;
    std::vector<ResizeTab> rtab;
    std::vector<ResizeVec> rvec;      // per level: vectorised tables (groups == 0 -> use rtab)
    std::vector<void*> rtab_mem;
    uint8_t* d_pyr = nullptr;         // pyramid set of the current / last call (a slot of d_pyr_ring)
    uint8_t* d_pyr_ring = nullptr;    // pyr_ring sets of max_batch pyramids: a caller that reads the pyramid of call
    int pyr_ring = 1;                 // k (Frame::ComputeStereoMatches' SAD step) on another stream can overlap call
    unsigned long long ncalls = 0;    // k+1, which writes the next set
    uint8_t* d_blur = nullptr;        // desc_sets sets of the blurred pyramid / kept keypoints (d_*_c: the current call's)
    uint8_t* d_blur_c = nullptr;
    // k_describe_sb (blur at the BRIEF sample points) instead of k_blur7 + k_describe_m: no blurred pyramid is kept
    // (ORBX_DESC_SB, read at create)
    bool desc_sb = false;
    int resize_tail = 0;              // ORBX_RESIZE_TAIL=l (>= 2): levels l .. n-1 in one k_resize_tail launch
    uint8_t* d_blur_diag = nullptr;   // one image's blurred pyramid, made on demand by orbx_extractor_copy_blurred_level
    int desc_sets = 2;                // call k + 1's blur and DistributeOctTree write the other set
    unsigned long long dcalls = 0;    // while call k's describe reads its own (no wait on that describe)
    int dset_call[2] = {-1, -1};      // event-pool index of the last call that used each set
    uint32_t* d_cand_xy = nullptr;
    uint8_t* d_cand_s = nullptr;
    int* d_cell_cnt = nullptr;
    uint32_t* d_key_xy = nullptr;
    uint8_t* d_key_r = nullptr;
    int16_t* d_key_node = nullptr;
    uint32_t* d_lvl_xy = nullptr;
    uint8_t* d_lvl_r = nullptr;
    int* d_lvl_cnt = nullptr;
    uint32_t* d_lvl_xy_c = nullptr;
    uint8_t* d_lvl_r_c = nullptr;
    int* d_lvl_cnt_c = nullptr;
    int* d_err = nullptr;
    // host-API staging: the image is packed into pinned host memory and goes over PCIe as one DMA (a pageable
    // 2-D copy of an odd-width image falls back to per-row transfers); results come back through pinned memory
    uint8_t* d_in = nullptr;
    size_t in_bytes = 0;
    uint8_t* h_in = nullptr;
    uint8_t* h_out = nullptr;      // pinned: count | keypoints | descriptors of one image
    size_t h_out_bytes = 0;
    uint8_t* d_hblk = nullptr;      // host API outputs on the device, laid out as h_out: count, keypoints, descriptors
    orbx_keypoint* d_kps = nullptr; // (pointers into d_hblk: one D2H copy brings all three back)
    uint8_t* d_desc = nullptr;
    int32_t* d_cnt = nullptr;
    int last_batch = 0;
    Src0 last_src0{nullptr, 0, 0};   // level 0 of the last device call = the caller's images

    // timing: a pool of event sets recorded on the launch streams, resolved lazily (no host sync per call).
    // Launch stream: 0 start, 1 pyramid done, 10 FAST (levels >= 1) start, 2 its end, 3 quadtree (levels >= 1) done,
    // 4 describe start (after the join), 5 describe done.  Side stream: 6 start, 7 FAST level 0 done, 8 quadtree
    // level 0 done, 9 blur done (level 0, the wait for the pyramid, levels >= 1; pure blur time when serial).
    static constexpr int kEvents = 11;
    static constexpr int kStageEv[kSpanStages][2] = {{0, 1}, {10, 2}, {8, 9}, {2, 3}, {4, 5}, {6, 7}, {7, 8}};
    struct EventSet { hipEvent_t ev[kEvents]; bool pending; };
    bool timing = false;
    std::vector<EventSet> tpool;
    size_t tnext = 0;
    double stage_ms[ST_COUNT] = {};
    int timed_calls = 0;
    int resolve(EventSet& es) {
        if (!es.pending) return ORBX_OK;
        ORBX_HIP(hipEventSynchronize(es.ev[5]));
        ORBX_HIP(hipEventSynchronize(es.ev[9]));
        for (int k = 0; k < kSpanStages; ++k) {
            float ms = 0;
            ORBX_HIP(hipEventElapsedTime(&ms, es.ev[kStageEv[k][0]], es.ev[kStageEv[k][1]]));
            stage_ms[k] += ms;
        }
        // union of two spans [a, b] (level 0) and [c, d] (levels >= 1), all relative to a
        auto busy = [&](int a, int b, int c, int d, double& acc) -> int {
            float tb = 0, tc = 0, td = 0;
            ORBX_HIP(hipEventElapsedTime(&tb, es.ev[a], es.ev[b]));
            ORBX_HIP(hipEventElapsedTime(&tc, es.ev[a], es.ev[c]));
            ORBX_HIP(hipEventElapsedTime(&td, es.ev[a], es.ev[d]));
            const double overlap = std::max(0.0, (double)std::min(tb, td) - (double)std::max(0.f, tc));
            acc += (double)tb + ((double)td - (double)tc) - overlap;
            return ORBX_OK;
        };
        if (int st = busy(6, 7, 10, 2, stage_ms[ST_FAST_BUSY])) return st;
        if (int st = busy(7, 8, 2, 3, stage_ms[ST_QUADTREE_BUSY])) return st;
        es.pending = false;
        timed_calls++;
        return ORBX_OK;
    }

    void free_buffers();
    int configure(int r, int c, int batch);
};

static void compute_tables(Extractor* e) {
    const int nl = e->nlevels;
    e->scale.assign(nl, 1.0f);
    e->sigma2.assign(nl, 1.0f);
    for (int i = 1; i < nl; ++i) {
        e->scale[i] = (float)((double)e->scale[i - 1] * e->scaleFactor);
        e->sigma2[i] = e->scale[i] * e->scale[i];
    }
    e->invScale.resize(nl);
    e->invSigma2.resize(nl);
    for (int i = 0; i < nl; ++i) {
        e->invScale[i] = 1.0f / e->scale[i];
        e->invSigma2[i] = 1.0f / e->sigma2[i];
    }
    const float factor = (float)(1.0f / e->scaleFactor);
    float want = (float)e->nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nl));
    e->nPerLevel.assign(nl, 0);
    int acc = 0;
    for (int l = 0; l < nl - 1; ++l) {
        e->nPerLevel[l] = round_even_f(want);
        acc += e->nPerLevel[l];
        want *= factor;
    }
    e->nPerLevel[nl - 1] = std::max(e->nfeatures - acc, 0);
    const int R = kHalfPatch;
    const int vmax = (int)std::floor(R * std::sqrt(2.f) / 2 + 1);
    const int vmin = (int)std::ceil(R * std::sqrt(2.f) / 2);
    for (int v = 0; v <= vmax; ++v) e->umax[v] = round_even_d(std::sqrt((double)R * R - v * v));
    for (int v = R, v0 = 0; v >= vmin; --v) {
        while (e->umax[v0] == e->umax[v0 + 1]) ++v0;
        e->umax[v] = v0;
        ++v0;
    }
}

static void level_dims(const Extractor* e, int rows, int cols, int l, int* w, int* h) {
    *w = round_even_f((float)cols * e->invScale[l]);
    *h = round_even_f((float)rows * e->invScale[l]);
}

void Extractor::free_buffers() {
    drop_graph();                                          // it names the buffers freed below
    auto F = [](auto*& p) { if (p) { (void)hipFree((void*)p); p = nullptr; } };
    F(d_levels); F(d_cells); F(d_tiles); F(d_pyr_ring); F(d_blur); F(d_blur_diag); F(d_cand_xy); F(d_cand_s); F(d_cell_cnt);
    F(d_key_xy); F(d_key_r); F(d_key_node); F(d_lvl_xy); F(d_lvl_r); F(d_lvl_cnt); F(d_err); F(d_in);
    F(d_hblk);
    d_kps = nullptr; d_desc = nullptr; d_cnt = nullptr;
    d_pyr = nullptr;                                       // a slot of the freed ring
    if (h_in) { (void)hipHostFree(h_in); h_in = nullptr; }
    if (h_out) { (void)hipHostFree(h_out); h_out = nullptr; }
    h_out_bytes = 0;
    for (void* p : rtab_mem) (void)hipFree(p);
    rtab_mem.clear();
    rtab.clear();
    rvec.clear();
    rows = cols = max_batch = 0;
    in_bytes = 0;
    d_pyr = nullptr;
}

static size_t qt_lds_bytes(int cap, int scan_cap);

template <typename T>
static int dev_alloc(T** p, size_t count) {
    ORBX_HIP(hipMalloc((void**)p, std::max<size_t>(count, 1) * sizeof(T)));
    return ORBX_OK;
}

int Extractor::configure(int r, int c, int batch) {
    if (r == rows && c == cols && batch <= max_batch) return ORBX_OK;
    ORBX_HIP(hipSetDevice(device));
    ::orbx::LegacyLock legacy_;                              // frees, synchronous uploads and memsets below
    ORBX_HIP(::orbx::device_sync());                       // callers' streams may still read the buffers freed below
    for (int& k : slot_call) k = -1;
    last_call = -1;
    const int keep_batch = std::max(batch, (r == rows && c == cols) ? max_batch : 0);
    free_buffers();
    ORBX_REQUIRE(r > 0 && c > 0 && batch > 0, ORBX_ERR_ARG, "configure: bad size %dx%d batch %d", r, c, batch);
    ORBX_REQUIRE(c < 32768 && r < 32768, ORBX_ERR_UNSUPPORTED, "image too large (%dx%d)", r, c);
    batch = keep_batch;

    // ---- level geometry, cells (ComputeKeyPointsOctTree :771-807), DistributeOctTree roots (:543-545)
    lv.assign(nlevels, LevelDev{});
    cellv.clear();
    tilev.clear();
    tile_off.clear();
    size_t poff = 0;
    int cand = 0, outs = 0, cap = 4;
    for (int l = 0; l < nlevels; ++l) {
        LevelDev& L = lv[l];
        level_dims(this, r, c, l, &L.w, &L.h);
        ORBX_REQUIRE(L.w > 0 && L.h > 0, ORBX_ERR_UNSUPPORTED, "level %d is empty for %dx%d", l, r, c);
        L.pyr_off = (int)poff;
        poff += (size_t)L.w * L.h;
        L.scale = scale[l];
        L.patch = (int)(31 * scale[l]);
        L.N = nPerLevel[l];
        const int minB = kEdge - 3, maxBX = L.w - kEdge + 3, maxBY = L.h - kEdge + 3;
        L.win_w = maxBX - minB;
        L.win_h = maxBY - minB;
        L.cell_begin = (int)cellv.size();
        L.cand_off = cand;
        const float width = (float)(maxBX - minB), height = (float)(maxBY - minB);
        const int nCols = (int)(width / 30.f), nRows = (int)(height / 30.f);
        if (nCols > 0 && nRows > 0 && L.win_w > 0 && L.win_h > 0) {
            const int wCell = (int)std::ceil(width / nCols), hCell = (int)std::ceil(height / nRows);
            for (int i = 0; i < nRows; ++i) {
                const float iniY = (float)(minB + i * hCell);
                float maxY = iniY + hCell + 6;
                if (iniY >= maxBY - 3) continue;
                if (maxY > maxBY) maxY = (float)maxBY;
                for (int j = 0; j < nCols; ++j) {
                    const float iniX = (float)(minB + j * wCell);
                    float maxX = iniX + wCell + 6;
                    if (iniX >= maxBX - 6) continue;
                    if (maxX > maxBX) maxX = (float)maxBX;
                    CellDev cd{};
                    cd.level = l;
                    cd.x0 = (int)iniX; cd.y0 = (int)iniY;
                    cd.W = (int)maxX - cd.x0; cd.H = (int)maxY - cd.y0;
                    ORBX_REQUIRE(cd.W <= kMaxRoi && cd.H <= kMaxRoi, ORBX_ERR_UNSUPPORTED, "cell ROI too large");
                    ORBX_REQUIRE((cd.H - 6) * ((cd.W - 5) / 2) <= 8 * 256, ORBX_ERR_UNSUPPORTED, "cell too large");
                    const int wd = std::max(cd.W - 6, 0), hd = std::max(cd.H - 6, 0);
                    cd.slot_cap = ((wd + 1) / 2) * ((hd + 1) / 2);   // strict 3x3 NMS: <= 1 per 2x2 block
                    cd.slot_off = cand;
                    cand += cd.slot_cap;
                    cellv.push_back(cd);
                }
            }
        }
        L.cell_end = (int)cellv.size();
        L.cand_cap = cand - L.cand_off;
        // k_quadtree's phase-2 sort keys hold a node's key count in bits 40..63 (< 2^24 keys per level) and the key
        // gather stores a key's cell as int16 (< 2^15 cells per level); a 4K frame's level 0 has ~2.3M candidate slots
        // in ~8.8k cells
        ORBX_REQUIRE(L.cand_cap < (1 << 24), ORBX_ERR_UNSUPPORTED, "too many FAST candidates per level");
        ORBX_REQUIRE(L.cell_end - L.cell_begin < 32768, ORBX_ERR_UNSUPPORTED, "too many FAST cells per level");
        if (L.win_w > 0 && L.win_h > 0) {
            // nIni = 0 (window more than twice as tall as wide) is undefined in the reference; pinned to 1
            L.nIni = std::max(1, (int)std::round((float)(maxBX - minB) / (maxBY - minB)));
            L.hX = (float)(maxBX - minB) / L.nIni;
        } else {
            L.nIni = 1; L.hX = 1.f;
        }
        L.out_cap = std::max(L.N + 3, 4 * L.nIni + 1);
        L.out_off = outs;
        outs += L.out_cap;
        cap = std::max(cap, L.out_cap);
        // blur tiles
        tile_off.push_back((int)tilev.size());
        for (int ty = 0; ty < (L.h + kBlurBand - 1) / kBlurBand; ++ty)
            for (int tx = 0; tx < (L.w + kBlurStrip - 1) / kBlurStrip; ++tx) tilev.push_back(BlurTile{l, tx, ty, 0});
    }
    tile_off.push_back((int)tilev.size());
    ORBX_REQUIRE(cap < 32768 && cap < (1 << 20), ORBX_ERR_UNSUPPORTED, "node capacity %d too large", cap);
    // k_quadtree's phase 1 scans (children << 16 | survivors) in one int: children <= 4 * cap must stay below 2^15
    ORBX_REQUIRE(4 * cap < (1 << 15), ORBX_ERR_UNSUPPORTED, "node capacity %d too large for the packed split scan", cap);
    // k_fast_wave launches: level 0 (side stream) and levels 1..n-1, each wave's LDS slice sized for the launch's
    // largest cell.  Cells up to 38 px wide (every cell of the KITTI and EuRoC grids) use the padded 19-dword rows
    // (fastw_row: bank-conflict-free pre-test, 20 dwords per row on average against 24 before); wider ones 40-dword
    // rows, 16-byte aligned.
    for (int k = 0; k < 3; ++k) {
        WaveLaunch& wl = wave_launch[k];
        wl.cell0 = k == 1 ? lv[0].cell_end : 0;
        wl.n = k == 0 ? lv[0].cell_end : k == 1 ? (int)cellv.size() - lv[0].cell_end : (int)cellv.size();
        int rows = 8, sw = 8, np = 1, kcap = 1, lr = 1, psn = 1;
        for (int i = wl.cell0; i < wl.cell0 + wl.n; ++i) {
            const CellDev& cd = cellv[i];
            const int Wd = std::max(cd.W - 6, 0), Hd = std::max(cd.H - 6, 0);
            const int PR = (Wd + 1) / 2, QR = (PR + 3) / 4;
            rows = std::max(rows, cd.H);
            sw = std::max(sw, (Wd + 5) & ~1);
            np = std::max(np, Hd * PR);
            kcap = std::max(kcap, cd.slot_cap);
            lr = std::max({lr, (cd.W + 1) / 2, 4 * QR + 3});          // ROI words; quad reads up to 4 * QR + 2
            psn = std::max({psn, 4 * ((cd.W + 7) / 8), 4 * QR + 3});   // the same with 16-byte ROI chunks
        }
        ORBX_REQUIRE(psn <= 40, ORBX_ERR_UNSUPPORTED, "cell too wide for k_fast_wave");
        wl.ps = lr <= 19 ? 19 : 40;
        wl.pc = wl.ps == 19 ? 4 : 0;
        ORBX_REQUIRE(sw <= fastw_sw(wl.ps), ORBX_ERR_UNSUPPORTED, "k_fast_wave score-map row");
        sw = fastw_sw(wl.ps);
        const int iw = fastw_image_words(rows, wl.ps, wl.pc);
        wl.kcap = kcap;                                     // two u16 key lists inside the pair image: 4 * kcap bytes
        ORBX_REQUIRE(4 * kcap <= iw * 4, ORBX_ERR_UNSUPPORTED, "k_fast_wave key lists exceed the pair image");
        wl.lay = wave_lds(rows, fastw_scrow(wl.ps), np, iw);
        const int bytes = kWaveWpg * wl.lay.bytes;
        ORBX_REQUIRE(bytes <= 160 * 1024, ORBX_ERR_UNSUPPORTED, "k_fast_wave LDS %d B", bytes);
        if (bytes > 64 * 1024) {
            ORBX_HIP(hipFuncSetAttribute((const void*)k_fast_wave<19, 4, kWaveWpg>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
            ORBX_HIP(hipFuncSetAttribute((const void*)k_fast_wave<40, 0, kWaveWpg>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
        }
    }
    int scap = cap;
    for (const LevelDev& L : lv) scap = std::max(scap, std::max(L.cell_end - L.cell_begin, L.nIni));
    scan_cap = scap + 1;
    {
        const size_t lds = (qt_lds_bytes(cap, scan_cap) + 15) & ~(size_t)15;
        ORBX_REQUIRE(lds <= 160 * 1024, ORBX_ERR_UNSUPPORTED, "quadtree LDS %zu B exceeds 160 KiB", lds);
        qt_lds = lds;
        // LDS key region (7 B per key: xy, node, response) per launch: level 0 (one workgroup per image, ~2-4k keys on a
        // KITTI frame) and levels >= 1 (seven workgroups per image, ~1-1.5k keys at level 1), each bounded by the
        // largest candidate count its levels can produce; levels whose keys overflow it use the HBM scratch
        int lcap[2] = {0, 0};
        for (int l = 0; l < nlevels; ++l) lcap[l ? 1 : 0] = std::max(lcap[l ? 1 : 0], lv[l].cand_cap);
        // sized so that two level-0 workgroups (256 threads) and three of levels >= 1 share a CU's 160 KiB. The budget is
        // rounded down to 1,280 B, the allocation granule that fits the measured packing: levels >= 1 with 53,344 B per
        // workgroup run three per CU, with 53,792 B two (0.156 -> 0.212 ms alone, r4y), level 0 with 81,904 B two (r4x;
        // a 512 B granule would give three at 53,792 B, a 2 KiB one two at 53,344 B). No LDS keys at levels >= 1: 0.186 ms.
        // r5bg: level 0 at 3,072 LDS keys (62.7 KB per workgroup) instead of the two-per-CU budget's 5,808 (81.9 KB):
        // the rest in the HBM scratch, and the LDS the two workgroups leave on their CU goes to FAST beside them --
        // step +0.8 % (75.2k -> 75.8k frames/s; 0 / 1k / 2k / 4k keys 75.7k / 75.8k / 75.4k / 75.8k, two rounds each)
        const int per_cu[2] = {2, 3};
        constexpr int kQtKeys0Max = 3072;
        int want[2];
        for (int k = 0; k < 2; ++k) {
            const size_t budget = (size_t)160 * 1024 / per_cu[k] / 1280 * 1280;
            want[k] = budget > lds ? (int)((budget - lds) / 7) : 0;
        }
        want[0] = std::min(want[0], kQtKeys0Max);
        size_t maxl = lds;
        for (int k = 0; k < 2; ++k) {
            int kc = std::min(want[k], lcap[k]);
            kc = (int)std::min<size_t>((size_t)kc, (160 * 1024 - lds) / 7) & ~7;
            qt_keys[k] = std::max(kc, 0);
            maxl = std::max(maxl, lds + 7 * (size_t)qt_keys[k]);
        }
        if (maxl > 64 * 1024)
            ORBX_HIP(hipFuncSetAttribute((const void*)k_quadtree, hipFuncAttributeMaxDynamicSharedMemorySize, (int)maxl));
    }
    pyr_size = (poff + 255) & ~(size_t)255;
    cand_stride = std::max(cand, 1);
    out_stride = outs;
    node_cap = cap;
    out_capacity = outs;
    rows = r; cols = c; max_batch = batch;

    int st;
    if ((st = dev_alloc(&d_levels, nlevels))) return st;
    if ((st = dev_alloc(&d_cells, cellv.size()))) return st;
    if ((st = dev_alloc(&d_tiles, tilev.size()))) return st;
    ORBX_HIP(hipMemcpy(d_levels, lv.data(), sizeof(LevelDev) * nlevels, hipMemcpyHostToDevice));
    if (!cellv.empty()) ORBX_HIP(hipMemcpy(d_cells, cellv.data(), sizeof(CellDev) * cellv.size(), hipMemcpyHostToDevice));
    ORBX_HIP(hipMemcpy(d_tiles, tilev.data(), sizeof(BlurTile) * tilev.size(), hipMemcpyHostToDevice));

    // ---- resize tables (pinned OpenCV 3.2 INTER_LINEAR fixed point), level l from level l-1
    rtab.assign(nlevels, ResizeTab{});
    rvec.assign(nlevels, ResizeVec{});
    for (int l = 1; l < nlevels; ++l) {
        const int sw = lv[l - 1].w, sh = lv[l - 1].h, dw = lv[l].w, dh = lv[l].h;
        const double sxs = 1.0 / ((double)dw / sw), sys = 1.0 / ((double)dh / sh);
        std::vector<int> hx0(dw), hx1(dw), ha0(dw), ha1(dw), hy0(dh), hy1(dh), hb0(dh), hb1(dh);
        int xlim = dw;
        for (int x = 0; x < dw; ++x) {
            float fx = (float)((x + 0.5) * sxs - 0.5);
            int ix = (int)std::floor(fx);
            fx -= ix;
            if (ix < 0) { fx = 0; ix = 0; }
            if (ix + 1 >= sw) {
                xlim = std::min(xlim, x);
                if (ix >= sw - 1) { fx = 0; ix = sw - 1; }
            }
            hx0[x] = ix;
            hx1[x] = std::min(ix + 1, sw - 1);
            ha0[x] = std::min(std::max(round_even_f((1.f - fx) * 2048), -32768), 32767);
            ha1[x] = std::min(std::max(round_even_f(fx * 2048), -32768), 32767);
        }
        for (int x = xlim; x < dw; ++x) { ha0[x] = 2048; ha1[x] = 0; hx1[x] = hx0[x]; }
        for (int y = 0; y < dh; ++y) {
            float fy = (float)((y + 0.5) * sys - 0.5);
            int iy = (int)std::floor(fy);
            fy -= iy;
            hb0[y] = std::min(std::max(round_even_f((1.f - fy) * 2048), -32768), 32767);
            hb1[y] = std::min(std::max(round_even_f(fy * 2048), -32768), 32767);
            hy0[y] = std::min(std::max(iy, 0), sh - 1);
            hy1[y] = std::min(std::max(iy + 1, 0), sh - 1);
        }
        int* mem;
        if ((st = dev_alloc(&mem, 4 * (size_t)dw + 4 * (size_t)dh))) return st;
        rtab_mem.push_back(mem);
        ResizeTab t;
        t.x0 = mem; t.x1 = mem + dw; t.a0 = mem + 2 * dw; t.a1 = mem + 3 * dw;
        t.y0 = mem + 4 * dw; t.y1 = t.y0 + dh; t.b0 = t.y1 + dh; t.b1 = t.b0 + dh;
        std::vector<int> host;
        host.reserve(4 * dw + 4 * dh);
        for (auto* v : {&hx0, &hx1, &ha0, &ha1, &hy0, &hy1, &hb0, &hb1}) host.insert(host.end(), v->begin(), v->end());
        ORBX_HIP(hipMemcpy(mem, host.data(), host.size() * sizeof(int), hipMemcpyHostToDevice));
        rtab[l] = t;
        // vectorised tables: 4 columns per group, their taps inside an 8-byte window at xb
        const int G = (dw + 3) / 4;
        std::vector<int> vxb(G);
        std::vector<uint32_t> vsel(4 * (size_t)G, 0), vcoef(4 * (size_t)G, 0);
        bool fits = true;
        for (int g = 0; g < G; ++g) {
            vxb[g] = hx0[4 * g];
            for (int k = 0; k < 4 && 4 * g + k < dw; ++k) {
                const int x = 4 * g + k, oL = hx0[x] - vxb[g], oR = hx1[x] - vxb[g];
                if (oL < 0 || oR < 0 || oL > 7 || oR > 7 || ha0[x] < 0 || ha1[x] < 0 || ha0[x] + ha1[x] > 2049) fits = false;
                vsel[4 * g + k] = (uint32_t)(oL & 7) | 0x0c00u | ((uint32_t)(oR & 7) << 16) | 0x0c000000u;
                vcoef[4 * g + k] = (uint32_t)(ha0[x] & 0xffff) | ((uint32_t)(ha1[x] & 0xffff) << 16);
            }
        }
        for (int y = 0; y < dh; ++y) if (hb0[y] < 0 || hb1[y] < 0 || hb0[y] + hb1[y] > 2049) fits = false;   // resize_acc
        if (fits) {
            uint8_t* vm;
            const size_t bx = ((size_t)G * 4 + 15) & ~(size_t)15, bs = (size_t)G * 16, by = (size_t)dh * 16;
            if ((st = dev_alloc(&vm, bx + 2 * bs + by))) return st;
            rtab_mem.push_back(vm);
            std::vector<int32_t> yr(4 * (size_t)dh);
            for (int y = 0; y < dh; ++y) { yr[4 * y] = hy0[y]; yr[4 * y + 1] = hy1[y]; yr[4 * y + 2] = hb0[y]; yr[4 * y + 3] = hb1[y]; }
            ORBX_HIP(hipMemcpy(vm, vxb.data(), (size_t)G * 4, hipMemcpyHostToDevice));
            ORBX_HIP(hipMemcpy(vm + bx, vsel.data(), bs, hipMemcpyHostToDevice));
            ORBX_HIP(hipMemcpy(vm + bx + bs, vcoef.data(), bs, hipMemcpyHostToDevice));
            ORBX_HIP(hipMemcpy(vm + bx + 2 * bs, yr.data(), by, hipMemcpyHostToDevice));
            ResizeVec rv;
            rv.xb = (const int*)vm; rv.sel = (const uint4*)(vm + bx); rv.coef = (const uint4*)(vm + bx + bs);
            rv.yrow = (const int4*)(vm + bx + 2 * bs); rv.groups = G; rv.sxs = sxs;
            rvec[l] = rv;
        }
    }

    // ---- batch buffers (HBM): pyramid + blurred pyramid + candidates + quadtree scratch
    const size_t B = (size_t)batch;
    if ((st = dev_alloc(&d_pyr_ring, (size_t)pyr_ring * B * pyr_size))) return st;
    d_pyr = d_pyr_ring;
    ncalls = 0;
    desc_sets = 2;                                                // r5n: 2 sets +0.8 % in the step against 1
    dcalls = 0;
    dset_call[0] = dset_call[1] = -1;
    if (!desc_sb && (st = dev_alloc(&d_blur, (size_t)desc_sets * B * pyr_size))) return st;
    d_blur_c = d_blur;
    if ((st = dev_alloc(&d_cand_xy, B * cand_stride))) return st;
    if ((st = dev_alloc(&d_cand_s, B * cand_stride))) return st;
    if ((st = dev_alloc(&d_cell_cnt, B * std::max<size_t>(cellv.size(), 1)))) return st;
    if ((st = dev_alloc(&d_key_xy, B * cand_stride))) return st;
    if ((st = dev_alloc(&d_key_r, B * cand_stride))) return st;
    if ((st = dev_alloc(&d_key_node, B * cand_stride))) return st;
    if ((st = dev_alloc(&d_lvl_xy, (size_t)desc_sets * B * out_stride))) return st;
    if ((st = dev_alloc(&d_lvl_r, (size_t)desc_sets * B * out_stride))) return st;
    if ((st = dev_alloc(&d_lvl_cnt, (size_t)desc_sets * B * nlevels))) return st;
    d_lvl_xy_c = d_lvl_xy; d_lvl_r_c = d_lvl_r; d_lvl_cnt_c = d_lvl_cnt;
    if ((st = dev_alloc(&d_err, 1))) return st;
    // diagnostics: delay the null stream right before the counter initialisation (tests/test_gpu_ordering.py)
    if (const char* dl = std::getenv("ORBX_DEBUG_UPLOAD_DELAY_MS")) ORBX_HIP(debug_spin(nullptr, std::atof(dl)));
    ORBX_HIP(hipMemset(d_err, 0, sizeof(int)));
    ORBX_HIP(hipMemset(d_cell_cnt, 0, sizeof(int) * B * std::max<size_t>(cellv.size(), 1)));
#ifndef ORBX_LEGACY_UPLOADS
    // The first call's FAST runs on the non-blocking side stream right after this returns; the null-stream uploads
    // above must be complete by then (until r2 they were not waited for: the delayed memset could zero cell counts
    // FAST had already stored -- the intermittent cross-call mismatch of DESIGN §7, reproduced by the test above).
    ORBX_HIP(init_done());
#endif
    return ORBX_OK;
}

static size_t qt_lds_bytes(int cap, int scan_cap) {   // k_quadtree's layout (QtState)
    int p2 = 64;                                            // the sort keys: >= 64 for the one-wave sort's padding
    while (p2 < cap) p2 <<= 1;
    const size_t cs = ((size_t)cap + 3) & ~(size_t)3;
    const size_t ints = 10 * cs + 8 * cs + cs + 2 * (size_t)scan_cap + 32 + 16 + 2;
    return ints * 4 + (size_t)p2 * 8;
}


static int run_batch(Extractor* e, const uint8_t* d_images, int batch, size_t step, size_t istride,
                     orbx_keypoint* d_kps, uint8_t* d_desc, int32_t* d_counts, int capacity, hipStream_t s,
                     hipStream_t so, bool pipelined, bool merged = false) {
    const int nl = e->nlevels;
    const size_t ps = e->pyr_size;
    Extractor::EventSet* es = nullptr;
    if (e->timing && !e->tpool.empty() && !e->capturing) {
        es = &e->tpool[e->tnext++ % e->tpool.size()];
        int st = e->resolve(*es);
        if (st) return st;
        es->pending = true;
    }
    const Src0 s0{d_images, step, istride};
    e->last_src0 = s0;
    const unsigned seq = ++e->call_seq;                             // ordering canary stamp (k_quadtree -> describe)
    const int slot = (int)(e->ncalls++ % (unsigned long long)e->pyr_ring);
    e->d_pyr = e->d_pyr_ring + (size_t)slot * e->max_batch * ps;
    const int dset = (int)(e->dcalls++ % (unsigned long long)e->desc_sets);
    {
        const size_t B = (size_t)e->max_batch;
        e->d_blur_c = e->d_blur ? e->d_blur + (size_t)dset * B * ps : nullptr;
        e->d_lvl_xy_c = e->d_lvl_xy + (size_t)dset * B * e->out_stride;
        e->d_lvl_r_c = e->d_lvl_r + (size_t)dset * B * e->out_stride;
        e->d_lvl_cnt_c = e->d_lvl_cnt + (size_t)dset * B * nl;
    }
    // this call's events: the pool entry of 32 calls ago, whose describe (and every wait on its events) is long done
    const int ci = (int)(e->cev_next++ % Extractor::kCallEv);
    Extractor::CallEvents& ce = e->cev[ci];
    if (ce.used && !e->capturing) ORBX_HIP(hipEventSynchronize(ce.desc));
    hipStream_t side = pipelined ? e->side : s;
    if (!pipelined) so = s;
    // DistributeOctTree of levels 1..n-1 on the output stream ahead of the describe (qt_out), so that the launch stream
    // goes on to the next call's resize chain right after FAST; the next call's FAST of levels >= 1 then waits for it
    // (it overwrites the candidates this quadtree reads).  Step +1.0 % (r5bj: 75.7k -> 76.4k) / +0.4 % (r5bk: 75.7k -> 76.1k
    // against both other schedules), EuRoC +0.6 %.
    const bool qto = e->qt_out && pipelined && so != s && !e->capturing;
    auto mark = [&](int k) {
        if (es) (void)hipEventRecord(es->ev[k], (k >= 6 && k <= 9) ? side : (k == 4 || k == 5 || (qto && k == 3)) ? so : s);
    };
    // the previous call's describe (possibly on another stream) reads the kept keypoints and the blurred pyramid
    // the last describe that read this call's set of kept keypoints / blurred pyramid (the previous call's with one set)
    auto after_prev_describe = [&](hipStream_t q) -> int {
        const int prev = e->dset_call[dset];
        if (prev >= 0 && !e->dbg_skip_desc_wait && !e->capturing) ORBX_HIP(hipStreamWaitEvent(q, e->cev[prev].desc, 0));
        return ORBX_OK;
    };
    const int ncells = (int)e->cellv.size();
    const std::vector<int>& toff = e->tile_off;                     // blur tiles of level l: [toff[l], toff[l + 1])
    QtScratch qs{e->d_key_xy, e->d_key_r, e->d_key_node};
    auto fast = [&](hipStream_t q, int k) -> int {
        const Extractor::WaveLaunch& wl = e->wave_launch[k];
        if (wl.n <= 0) return ORBX_OK;
        if (k != 0 && e->qt_prev >= 0) {                            // the previous call's quadtree on its output stream
            // (a capture follows sync_calls and stream synchronisations, so that quadtree is done: no edge into it)
            if (!e->capturing) ORBX_HIP(hipStreamWaitEvent(q, e->cev[e->qt_prev].qt, 0));
            if (!qto) e->qt_prev = -1;
        }
        constexpr int wpg = Extractor::kWaveWpg;
        const int nwg = (wl.n * batch + wpg - 1) / wpg;
        auto kw = wl.ps == 19 ? k_fast_wave<19, 4, wpg> : k_fast_wave<40, 0, wpg>;
        hipLaunchKernelGGL(kw, dim3(kXcds * xcd_chunk(nwg)), dim3(64 * wpg), (size_t)wpg * wl.lay.bytes, q, e->d_pyr, ps,
                           e->d_levels, e->d_cells, wl.cell0, wl.n, e->iniTh, e->minTh, e->d_cand_xy, e->d_cand_s,
                           e->cand_stride, e->d_cell_cnt, ncells, batch, s0, wl.lay, wl.kcap, e->wave_twopass);
        return ORBX_OK;
    };
    auto quadtree = [&](hipStream_t q, int lvl0, int n) {
        if (n <= 0) return;
        const int kc = lvl0 == 0 ? e->qt_keys[0] : e->qt_keys[1];  // LDS key capacity: level 0 / levels >= 1
        hipLaunchKernelGGL(k_quadtree, dim3(n, batch), dim3(kQtThreads), e->qt_lds + 7 * (size_t)kc, q, e->d_levels, e->d_cells,
                           e->d_cand_xy, e->d_cand_s, e->cand_stride, e->d_cell_cnt, std::max(ncells, 1), qs, e->d_lvl_xy_c,
                           e->d_lvl_r_c, e->out_stride, e->d_lvl_cnt_c, nl, e->node_cap, e->scan_cap, e->d_err, lvl0,
                           (int)e->qt_lds, kc, seq);
    };
    auto blur = [&](hipStream_t q, int tile0, int n) {
        if (n <= 0 || e->desc_sb) return;                           // k_describe_sb blurs at the sample points
        hipLaunchKernelGGL(k_blur7, dim3(kXcds * xcd_chunk((n + 3) / 4 * batch)), dim3(256), 0, q, e->d_pyr, e->d_blur_c, ps,
                           e->d_levels, e->d_tiles, n, batch, s0, tile0);
    };

    mark(0);
    if (side != s) {
        ORBX_HIP(hipEventRecord(ce.fork, s));
        ORBX_HIP(hipStreamWaitEvent(side, ce.fork, 0));
    }
    auto resize_chain = [&]() -> int {
        if (e->slot_call[slot] >= 0 && !e->capturing)               // this set's last reader
            ORBX_HIP(hipStreamWaitEvent(s, e->cev[e->slot_call[slot]].desc, 0));
        for (int l = 1; l < nl; ++l) {
            const uint8_t* src = (l == 1) ? d_images : e->d_pyr + e->lv[l - 1].pyr_off;
            const size_t sstep = (l == 1) ? step : (size_t)e->lv[l - 1].w, sis = (l == 1) ? istride : ps;
            const LevelDev& L = e->lv[l];
            if (e->resize_tail > 1 && l == e->resize_tail && nl - l <= kTailMax) {
                bool ok = true;
                for (int k = l; k < nl; ++k) ok = ok && e->rvec[k].groups > 0 && e->lv[k - 1].w >= 8;
                if (ok) {                                           // levels l .. nl-1 in one launch
                    TailArgs A{};
                    A.n = nl - l;
                    for (int k = l; k < nl; ++k) {
                        TailLevel& T = A.lv[k - l];
                        T.t = e->rvec[k]; T.sw = e->lv[k - 1].w; T.src_off = e->lv[k - 1].pyr_off; T.dst_off = e->lv[k].pyr_off;
                        T.dw = e->lv[k].w; T.dh = e->lv[k].h;
                        T.nstrips = (T.dw + kResizeStrip - 1) / kResizeStrip; T.nbands = (T.dh + kResizeBand - 1) / kResizeBand;
                    }
                    hipLaunchKernelGGL(k_resize_tail, dim3(batch), dim3(256), 0, s, e->d_pyr, ps, A, batch);
                    break;
                }
            }
            if (e->rvec[l].groups > 0) {
                const int nstrips = (L.w + kResizeStrip - 1) / kResizeStrip, nbands = (L.h + kResizeBand - 1) / kResizeBand;
                const int nwg = (nstrips * nbands * batch + 3) / 4;
                hipLaunchKernelGGL(k_resize4, dim3(kXcds * xcd_chunk(nwg)), dim3(256), 0, s, e->d_pyr, ps, src, sstep, sis,
                                   e->lv[l - 1].w, L.pyr_off, L.w, L.h, e->rvec[l], nstrips, nbands, batch);
            } else {                                                // taps outside an 8-byte window: the scalar form
                dim3 g((L.w + 255) / 256, L.h, batch);
                hipLaunchKernelGGL(k_resize, g, dim3(256), 0, s, e->d_pyr, ps, src, sstep, sis, L.pyr_off, L.w, L.h, e->rtab[l]);
            }
        }
        mark(1);
        return ORBX_OK;
    };
    if (side == s) { int st = resize_chain(); if (st) return st; }  // serial: every stage contiguous on one stream
    if (merged && side == s) {
        // one launch per stage over every level (the host API's one-image calls, where the chain of dependent launches
        // is the latency): FAST, DistributeOctTree, blur
        mark(6);
        if (int st = fast(s, 2)) return st;
        mark(7);
        if (int st = after_prev_describe(s)) return st;
        quadtree(s, 0, nl);
        mark(8);
        blur(s, toff[0], toff[nl] - toff[0]);
        mark(9);
        mark(10);
        mark(2);
        mark(3);
    } else {
    // side stream, level 0 (reads only the caller's images)
    mark(6);
    if (int st = fast(side, 0)) return st;
    mark(7);
    if (int st = after_prev_describe(side)) return st;
    quadtree(side, 0, nl > 0 ? 1 : 0);
    mark(8);
    blur(side, toff[0], toff[1] - toff[0]);
    if (side != s) {
        int st = resize_chain();                                    // launch stream: levels 1..nl-1 of the pyramid
        if (st) return st;
        ORBX_HIP(hipEventRecord(ce.pyr, s));
        ORBX_HIP(hipStreamWaitEvent(side, ce.pyr, 0));
    }
    blur(side, toff[1], toff[nl] - toff[1]);                        // side: levels 1..nl-1 once the pyramid exists
    mark(9);
    if (side != s) ORBX_HIP(hipEventRecord(ce.join, side));
    mark(10);                                                       // launch stream: FAST, DistributeOctTree 1..nl-1
    if (int st = fast(s, 1)) return st;
    mark(2);
    if (!qto) {
        if (int st = after_prev_describe(s)) return st;
        quadtree(s, 1, nl - 1);
        mark(3);
    }
    }
    // the descriptor stage on the output stream, once both streams are done; the next call's resize chain (launch
    // stream) runs beside it
    if (so != s) {
        ORBX_HIP(hipEventRecord(ce.front, s));
        ORBX_HIP(hipStreamWaitEvent(so, ce.front, 0));
    }
    if (side != so) ORBX_HIP(hipStreamWaitEvent(so, ce.join, 0));
    if (qto) {
        if (int st = after_prev_describe(so)) return st;
        quadtree(so, 1, nl - 1);
        mark(3);
        ORBX_HIP(hipEventRecord(ce.qt, so));
        e->qt_prev = ci;
    }
    mark(4);
    {
        SlotTable tab{};
        for (int l = 0; l < nl; ++l) tab.out_off[l] = e->lv[l].out_off;
        const int nslots = e->out_stride;                           // every level's slots; the launch writes the counts
        constexpr int kpw = 2;                                      // keypoints per wave
        dim3 g(kXcds * xcd_chunk((nslots + 4 * kpw - 1) / (4 * kpw) * batch));
        if (e->desc_sb)
            hipLaunchKernelGGL(k_describe_sb, g, dim3(256), 0, so, e->d_pyr, ps, e->d_levels, nl, e->d_lvl_xy_c, e->d_lvl_r_c,
                               e->out_stride, e->d_lvl_cnt_c, d_kps, d_desc, d_counts, capacity, 0, nslots, 1, batch, s0, tab,
                               seq, e->d_err);
        else
            hipLaunchKernelGGL(k_describe_m<kpw>, g, dim3(256), 0, so, e->d_pyr, e->d_blur_c, ps, e->d_levels, nl,
                               e->d_lvl_xy_c, e->d_lvl_r_c, e->out_stride, e->d_lvl_cnt_c, d_kps, d_desc, d_counts, capacity, 0,
                               nslots, 1, batch, s0, tab, seq, e->d_err);
    }
    mark(5);
    ORBX_HIP(hipEventRecord(ce.desc, so));
    if (e->capturing) {                                             // replays are synchronous: nothing to wait on
        ce.used = false;
        e->slot_call[slot] = -1;
        e->last_call = -1;
        e->dset_call[dset] = -1;
    } else {
        ce.used = true;
        e->slot_call[slot] = ci;
        e->last_call = ci;
        e->dset_call[dset] = ci;
        e->async_pending = true;
    }
    ORBX_HIP(hipGetLastError());
    e->last_batch = batch;
    return ORBX_OK;
}

static int check_constants(const Extractor* e) {
    // umax is the same for every extractor (depends only on HALF_PATCH_SIZE); the kernels use kUmax
    for (int v = 0; v < 16; ++v)
        ORBX_REQUIRE(e->umax[v] == kUmax[v], ORBX_ERR_UNSUPPORTED, "umax table mismatch at %d", v);
    return ORBX_OK;
}

}  // namespace orbx

// =============================================================================================
// C ABI
// =============================================================================================
using namespace orbx;

struct orbx_extractor : public orbx::Extractor {};

extern "C" {

const char* orbx_last_error(void) { return orbx::g_err.c_str(); }
const char* orbx_version(void) { return "orbx 0.1 (gfx950)"; }
int orbx_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int orbx_stream_create(int device, int priority, int cu_exclude, void** out) {
    if (!out) return ORBX_ERR_ARG;
    *out = nullptr;
    int cur = 0;
    ORBX_HIP(hipGetDevice(&cur));
    ORBX_HIP(hipSetDevice(device));
    hipStream_t s = nullptr;
    const hipError_t he = create_stream_masked(&s, priority, cu_exclude);
    (void)hipSetDevice(cur);
    if (he != hipSuccess) {
        set_error("stream create: %s", hipGetErrorString(he));
        return ORBX_ERR_HIP;
    }
    *out = (void*)s;
    return ORBX_OK;
}

int orbx_device_check(int device) {
    ORBX_HIP(hipSetDevice(device));
    ORBX_HIP(::orbx::device_sync());
    ORBX_HIP(hipGetLastError());
    return ORBX_OK;
}

int orbx_stream_destroy(void* stream) {
    if (!stream) return ORBX_ERR_ARG;
    ORBX_HIP(hipStreamDestroy((hipStream_t)stream));
    return ORBX_OK;
}

int orbx_extractor_create(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST, int device,
                          orbx_extractor** out) {
    ORBX_REQUIRE(out, ORBX_ERR_ARG, "out is NULL");
    *out = nullptr;
    ORBX_REQUIRE(nfeatures >= 0 && nlevels >= 1 && nlevels <= kMaxLevels && scaleFactor > 1.0f, ORBX_ERR_ARG,
                 "bad extractor parameters");
    int ndev = 0;
    ORBX_HIP(hipGetDeviceCount(&ndev));
    ORBX_REQUIRE(device >= 0 && device < ndev, ORBX_ERR_ARG, "device %d out of range (%d devices)", device, ndev);
    orbx_extractor* e = new orbx_extractor();
    e->nfeatures = nfeatures;
    e->nlevels = nlevels;
    e->iniTh = iniThFAST;
    e->minTh = minThFAST;
    e->scaleFactor = (double)scaleFactor;
    e->device = device;
    compute_tables(e);
    hipError_t he = hipSetDevice(device);
    e->own_stream = true;
    // High priority for the side stream: its level-0 quadtree (128 long-lived workgroups) must not queue behind the
    // launch stream's FAST grid (measured: 35.1k -> 37.6k frames/s; at normal priority -1 %, r5bu).
    const int side_prio = -1;
    const int cu_ex = std::getenv("ORBX_CU_EXCLUDE") ? std::atoi(std::getenv("ORBX_CU_EXCLUDE")) : 0;
    if (he == hipSuccess) he = create_stream_masked(&e->side, side_prio, cu_ex);
    for (auto& c : e->cev)
        for (hipEvent_t* ev : {&c.fork, &c.pyr, &c.join, &c.front, &c.desc, &c.qt})
            if (he == hipSuccess) he = hipEventCreateWithFlags(ev, hipEventDisableTiming);
    if (he != hipSuccess) {
        set_error("stream create: %s", hipGetErrorString(he));
        orbx_extractor_destroy(e);
        return ORBX_ERR_HIP;
    }
    if (const char* pl = std::getenv("ORBX_PIPELINE")) e->pipeline = std::atoi(pl) != 0;
    if (const char* tp = std::getenv("ORBX_FAST_TWOPASS")) e->wave_twopass = std::atoi(tp) != 0;
    if (const char* hg = std::getenv("ORBX_HOST_GRAPH")) e->host_graph = std::atoi(hg) != 0;
    if (const char* hs = std::getenv("ORBX_HOST_SERIAL")) e->host_serial = std::atoi(hs) != 0;
    if (const char* hm = std::getenv("ORBX_HOST_MERGED")) e->host_merged = std::atoi(hm) != 0;
    if (const char* sw = std::getenv("ORBX_DEBUG_SKIP_DESC_WAIT")) e->dbg_skip_desc_wait = std::atoi(sw) != 0;
    if (const char* qo = std::getenv("ORBX_QT_OUT")) e->qt_out = std::atoi(qo) != 0;
    if (const char* sb = std::getenv("ORBX_DESC_SB")) e->desc_sb = std::atoi(sb) != 0;
    if (const char* rt = std::getenv("ORBX_RESIZE_TAIL")) e->resize_tail = std::atoi(rt);
    if (int st = check_constants(e)) {
        orbx_extractor_destroy(e);
        return st;
    }
    *out = e;
    return ORBX_OK;
}

int orbx_extractor_destroy(orbx_extractor* e) {
    if (!e) return ORBX_OK;
    (void)hipSetDevice(e->device);
    // Every stream of the device, not only the extractor's own: callers' streams read its pyramid ring and outputs
    // (the stereo SAD step reads orbx_extractor_pyramid_device's levels); hipFree was measured to wait for them too,
    // but the guarantee should not rest on that.
    ::orbx::LegacyLock legacy_;
    (void)::orbx::device_sync();
    e->free_buffers();                                      // (and the host-API graph)
    for (auto& es : e->tpool)
        for (auto& ev : es.ev) (void)hipEventDestroy(ev);
    if (e->own_stream && e->stream) (void)hipStreamDestroy(e->stream);
    if (e->side) (void)hipStreamDestroy(e->side);
    for (auto& c : e->cev)
        for (hipEvent_t ev : {c.fork, c.pyr, c.join, c.front, c.desc, c.qt})
            if (ev) (void)hipEventDestroy(ev);
    delete e;
    return ORBX_OK;
}

int orbx_extractor_get_levels(const orbx_extractor* e) { return e ? e->nlevels : ORBX_ERR_ARG; }
float orbx_extractor_get_scale_factor(const orbx_extractor* e) { return e ? (float)e->scaleFactor : 0.f; }

static int copy_vec(const std::vector<float>& v, float* out) {
    ORBX_REQUIRE(out, ORBX_ERR_ARG, "out is NULL");
    std::memcpy(out, v.data(), v.size() * sizeof(float));
    return ORBX_OK;
}
int orbx_extractor_get_scale_factors(const orbx_extractor* e, float* out) {
    ORBX_REQUIRE(e, ORBX_ERR_ARG, "null extractor");
    return copy_vec(e->scale, out);
}
int orbx_extractor_get_inverse_scale_factors(const orbx_extractor* e, float* out) {
    ORBX_REQUIRE(e, ORBX_ERR_ARG, "null extractor");
    return copy_vec(e->invScale, out);
}
int orbx_extractor_get_scale_sigma_squares(const orbx_extractor* e, float* out) {
    ORBX_REQUIRE(e, ORBX_ERR_ARG, "null extractor");
    return copy_vec(e->sigma2, out);
}
int orbx_extractor_get_inverse_scale_sigma_squares(const orbx_extractor* e, float* out) {
    ORBX_REQUIRE(e, ORBX_ERR_ARG, "null extractor");
    return copy_vec(e->invSigma2, out);
}
int orbx_extractor_get_features_per_level(const orbx_extractor* e, int* out) {
    ORBX_REQUIRE(e && out, ORBX_ERR_ARG, "null argument");
    std::memcpy(out, e->nPerLevel.data(), e->nPerLevel.size() * sizeof(int));
    return ORBX_OK;
}

int orbx_extractor_reserve(orbx_extractor* e, int rows, int cols, int max_batch) {
    ORBX_REQUIRE(e, ORBX_ERR_ARG, "null extractor");
    return e->configure(rows, cols, max_batch);
}

int orbx_extractor_set_pyramid_ring(orbx_extractor* e, int n) {
    ORBX_REQUIRE(e && n >= 1 && n <= 8, ORBX_ERR_ARG, "pyramid ring must be 1..8");
    if (n == e->pyr_ring) return ORBX_OK;
    const int r = e->rows, c = e->cols, b = e->max_batch;
    ORBX_HIP(hipSetDevice(e->device));
    ::orbx::LegacyLock legacy_;
    ORBX_HIP(::orbx::device_sync());                       // callers' streams may still read the pyramid ring
    e->free_buffers();
    for (int& k : e->slot_call) k = -1;
    e->last_call = -1;
    e->pyr_ring = n;
    return (r > 0 && c > 0 && b > 0) ? e->configure(r, c, b) : ORBX_OK;
}

int orbx_extractor_max_keypoints(orbx_extractor* e, int rows, int cols) {
    ORBX_REQUIRE(e, ORBX_ERR_ARG, "null extractor");
    int st = e->configure(rows, cols, std::max(e->max_batch, 1));
    if (st) return st;
    return e->out_capacity;
}

int orbx_extractor_level_sizes(orbx_extractor* e, int rows, int cols, int* lr, int* lc) {
    ORBX_REQUIRE(e && lr && lc, ORBX_ERR_ARG, "null argument");
    for (int l = 0; l < e->nlevels; ++l) level_dims(e, rows, cols, l, &lc[l], &lr[l]);
    return ORBX_OK;
}

int orbx_extract_batch_device(orbx_extractor* e, const uint8_t* d_images, int batch, int rows, int cols, size_t step,
                              size_t image_stride, orbx_keypoint* d_keypoints, uint8_t* d_descriptors, int32_t* d_counts,
                              int capacity, void* stream) {
    ORBX_REQUIRE(e && d_images && d_keypoints && d_descriptors && d_counts, ORBX_ERR_ARG, "null argument");
    ORBX_REQUIRE(batch > 0 && rows > 0 && cols > 0 && step >= (size_t)cols, ORBX_ERR_ARG, "bad batch geometry");
    ORBX_HIP(hipSetDevice(e->device));
    int st = e->configure(rows, cols, batch);
    if (st) return st;
    ORBX_REQUIRE(capacity >= e->out_capacity, ORBX_ERR_CAPACITY, "capacity %d < required %d", capacity, e->out_capacity);
    hipStream_t s = (hipStream_t)stream;   // NULL = the HIP null stream
    return run_batch(e, d_images, batch, step, image_stride, d_keypoints, d_descriptors, d_counts, capacity, s, s,
                     e->pipeline);
}

int orbx_extract_batch_device_split(orbx_extractor* e, const uint8_t* d_images, int batch, int rows, int cols, size_t step,
                                    size_t image_stride, orbx_keypoint* d_keypoints, uint8_t* d_descriptors,
                                    int32_t* d_counts, int capacity, void* in_stream, void* out_stream) {
    ORBX_REQUIRE(e && d_images && d_keypoints && d_descriptors && d_counts, ORBX_ERR_ARG, "null argument");
    ORBX_REQUIRE(batch > 0 && rows > 0 && cols > 0 && step >= (size_t)cols, ORBX_ERR_ARG, "bad batch geometry");
    ORBX_HIP(hipSetDevice(e->device));
    int st = e->configure(rows, cols, batch);
    if (st) return st;
    ORBX_REQUIRE(capacity >= e->out_capacity, ORBX_ERR_CAPACITY, "capacity %d < required %d", capacity, e->out_capacity);
    return run_batch(e, d_images, batch, step, image_stride, d_keypoints, d_descriptors, d_counts, capacity,
                     (hipStream_t)in_stream, (hipStream_t)out_stream, e->pipeline);
}

// The host call in two halves: extract_begin stages the image and enqueues the extraction and the result copy on the
// extractor's stream (no synchronisation); extract_end waits for that stream and hands the results out.  orbx_extract
// is begin + end; orbx_extract_pair begins both extractors before ending either, so one host thread keeps the left and
// right extractions in flight together (what Frame.cc:78-81 gets from two threads).
static int extract_begin(orbx_extractor* e, const uint8_t* image, int rows, int cols, size_t step) {
    ORBX_REQUIRE(step >= (size_t)cols, ORBX_ERR_ARG, "step < cols");
    ORBX_HIP(hipSetDevice(e->device));
    int st = e->configure(rows, cols, std::max(e->max_batch, 1));
    if (st) return st;
    const size_t nb = (size_t)rows * cols;
    // buffer (re)allocation and the capture of this configuration's graph hold the process-wide legacy lock: another
    // thread's device synchronisation or synchronous upload during the capture would invalidate it (orbx_common.h)
    std::unique_lock<std::recursive_mutex> legacy_(::orbx::legacy_mutex(), std::defer_lock);
    if (!(e->host_graph && e->hgexec) || e->in_bytes < nb || !e->d_hblk) legacy_.lock();
    if (e->in_bytes < nb) {
        e->drop_graph();                                     // it names the buffers replaced here
        if (e->d_in) (void)hipFree(e->d_in);
        if (e->h_in) (void)hipHostFree(e->h_in);
        e->d_in = nullptr;
        e->h_in = nullptr;
        e->in_bytes = 0;
        if ((st = dev_alloc(&e->d_in, nb))) return st;
        ORBX_HIP(hipHostMalloc((void**)&e->h_in, nb, hipHostMallocDefault));
        e->in_bytes = nb;
    }
    // output block (device and pinned host alike): count at 0, keypoints at 64, descriptors 64-byte aligned after them
    const size_t odesc = (64 + (size_t)e->out_capacity * sizeof(orbx_keypoint) + 63) & ~(size_t)63;
    const size_t ob = odesc + (size_t)e->out_capacity * 32;
    if (!e->d_hblk) {
        if ((st = dev_alloc(&e->d_hblk, ob))) return st;
        e->d_cnt = reinterpret_cast<int32_t*>(e->d_hblk);
        e->d_kps = reinterpret_cast<orbx_keypoint*>(e->d_hblk + 64);
        e->d_desc = e->d_hblk + odesc;
    }
    if (e->h_out_bytes < ob) {
        e->drop_graph();
        if (e->h_out) (void)hipHostFree(e->h_out);
        e->h_out = nullptr;
        e->h_out_bytes = 0;
        ORBX_HIP(hipHostMalloc((void**)&e->h_out, ob, hipHostMallocDefault));
        e->h_out_bytes = ob;
    }
    int32_t* h_cnt = (int32_t*)e->h_out;                    // count, then the error word (extract_end reads both)
    hipStream_t s = e->own();
    // The image in, outside the graph (its source changes every call): packed into pinned staging, one H2D copy.  (r4n,
    // native per-call path: one staged copy 0.397 / 0.396 ms per frame, a pageable copy 0.398 / 0.393, four row bands
    // each copied as soon as packed 0.427 / 0.424.)  The previous call's transfers out of h_in completed before it
    // returned (stream synchronised).
    if (step == (size_t)cols) {
        std::memcpy(e->h_in, image, nb);
    } else {
        for (int r = 0; r < rows; ++r) std::memcpy(e->h_in + (size_t)r * cols, image + (size_t)r * step, (size_t)cols);
    }
    ORBX_HIP(hipMemcpyAsync(e->d_in, e->h_in, nb, hipMemcpyHostToDevice, s));
    // the call's other stream operations: the extraction, count + keypoints + descriptors of the whole capacity in one
    // copy (a count-sized copy would need a second synchronisation; only the first n are read), the error word
    auto enqueue = [&]() -> int {
        int r = run_batch(e, e->d_in, 1, cols, nb, e->d_kps, e->d_desc, e->d_cnt, e->out_capacity, s, s,
                          e->pipeline && !e->host_serial, e->host_serial && e->host_merged);
        if (r) return r;
        ORBX_HIP(hipMemcpyAsync(e->h_out, e->d_hblk, ob, hipMemcpyDeviceToHost, s));
        ORBX_HIP(hipMemcpyAsync(h_cnt + 1, e->d_err, sizeof(int), hipMemcpyDeviceToHost, s));
        return ORBX_OK;
    };
    if (e->host_graph && !e->hgexec) {
        // first call of this configuration: finish every earlier call, then capture this one's operations
        if (int r = e->sync_calls()) return r;
        if (e->side) ORBX_HIP(hipStreamSynchronize(e->side));
        ORBX_HIP(hipStreamSynchronize(s));
        e->async_pending = false;
        ORBX_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
        e->capturing = true;
        const int r = enqueue();
        e->capturing = false;
        hipGraph_t g = nullptr;
        const hipError_t ec = hipStreamEndCapture(s, &g);
        hipGraphExec_t x = nullptr;
        const hipError_t ei = (r == ORBX_OK && ec == hipSuccess) ? hipGraphInstantiate(&x, g, nullptr, nullptr, 0) : ec;
        if (r != ORBX_OK || ei != hipSuccess) {              // no graph for this extractor: per-call stream operations
            if (g) (void)hipGraphDestroy(g);
            (void)hipGetLastError();
            e->host_graph = false;
            // A capture invalidated part-way (another thread synchronised the device: liborbx's own such operations
            // wait for the legacy lock, a caller's cannot) can leave the extractor's streams in the capture sequence and
            // its call events recorded inside it.  The extractor continues on fresh streams and events; the old ones
            // are left alone (neither ended nor destroyed: both crash or fail on a stream still in the sequence, r7z).
            hipStream_t ns = nullptr, nside = nullptr;
            ORBX_HIP(hipStreamCreateWithFlags(&ns, hipStreamNonBlocking));
            ORBX_HIP(create_stream_masked(&nside, -1, std::getenv("ORBX_CU_EXCLUDE") ? std::atoi(std::getenv("ORBX_CU_EXCLUDE")) : 0));
            e->stream = ns;
            e->side = nside;
            s = ns;
            for (auto& c : e->cev) {
                for (hipEvent_t* ev : {&c.fork, &c.pyr, &c.join, &c.front, &c.desc, &c.qt})
                    ORBX_HIP(hipEventCreateWithFlags(ev, hipEventDisableTiming));
                c.used = false;
            }
            for (int& k : e->slot_call) k = -1;
            e->dset_call[0] = e->dset_call[1] = -1;
            e->last_call = -1;
            e->qt_prev = -1;
        } else {
            e->hgraph = g;
            e->hgexec = x;
            e->hg_pyr = e->d_pyr;                            // the pyramid set the graph writes
        }
    }
    if (e->host_graph && e->hgexec) {
        if (e->async_pending) {                              // a device-API call may still use the buffers
            if (int r = e->sync_calls()) return r;
            e->async_pending = false;
        }
        ORBX_HIP(hipGraphLaunch(e->hgexec, s));
        e->d_pyr = e->hg_pyr;                                // what orbx_extractor_pyramid_device now names
        e->last_src0 = Src0{e->d_in, (size_t)cols, nb};
        e->last_batch = 1;
    } else {
        if ((st = enqueue())) return st;
    }
    return ORBX_OK;
}

static int extract_end(orbx_extractor* e, orbx_keypoint* kps, uint8_t* desc, int capacity, int* n_out) {
    ORBX_HIP(hipSetDevice(e->device));
    const size_t odesc = (64 + (size_t)e->out_capacity * sizeof(orbx_keypoint) + 63) & ~(size_t)63;
    const int32_t* h_cnt = (const int32_t*)e->h_out;
    const orbx_keypoint* h_kps = (const orbx_keypoint*)(e->h_out + 64);
    const uint8_t* h_desc = e->h_out + odesc;
    ORBX_HIP(hipStreamSynchronize(e->own()));
    const int n = h_cnt[0], err = h_cnt[1];
    ORBX_REQUIRE(!(err & kErrStale), ORBX_ERR_HIP, "ordering canary: a describe read another call's keypoints (err=%d)", err);
    ORBX_REQUIRE(err == 0, ORBX_ERR_UNSUPPORTED, "quadtree node capacity exceeded (err=%d)", err);
    *n_out = n;
    if (n > capacity) {
        set_error("capacity %d < %d keypoints", capacity, n);
        return ORBX_ERR_CAPACITY;
    }
    if (n > 0) {
        ORBX_REQUIRE(kps && desc, ORBX_ERR_ARG, "null output buffers");
        std::memcpy(kps, h_kps, sizeof(orbx_keypoint) * (size_t)n);
        std::memcpy(desc, h_desc, (size_t)n * 32);
    }
    return ORBX_OK;
}

int orbx_extract(orbx_extractor* e, const uint8_t* image, int rows, int cols, size_t step, orbx_keypoint* kps,
                 uint8_t* desc, int capacity, int* n_out) {
    ORBX_REQUIRE(e && n_out, ORBX_ERR_ARG, "null argument");
    *n_out = 0;
    if (!image || rows <= 0 || cols <= 0) return ORBX_OK;   // _image.empty() -> return (:1046-1047)
    if (int st = extract_begin(e, image, rows, cols, step)) return st;
    return extract_end(e, kps, desc, capacity, n_out);
}

int orbx_extract_pair(orbx_extractor* left, orbx_extractor* right, const uint8_t* image_left, size_t step_left,
                      const uint8_t* image_right, size_t step_right, int rows, int cols, orbx_keypoint* kps_left,
                      uint8_t* desc_left, int capacity_left, int* n_left, orbx_keypoint* kps_right, uint8_t* desc_right,
                      int capacity_right, int* n_right) {
    ORBX_REQUIRE(left && right && left != right && n_left && n_right, ORBX_ERR_ARG,
                 "two distinct extractors and both counts are required");
    *n_left = *n_right = 0;
    const bool l_ok = image_left && rows > 0 && cols > 0, r_ok = image_right && rows > 0 && cols > 0;
    if (l_ok) if (int st = extract_begin(left, image_left, rows, cols, step_left)) return st;
    if (r_ok) {
        if (int st = extract_begin(right, image_right, rows, cols, step_right)) {
            if (l_ok) (void)hipStreamSynchronize(left->own());   // leave the left call finished, not half-done
            return st;
        }
    }
    int st = l_ok ? extract_end(left, kps_left, desc_left, capacity_left, n_left) : ORBX_OK;
    const int sr = r_ok ? extract_end(right, kps_right, desc_right, capacity_right, n_right) : ORBX_OK;
    return st ? st : sr;
}

// The host call's halves and its device outputs, for orbx_stereo_frame (orbx_match.hip; declared in orbx_common.h, not a
// public entry point): the stereo search of a Frame reads the extractions' device outputs where extract_begin leaves
// them (count, keypoints, descriptors of the whole capacity), on the extractor's own stream.
int orbx_internal_extract_begin(orbx_extractor* e, const uint8_t* image, int rows, int cols, size_t step) {
    return extract_begin(e, image, rows, cols, step);
}
int orbx_internal_extract_end(orbx_extractor* e, orbx_keypoint* kps, uint8_t* desc, int capacity, int* n_out) {
    return extract_end(e, kps, desc, capacity, n_out);
}
int orbx_internal_host_outputs(orbx_extractor* e, const orbx_keypoint** kps, const uint8_t** desc, const int32_t** count,
                               int* capacity, void** stream) {
    ORBX_REQUIRE(e && e->d_hblk, ORBX_ERR_ARG, "no host call in flight on this extractor");
    *kps = e->d_kps;
    *desc = e->d_desc;
    *count = e->d_cnt;
    *capacity = e->out_capacity;
    *stream = (void*)e->own();
    return ORBX_OK;
}

int orbx_extractor_status(orbx_extractor* e, int* flags, int reset) {
    ORBX_REQUIRE(e && flags, ORBX_ERR_ARG, "null argument");
    *flags = 0;
    if (!e->d_err) return ORBX_OK;
    ORBX_HIP(hipSetDevice(e->device));
    if (e->stream) ORBX_HIP(hipStreamSynchronize(e->stream));
    if (e->side) ORBX_HIP(hipStreamSynchronize(e->side));
    if (int st = e->sync_calls()) return st;
    hipStream_t q = e->side ? e->side : e->own();
    int h = 0;
    ORBX_HIP(hipMemcpyAsync(&h, e->d_err, sizeof(int), hipMemcpyDeviceToHost, q));
    if (reset) ORBX_HIP(hipMemsetAsync(e->d_err, 0, sizeof(int), q));
    ORBX_HIP(hipStreamSynchronize(q));
    *flags = h;
    return ORBX_OK;
}

int orbx_debug_spin_device(void* stream, double ms) {
    ORBX_HIP(debug_spin((hipStream_t)stream, ms));
    return ORBX_OK;
}

int orbx_extractor_pyramid_device(const orbx_extractor* e, orbx_pyramid* out) {
    ORBX_REQUIRE(e && out, ORBX_ERR_ARG, "null argument");
    ORBX_REQUIRE(e->d_pyr && e->last_src0.p && e->last_batch > 0, ORBX_ERR_ARG, "no pyramid: extract first");
    std::memset(out, 0, sizeof(*out));
    out->nlevels = e->nlevels;
    out->batch = e->last_batch;
    out->level0 = e->last_src0.p;
    out->level0_step = e->last_src0.step;
    out->level0_image_stride = e->last_src0.istride;
    out->levels = e->d_pyr;
    out->image_stride = e->pyr_size;
    for (int l = 0; l < e->nlevels; ++l) {
        out->offset[l] = (size_t)e->lv[l].pyr_off;
        out->rows[l] = e->lv[l].h;
        out->cols[l] = e->lv[l].w;
        out->scale[l] = e->scale[l];
        out->inv_scale[l] = e->invScale[l];
    }
    return ORBX_OK;
}

int orbx_extractor_level_device(orbx_extractor* e, int index, int level, const uint8_t** d_level, int* rows, int* cols,
                                size_t* step) {
    ORBX_REQUIRE(e && d_level && rows && cols && step, ORBX_ERR_ARG, "null argument");
    ORBX_REQUIRE(e->d_pyr && e->last_src0.p && level >= 0 && level < e->nlevels && index >= 0 && index < e->last_batch,
                 ORBX_ERR_ARG, "no pyramid for index %d level %d", index, level);
    if (level == 0) {
        *d_level = e->last_src0.p + (size_t)index * e->last_src0.istride;
        *step = e->last_src0.step;
    } else {
        *d_level = e->d_pyr + (size_t)index * e->pyr_size + e->lv[level].pyr_off;
        *step = (size_t)e->lv[level].w;
    }
    *rows = e->lv[level].h;
    *cols = e->lv[level].w;
    return ORBX_OK;
}

int orbx_extractor_copy_blurred_level(orbx_extractor* e, int index, int level, uint8_t* dst, size_t dst_step) {
    ORBX_REQUIRE(e && dst, ORBX_ERR_ARG, "null argument");
    ORBX_REQUIRE(e->d_pyr && e->last_src0.p && level >= 0 && level < e->nlevels && index >= 0 &&
                     index < e->last_batch,
                 ORBX_ERR_ARG, "no blurred level for index %d level %d", index, level);
    const int w = e->lv[level].w, h = e->lv[level].h;
    ORBX_REQUIRE(dst_step >= (size_t)w, ORBX_ERR_ARG, "bad destination");
    ORBX_HIP(hipSetDevice(e->device));
    ::orbx::LegacyLock legacy_;
    ORBX_HIP(::orbx::device_sync());                                  // the last call's kernels may run on any stream
    // k_blur7 over every tile of image `index` of the last call's pyramid (d_pyr, and level 0 = the caller's image),
    // into a one-image buffer: whatever the describe form, and whichever describe-input set the last call used
    if (!e->d_blur_diag) ORBX_HIP(hipMalloc((void**)&e->d_blur_diag, e->pyr_size));
    const int ntiles = e->tile_off[e->nlevels] - e->tile_off[0];
    const Src0 s0{e->last_src0.p + (size_t)index * e->last_src0.istride, e->last_src0.step, e->last_src0.istride};
    hipLaunchKernelGGL(k_blur7, dim3(kXcds * xcd_chunk((ntiles + 3) / 4)), dim3(256), 0, e->own(),
                       e->d_pyr + (size_t)index * e->pyr_size, e->d_blur_diag, e->pyr_size, e->d_levels, e->d_tiles, ntiles, 1,
                       s0, e->tile_off[0]);
    ORBX_HIP(hipGetLastError());
    ORBX_HIP(hipStreamSynchronize(e->own()));
    const uint8_t* p = e->d_blur_diag + e->lv[level].pyr_off;          // as k_blur7 writes it
    ORBX_HIP(hipMemcpy2D(dst, dst_step, p, (size_t)w, (size_t)w, (size_t)h, hipMemcpyDeviceToHost));
    return ORBX_OK;
}

int orbx_extractor_copy_level(orbx_extractor* e, int index, int level, uint8_t* dst, size_t dst_step) {
    const uint8_t* p;
    int r, c;
    size_t sp;
    int st = orbx_extractor_level_device(e, index, level, &p, &r, &c, &sp);
    if (st) return st;
    ORBX_REQUIRE(dst && dst_step >= (size_t)c, ORBX_ERR_ARG, "bad destination");
    ORBX_HIP(hipSetDevice(e->device));
    ORBX_HIP(hipMemcpy2DAsync(dst, dst_step, p, sp, c, r, hipMemcpyDeviceToHost, e->own()));
    ORBX_HIP(hipStreamSynchronize(e->own()));
    return ORBX_OK;
}

int orbx_extractor_enable_timing(orbx_extractor* e, int enable) {
    ORBX_REQUIRE(e, ORBX_ERR_ARG, "null extractor");
    ORBX_HIP(hipSetDevice(e->device));
    for (auto& es : e->tpool) es.pending = false;
    if (enable && e->tpool.empty()) {
        e->tpool.resize(64);
        for (auto& es : e->tpool) {
            es.pending = false;
            for (auto& ev : es.ev) ORBX_HIP(hipEventCreate(&ev));
        }
    }
    e->timing = enable != 0;
    for (double& v : e->stage_ms) v = 0;
    e->timed_calls = 0;
    return ORBX_OK;
}
int orbx_extractor_stage_count(void) { return ST_COUNT; }
const char* orbx_extractor_stage_name(int s) { return (s >= 0 && s < ST_COUNT) ? kStageNames[s] : ""; }
#ifdef ORBX_QT_PROF
int orbx_debug_qt_prof(unsigned long long* out) {   // 2 x 64 stamps (diagnostics build only)
    ORBX_HIP(::orbx::device_sync());
    ORBX_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(orbx::g_qtprof), sizeof(orbx::g_qtprof)));
    return ORBX_OK;
}
#endif

int orbx_extractor_stage_times(orbx_extractor* e, double* ms, int* calls) {
    ORBX_REQUIRE(e && ms, ORBX_ERR_ARG, "null argument");
    ORBX_HIP(hipSetDevice(e->device));
    for (auto& es : e->tpool) {
        int st = e->resolve(es);
        if (st) return st;
    }
    for (int k = 0; k < ST_COUNT; ++k) ms[k] = e->stage_ms[k];
    if (calls) *calls = e->timed_calls;
    return ORBX_OK;
}

}  // extern "C"
