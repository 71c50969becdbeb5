// =====================================================================================================
// orbx_proj.hip — keypoint grid and the projection / radius matchers on gfx950.
//
//   k_grid_build   Frame::AssignFeaturesToGrid (src/Frame.cc:230-245, PosInGrid :382-392): one workgroup per
//                  keypoint set; (cell, index) keys bitonic-sorted in LDS, cell starts by binary search ->
//                  CSR cell lists with indices ascending inside a cell, the reference's mGrid[ix][iy] order.
//   k_proj_search  the window search of SearchByProjection x4, Fuse x2 and SearchBySim3 (modes in
//                  include/orbx.h): one workgroup per (query set, target view), one query per thread, the
//                  candidate walk in GetFeaturesInArea order (src/Frame.cc:327-380) so the first-minimum tie
//                  rule holds.  The assigning modes exclude keypoints that EARLIER queries of the same call
//                  were assigned to (the reference's sequential mvpMapPoints check); that dependency is solved
//                  exactly by a fixed-point iteration: every query re-evaluates its window with the keypoints
//                  claimed by earlier accepted (blocking) queries of the previous round excluded, until no
//                  choice changes.  Query 0 is final after one round and, by induction over the query order,
//                  the unique fixed point is the sequential result; real calls settle in a few rounds.
//   k_proj_init    SearchForInitialization (src/ORBmatcher.cc:407-522), whose exclusion depends on the distance
//                  of the current owner (stealing): one wave walks the queries in order, lanes over candidates.
//   k_project      the per-MapPoint projection in front of the searches (LASTFRAME :1363-1392, isInFrustum
//                  Frame.cc:269-325 + the MAPPOINTS window :62-71, Fuse :854-893): one thread per point.
// Float arithmetic is written with explicit __f*_rn (no contraction) in the reference's operation order.
// =====================================================================================================
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "orbx_common.h"

namespace orbx {

constexpr int kProjThreads = 1024;
constexpr int kGridMaxKps = 8192;          // keypoints per view (13-bit index in the sort key)
constexpr int kGridMaxCells = (1 << 19) - 1;
constexpr int kProjHisto = 30;             // HISTO_LENGTH (src/ORBmatcher.cc:39)

__device__ __forceinline__ int grid_cell(const orbx_grid& g, float x, float y) {   // PosInGrid (:382-392)
    const int px = (int)roundf(__fmul_rn(__fsub_rn(x, g.min_x), g.inv_w));
    const int py = (int)roundf(__fmul_rn(__fsub_rn(y, g.min_y), g.inv_h));
    if (px < 0 || px >= g.cols || py < 0 || py >= g.rows) return -1;
    return px * g.rows + py;
}

__device__ __forceinline__ int lower_bound_u32(const uint32_t* a, int n, uint32_t v) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (a[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(kProjThreads) void k_grid_build(const orbx_keypoint* __restrict__ kps, const int32_t* __restrict__ counts,
                                                             int n_fixed, int capacity, orbx_grid g,
                                                             int32_t* __restrict__ cell_start, int32_t* __restrict__ cell_idx) {
    extern __shared__ uint32_t gkey[];
    const int set = blockIdx.x, tid = threadIdx.x, T = blockDim.x;
    const int n = min(counts ? counts[set] : n_fixed, capacity);
    const int ncell = g.cols * g.rows;
    const orbx_keypoint* K = kps + (size_t)set * capacity;
    int32_t* cs = cell_start + (size_t)set * (ncell + 1);
    int32_t* ci = cell_idx + (size_t)set * capacity;
    int P2 = 1;
    while (P2 < n) P2 <<= 1;
    for (int i = tid; i < P2; i += T) {
        uint32_t key = 0xffffffffu;
        if (i < n) {
            const int c = grid_cell(g, K[i].x, K[i].y);
            if (c >= 0) key = ((uint32_t)c << 13) | (uint32_t)i;
        }
        gkey[i] = key;
    }
    __syncthreads();
    for (int k = 2; k <= P2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < P2; i += T) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint32_t a = gkey[i], b = gkey[ixj];
                    if ((a > b) == ((i & k) == 0)) { gkey[i] = b; gkey[ixj] = a; }
                }
            }
            __syncthreads();
        }
    for (int c = tid; c <= ncell; c += T) cs[c] = lower_bound_u32(gkey, P2, (uint32_t)c << 13);
    for (int i = tid; i < n; i += T)
        if (gkey[i] != 0xffffffffu) ci[i] = (int32_t)(gkey[i] & 0x1fffu);
}

// Counting form of the same grid (grids of < 32767 cells, the reference's 64 x 48 among them): cell counts by LDS
// atomics, an exclusive scan gives the cell starts, the keypoints are scattered into their cells by atomic cursors
// (after the scatter the cursor of cell c is the start of cell c + 1), and each cell's few indices are put back in
// ascending order by one thread -- the CSR arrays of k_grid_build (cells ascending, indices ascending inside a cell)
// from O(n) work and 4 barriers instead of the 66 stages of a 2048-key bitonic sort.
// LDS: cnt[ncell + 1] ints, then cell[cap] and idx[cap] as u16.
// The counting grid of keypoint set 'set' (its first n keypoints) by the whole workgroup; dynamic LDS gcs: (ncell + 1)
// ints + 2 x capacity u16.
__device__ __forceinline__ void grid_count_set(const orbx_keypoint* __restrict__ kps, int n, int capacity, const orbx_grid& g,
                                               int32_t* __restrict__ cell_start, int32_t* __restrict__ cell_idx, int set) {
    extern __shared__ int gcs[];
    __shared__ int tmp[kProjThreads / 64 + 1];
    const int tid = threadIdx.x, T = blockDim.x;
    const int ncell = g.cols * g.rows;
    const orbx_keypoint* K = kps + (size_t)set * capacity;
    int32_t* cs = cell_start + (size_t)set * (ncell + 1);
    int32_t* ci = cell_idx + (size_t)set * capacity;
    int* cnt = gcs;
    uint16_t* cof = reinterpret_cast<uint16_t*>(cnt + ncell + 1);
    uint16_t* idx = cof + capacity;
    for (int c = tid; c <= ncell; c += T) cnt[c] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += T) {
        const int c = grid_cell(g, K[i].x, K[i].y);
        cof[i] = (uint16_t)(c < 0 ? 0xffff : c);
        if (c >= 0) atomicAdd(&cnt[c], 1);
    }
    __syncthreads();
    block_scan_array(cnt, ncell + 1, tmp);               // cnt[c] = start of cell c; cnt[ncell] = valid keypoints
    for (int c = tid; c <= ncell; c += T) cs[c] = cnt[c];
    __syncthreads();
    for (int i = tid; i < n; i += T) {
        const int c = cof[i];
        if (c != 0xffff) idx[atomicAdd(&cnt[c], 1)] = (uint16_t)i;
    }
    __syncthreads();
    for (int c = tid; c < ncell; c += T) {               // cell c: [end of cell c - 1, cnt[c])
        const int b = c ? cnt[c - 1] : 0, e = cnt[c];
        for (int j = b + 1; j < e; ++j) {
            const uint16_t v = idx[j];
            int k = j - 1;
            while (k >= b && idx[k] > v) { idx[k + 1] = idx[k]; --k; }
            idx[k + 1] = v;
        }
    }
    __syncthreads();
    const int total = ncell ? cnt[ncell - 1] : 0;
    for (int j = tid; j < total; j += T) ci[j] = idx[j];
}

__global__ __launch_bounds__(kProjThreads) void k_grid_count(const orbx_keypoint* __restrict__ kps, const int32_t* __restrict__ counts,
                                                             int n_fixed, int capacity, orbx_grid g,
                                                             int32_t* __restrict__ cell_start, int32_t* __restrict__ cell_idx) {
    const int set = blockIdx.x;
    grid_count_set(kps, min(counts ? counts[set] : n_fixed, capacity), capacity, g, cell_start, cell_idx, set);
}

__device__ __forceinline__ int proj_rot_bin(float a1, float a2) {   // e.g. src/ORBmatcher.cc:1435-1440
    float rot = __fsub_rn(a1, a2);
    if (rot < 0.0f) rot = __fadd_rn(rot, 360.0f);
    int bin = (int)roundf(__fmul_rn(rot, 1.0f / kProjHisto));
    if (bin == kProjHisto) bin = 0;
    return bin;
}

// ---------------------------------------------------------------------------------------------
// k_proj_search.  A problem's target keypoints are staged into LDS once, in CSR (grid) order, as 16-byte entries
// {x, y, uright, meta = idx | octave << 13 | blocked << 18 | has-uright << 19} next to the cell starts, so a window walk
// costs LDS reads; only the descriptors of the candidates that pass the window's geometric tests are read from
// memory, two at a time (independent loads in flight).  Assigning modes record each query's passing candidates
// (keypoint, distance, octave) in walk order in an LDS list, so the fixed-point rounds re-evaluate a query from its
// list with the current claims and touch no descriptor again; a query with more candidates than the list holds walks
// again.  Problems whose cells and keypoints do not fit in LDS read them from memory (same walk, kLds = false).
// ---------------------------------------------------------------------------------------------
constexpr uint32_t kMetaBlocked = 1u << 18, kMetaUr = 1u << 19;
constexpr int kProjListMax = 16;           // candidates recorded per query (assigning modes)
constexpr int kProjBatch = 2;              // descriptor loads in flight per query walk (2: <= 64 VGPRs, two 16-wave
                                           // workgroups per CU)
constexpr uint8_t kQmBlocks = 0x80, kQmSkip = 0x40, kQmCount = 0x3f;   // per-query byte: flags + list count
constexpr uint8_t kQmOverflow = 0x3f;

// The reference's running minimum and second minimum over the window in walk order (e.g. src/ORBmatcher.cc:96-110):
// (bestDist, bestLevel, bestIdx) and (bestDist2, bestLevel2).
struct ProjBest {
    int d1, l1, i1, d2, l2;
    __device__ __forceinline__ void init(int v) { d1 = d2 = v; l1 = l2 = i1 = -1; }
    __device__ __forceinline__ void add(int dist, int lvl, int idx) {
        if (dist < d1) { d2 = d1; l2 = l1; d1 = dist; l1 = lvl; i1 = idx; }
        else if (dist < d2) { l2 = lvl; d2 = dist; }
    }
};
__device__ __forceinline__ int proj_accept(const orbx_proj_params& P, const ProjBest& b) {
    if (b.i1 < 0 || b.d1 > P.accept_max) return -1;
    if (P.mode == ORBX_PROJ_MAPPOINTS && b.l1 == b.l2 && (float)b.d1 > __fmul_rn(P.nnratio, (float)b.d2)) return -1;   // :122
    return b.i1;
}

struct ProjWin { int x0, x1, y0, y1; };
__device__ __forceinline__ bool proj_window(const orbx_grid& g, const orbx_proj_query& Q, ProjWin& w) {   // Frame.cc:327-345
    const float x = Q.x, y = Q.y, r = Q.r;
    w.x0 = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(x, g.min_x), r), g.inv_w)));
    if (w.x0 >= g.cols) return false;
    w.x1 = min(g.cols - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(x, g.min_x), r), g.inv_w)));
    if (w.x1 < 0) return false;
    w.y0 = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(y, g.min_y), r), g.inv_h)));
    if (w.y0 >= g.rows) return false;
    w.y1 = min(g.rows - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(y, g.min_y), r), g.inv_h)));
    return w.y1 >= 0;
}

// CSR entry j of a problem: staged in LDS, or assembled from the problem's arrays
__device__ __forceinline__ float4 proj_entry_of(const orbx_proj_problem& pb, int idx);
template <bool kLds>
__device__ __forceinline__ float4 proj_entry(const orbx_proj_problem& pb, const float4* ent, int j) {
    if constexpr (kLds) return ent[j];
    return proj_entry_of(pb, pb.cell_idx[j]);
}
// the 16-byte staged entry of target keypoint idx: {x, y, uright, idx | octave << 13 | blocked | has-uright}
__device__ __forceinline__ float4 proj_entry_of(const orbx_proj_problem& pb, int idx) {
    const orbx_keypoint kp = pb.kps[idx];
    uint32_t meta = (uint32_t)idx | ((uint32_t)kp.octave << 13);
    if (pb.blocked && pb.blocked[idx]) meta |= kMetaBlocked;
    float ur = 0.0f;
    if (pb.uright) { ur = pb.uright[idx]; meta |= kMetaUr; }
    return make_float4(kp.x, kp.y, ur, __uint_as_float(meta));
}

// The geometric / level / stereo / reprojection tests of one candidate (everything but the descriptor and the claims),
// in the reference's order of checks (GetFeaturesInArea :352-372, then e.g. :81-94, :1406-1426, :906-941).
template <bool kAssign>
__device__ __forceinline__ bool proj_pass(const orbx_proj_params& P, const float* isg, const orbx_proj_query& Q, bool check,
                                          bool stereo_tol, float4 e) {
    const uint32_t meta = __float_as_uint(e.w);
    const int oct = (int)((meta >> 13) & 31u);
    if (check) {
        if (oct < Q.min_level) return false;
        if (Q.max_level >= 0 && oct > Q.max_level) return false;
    }
    if (!(fabsf(__fsub_rn(e.x, Q.x)) < Q.r && fabsf(__fsub_rn(e.y, Q.y)) < Q.r)) return false;
    if (kAssign && (meta & kMetaBlocked)) return false;
    if (kAssign && stereo_tol && (meta & kMetaUr) && e.z > 0.0f && fabsf(__fsub_rn(Q.ur, e.z)) > Q.ur_tol) return false;
    if (!kAssign && P.mode == ORBX_PROJ_FUSE) {
        const float ex = __fsub_rn(Q.x, e.x), ey = __fsub_rn(Q.y, e.y);
        if ((meta & kMetaUr) && e.z >= 0.0f) {
            const float er = __fsub_rn(Q.ur, e.z);
            const float e2 = __fadd_rn(__fadd_rn(__fmul_rn(ex, ex), __fmul_rn(ey, ey)), __fmul_rn(er, er));
            if ((double)__fmul_rn(e2, isg[oct]) > 7.8) return false;
        } else {
            const float e2 = __fadd_rn(__fmul_rn(ex, ex), __fmul_rn(ey, ey));
            if ((double)__fmul_rn(e2, isg[oct]) > 5.99) return false;
        }
    }
    return true;
}

// One query's window walk in GetFeaturesInArea order (cells ix-major, indices ascending inside a cell).  claim: skip
// keypoints claimed by an earlier blocking query (nullptr: no claims).  list (stride nq, nullptr: none) receives the
// passing candidates as idx | dist << 13 | octave << 22; returns their count, or kQmOverflow past kcap.
template <bool kLds, bool kAssign>
__device__ int proj_walk(const orbx_proj_params& P, const float* isg, const orbx_grid& g, const orbx_proj_problem& pb, int q,
                         const orbx_proj_query& Q, const int* cs, const float4* ent, const int* claim, uint32_t* list,
                         int nq, int kcap, ProjBest& best) {
    best.init((!kAssign && P.mode == ORBX_PROJ_BEST) ? INT_MAX : 256);
    ProjWin w;
    if (!proj_window(g, Q, w)) return 0;
    const bool check = (Q.min_level > 0) || (Q.max_level >= 0);
    const bool stereo_tol = (P.mode == ORBX_PROJ_MAPPOINTS || P.mode == ORBX_PROJ_LASTFRAME) && pb.uright && Q.ur_tol >= 0.0f;
    const uint4* qd = reinterpret_cast<const uint4*>(pb.qdesc + 32 * (size_t)q);
    const uint4 a0 = qd[0], a1 = qd[1];
    int nrec = 0;
    uint32_t pm[kProjBatch];            // pending candidates: idx | octave << 22
    int np = 0;
    auto flush = [&]() {
        uint4 d[kProjBatch][2];
#pragma unroll
        for (int k = 0; k < kProjBatch; ++k)
            if (k < np) {
                const uint4* kd = reinterpret_cast<const uint4*>(pb.desc + 32 * (size_t)(pm[k] & 0x1fffu));
                d[k][0] = kd[0];
                d[k][1] = kd[1];
            }
#pragma unroll
        for (int k = 0; k < kProjBatch; ++k)
            if (k < np) {
                const int idx = (int)(pm[k] & 0x1fffu), oct = (int)(pm[k] >> 22);
                const int dist = hamming256(a0, a1, d[k][0], d[k][1]);
                best.add(dist, oct, idx);
                if (kAssign && list) {
                    if (nrec < kcap) list[(size_t)nrec * nq + q] = (uint32_t)idx | ((uint32_t)dist << 13) | ((uint32_t)oct << 22);
                    ++nrec;
                }
            }
        np = 0;
    };
    for (int ix = w.x0; ix <= w.x1; ++ix)
        for (int iy = w.y0; iy <= w.y1; ++iy) {
            const int c = ix * g.rows + iy;
            const int j1 = cs[c + 1];
            for (int j = cs[c]; j < j1; ++j) {
                const float4 e = proj_entry<kLds>(pb, ent, j);
                if (!proj_pass<kAssign>(P, isg, Q, check, stereo_tol, e)) continue;
                const uint32_t meta = __float_as_uint(e.w);
                const int idx = (int)(meta & 0x1fffu);
                if (kAssign && claim && claim[idx] < q) continue;
                const uint32_t v = (uint32_t)idx | (((meta >> 13) & 31u) << 22);
                if (np == 0) pm[0] = v; else pm[kProjBatch - 1] = v;
                if (++np == kProjBatch) flush();
            }
        }
    flush();
    return nrec > kcap ? (int)kQmOverflow : nrec;
}

// A problem larger than the launch's LDS plan (max_n / max_nq of orbx_proj_search_batch_device) is not searched:
// its q_idx / q_dist are -1 and *nmatches = -1, never an LDS overrun.  Workgroup-uniform (one problem per workgroup).
// When the launch builds the grid (ncell >= 0: orbx_proj_search_grid_batch_device) the problem's grid is written empty
// (every cell_start 0), so a later search of the same frame walks no stale CSR entries.
__device__ __forceinline__ bool proj_over_cap(const orbx_proj_problem& pb, int n_cap, int nq_cap, int tid, int T,
                                              int ncell = -1) {
    if (pb.n <= n_cap && pb.nq <= nq_cap) return false;
    for (int q = tid; q < pb.nq; q += T) { pb.q_idx[q] = -1; pb.q_dist[q] = -1; }
    if (tid == 0 && pb.nmatches) *pb.nmatches = -1;
    if (ncell >= 0)
        for (int c = tid; c <= ncell; c += T) const_cast<int32_t*>(pb.cell_start)[c] = 0;
    return true;
}

// Frame::AssignFeaturesToGrid (src/Frame.cc:230-245) of a problem's first ng target keypoints inside its search
// workgroup -- the counting form of k_grid_count (cell counts by LDS atomics, exclusive scan, scatter by atomic cursors,
// each cell's indices put back in ascending order by one thread), so the CSR arrays are the same -- leaving the cell
// starts in cs_l[0 .. ncell] and the entries in CSR order in ent_l, and writing both arrays to the problem's cell_start /
// cell_idx for later searches of the same frame.  cof / idx: 2 x ng u16 of scratch LDS; tmp: nwaves + 1 ints.
__device__ void proj_grid_stage(const orbx_proj_problem& pb, const orbx_grid& g, int ng, int ncell, int* cs_l, float4* ent_l,
                                uint16_t* cof, uint16_t* idx, int* tmp) {
    const int tid = threadIdx.x, T = blockDim.x;
    for (int c = tid; c <= ncell; c += T) cs_l[c] = 0;
    __syncthreads();
    for (int i = tid; i < ng; i += T) {
        const int c = grid_cell(g, pb.kps[i].x, pb.kps[i].y);
        cof[i] = (uint16_t)(c < 0 ? 0xffff : c);
        if (c >= 0) atomicAdd(&cs_l[c], 1);
    }
    __syncthreads();
    block_scan_array(cs_l, ncell + 1, tmp);              // cs_l[c] = start of cell c; cs_l[ncell] = keypoints in cells
    int32_t* gcs = const_cast<int32_t*>(pb.cell_start);
    for (int c = tid; c <= ncell; c += T) gcs[c] = cs_l[c];
    __syncthreads();
    for (int i = tid; i < ng; i += T) {
        const int c = cof[i];
        if (c != 0xffff) idx[atomicAdd(&cs_l[c], 1)] = (uint16_t)i;
    }
    __syncthreads();                                     // cs_l[c] = end of cell c
    for (int c = tid; c < ncell; c += T) {
        const int b = c ? cs_l[c - 1] : 0, e = cs_l[c];
        for (int j = b + 1; j < e; ++j) {
            const uint16_t v = idx[j];
            int k = j - 1;
            while (k >= b && idx[k] > v) { idx[k + 1] = idx[k]; --k; }
            idx[k + 1] = v;
        }
    }
    __syncthreads();
    const int total = ncell ? cs_l[ncell - 1] : 0;
    int32_t* gci = const_cast<int32_t*>(pb.cell_idx);
    for (int j = tid; j < total; j += T) {
        const int k = idx[j];
        gci[j] = k;
        ent_l[j] = proj_entry_of(pb, k);
    }
    // starts back in place (start[c] = end[c - 1], start[ncell] = total): chunks of 4 T cells from the top down, so a
    // chunk reads its lower neighbour before that neighbour is rewritten
    const int nch = (ncell + 1 + 4 * T - 1) / (4 * T);
    for (int ch = nch - 1; ch >= 0; --ch) {
        int v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int c = ch * 4 * T + r * T + tid;
            v[r] = (c <= ncell && c > 0) ? cs_l[c - 1] : 0;
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int c = ch * 4 * T + r * T + tid;
            if (c <= ncell) cs_l[c] = v[r];
        }
        __syncthreads();
    }
}

// Modes MAPPOINTS .. BEST.  Dynamic LDS: [kLds: cell starts (ncell + 1), entries (16 B x n)] then, for the assigning
// modes, claim[n], own[n], res[nq] (idx | dist << 13, or -1), qm[nq] (kQm* byte) and the lists (kcap x nq).
template <bool kLds, bool kAssign>
__global__ __launch_bounds__(kProjThreads, kAssign ? 4 : 8) void k_proj_search(orbx_proj_params P, orbx_grid g,
                                                              const orbx_proj_problem* __restrict__ probs, int n_cap,
                                                              int nq_cap, int kcap, const int32_t* __restrict__ grid_counts) {
    extern __shared__ __attribute__((aligned(16))) int psm[];
    __shared__ int changed, hist[32], keep[3], acc_sh, bad_sh;
    __shared__ float isg[32];                          // mvInvLevelSigma2 (a per-lane index into the kernel arguments
                                                       // would be a vector load from the argument buffer per candidate)
    const orbx_proj_problem pb = probs[blockIdx.x];
    const int tid = threadIdx.x, T = blockDim.x, nq = pb.nq, n = pb.n;
    const int ncell = g.cols * g.rows;
    // grid_counts[p] >= 0: this problem's grid is built here from its first grid_counts[p] keypoints and written out;
    // < 0: it is read (staged) from cell_start / cell_idx as without grid_counts
    const int gcount = grid_counts ? grid_counts[blockIdx.x] : -1;
    if (proj_over_cap(pb, n_cap, nq_cap, tid, T, (kLds && gcount >= 0) ? ncell : -1)) return;
    if (tid < 32) isg[tid] = P.inv_sigma2[tid];
    char* lp = reinterpret_cast<char*>(psm);
    const int* cs = pb.cell_start;
    const float4* ent = nullptr;
    if constexpr (kLds) {
        int* cs_l = reinterpret_cast<int*>(lp);
        lp += ((size_t)(ncell + 1) * 4 + 15) & ~(size_t)15;
        float4* ent_l = reinterpret_cast<float4*>(lp);
        lp += (size_t)16 * n_cap;
        if (gcount >= 0) {
            // the grid built here (orbx_proj_search_grid_batch_device); scratch: the LDS after the entries, free until the
            // assigning modes' arrays are initialised below (the launch reserves it for the non-assigning ones)
            uint16_t* cof = reinterpret_cast<uint16_t*>(lp);
            proj_grid_stage(pb, g, min(gcount, n), ncell, cs_l, ent_l, cof, cof + n_cap, hist);
        } else {
            for (int c = tid; c <= ncell; c += T) cs_l[c] = pb.cell_start[c];
            const int ncsr = min(pb.cell_start[ncell], n);
            for (int j = tid; j < ncsr; j += T) ent_l[j] = proj_entry<false>(pb, nullptr, j);
        }
        cs = cs_l;
        ent = ent_l;
    }
    if (tid == 0) { acc_sh = 0; bad_sh = 0; }
    if (tid < 32) hist[tid] = 0;
    __syncthreads();
    if constexpr (!kAssign) {
        int acc = 0;
        for (int q = tid; q < nq; q += T) {
            const orbx_proj_query Q = pb.queries[q];
            int r = -1;
            ProjBest b;
            if (!(Q.flags & ORBX_QF_SKIP)) {
                proj_walk<kLds, false>(P, isg, g, pb, q, Q, cs, ent, nullptr, nullptr, nq, 0, b);
                r = proj_accept(P, b);
            }
            pb.q_idx[q] = r;
            pb.q_dist[q] = r >= 0 ? b.d1 : -1;
            acc += r >= 0;
        }
        acc = wave_sum(acc);
        if (lane_id() == 0 && acc) atomicAdd(&acc_sh, acc);
        __syncthreads();
        if (tid == 0) *pb.nmatches = acc_sh;
        return;
    } else {
    int* claim = reinterpret_cast<int*>(lp);
    int* own = claim + n_cap;
    int* res = own + n_cap;
    uint8_t* qm = reinterpret_cast<uint8_t*>(res + nq_cap);
    uint32_t* list = reinterpret_cast<uint32_t*>(lp + (((size_t)8 * n_cap + 4 * (size_t)nq_cap + nq_cap + 15) & ~(size_t)15));
    // round 0: every query's walk without claims, its candidates recorded
    for (int q = tid; q < nq; q += T) {
        const orbx_proj_query Q = pb.queries[q];
        int r = -1, m = (Q.flags & ORBX_QF_BLOCKS) ? kQmBlocks : 0;
        if (Q.flags & ORBX_QF_SKIP) {
            m |= kQmSkip;
        } else {
            ProjBest b;
            const int cnt = proj_walk<kLds, true>(P, isg, g, pb, q, Q, cs, ent, nullptr, kcap > 0 ? list : nullptr, nq, kcap, b);
            m |= kcap > 0 ? cnt : kQmOverflow;                // no list room: every round walks again
            r = proj_accept(P, b);
            if (r >= 0) r |= b.d1 << 13;
        }
        res[q] = r;
        qm[q] = (uint8_t)m;
    }
    // fixed-point rounds: claims from the current results, every query re-evaluated with them (from its list, or by a
    // new walk when the list overflowed), until no result changes (at most nq rounds: query q is final after q + 1)
    for (int round = 1; round <= nq; ++round) {
        for (int i = tid; i < n; i += T) claim[i] = INT_MAX;
        __syncthreads();                               // every thread has read the previous round's 'changed'
        if (tid == 0) changed = 0;
        for (int q = tid; q < nq; q += T) {
            const int r = res[q];
            if (r >= 0 && (qm[q] & kQmBlocks)) atomicMin(&claim[r & 0x1fff], q);
        }
        __syncthreads();
        int ch = 0;
        for (int q = tid; q < nq; q += T) {
            const int m = qm[q];
            if (m & kQmSkip) continue;
            const int cnt = m & kQmCount;
            ProjBest b;
            if (cnt != kQmOverflow) {
                b.init(256);
                for (int k = 0; k < cnt; ++k) {
                    const uint32_t v = list[(size_t)k * nq + q];
                    const int idx = (int)(v & 0x1fffu);
                    if (claim[idx] < q) continue;
                    b.add((int)((v >> 13) & 0x1ffu), (int)(v >> 22), idx);
                }
            } else {
                proj_walk<kLds, true>(P, isg, g, pb, q, pb.queries[q], cs, ent, claim, nullptr, nq, 0, b);
            }
            int r = proj_accept(P, b);
            if (r >= 0) r |= b.d1 << 13;
            if (r != res[q]) { ch = 1; res[q] = r; }
        }
        if (ch) changed = 1;
        __syncthreads();
        if (!changed) break;                           // workgroup-uniform
    }
    // final assignment: the last accepted query writes mvpMapPoints[idx] (src/ORBmatcher.cc:125, :1430, :1559, :398)
    for (int i = tid; i < n; i += T) own[i] = -1;
    __syncthreads();
    const bool rot = P.check_ori && (P.mode == ORBX_PROJ_LASTFRAME || P.mode == ORBX_PROJ_KEYFRAME);
    int acc = 0;
    for (int q = tid; q < nq; q += T) {
        const int v = res[q];
        pb.q_idx[q] = v >= 0 ? (v & 0x1fff) : -1;
        pb.q_dist[q] = v >= 0 ? (v >> 13) : -1;
        if (v < 0) continue;
        const int r = v & 0x1fff;
        ++acc;
        atomicMax(&own[r], q);
        if (rot) atomicAdd(&hist[proj_rot_bin(pb.queries[q].angle, pb.kps[r].angle)], 1);
    }
    acc = wave_sum(acc);
    if (lane_id() == 0 && acc) atomicAdd(&acc_sh, acc);
    __syncthreads();
    if (rot) {
        // ComputeThreeMaxima (:1603-1644), then every entry of the other bins sets mvpMapPoints[idx] = NULL
        if (tid == 0) {
            int m1 = 0, m2 = 0, m3 = 0, i1 = -1, i2 = -1, i3 = -1;
            for (int i = 0; i < kProjHisto; ++i) {
                const int s = hist[i];
                if (s > m1) { m3 = m2; m2 = m1; m1 = s; i3 = i2; i2 = i1; i1 = i; }
                else if (s > m2) { m3 = m2; m2 = s; i3 = i2; i2 = i; }
                else if (s > m3) { m3 = s; i3 = i; }
            }
            if (m2 < 0.1f * (float)m1) { i2 = -1; i3 = -1; }
            else if (m3 < 0.1f * (float)m1) { i3 = -1; }
            keep[0] = i1; keep[1] = i2; keep[2] = i3;
        }
        __syncthreads();
        int bad = 0;
        for (int q = tid; q < nq; q += T) {
            const int v = res[q];
            if (v < 0) continue;
            const int r = v & 0x1fff;
            const int b = proj_rot_bin(pb.queries[q].angle, pb.kps[r].angle);
            if (b == keep[0] || b == keep[1] || b == keep[2]) continue;
            own[r] = -2;
            ++bad;
        }
        bad = wave_sum(bad);
        if (lane_id() == 0 && bad) atomicAdd(&bad_sh, bad);
        __syncthreads();
    }
    for (int i = tid; i < n; i += T) pb.owner[i] = own[i];
    if (tid == 0) *pb.nmatches = acc_sh - bad_sh;
    }
}

// SearchForInitialization: one wave per problem walks the queries in order.  Dynamic LDS: matchedDist[n],
// m21[n] (vMatchedDistance / vnMatches21 of :417-418) and res[nq] (vnMatches12).
constexpr int kInitNone = 1023;   // "INT_MAX" distance inside the packed (distance << 20 | position) key

__global__ __launch_bounds__(64) void k_proj_init(orbx_proj_params P, orbx_grid g, const orbx_proj_problem* __restrict__ probs,
                                                  int n_cap, int nq_cap) {
    extern __shared__ int ism[];
    __shared__ int hist[32];
    const orbx_proj_problem pb = probs[blockIdx.x];
    const int ln = lane_id(), nq = pb.nq, n = pb.n;
    if (proj_over_cap(pb, n_cap, nq_cap, ln, kWave)) return;
    int* mdist = ism;
    int* m21 = ism + n;
    int* res = ism + 2 * n;
    for (int i = ln; i < n; i += kWave) { mdist[i] = INT_MAX; m21[i] = -1; }
    for (int i = ln; i < nq; i += kWave) res[i] = -1;
    if (ln < 32) hist[ln] = 0;
    __syncthreads();
    int nm = 0;
    for (int q = 0; q < nq; ++q) {
        const orbx_proj_query Q = pb.queries[q];
        if (Q.flags & ORBX_QF_SKIP) continue;
        const float x = Q.x, y = Q.y, r = Q.r;
        const int nMinCellX = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(x, g.min_x), r), g.inv_w)));
        if (nMinCellX >= g.cols) continue;
        const int nMaxCellX = min(g.cols - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(x, g.min_x), r), g.inv_w)));
        if (nMaxCellX < 0) continue;
        const int nMinCellY = max(0, (int)floorf(__fmul_rn(__fsub_rn(__fsub_rn(y, g.min_y), r), g.inv_h)));
        if (nMinCellY >= g.rows) continue;
        const int nMaxCellY = min(g.rows - 1, (int)ceilf(__fmul_rn(__fadd_rn(__fsub_rn(y, g.min_y), r), g.inv_h)));
        if (nMaxCellY < 0) continue;
        const bool check = (Q.min_level > 0) || (Q.max_level >= 0);
        const uint4* qd = reinterpret_cast<const uint4*>(pb.qdesc + 32 * (size_t)q);
        const uint4 a0 = qd[0], a1 = qd[1];
        // running best (b1, position bp, keypoint bi) and second b2 over the candidates in walk order; the
        // sequential update rule keeps as second the smallest value among the non-best candidates
        int b1 = kInitNone, b2 = kInitNone, bi = -1, pos = 0;
        for (int ix = nMinCellX; ix <= nMaxCellX; ++ix)
            for (int iy = nMinCellY; iy <= nMaxCellY; ++iy) {
                const int c = ix * g.rows + iy;
                const int j0 = pb.cell_start[c], j1 = pb.cell_start[c + 1];
                for (int jb = j0; jb < j1; jb += kWave) {
                    const int j = jb + ln;
                    int d = kInitNone, idx = -1;
                    if (j < j1) {
                        idx = pb.cell_idx[j];
                        const orbx_keypoint kp = pb.kps[idx];
                        bool ok = true;
                        if (check) {
                            if (kp.octave < Q.min_level) ok = false;
                            if (Q.max_level >= 0 && kp.octave > Q.max_level) ok = false;
                        }
                        if (!(fabsf(__fsub_rn(kp.x, x)) < r && fabsf(__fsub_rn(kp.y, y)) < r)) ok = false;
                        if (ok) {
                            const uint4* kd = reinterpret_cast<const uint4*>(pb.desc + 32 * (size_t)idx);
                            const int dist = hamming256(a0, a1, kd[0], kd[1]);
                            if (!(mdist[idx] <= dist)) d = dist;           // :446-447
                        }
                    }
                    const uint32_t key = ((uint32_t)d << 20) | (uint32_t)(pos + ln);
                    const uint32_t m = wave_min_u32(key);
                    const int cb1 = (int)(m >> 20);
                    const int cb2 = (int)wave_min_u32(key == m ? (uint32_t)kInitNone : (uint32_t)d);
                    const int cidx = __builtin_amdgcn_readlane(idx, (int)(m & 0xfffff) - pos);
                    if (cb1 < b1) { b2 = min(b1, cb2); b1 = cb1; bi = cidx; }
                    else { b2 = min(b2, min(cb1, cb2)); }
                    pos += min(kWave, j1 - jb);
                }
            }
        if (bi < 0 || b1 == kInitNone || b1 > P.accept_max) continue;
        const float second = b2 == kInitNone ? (float)INT_MAX : (float)b2;
        if (!((float)b1 < __fmul_rn(second, P.nnratio))) continue;         // :463
        if (ln == 0) {
            if (m21[bi] >= 0) res[m21[bi]] = -1;                            // :465-469
            res[q] = bi;
            m21[bi] = q;
            mdist[bi] = b1;
            if (P.check_ori) hist[proj_rot_bin(Q.angle, pb.kps[bi].angle)] += 1;
        }
        nm += 1;
        __syncthreads();
    }
    __syncthreads();
    // nmatches = accepted - stolen - rotation-filtered (:461-514); stolen entries have res == -1 already
    int owners = 0;
    for (int q = ln; q < nq; q += kWave) owners += res[q] >= 0;
    owners = wave_sum(owners);
    int keep0 = -1, keep1 = -1, keep2 = -1;
    if (P.check_ori) {
        int m1 = 0, m2 = 0, m3 = 0, i1 = -1, i2 = -1, i3 = -1;
        for (int i = 0; i < kProjHisto; ++i) {
            const int s = hist[i];
            if (s > m1) { m3 = m2; m2 = m1; m1 = s; i3 = i2; i2 = i1; i1 = i; }
            else if (s > m2) { m3 = m2; m2 = s; i3 = i2; i2 = i; }
            else if (s > m3) { m3 = s; i3 = i; }
        }
        if (m2 < 0.1f * (float)m1) { i2 = -1; i3 = -1; }
        else if (m3 < 0.1f * (float)m1) { i3 = -1; }
        keep0 = i1; keep1 = i2; keep2 = i3;
    }
    int dropped = 0;
    for (int q = ln; q < nq; q += kWave) {
        int r = res[q];
        if (r >= 0 && P.check_ori) {
            const int b = proj_rot_bin(pb.queries[q].angle, pb.kps[r].angle);
            if (b != keep0 && b != keep1 && b != keep2) { r = -1; ++dropped; }
        }
        pb.q_idx[q] = r;
        pb.q_dist[q] = r >= 0 ? mdist[r] : -1;
    }
    dropped = wave_sum(dropped);
    (void)nm;
    if (ln == 0) *pb.nmatches = owners - dropped;
}

// ---------------------------------------------------------------------------------------------
// Projection step (include/orbx.h orbx_proj_project): one thread per MapPoint, the reference's operation order for
// each caller, pinned as the oracle (oracle/proj_oracle.cpp orc_project): Rcw * X + tcw as float products summed left
// to right (OpenCV's 3x3 gemm fast path), cv::norm / Mat::dot of a 3-vector with double products accumulated left to
// right in double (OpenCV 3.2 normL2Sqr<float, double> / dotProd_), PredictScale's log in double.
// ---------------------------------------------------------------------------------------------
struct ProjScales { float s[32]; };

__device__ __forceinline__ double norm2_d(float x, float y, float z) {          // ((0 + x*x) + y*y) + z*z in double
    const double a = x, b = y, c = z;
    return __dadd_rn(__dadd_rn(__dmul_rn(a, a), __dmul_rn(b, b)), __dmul_rn(c, c));
}
__device__ __forceinline__ double dot3_d(float x, float y, float z, float u, float v, float w) {
    return __dadd_rn(__dadd_rn(__dmul_rn((double)x, (double)u), __dmul_rn((double)y, (double)v)),
                     __dmul_rn((double)z, (double)w));
}

__device__ __forceinline__ int predict_scale(float max_dist, float dist, float log_sf, int nlevels) {   // MapPoint.cc:389-421
    const float ratio = __fdiv_rn(max_dist, dist);
    int n = (int)ceil(__ddiv_rn(log((double)ratio), (double)log_sf));
    if (n < 0) n = 0;
    else if (n >= nlevels) n = nlevels - 1;
    return n;
}

__global__ __launch_bounds__(256) void k_project(int mode, const orbx_map_point* __restrict__ pts, const int32_t* __restrict__ counts,
                                                 int n_fixed, int capacity, const orbx_view* __restrict__ views,
                                                 const int32_t* __restrict__ view_points, ProjScales sc, int nlevels,
                                                 float log_sf, const int32_t* __restrict__ found,
                                                 orbx_proj_query* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x, vi = blockIdx.y;
    if (i >= capacity) return;
    const int set = view_points ? view_points[vi] : vi;
    const int n = counts ? min(counts[set], capacity) : n_fixed;
    const orbx_view& V = views[vi];
    orbx_proj_query q;
    q.x = q.y = q.r = 0.0f;
    q.min_level = -1; q.max_level = -1;
    q.ur = 0.0f; q.ur_tol = -1.0f; q.angle = 0.0f;
    q.level = -1;
    q.flags = ORBX_QF_SKIP;
    orbx_proj_query* o = out + (size_t)vi * capacity + i;
    if (i >= n) { *o = q; return; }                                    // rows past the set's count: skipped
    const orbx_map_point p = pts[(size_t)set * capacity + i];
    auto dot3 = [](float a, float b, float c, float x, float y, float z, float t) {   // ((a x + b y) + c z) + t
        return __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(a, x), __fmul_rn(b, y)), __fmul_rn(c, z)), t);
    };
    const float xc = dot3(V.R[0], V.R[1], V.R[2], p.x, p.y, p.z, V.t[0]);
    const float yc = dot3(V.R[3], V.R[4], V.R[5], p.x, p.y, p.z, V.t[1]);
    const float zc = dot3(V.R[6], V.R[7], V.R[8], p.x, p.y, p.z, V.t[2]);
    if ((p.flags & ORBX_QF_SKIP) || (found && found[(size_t)vi * capacity + i] >= 0)) { *o = q; return; }
    if (mode == ORBX_PROJ_LASTFRAME) {
        const float invzc = (float)__ddiv_rn(1.0, (double)zc);                           // :1368
        const float u = __fadd_rn(__fmul_rn(__fmul_rn(V.fx, xc), invzc), V.cx);
        const float v = __fadd_rn(__fmul_rn(__fmul_rn(V.fy, yc), invzc), V.cy);
        if (invzc < 0 || u < V.min_x || u > V.max_x || v < V.min_y || v > V.max_y) { *o = q; return; }
        const int oct = p.octave;
        const float radius = __fmul_rn(V.th, sc.s[oct]);                                   // :1384
        q.x = u; q.y = v; q.r = radius;
        if (V.level_mode > 0) { q.min_level = oct; q.max_level = -1; }                     // :1388-1393
        else if (V.level_mode < 0) { q.min_level = 0; q.max_level = oct; }
        else { q.min_level = oct - 1; q.max_level = oct + 1; }
        q.ur = __fsub_rn(u, __fmul_rn(V.bf, invzc));                                        // :1418-1426
        q.ur_tol = radius;
        q.angle = p.angle;
        q.level = oct;
    } else {
        float u, v, invz;
        if (zc < 0.0f) { *o = q; return; }
        if (mode == ORBX_PROJ_MAPPOINTS) {                                                  // Frame::isInFrustum
            invz = __fdiv_rn(1.0f, zc);
            u = __fadd_rn(__fmul_rn(__fmul_rn(V.fx, xc), invz), V.cx);
            v = __fadd_rn(__fmul_rn(__fmul_rn(V.fy, yc), invz), V.cy);
            if (u < V.min_x || u > V.max_x || v < V.min_y || v > V.max_y) { *o = q; return; }
        } else {                                                                            // Fuse :857-871
            invz = __fdiv_rn(1.0f, zc);
            u = __fadd_rn(__fmul_rn(V.fx, __fmul_rn(xc, invz)), V.cx);
            v = __fadd_rn(__fmul_rn(V.fy, __fmul_rn(yc, invz)), V.cy);
            if (!(u >= V.min_x && u < V.max_x && v >= V.min_y && v < V.max_y)) { *o = q; return; }
        }
        const float maxD = __fmul_rn(1.2f, p.max_dist), minD = __fmul_rn(0.8f, p.min_dist);  // MapPoint.cc:377-387
        const float POx = __fsub_rn(p.x, V.Ow[0]), POy = __fsub_rn(p.y, V.Ow[1]), POz = __fsub_rn(p.z, V.Ow[2]);
        const float dist = (float)__dsqrt_rn(norm2_d(POx, POy, POz));                   // cv::norm
        if (dist < minD || dist > maxD) { *o = q; return; }
        const double dot = dot3_d(POx, POy, POz, p.nx, p.ny, p.nz);                         // PO.dot(Pn)
        const int pred = predict_scale(p.max_dist, dist, log_sf, nlevels);
        if (mode == ORBX_PROJ_MAPPOINTS) {
            const float viewCos = (float)__ddiv_rn(dot, (double)dist);                       // Frame.cc:308-311
            if (viewCos < V.view_cos_limit) { *o = q; return; }
            float r = (double)viewCos > 0.998 ? 2.5f : 4.0f;                                 // RadiusByViewingCos
            if (V.th != 1.0f) r = __fmul_rn(r, V.th);
            q.x = u; q.y = v; q.r = __fmul_rn(r, sc.s[pred]);
            q.min_level = pred - 1; q.max_level = pred;
            q.ur = __fsub_rn(u, __fmul_rn(V.bf, invz));                                     // mTrackProjXR
            q.ur_tol = __fmul_rn(r, sc.s[pred]);
        } else {
            if (dot < __dmul_rn(0.5, (double)dist)) { *o = q; return; }                    // :887-888
            q.x = u; q.y = v; q.r = __fmul_rn(V.th, sc.s[pred]);
            q.min_level = pred - 1; q.max_level = pred;
            q.ur = __fsub_rn(u, __fmul_rn(V.bf, invz));
        }
        q.level = pred;
    }
    q.flags = p.flags & ~ORBX_QF_SKIP;
    *o = q;
}

// MapPoints of stereo frames: Frame::UnprojectStereo (src/Frame.cc:666-680) and the Frame form of the MapPoint
// constructor (src/MapPoint.cc:47-68).  One thread per keypoint.  Pinned as the projection: Rwc * x3Dc + Ow as float
// products summed left to right; cv::norm with double squares summed in double and a double sqrt; the normal divided as
// cv::Mat / double (the scale 1 / norm rounded to float, then a float product per component).
__device__ __forceinline__ void stereo_mappoint(const orbx_keypoint* __restrict__ kps, const float* __restrict__ depth,
                                                int capacity, const float* __restrict__ twc, const float4& cam,
                                                const ProjScales& sc, int nlevels, int flags, orbx_map_point* __restrict__ out,
                                                int b, int i) {
    const size_t o = (size_t)b * capacity + i;
    const orbx_keypoint kp = kps[o];
    const float z = depth[o];
    orbx_map_point p{};
    p.octave = kp.octave;
    p.angle = kp.angle;
    p.flags = ORBX_QF_SKIP;
    if (z > 0) {
        const float* T = twc + 12 * (size_t)b;
        const float x = __fmul_rn(__fmul_rn(__fsub_rn(kp.x, cam.z), z), __fdiv_rn(1.0f, cam.x));   // (u-cx)*z*invfx
        const float y = __fmul_rn(__fmul_rn(__fsub_rn(kp.y, cam.w), z), __fdiv_rn(1.0f, cam.y));
        auto row = [&](int r) {
            return __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(T[3 * r], x), __fmul_rn(T[3 * r + 1], y)), __fmul_rn(T[3 * r + 2], z)),
                             T[9 + r]);
        };
        p.x = row(0); p.y = row(1); p.z = row(2);
        const float dx = __fsub_rn(p.x, T[9]), dy = __fsub_rn(p.y, T[10]), dz = __fsub_rn(p.z, T[11]);
        const double nrm = __dsqrt_rn(norm2_d(dx, dy, dz));                                   // cv::norm
        const float inv = (float)__ddiv_rn(1.0, nrm);
        p.nx = __fmul_rn(dx, inv); p.ny = __fmul_rn(dy, inv); p.nz = __fmul_rn(dz, inv);
        const float dist = (float)nrm;
        p.max_dist = __fmul_rn(dist, sc.s[kp.octave]);
        p.min_dist = __fdiv_rn(p.max_dist, sc.s[nlevels - 1]);
        p.flags = flags & ~ORBX_QF_SKIP;
    }
    out[o] = p;
}

__global__ __launch_bounds__(256) void k_stereo_mappoints(const orbx_keypoint* __restrict__ kps, const float* __restrict__ depth,
                                                          const int32_t* __restrict__ counts, int capacity,
                                                          const float* __restrict__ twc, float4 cam, ProjScales sc, int nlevels,
                                                          int flags, orbx_map_point* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x, b = blockIdx.y;
    const int n = min(counts[b], capacity);
    if (i >= n) return;
    stereo_mappoint(kps, depth, capacity, twc, cam, sc, nlevels, flags, out, b, i);
}

// A new keyframe's stereo MapPoints and its grid (Frame::AssignFeaturesToGrid, src/Frame.cc:230-245) in one
// workgroup: the MapPoints as k_stereo_mappoints, then the counting grid of k_grid_count (the same CSR arrays) -- one
// launch of one 256-thread workgroup per keyframe instead of a MapPoint launch and a 1,024-thread grid launch
// (LocalMapping's new keyframes).  Dynamic LDS: k_grid_count's.
#ifndef ORBX_KF_PREP_WG
#define ORBX_KF_PREP_WG 1024   // threads per keyframe workgroup (compile-time; A/B builds: make variant)
#endif
__global__ __launch_bounds__(kProjThreads) void k_kf_prep(const orbx_keypoint* __restrict__ kps, const float* __restrict__ depth,
                                                 const int32_t* __restrict__ counts, int capacity, const float* __restrict__ twc,
                                                 float4 cam, ProjScales sc, int nlevels, int flags,
                                                 orbx_map_point* __restrict__ out, orbx_grid g, int32_t* __restrict__ cell_start,
                                                 int32_t* __restrict__ cell_idx) {
    const int b = blockIdx.x;
    const int n = min(counts[b], capacity);
    for (int i = threadIdx.x; i < n; i += blockDim.x) stereo_mappoint(kps, depth, capacity, twc, cam, sc, nlevels, flags, out, b, i);
    grid_count_set(kps, n, capacity, g, cell_start, cell_idx, b);
}

// ---------------------------------------------------------------------------------------------
// Frame::UndistortKeyPoints (src/Frame.cc:404-434) and ComputeImageBounds (:436-464): cv::undistortPoints(pts,
// K, DistCoef, R = I, P = K), pinned to OpenCV 3.2's cvUndistortPoints (README.md:68 "Tested with ... OpenCV 3.2"):
// double precision, normalise with 1/fx, 1/fy, five fixed iterations of
//   icdist = (1 + ((k7 r2 + k6) r2 + k5) r2) / (1 + ((k4 r2 + k1) r2 + k0) r2)
//   dx = 2 k2 x y + k3 (r2 + 2 x^2) + k8 r2 + k9 r2^2,   dy = k2 (r2 + 2 y^2) + 2 k3 x y + k10 r2 + k11 r2^2
//   x = (x0 - dx) icdist,  y = (y0 - dy) icdist
// then P = K: u = fx x + 0 y + cx, v = 0 x + fy y + cy, w = 1 / (0 x + 0 y + 1).  No FMA (explicit __d*_rn), so the
// oracle's plain C++ gives the same bits.  Thin-prism / tilt terms (k12, k13) are not supported (ORB-SLAM2 reads at
// most k1 k2 p1 p2 k3, Tracking.cc).
// ---------------------------------------------------------------------------------------------
struct Undist {
    double fx, fy, cx, cy, ifx, ify, k[12];
    double r[9];         // RR = P * I = K in double (cvMatMul with the identity is exact)
};

__device__ __forceinline__ void undistort_point(const Undist& U, float fu, float fv, float& ou, float& ov) {
    double x = __dmul_rn(__dsub_rn((double)fu, U.cx), U.ifx);
    double y = __dmul_rn(__dsub_rn((double)fv, U.cy), U.ify);
    const double x0 = x, y0 = y;
    const double* k = U.k;
    for (int j = 0; j < 5; ++j) {
        const double r2 = __dadd_rn(__dmul_rn(x, x), __dmul_rn(y, y));
        const double num = __dadd_rn(1.0, __dmul_rn(__dadd_rn(__dmul_rn(__dadd_rn(__dmul_rn(k[7], r2), k[6]), r2), k[5]), r2));
        const double den = __dadd_rn(1.0, __dmul_rn(__dadd_rn(__dmul_rn(__dadd_rn(__dmul_rn(k[4], r2), k[1]), r2), k[0]), r2));
        const double icdist = __ddiv_rn(num, den);
        const double dx = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(__dmul_rn(__dmul_rn(2.0, k[2]), x), y),
                                                        __dmul_rn(k[3], __dadd_rn(r2, __dmul_rn(__dmul_rn(2.0, x), x)))),
                                              __dmul_rn(k[8], r2)),
                                    __dmul_rn(__dmul_rn(k[9], r2), r2));
        const double dy = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(k[2], __dadd_rn(r2, __dmul_rn(__dmul_rn(2.0, y), y))),
                                                        __dmul_rn(__dmul_rn(__dmul_rn(2.0, k[3]), x), y)),
                                              __dmul_rn(k[10], r2)),
                                    __dmul_rn(__dmul_rn(k[11], r2), r2));
        x = __dmul_rn(__dsub_rn(x0, dx), icdist);
        y = __dmul_rn(__dsub_rn(y0, dy), icdist);
    }
    const double* R = U.r;
    const double xx = __dadd_rn(__dadd_rn(__dmul_rn(R[0], x), __dmul_rn(R[1], y)), R[2]);
    const double yy = __dadd_rn(__dadd_rn(__dmul_rn(R[3], x), __dmul_rn(R[4], y)), R[5]);
    const double ww = __ddiv_rn(1.0, __dadd_rn(__dadd_rn(__dmul_rn(R[6], x), __dmul_rn(R[7], y)), R[8]));
    ou = (float)__dmul_rn(xx, ww);
    ov = (float)__dmul_rn(yy, ww);
}

// One thread per keypoint of 'batch' sets (extractor batch layout); a zero first coefficient copies (Frame.cc:406-410).
__global__ __launch_bounds__(256) void k_undistort(Undist U, int copy_only, const orbx_keypoint* __restrict__ kps,
                                                   const int32_t* __restrict__ counts, int n_fixed, int capacity,
                                                   orbx_keypoint* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x, b = blockIdx.y;
    const int n = counts ? counts[b] : n_fixed;
    if (i >= n || i >= capacity) return;
    orbx_keypoint kp = kps[(size_t)b * capacity + i];
    if (!copy_only) undistort_point(U, kp.x, kp.y, kp.x, kp.y);
    out[(size_t)b * capacity + i] = kp;
}

// SearchLocalPoints' skip rule after the motion-model search (src/Tracking.cc:1160-1182): one thread per (set, query) and
// per (set, keypoint); the grid's x covers max(n_queries, n_keypoints).
__global__ __launch_bounds__(256) void k_proj_found(const int32_t* __restrict__ q_idx, const int32_t* __restrict__ owner,
                                                    int nq, int nk, int32_t* __restrict__ found, uint8_t* __restrict__ blocked) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x, s = blockIdx.y;
    const int32_t* ow = owner + (size_t)s * nk;
    if (i < nq) {
        const int k = q_idx[(size_t)s * nq + i];
        found[(size_t)s * nq + i] = (k >= 0 && k < nk && ow[k] == i) ? 0 : -1;
    }
    if (blocked && i < nk) blocked[(size_t)s * nk + i] = ow[i] >= 0 ? 1 : 0;
}

}  // namespace orbx

using namespace orbx;

static size_t a256p(size_t b) { return (b + 255) & ~(size_t)255; }

static int grid_check(const orbx_grid& g) {
    ORBX_REQUIRE(g.cols > 0 && g.rows > 0 && (long long)g.cols * g.rows <= kGridMaxCells, ORBX_ERR_ARG, "bad grid %d x %d",
                 g.cols, g.rows);
    return ORBX_OK;
}


static int make_undist(const float* K, const float* dist, int n_dist, Undist* U, int* copy_only) {
    ORBX_REQUIRE(K && (n_dist == 0 || dist) && (n_dist == 0 || n_dist == 4 || n_dist == 5 || n_dist == 8 || n_dist == 12),
                 ORBX_ERR_ARG, "distortion coefficients: 0, 4, 5, 8 or 12 expected (got %d)", n_dist);
    std::memset(U, 0, sizeof(*U));
    for (int i = 0; i < n_dist; ++i) U->k[i] = (double)dist[i];
    U->fx = K[0]; U->fy = K[4]; U->cx = K[2]; U->cy = K[5];
    ORBX_REQUIRE(U->fx != 0.0 && U->fy != 0.0, ORBX_ERR_ARG, "bad camera matrix");
    U->ifx = 1.0 / U->fx;
    U->ify = 1.0 / U->fy;
    for (int i = 0; i < 9; ++i) U->r[i] = (double)K[i];
    *copy_only = n_dist == 0 || dist[0] == 0.0f;       // mDistCoef.at<float>(0) == 0.0 (Frame.cc:406)
    return ORBX_OK;
}

extern "C" {

int orbx_undistort_keypoints_device(orbx_matcher* m, const orbx_keypoint* d_kps, const int32_t* d_counts, int batch, int capacity,
                                    const float* K, const float* dist, int n_dist, orbx_keypoint* d_out, void* stream) {
    ORBX_REQUIRE(m && d_kps && d_counts && d_out && batch >= 0 && capacity > 0, ORBX_ERR_ARG, "bad argument");
    Undist U;
    int copy_only = 0;
    int st = make_undist(K, dist, n_dist, &U, &copy_only);
    if (st) return st;
    if (batch == 0) return ORBX_OK;
    ORBX_REQUIRE(batch <= 65535, ORBX_ERR_UNSUPPORTED, "batch too large");
    ORBX_HIP(hipSetDevice(matcher_device(m)));
    hipLaunchKernelGGL(k_undistort, dim3((capacity + 255) / 256, batch), dim3(256), 0, (hipStream_t)stream, U, copy_only, d_kps,
                       d_counts, 0, capacity, d_out);
    ORBX_HIP(hipGetLastError());
    return ORBX_OK;
}

int orbx_undistort_keypoints(orbx_matcher* m, const orbx_keypoint* kps, int n, const float* K, const float* dist, int n_dist,
                             orbx_keypoint* out) {
    ORBX_REQUIRE(m && n >= 0 && (n == 0 || (kps && out)), ORBX_ERR_ARG, "bad argument");
    Undist U;
    int copy_only = 0;
    int st = make_undist(K, dist, n_dist, &U, &copy_only);
    if (st) return st;
    if (n == 0) return ORBX_OK;
    uint8_t* base = nullptr;
    hipStream_t s = nullptr;
    const size_t b = a256p(sizeof(orbx_keypoint) * (size_t)n);
    MatcherLease lease_(m);
    if ((st = matcher_scratch(m, 2 * b, (void**)&base, (void**)&s))) return st;
    lease_.on(s);
    ORBX_HIP(hipSetDevice(matcher_device(m)));
    orbx_keypoint* din = (orbx_keypoint*)base;
    orbx_keypoint* dout = (orbx_keypoint*)(base + b);
    ORBX_HIP(hipMemcpyAsync(din, kps, sizeof(orbx_keypoint) * (size_t)n, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_undistort, dim3((n + 255) / 256, 1), dim3(256), 0, s, U, copy_only, din, nullptr, n, n, dout);
    ORBX_HIP(hipGetLastError());
    ORBX_HIP(hipMemcpyAsync(out, dout, sizeof(orbx_keypoint) * (size_t)n, hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipStreamSynchronize(s));
    return ORBX_OK;
}

int orbx_compute_image_bounds(orbx_matcher* m, const float* K, const float* dist, int n_dist, int cols, int rows,
                              float* bounds) {
    ORBX_REQUIRE(m && bounds && cols > 0 && rows > 0, ORBX_ERR_ARG, "bad argument");
    Undist U;
    int copy_only = 0;
    int st = make_undist(K, dist, n_dist, &U, &copy_only);
    if (st) return st;
    if (copy_only) {   // Frame.cc:457-463
        bounds[0] = 0.0f; bounds[1] = (float)cols; bounds[2] = 0.0f; bounds[3] = (float)rows;
        return ORBX_OK;
    }
    orbx_keypoint c[4] = {};
    c[0].x = 0.0f; c[0].y = 0.0f; c[1].x = (float)cols; c[1].y = 0.0f;
    c[2].x = 0.0f; c[2].y = (float)rows; c[3].x = (float)cols; c[3].y = (float)rows;
    orbx_keypoint u[4];
    if ((st = orbx_undistort_keypoints(m, c, 4, K, dist, n_dist, u))) return st;
    bounds[0] = std::min(u[0].x, u[2].x);   // mnMinX, mnMaxX, mnMinY, mnMaxY (:451-454)
    bounds[1] = std::max(u[1].x, u[3].x);
    bounds[2] = std::min(u[0].y, u[1].y);
    bounds[3] = std::max(u[2].y, u[3].y);
    return ORBX_OK;
}

static int project_check(int mode, const float* scale_factors, int nlevels, ProjScales* sc) {
    ORBX_REQUIRE(mode == ORBX_PROJ_LASTFRAME || mode == ORBX_PROJ_MAPPOINTS || mode == ORBX_PROJ_FUSE, ORBX_ERR_ARG,
                 "projection mode %d (LASTFRAME, MAPPOINTS or FUSE)", mode);
    ORBX_REQUIRE(scale_factors && nlevels >= 1 && nlevels <= 32, ORBX_ERR_ARG, "bad scale factors");
    std::memset(sc, 0, sizeof(*sc));
    for (int l = 0; l < nlevels; ++l) sc->s[l] = scale_factors[l];
    return ORBX_OK;
}

int orbx_proj_project_device(orbx_matcher* m, int mode, const orbx_map_point* d_points, const int32_t* d_counts, int n_views,
                             int capacity, const orbx_view* d_views, const int32_t* d_view_points, const float* scale_factors,
                             int nlevels, float log_scale_factor, const int32_t* d_found, orbx_proj_query* d_queries,
                             void* stream) {
    ORBX_REQUIRE(m && d_points && d_counts && d_views && d_queries && n_views >= 0 && capacity > 0, ORBX_ERR_ARG,
                 "bad argument");
    ProjScales sc;
    int st = project_check(mode, scale_factors, nlevels, &sc);
    if (st) return st;
    if (n_views == 0) return ORBX_OK;
    ORBX_REQUIRE(n_views <= 65535, ORBX_ERR_UNSUPPORTED, "too many views");
    ORBX_HIP(hipSetDevice(matcher_device(m)));
    hipLaunchKernelGGL(k_project, dim3((capacity + 255) / 256, n_views), dim3(256), 0, (hipStream_t)stream, mode, d_points,
                       d_counts, 0, capacity, d_views, d_view_points, sc, nlevels, log_scale_factor, d_found, d_queries);
    ORBX_HIP(hipGetLastError());
    return ORBX_OK;
}

int orbx_proj_found_device(orbx_matcher* m, const int32_t* d_q_idx, const int32_t* d_owner, int n_sets, int n_queries,
                           int n_keypoints, int32_t* d_found, uint8_t* d_blocked, void* stream) {
    ORBX_REQUIRE(m && d_q_idx && d_owner && d_found && n_sets >= 0 && n_queries >= 0 && n_keypoints >= 0, ORBX_ERR_ARG,
                 "bad argument");
    const int n = std::max(n_queries, n_keypoints);
    if (n_sets == 0 || n == 0) return ORBX_OK;
    ORBX_REQUIRE(n_sets <= 65535, ORBX_ERR_UNSUPPORTED, "too many sets");
    ORBX_HIP(hipSetDevice(matcher_device(m)));
    hipLaunchKernelGGL(k_proj_found, dim3((n + 255) / 256, n_sets), dim3(256), 0, (hipStream_t)stream, d_q_idx, d_owner,
                       n_queries, n_keypoints, d_found, d_blocked);
    ORBX_HIP(hipGetLastError());
    return ORBX_OK;
}

int orbx_stereo_mappoints_device(orbx_matcher* m, const orbx_keypoint* d_kps, const float* d_depth, const int32_t* d_counts,
                                 int batch, int capacity, const float* d_twc, const float* camera, const float* scale_factors,
                                 int nlevels, int flags, orbx_map_point* d_points, void* stream) {
    ORBX_REQUIRE(m && d_kps && d_depth && d_counts && d_twc && camera && d_points && batch >= 0 && capacity > 0, ORBX_ERR_ARG,
                 "bad argument");
    ProjScales sc;
    int st = project_check(ORBX_PROJ_FUSE, scale_factors, nlevels, &sc);
    if (st) return st;
    ORBX_REQUIRE(camera[0] != 0.0f && camera[1] != 0.0f, ORBX_ERR_ARG, "bad camera");
    if (batch == 0) return ORBX_OK;
    ORBX_REQUIRE(batch <= 65535, ORBX_ERR_UNSUPPORTED, "batch too large");
    ORBX_HIP(hipSetDevice(matcher_device(m)));
    hipLaunchKernelGGL(k_stereo_mappoints, dim3((capacity + 255) / 256, batch), dim3(256), 0, (hipStream_t)stream, d_kps, d_depth,
                       d_counts, capacity, d_twc, make_float4(camera[0], camera[1], camera[2], camera[3]), sc, nlevels, flags,
                       d_points);
    ORBX_HIP(hipGetLastError());
    return ORBX_OK;
}

int orbx_keyframe_prep_device(orbx_matcher* m, const orbx_keypoint* d_kps, const float* d_depth, const int32_t* d_counts,
                              int batch, int capacity, const float* d_twc, const float* camera, const float* scale_factors,
                              int nlevels, int flags, orbx_map_point* d_points, orbx_grid grid, int32_t* d_cell_start,
                              int32_t* d_cell_idx, void* stream) {
    ORBX_REQUIRE(m && d_kps && d_depth && d_counts && d_twc && camera && d_points && d_cell_start && d_cell_idx && batch >= 0 &&
                     capacity > 0, ORBX_ERR_ARG, "bad argument");
    ProjScales sc;
    int st = project_check(ORBX_PROJ_FUSE, scale_factors, nlevels, &sc);
    if (st) return st;
    if ((st = grid_check(grid))) return st;
    ORBX_REQUIRE(camera[0] != 0.0f && camera[1] != 0.0f, ORBX_ERR_ARG, "bad camera");
    if (batch == 0) return ORBX_OK;
    const size_t ncell = (size_t)grid.cols * grid.rows;
    const size_t lds = ((ncell + 1) * 4 + 4 * (size_t)capacity + 15) & ~(size_t)15;
    ORBX_REQUIRE(ncell < 0xffff && capacity < 0xffff && lds <= 64 * 1024, ORBX_ERR_UNSUPPORTED,
                 "keyframe grid of %d cells x %d keypoints does not fit the one-workgroup form", (int)ncell, capacity);
    ORBX_REQUIRE(batch <= 65535, ORBX_ERR_UNSUPPORTED, "batch too large");
    ORBX_HIP(hipSetDevice(matcher_device(m)));
    // 1,024 threads: r6q +0.4 % against the two launches; 256 threads -1.5 % (r6p: the workgroups run ~4x longer)
    hipLaunchKernelGGL(k_kf_prep, dim3(batch), dim3(ORBX_KF_PREP_WG), lds, (hipStream_t)stream, d_kps, d_depth, d_counts, capacity, d_twc,
                       make_float4(camera[0], camera[1], camera[2], camera[3]), sc, nlevels, flags, d_points, grid, d_cell_start,
                       d_cell_idx);
    ORBX_HIP(hipGetLastError());
    return ORBX_OK;
}

int orbx_proj_project(orbx_matcher* m, int mode, const orbx_map_point* points, int n, const orbx_view* view,
                      const float* scale_factors, int nlevels, float log_scale_factor, orbx_proj_query* queries) {
    ORBX_REQUIRE(m && view && n >= 0 && (n == 0 || (points && queries)), ORBX_ERR_ARG, "bad argument");
    ProjScales sc;
    int st = project_check(mode, scale_factors, nlevels, &sc);
    if (st) return st;
    if (n == 0) return ORBX_OK;
    uint8_t* base = nullptr;
    hipStream_t s = nullptr;
    const size_t bp = a256p(sizeof(orbx_map_point) * (size_t)n), bv = a256p(sizeof(orbx_view)),
                 bq = a256p(sizeof(orbx_proj_query) * (size_t)n);
    MatcherLease lease_(m);
    if ((st = matcher_scratch(m, bp + bv + bq, (void**)&base, (void**)&s))) return st;
    lease_.on(s);
    ORBX_HIP(hipSetDevice(matcher_device(m)));
    orbx_map_point* dp = (orbx_map_point*)base;
    orbx_view* dv = (orbx_view*)(base + bp);
    orbx_proj_query* dq = (orbx_proj_query*)(base + bp + bv);
    ORBX_HIP(hipMemcpyAsync(dp, points, sizeof(orbx_map_point) * (size_t)n, hipMemcpyHostToDevice, s));
    ORBX_HIP(hipMemcpyAsync(dv, view, sizeof(orbx_view), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_project, dim3((n + 255) / 256, 1), dim3(256), 0, s, mode, dp, (const int32_t*)nullptr, n, n, dv,
                       (const int32_t*)nullptr, sc, nlevels, log_scale_factor, (const int32_t*)nullptr, dq);
    ORBX_HIP(hipGetLastError());
    ORBX_HIP(hipMemcpyAsync(queries, dq, sizeof(orbx_proj_query) * (size_t)n, hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipStreamSynchronize(s));
    return ORBX_OK;
}

}  // extern "C"

// k_grid_count when its LDS (cell counts + two u16 arrays) fits and cells and indices fit in u16, else k_grid_build
static void launch_grid_build(const orbx_grid& grid, const orbx_keypoint* d_kps, const int32_t* d_counts, int n_fixed,
                              int capacity, int batch, int32_t* d_cs, int32_t* d_ci, hipStream_t s) {
    const size_t ncell = (size_t)grid.cols * grid.rows;
    const size_t lds_c = ((ncell + 1) * 4 + 4 * (size_t)capacity + 15) & ~(size_t)15;
    if (ncell < 0xffff && capacity < 0xffff && lds_c <= 64 * 1024) {
        // r4at/r4au: 11 us against the bitonic form's 29 us per launch at least (the tracking frames' grids, 256 sets);
        // in the step the two are even (3.59-3.64 ms), 256 threads slower (3.66)
        hipLaunchKernelGGL(k_grid_count, dim3(batch), dim3(kProjThreads), lds_c, s, d_kps, d_counts, n_fixed, capacity, grid,
                           d_cs, d_ci);
        return;
    }
    int p2 = 1;
    while (p2 < capacity) p2 <<= 1;
    hipLaunchKernelGGL(k_grid_build, dim3(batch), dim3(kProjThreads), (size_t)p2 * 4, s, d_kps, d_counts, n_fixed, capacity,
                       grid, d_cs, d_ci);
}

extern "C" {

int orbx_grid_build_device(orbx_matcher* m, orbx_grid grid, const orbx_keypoint* d_kps, const int32_t* d_counts, int batch,
                           int capacity, int32_t* d_cell_start, int32_t* d_cell_idx, void* stream) {
    ORBX_REQUIRE(m && d_kps && d_counts && d_cell_start && d_cell_idx && batch >= 0 && capacity > 0, ORBX_ERR_ARG,
                 "bad argument");
    int st = grid_check(grid);
    if (st) return st;
    ORBX_REQUIRE(capacity <= kGridMaxKps, ORBX_ERR_UNSUPPORTED, "capacity %d > %d", capacity, kGridMaxKps);
    if (batch == 0) return ORBX_OK;
    ORBX_HIP(hipSetDevice(matcher_device(m)));
    launch_grid_build(grid, d_kps, d_counts, 0, capacity, batch, d_cell_start, d_cell_idx, (hipStream_t)stream);
    ORBX_HIP(hipGetLastError());
    return ORBX_OK;
}

static int proj_search_batch(orbx_matcher* m, const orbx_proj_params* params, orbx_grid grid,
                             const orbx_proj_problem* d_problems, int n_problems, int max_n, int max_nq,
                             const int32_t* d_grid_counts, void* stream) {
    // (an empty batch may pass a NULL problem array -- an empty torch slice's data pointer: r5bab failed on exactly that)
    ORBX_REQUIRE(m && params && (d_problems || n_problems == 0) && n_problems >= 0 && max_n >= 0 && max_nq >= 0, ORBX_ERR_ARG,
                 "bad argument");
    int st = grid_check(grid);
    if (st) return st;
    const orbx_proj_params& P = *params;
    ORBX_REQUIRE(P.mode >= ORBX_PROJ_MAPPOINTS && P.mode <= ORBX_PROJ_INIT, ORBX_ERR_ARG, "bad mode %d", P.mode);
    ORBX_REQUIRE(P.nlevels >= 1 && P.nlevels <= 32, ORBX_ERR_ARG, "bad nlevels %d", P.nlevels);
    if (n_problems == 0) return ORBX_OK;
    ORBX_HIP(hipSetDevice(matcher_device(m)));
    hipStream_t s = (hipStream_t)stream;
    ORBX_REQUIRE(!d_grid_counts || P.mode != ORBX_PROJ_INIT, ORBX_ERR_UNSUPPORTED, "grid built in the search: not for INIT");
    if (P.mode == ORBX_PROJ_INIT) {
        const size_t lds = (size_t)(2 * std::max(max_n, 1) + std::max(max_nq, 1)) * 4;
        ORBX_REQUIRE(lds <= 160 * 1024, ORBX_ERR_UNSUPPORTED, "too many keypoints for SearchForInitialization (%d, %d)", max_n,
                     max_nq);
        if (lds > 64 * 1024)
            ORBX_HIP(hipFuncSetAttribute((const void*)k_proj_init, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL(k_proj_init, dim3(n_problems), dim3(64), lds, s, P, grid, d_problems, std::max(max_n, 1),
                           std::max(max_nq, 1));
    } else {
        // LDS plan (k_proj_search): staged cells + entries when they fit, then the assigning modes' claim / own / res /
        // qm arrays and as many list slots per query (<= kProjListMax) as the rest of the 160 KiB holds
        const size_t N = std::max(max_n, 1), NQ = std::max(max_nq, 1), ncell = (size_t)grid.cols * grid.rows;
        const bool assigning = P.mode <= ORBX_PROJ_SIM3;
        const size_t core = assigning ? ((8 * N + 4 * NQ + NQ + 15) & ~(size_t)15) : 0;
        const size_t stage = ((4 * (ncell + 1) + 15) & ~(size_t)15) + 16 * N;
        const size_t cap = 160 * 1024;
        ORBX_REQUIRE(core <= cap, ORBX_ERR_UNSUPPORTED, "too many target keypoints (%d) / queries (%d)", max_n, max_nq);
        // a grid built in the search needs 4 B per target keypoint of scratch after the entries (the assigning modes'
        // claim / own arrays serve) and the staged form, u16 cells and indices
        const size_t gscr = (d_grid_counts && !assigning) ? ((4 * N + 15) & ~(size_t)15) : 0;
        // (the non-assigning modes walking cells and entries in memory instead: 70.9k against 75.4k frames/s, r5bi)
        const bool staged = stage + core + gscr <= cap;
        ORBX_REQUIRE(!d_grid_counts || (staged && ncell < 0xffff && N < 0xffff), ORBX_ERR_UNSUPPORTED,
                     "grid built in the search: %d keypoints, %d cells do not fit the staged plan", max_n, (int)ncell);
        const size_t used = core + (staged ? stage + gscr : 0);
        // list slots per query: as many as fit up to kProjListMax (0 / 2 / 4 / 8 slots: -7 % .. -0.1 %, r5bb)
        int kcap = 0;
        if (assigning) kcap = (int)std::min<size_t>(kProjListMax, (cap - used) / (4 * NQ));
        const size_t lds = std::max<size_t>(used + (size_t)kcap * 4 * NQ, 16);
        auto kern = assigning ? (staged ? k_proj_search<true, true> : k_proj_search<false, true>)
                              : (staged ? k_proj_search<true, false> : k_proj_search<false, false>);
        if (lds > 64 * 1024) ORBX_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        // 1024-thread workgroups for the assigning modes (their fixed-point rounds are workgroup-wide), 512 for the
        // non-assigning ones (Fuse: a workgroup waits for a CU with as many free wave slots beside the front end;
        // r4ao/r4ap, step 3.66-3.69 ms at 1024, 3.59-3.63 at 512, 3.62-3.64 at 384 / 768, 256 unstable 3.62-3.87).
        // (assigning modes at 512 / 768 threads: -2 % / -0.4 %, r5al)
        const int threads = assigning ? kProjThreads : 512;
        hipLaunchKernelGGL(kern, dim3(n_problems), dim3(threads), lds, s, P, grid, d_problems, (int)N, (int)NQ, kcap,
                           d_grid_counts);
    }
    ORBX_HIP(hipGetLastError());
    return ORBX_OK;
}

int orbx_proj_search_batch_device(orbx_matcher* m, const orbx_proj_params* params, orbx_grid grid,
                                  const orbx_proj_problem* d_problems, int n_problems, int max_n, int max_nq, void* stream) {
    return proj_search_batch(m, params, grid, d_problems, n_problems, max_n, max_nq, nullptr, stream);
}

int orbx_proj_search_grid_batch_device(orbx_matcher* m, const orbx_proj_params* params, orbx_grid grid,
                                       const orbx_proj_problem* d_problems, int n_problems, int max_n, int max_nq,
                                       const int32_t* d_grid_counts, void* stream) {
    ORBX_REQUIRE(d_grid_counts, ORBX_ERR_ARG, "bad argument");
    return proj_search_batch(m, params, grid, d_problems, n_problems, max_n, max_nq, d_grid_counts, stream);
}

// Host form: one query set against one view; builds the view's grid, runs the search, copies results back.
int orbx_proj_search(orbx_matcher* m, const orbx_proj_params* params, orbx_grid grid, const orbx_proj_query* queries,
                     const uint8_t* qdesc, int nq, const orbx_keypoint* kps, const uint8_t* desc, const float* uright,
                     const uint8_t* blocked, int n, int32_t* q_idx, int32_t* q_dist, int32_t* owner, int* n_matches) {
    ORBX_REQUIRE(m && params && n_matches && nq >= 0 && n >= 0, ORBX_ERR_ARG, "bad argument");
    ORBX_REQUIRE((nq == 0 || (queries && qdesc && q_idx && q_dist)) && (n == 0 || (kps && desc)), ORBX_ERR_ARG,
                 "null buffers");
    ORBX_REQUIRE(n <= kGridMaxKps, ORBX_ERR_UNSUPPORTED, "more than %d keypoints", kGridMaxKps);
    int st = grid_check(grid);
    if (st) return st;
    *n_matches = 0;
    const int ncell = grid.cols * grid.rows;
    const size_t N = std::max(n, 1), NQ = std::max(nq, 1);
    const size_t bytes = a256p(sizeof(orbx_proj_query) * NQ) + a256p(32 * NQ) + a256p(sizeof(orbx_keypoint) * N) +
                         a256p(32 * N) + a256p(4 * N) + a256p(N) + a256p(4 * ((size_t)ncell + 1)) + a256p(4 * N) +
                         3 * a256p(4 * NQ) + a256p(4 * N) + a256p(sizeof(orbx_proj_problem)) + 1024;
    uint8_t* base = nullptr;
    hipStream_t s = nullptr;
    MatcherLease lease_(m);
    if ((st = matcher_scratch(m, bytes, (void**)&base, (void**)&s))) return st;
    lease_.on(s);
    size_t off = 0;
    auto take = [&](size_t b) { uint8_t* p = base + off; off += a256p(b); return p; };
    orbx_proj_query* dq = (orbx_proj_query*)take(sizeof(orbx_proj_query) * NQ);
    uint8_t* dqd = take(32 * NQ);
    orbx_keypoint* dk = (orbx_keypoint*)take(sizeof(orbx_keypoint) * N);
    uint8_t* dd = take(32 * N);
    float* du = (float*)take(4 * N);
    uint8_t* db = take(N);
    int32_t* dcs = (int32_t*)take(4 * ((size_t)ncell + 1));
    int32_t* dci = (int32_t*)take(4 * N);
    int32_t* dqi = (int32_t*)take(4 * NQ);
    int32_t* dqdist = (int32_t*)take(4 * NQ);
    int32_t* dnm = (int32_t*)take(4 * NQ);
    int32_t* down = (int32_t*)take(4 * N);
    orbx_proj_problem* dpb = (orbx_proj_problem*)take(sizeof(orbx_proj_problem));
    if (nq) {
        ORBX_HIP(hipMemcpyAsync(dq, queries, sizeof(orbx_proj_query) * nq, hipMemcpyHostToDevice, s));
        ORBX_HIP(hipMemcpyAsync(dqd, qdesc, 32 * (size_t)nq, hipMemcpyHostToDevice, s));
    }
    if (n) {
        ORBX_HIP(hipMemcpyAsync(dk, kps, sizeof(orbx_keypoint) * n, hipMemcpyHostToDevice, s));
        ORBX_HIP(hipMemcpyAsync(dd, desc, 32 * (size_t)n, hipMemcpyHostToDevice, s));
        if (uright) ORBX_HIP(hipMemcpyAsync(du, uright, 4 * (size_t)n, hipMemcpyHostToDevice, s));
        if (blocked) ORBX_HIP(hipMemcpyAsync(db, blocked, (size_t)n, hipMemcpyHostToDevice, s));
    }
    orbx_proj_problem pb{};
    pb.queries = dq; pb.qdesc = dqd; pb.nq = nq;
    pb.kps = dk; pb.desc = dd; pb.uright = uright ? du : nullptr; pb.blocked = blocked ? db : nullptr; pb.n = n;
    pb.cell_start = dcs; pb.cell_idx = dci;
    pb.q_idx = dqi; pb.q_dist = dqdist; pb.owner = down; pb.nmatches = dnm;
    ORBX_HIP(hipMemcpyAsync(dpb, &pb, sizeof(pb), hipMemcpyHostToDevice, s));
    launch_grid_build(grid, dk, nullptr, n, std::max(n, 1), 1, dcs, dci, s);
    ORBX_HIP(hipGetLastError());
    if ((st = orbx_proj_search_batch_device(m, params, grid, dpb, 1, n, nq, s))) return st;
    int nm = 0;
    ORBX_HIP(hipMemcpyAsync(&nm, dnm, 4, hipMemcpyDeviceToHost, s));
    if (nq) {
        ORBX_HIP(hipMemcpyAsync(q_idx, dqi, 4 * (size_t)nq, hipMemcpyDeviceToHost, s));
        ORBX_HIP(hipMemcpyAsync(q_dist, dqdist, 4 * (size_t)nq, hipMemcpyDeviceToHost, s));
    }
    if (owner && n && params->mode <= ORBX_PROJ_SIM3) ORBX_HIP(hipMemcpyAsync(owner, down, 4 * (size_t)n, hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipStreamSynchronize(s));
    if (owner && n && params->mode > ORBX_PROJ_SIM3)
        for (int i = 0; i < n; ++i) owner[i] = -1;
    *n_matches = nm;
    return ORBX_OK;
}

}  // extern "C"
