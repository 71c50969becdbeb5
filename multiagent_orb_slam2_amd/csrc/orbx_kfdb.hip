// =====================================================================================================
// orbx_kfdb.hip — keyframe database (DBoW2 inverted file) queries on gfx950.
//
// Replaces KeyFrameDatabase (src/KeyFrameDatabase.cc): add / erase / clear (:40-73) and the three
// candidate queries that precede every SearchByBoW of the cross-agent path:
//   DetectLoopCandidates            :76-197   LoopClosing::DetectLoop (src/LoopClosing.cc:164),
//                                             MapFusion's fusion detection (src/MapFusion.cc:133)
//   DetectCovisibilityCandidates    :199-308  MapFusion covisibility discovery (src/MapFusion.cc:820)
//   DetectRelocalizationCandidates  :310-420  Tracking::Relocalization (src/Tracking.cc:1366)
// and ORBVocabulary::score (DBoW2 L1Scoring, Thirdparty/DBoW2/DBoW2/ScoringObject.cpp:23-66), which
// the callers also use directly for the minimum-score bound (src/MapFusion.cc:800-815).
//
// The database is a table of keyframe slots.  A slot holds a BowVector (word ids ascending, double
// values), its GetBestCovisibilityKeyFrames(10) list (src/KeyFrame.cc:189-197) and the per-keyframe
// scratch fields the reference keeps on KeyFrame (mnLoopQuery/mnLoopWords/mLoopScore and the Covis /
// Reloc triples, include/KeyFrame.h:155-163): results then equal the reference's even when a query
// id repeats and stale fields are read (the reference reads mCovisScore, which nothing assigns).
//
// Reference order -> data-parallel form.  The reference walks the query's words in ascending order and,
// per word, the inverted list in add order, pushing each keyframe at its first encounter.  The list
// order is therefore the order of (position of the first shared query word, add sequence number), a
// key every keyframe computes independently; all other steps are per-keyframe (word count, L1 score,
// covisibility accumulation) or order-free reductions (max).  Kernels per query batch:
//   k_kfdb_share    one thread per (query word): walk the word's inverted list, atomic word count and
//                   atomic-min first position per keyframe slot
//   (small databases: k_kfdb_bits + k_kfdb_pairwise_gb intersect every (query, slot) pair against a bitmap of the
//                   query's words instead of walking an inverted file; same word count and first position)
//   (<= 2048 slots: k_kfdb_wmap_count reads, per query word, the word's row of a word x slot bit matrix kept
//                   beside the BowVectors; same word count and first position from 1/32 of a word per slot)
//   k_kfdb_select   one workgroup per query: list membership from the scratch fields, max common words,
//                   compaction of the keyframes to score
//   k_kfdb_score    query BowVector staged in LDS; one wave per scored keyframe walks its words, finds
//                   the common ones by binary search in LDS and adds the L1 terms in ascending word order
//                   (sequential scalar double adds, exactly DBoW2's summation order)
//   k_kfdb_accum    one workgroup per query: covisibility accumulation, best-score retention, LDS
//                   bitonic sort by the reference's list key, first-occurrence de-duplication
//   k_kfdb_state    one thread per slot: applies the queries' updates to the scratch fields in query
//                   order and flags a batch whose queries interact through them (then the host form
//                   re-runs the batch one query at a time)
// The inverted file (CSR word -> slots) is rebuilt on the device when membership changed: count,
// exclusive scan over the vocabulary, scatter.
// =====================================================================================================
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "orbx_common.h"

namespace orbx {

constexpr int kKfdbCovis = 10;           // GetBestCovisibilityKeyFrames(10)
constexpr int kKfdbMaxWords = 4096;      // BowVector entries per slot (<= features per keyframe)
constexpr int kKfdbMaxRetained = 2048;   // retained candidates per query (LDS sort)
constexpr int kScanChunk = 4096;         // vocabulary entries per scan workgroup (1024 threads x 4)
constexpr uint32_t kNoSeq = 0xFFFFFFFFu;

enum { KIND_LOOP = ORBX_KFDB_LOOP, KIND_COVIS = ORBX_KFDB_COVIS, KIND_RELOC = ORBX_KFDB_RELOC };

// Per-query scratch, one row of S slots per query (see kfdb_scratch_layout).
struct QScratch {
    int32_t* cnt;        // words shared with the query (atomic)
    int32_t* first;      // position of the first shared query word (atomic min; INT_MAX-ish when none)
    uint8_t* excl;       // exclusion set of the query (connected / ignored keyframes); NULL = none in the batch
    float* si;           // L1 score of scored keyframes
    int32_t* cand;       // compacted scored keyframes (any order)
    float* acc;          // accumulated score of candidate i (by cand position)
    int32_t* best;       // best keyframe of candidate i
    int32_t* meta;       // per query: [0] npushed, [1] minCommon, [2] ncand
};

__device__ __forceinline__ bool excl_at(const QScratch& X, size_t i) { return X.excl && X.excl[i]; }

struct DbDev {
    const uint32_t* bw;      // [S][maxw] word ids ascending
    const double* bv;        // [S][maxw] values
    const int32_t* bn;       // [S] BowVector sizes
    const int32_t* covis;    // [S][10] best covisible slots, -1 padded
    const uint32_t* seq;     // [S] add sequence number, kNoSeq when not in the database
    const int32_t* if_off;   // [n_vocab + 1]
    const int32_t* if_slot;  // inverted file entries
    int S, maxw, n_vocab;
    uint32_t* wmap;          // [n_vocab][wdw] bit k % 32 of word dw k / 32: slot k's BowVector holds the word; or NULL
    int wdw;                 // dwords per word row: ceil(S / 32)
};

struct StateDev {
    unsigned long long* q;
    int32_t* w;
    float* s;
};

// ---------------------------------------------------------------------------------------------
// Inverted file rebuild
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_if_count(DbDev D, const int32_t* __restrict__ members, int32_t* __restrict__ cnt) {
    const int k = members[blockIdx.x];
    const int n = D.bn[k];
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t w = D.bw[(size_t)k * D.maxw + i];
        if (w < (uint32_t)D.n_vocab) atomicAdd(&cnt[w], 1);
    }
}

// Exclusive scan of n ints in place, pass 1: per-chunk totals.
__global__ __launch_bounds__(1024) void k_scan_chunks(const int32_t* __restrict__ a, int n, int32_t* __restrict__ sums) {
    __shared__ int tmp[1024 / kWave + 1];
    const int b = blockIdx.x * kScanChunk + threadIdx.x * 4;
    int s = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) s += (b + j < n) ? a[b + j] : 0;
    int total;
    block_excl_scan(s, tmp, &total);
    if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

// Pass 2: one workgroup scans the chunk totals (in place, exclusive).
__global__ __launch_bounds__(1024) void k_scan_top(int32_t* __restrict__ sums, int nb) {
    __shared__ int tmp[1024 / kWave + 1];
    int carry = 0;
    for (int base = 0; base < nb; base += 1024) {
        const int i = base + threadIdx.x;
        const int v = i < nb ? sums[i] : 0;
        int total;
        const int ex = block_excl_scan(v, tmp, &total);
        if (i < nb) sums[i] = carry + ex;
        carry += total;
        __syncthreads();
    }
}

// Pass 3: chunk-local exclusive scan plus the chunk offset; also writes the scatter cursor.
__global__ __launch_bounds__(1024) void k_scan_apply(int32_t* __restrict__ a, int n, const int32_t* __restrict__ sums,
                                                     int32_t* __restrict__ cur) {
    __shared__ int tmp[1024 / kWave + 1];
    const int b = blockIdx.x * kScanChunk + threadIdx.x * 4;
    int v[4], s = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        v[j] = (b + j < n) ? a[b + j] : 0;
        s += v[j];
    }
    int total;
    int off = block_excl_scan(s, tmp, &total) + sums[blockIdx.x];
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (b + j < n) {
            a[b + j] = off;
            if (cur) cur[b + j] = off;
            off += v[j];
        }
}

__global__ __launch_bounds__(256) void k_if_scatter(DbDev D, const int32_t* __restrict__ members, int32_t* __restrict__ cur,
                                                    int32_t* __restrict__ slot_out) {
    const int k = members[blockIdx.x];
    const int n = D.bn[k];
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t w = D.bw[(size_t)k * D.maxw + i];
        if (w < (uint32_t)D.n_vocab) slot_out[atomicAdd(&cur[w], 1)] = k;
    }
}

// slot k's first n words into (set) or out of the word map, by the workgroup (each slot owns its bit: atomics only
// against other slots' bits in the same dword)
__device__ __forceinline__ void wmap_slot(const DbDev& D, int k, int n, bool set) {
    const uint32_t bit = 1u << (k & 31);
    for (int j = threadIdx.x; j < n; j += blockDim.x) {
        const uint32_t w = D.bw[(size_t)k * D.maxw + j];
        if (w >= (uint32_t)D.n_vocab) continue;
        uint32_t* a = &D.wmap[(size_t)w * D.wdw + (k >> 5)];
        if (set) atomicOr(a, bit);
        else atomicAnd(a, ~bit);
    }
}

__global__ __launch_bounds__(256) void k_set_bow(DbDev D, uint32_t* __restrict__ bw, double* __restrict__ bv, int32_t* __restrict__ bn,
                                                 const int32_t* __restrict__ slots, const uint32_t* __restrict__ words, long long word_stride,
                                                 const double* __restrict__ values, long long value_stride,
                                                 const int32_t* __restrict__ n_words, long long n_stride) {
    const int i = blockIdx.x;
    const int k = slots[i];
    if (k < 0 || k >= D.S) return;
    const int n = max(0, min(n_words[(size_t)i * n_stride], D.maxw));
    if (D.wmap) {                                     // the old BowVector's bits out of the word map first
        wmap_slot(D, k, bn[k], false);
        __syncthreads();
    }
    for (int j = threadIdx.x; j < n; j += blockDim.x) {
        const uint32_t w = words[(size_t)i * word_stride + j];
        bw[(size_t)k * D.maxw + j] = w;
        bv[(size_t)k * D.maxw + j] = values[(size_t)i * value_stride + j];
        if (D.wmap && w < (uint32_t)D.n_vocab) atomicOr(&D.wmap[(size_t)w * D.wdw + (k >> 5)], 1u << (k & 31));
    }
    if (threadIdx.x == 0) bn[k] = n;
}

// the host form of set_bow: slot k's current words out of (set false) or into (set true) the word map
__global__ __launch_bounds__(256) void k_wmap_slot(DbDev D, int k, bool set) { wmap_slot(D, k, D.bn[k], set); }

// MapFusion keeps the first k candidates of another map (src/MapFusion.cc:136-144 drops same-map
// candidates) and matches the query against each (:275).  One thread per query; pairs (query, cand) or
// (query, -1) padding, k per query.
__global__ __launch_bounds__(64) void k_kfdb_pairs(const int32_t* __restrict__ cand, int cand_stride, const int32_t* __restrict__ n_cand,
                                                   const int32_t* __restrict__ qslots, int nq, const int32_t* __restrict__ slot_group,
                                                   const int32_t* __restrict__ query_group, int k, int32_t* __restrict__ pairs) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    const int qs = qslots[q];
    const int g = (slot_group && query_group) ? query_group[q] : 0;
    int m = 0;
    for (int i = 0; i < n_cand[q] && m < k; ++i) {
        const int c = cand[(size_t)q * cand_stride + i];
        if (slot_group && query_group && slot_group[c] == g) continue;
        pairs[2 * ((size_t)q * k + m)] = qs;
        pairs[2 * ((size_t)q * k + m) + 1] = c;
        ++m;
    }
    for (; m < k; ++m) {
        pairs[2 * ((size_t)q * k + m)] = qs;
        pairs[2 * ((size_t)q * k + m) + 1] = -1;
    }
}

// ---------------------------------------------------------------------------------------------
// L1 score (DBoW2 L1Scoring::score): score = -(sum over common words, ascending id, of
// |v - w| - |v| - |w|) / 2 with v from the first vector (the query) and w from the second.
// One wave; 'q' (the first vector, usually staged in LDS) is searched, 'c' drives the lanes.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ double readlane_f64(double v, int l) {
    const unsigned long long u = __double_as_longlong(v);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, l), hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), l);
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

__device__ double wave_l1_score(const uint32_t* qw, const double* qv, int nq, const uint32_t* cw, const double* cv, int nc) {
    double score = 0.0;
    for (int base = 0; base < nc; base += kWave) {
        const int i = base + lane_id();
        double term = 0.0;
        bool found = false;
        if (i < nc && nq > 0) {
            const uint32_t w = cw[i];
            int lo = 0, hi = nq;                 // lower_bound in the query's words
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (qw[mid] < w) lo = mid + 1; else hi = mid;
            }
            if (lo < nq && qw[lo] == w) {
                const double vi = qv[lo], wi = cv[i];
                term = __dsub_rn(__dsub_rn(fabs(__dsub_rn(vi, wi)), fabs(vi)), fabs(wi));
                found = true;
            }
        }
        uint64_t m = __ballot(found);
        while (m) {
            const int l = __builtin_ctzll(m);
            score = __dadd_rn(score, readlane_f64(term, l));
            m &= m - 1;
        }
    }
    return -score / 2.0;
}

// ---------------------------------------------------------------------------------------------
// Queries
// ---------------------------------------------------------------------------------------------
struct QueryIn {
    const int32_t* slot;              // [nq] query slots
    const unsigned long long* id;     // [nq] query ids (KeyFrame::mnId / Frame::mnId)
    const float* min_score;           // [nq] (LOOP, COVIS)
    const int32_t* excl_off;          // [nq + 1] or NULL
    const int32_t* excl;
    int seq_bounded;                  // query q sees only the members added before its own slot (MapFusion's
                                      // query-then-add order, src/MapFusion.cc:133, :149 / :222)
};

// Membership of slot k for query q: in the database and, for a sequentially bounded batch, added before the
// query's own slot (a query slot that is not a member sees every member).
__device__ __forceinline__ bool kf_visible(const DbDev& D, const QueryIn& Q, int q, int k) {
    const uint32_t sk = D.seq[k];
    if (sk == kNoSeq) return false;
    return !Q.seq_bounded || sk < D.seq[Q.slot[q]];
}

__global__ __launch_bounds__(256) void k_kfdb_mark_excl(QueryIn Q, QScratch X, int S) {
    const int q = blockIdx.x;
    if (!Q.excl_off) return;
    for (int e = Q.excl_off[q] + threadIdx.x; e < Q.excl_off[q + 1]; e += blockDim.x) {
        const int k = Q.excl[e];
        if (k >= 0 && k < S) X.excl[(size_t)q * S + k] = 1;
    }
}

__global__ __launch_bounds__(256) void k_kfdb_share(DbDev D, QueryIn Q, QScratch X, int kind) {
    const int q = blockIdx.y;
    const int qs = Q.slot[q];
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= D.bn[qs]) return;
    const uint32_t w = D.bw[(size_t)qs * D.maxw + p];
    if (w >= (uint32_t)D.n_vocab) return;
    const size_t row = (size_t)q * D.S;
    const uint32_t bound = Q.seq_bounded ? D.seq[qs] : kNoSeq;
    for (int e = D.if_off[w]; e < D.if_off[w + 1]; ++e) {
        const int k = D.if_slot[e];
        if (kind == KIND_COVIS && excl_at(X, row + k)) continue;   // :220 ignored keyframes are skipped
        if (D.seq[k] >= bound) continue;                           // added after the query (sequential batch)
        atomicAdd(&X.cnt[row + k], 1);
        atomicMin(&X.first[row + k], p);
    }
}

// Small databases: no inverted file.  One wave per (query, slot) intersects the slot's BowVector with the query's and
// produces the same word count and first shared query word as k_kfdb_share; the L1 scores are left to k_kfdb_score,
// for the keyframes that pass minCommonWords only (:113-126), as on the inverted-file path (summing the score for every
// (query, slot) pair was most of the pairwise time: r5, 0.07 ms per step at one agent, 0.36 at eight).  The query's
// words are a bitmap over the vocabulary, in memory (nbw words per query;
// DBoW2's k = 10, L = 6 tree has 10^6 leaves, 122 KB per query, L2-resident: the workgroups of one query are dealt to
// one XCD) -- no LDS, so it never holds a CU's LDS that FAST beside it could use.  Per slot wave: four slot words per
// lane in flight, then their four bitmap words; the hit count is the ballots' popcounts.  The words are ascending in
// both lists, so the first shared query word is the slot's first hit (the lowest lane of the first ballot that has
// one), and its position in the query's list is its rank there, found with two ballots over the list.  Words outside
// the vocabulary never match (as in k_kfdb_share's inverted file).  k_kfdb_bits sets the bits; k_kfdb_select clears
// the words it set once the counts are read.
__global__ __launch_bounds__(256) void k_kfdb_bits(DbDev D, QueryIn Q, uint32_t* __restrict__ qbits, int nbw) {
    const int q = blockIdx.x, qs = Q.slot[q], nq = D.bn[qs];
    uint32_t* bm = qbits + (size_t)q * nbw;
    for (int i = threadIdx.x; i < nq; i += blockDim.x) {
        const uint32_t w = D.bw[(size_t)qs * D.maxw + i];
        if (w < (uint32_t)D.n_vocab) atomicOr(&bm[w >> 5], 1u << (w & 31));
    }
}

__global__ __launch_bounds__(256) void k_kfdb_pairwise_gb(DbDev D, QueryIn Q, QScratch X, int kind,
                                                          const uint32_t* __restrict__ qbits, int nbw, int nqry, int gx) {
    const int item = xcd_item(xcd_chunk(gx * nqry));
    if (item >= gx * nqry) return;
    const int q = item / gx, bx = item - q * gx;
    const int qs = Q.slot[q];
    const int nq = D.bn[qs];
    const uint32_t nv = (uint32_t)D.n_vocab;
    const uint32_t* bm = qbits + (size_t)q * nbw;
    const uint32_t* ql = D.bw + (size_t)qs * D.maxw;
    const int waves = blockDim.x / kWave, ln = lane_id();
    const size_t row = (size_t)q * D.S;
    for (int k = bx * waves + (int)(threadIdx.x / kWave); k < D.S; k += gx * waves) {
        int c = 0;                                                    // wave-uniform
        uint32_t first = 0x7f7f7f7fu;
        if (kf_visible(D, Q, q, k) && !(kind == KIND_COVIS && excl_at(X, row + k)) && nq > 0) {
            const uint32_t* cw = D.bw + (size_t)k * D.maxw;
            const int nc = D.bn[k];
            bool found = false;
            uint32_t m = 0;                                           // the first (lowest) shared word
            for (int i0 = 0; i0 < nc; i0 += 4 * kWave) {
                uint32_t w[4], b[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int i = i0 + j * kWave + ln;
                    w[j] = i < nc ? cw[i] : 0xffffffffu;
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) b[j] = w[j] < nv ? bm[w[j] >> 5] : 0u;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint64_t hb = __ballot((b[j] >> (w[j] & 31)) & 1u);
                    c += __popcll(hb);
                    if (!found && hb) {
                        found = true;
                        m = __builtin_amdgcn_readlane(w[j], __builtin_ctzll(hb));
                    }
                }
            }
            if (found) {
                // rank of m in the query's list (nq <= 4096 = 64 segments of <= 64): its segment, then within it
                const int step = (nq + kWave - 1) / kWave;
                const int p0 = ln * step;
                const uint64_t sb = __ballot(p0 < nq && ql[min(p0, nq - 1)] <= m);
                const int base = (__popcll(sb) - 1) * step;
                const int p1 = base + ln;
                const uint64_t rb = __ballot(ln < step && p1 < nq && ql[min(p1, nq - 1)] < m);
                first = (uint32_t)(base + __popcll(rb));
            }
        }
        if (ln == 0) {
            X.cnt[row + k] = c;
            X.first[row + k] = (int)first;
        }
    }
}

// Word-map form of the same counts.  One workgroup per query: thread t owns slot dword d = t % wdw (32 slots) for the
// query words p = g, g + G, ... (g = t / wdw, G = 256 / wdw groups; wdw <= 64), reads word p's dword d, and counts
// its 32 slots' hits with a Harley-Seal carry-save tree (16 words per flush: ones / twos / fours / eights registers,
// the sixteens rippled into 9 bit planes) -- ~7 bit operations per word for 32 slots, instead of a wave per (query,
// slot) walking the slot's words.  Words are walked in ascending position, so a slot's first hit in a thread is that
// thread's smallest position; the groups' firsts and counts merge by LDS atomics (once per slot and group).
constexpr int kWmapMaxSlots = 2048;
__device__ __forceinline__ void csa(uint32_t& h, uint32_t& l, uint32_t a, uint32_t b, uint32_t c) {
    const uint32_t u = a ^ b;
    h = (a & b) | (u & c);
    l = u ^ c;
}

__global__ __launch_bounds__(256) void k_kfdb_wmap_count(DbDev D, QueryIn Q, QScratch X, int kind) {
    extern __shared__ int wsm[];
    int* s_cnt = wsm;                       // [S]
    int* s_first = wsm + D.S;               // [S]
    uint32_t* s_qw = (uint32_t*)(wsm + 2 * D.S);   // [maxw]
    const int q = blockIdx.x, tid = threadIdx.x;
    const int qs = Q.slot[q], nq = D.bn[qs];
    const uint32_t nv = (uint32_t)D.n_vocab;
    for (int k = tid; k < D.S; k += blockDim.x) { s_cnt[k] = 0; s_first[k] = 0x7f7f7f7f; }
    for (int i = tid; i < nq; i += blockDim.x) s_qw[i] = D.bw[(size_t)qs * D.maxw + i];
    __syncthreads();
    const int dw = D.wdw, G = blockDim.x / dw, g = tid / dw, d = tid - g * dw;
    if (g < G) {
        uint32_t ones = 0, twos = 0, fours = 0, eights = 0, seen = 0;
        uint32_t pl[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};   // sixteens, bit planes
        for (int p0 = g; p0 < nq; p0 += 16 * G) {
            uint32_t x[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int p = p0 + r * G;
                const uint32_t w = p < nq ? s_qw[p] : 0xffffffffu;
                x[r] = w < nv ? D.wmap[(size_t)w * dw + d] : 0u;
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const uint32_t nw = x[r] & ~seen;
                if (nw) {                                      // this thread's first hit of these slots: position p
                    seen |= nw;
                    uint32_t m = nw;
                    while (m) {
                        const int b = __builtin_ctz(m);
                        atomicMin(&s_first[d * 32 + b], p0 + r * G);
                        m &= m - 1;
                    }
                }
            }
            uint32_t ta, tb, fa, fb, ea, eb, six;
            csa(ta, ones, ones, x[0], x[1]);   csa(tb, ones, ones, x[2], x[3]);   csa(fa, twos, twos, ta, tb);
            csa(ta, ones, ones, x[4], x[5]);   csa(tb, ones, ones, x[6], x[7]);   csa(fb, twos, twos, ta, tb);
            csa(ea, fours, fours, fa, fb);
            csa(ta, ones, ones, x[8], x[9]);   csa(tb, ones, ones, x[10], x[11]); csa(fa, twos, twos, ta, tb);
            csa(ta, ones, ones, x[12], x[13]); csa(tb, ones, ones, x[14], x[15]); csa(fb, twos, twos, ta, tb);
            csa(eb, fours, fours, fa, fb);
            csa(six, eights, eights, ea, eb);
#pragma unroll
            for (int j = 0; j < 9; ++j) { const uint32_t t = pl[j] & six; pl[j] ^= six; six = t; }
        }
        if (seen) {
            for (int b = 0; b < 32; ++b) {
                if (!((seen >> b) & 1u)) continue;
                int c = (int)((ones >> b) & 1u) + 2 * (int)((twos >> b) & 1u) + 4 * (int)((fours >> b) & 1u) +
                        8 * (int)((eights >> b) & 1u);
#pragma unroll
                for (int j = 0; j < 9; ++j) c += (int)((pl[j] >> b) & 1u) << (4 + j);
                atomicAdd(&s_cnt[d * 32 + b], c);
            }
        }
    }
    __syncthreads();
    const size_t row = (size_t)q * D.S;
    for (int k = tid; k < D.S; k += blockDim.x) {
        int c = 0, first = 0x7f7f7f7f;
        if (kf_visible(D, Q, q, k) && !(kind == KIND_COVIS && excl_at(X, row + k)) && nq > 0 && s_cnt[k] > 0) {
            c = s_cnt[k];
            first = s_first[k];
        }
        X.cnt[row + k] = c;
        X.first[row + k] = first;
    }
}

// A keyframe enters lKFsSharingWords when it shares a word, its query field is not already this id
// (:93 / :221 / :325) and, for loop queries, it is not connected to the query (:96).
__device__ __forceinline__ bool kf_pushed(int kind, int c, bool stale, bool ex) {
    return c > 0 && !stale && !(kind == KIND_LOOP && ex);
}

__global__ __launch_bounds__(1024) void k_kfdb_select(DbDev D, QueryIn Q, QScratch X, StateDev St, int kind,
                                                      uint32_t* __restrict__ qbits, int nbw) {
    __shared__ int s_max, s_np, s_nc;
    const int q = blockIdx.x;
    if (qbits) {                                                      // k_kfdb_pairwise_gb is done with this query's bits
        const int qs = Q.slot[q], nq = D.bn[qs];
        for (int i = threadIdx.x; i < nq; i += blockDim.x) {
            const uint32_t w = D.bw[(size_t)qs * D.maxw + i];
            if (w < (uint32_t)D.n_vocab) qbits[(size_t)q * nbw + (w >> 5)] = 0u;
        }
    }
    const unsigned long long id = Q.id[q];
    const size_t row = (size_t)q * D.S;
    if (threadIdx.x == 0) { s_max = 0; s_np = 0; s_nc = 0; }
    __syncthreads();
    int mx = 0, np = 0;
    for (int k = threadIdx.x; k < D.S; k += blockDim.x) {
        const int c = X.cnt[row + k];
        if (kf_pushed(kind, c, St.q[k] == id, excl_at(X, row + k))) {
            mx = max(mx, c);
            ++np;
        }
    }
    atomicMax(&s_max, mx);
    atomicAdd(&s_np, np);
    __syncthreads();
    const int minCommon = (int)((float)s_max * 0.8f);          // int minCommonWords = maxCommonWords*0.8f
    for (int k = threadIdx.x; k < D.S; k += blockDim.x) {
        const int c = X.cnt[row + k];
        if (kf_pushed(kind, c, St.q[k] == id, excl_at(X, row + k)) && c > minCommon) {
            const int pos = atomicAdd(&s_nc, 1);
            X.cand[row + pos] = k;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        X.meta[q * 4 + 0] = s_np;
        X.meta[q * 4 + 1] = minCommon;
        X.meta[q * 4 + 2] = s_np ? s_nc : 0;
    }
}

__global__ __launch_bounds__(256) void k_kfdb_score(DbDev D, QueryIn Q, QScratch X) {
    extern __shared__ unsigned char smem[];
    double* qv = reinterpret_cast<double*>(smem);
    uint32_t* qw = reinterpret_cast<uint32_t*>(qv + D.maxw);
    const int q = blockIdx.y;
    const int nc = X.meta[q * 4 + 2];
    const int waves = blockDim.x / kWave;
    // a few candidates per query pass minCommonWords: the workgroups past them leave before staging the query
    if ((int)blockIdx.x * waves >= nc) return;
    const int qs = Q.slot[q];
    const int nq = D.bn[qs];
    for (int i = threadIdx.x; i < nq; i += blockDim.x) {
        qw[i] = D.bw[(size_t)qs * D.maxw + i];
        qv[i] = D.bv[(size_t)qs * D.maxw + i];
    }
    __syncthreads();
    const size_t row = (size_t)q * D.S;
    for (int c = blockIdx.x * waves + (int)(threadIdx.x / kWave); c < nc; c += gridDim.x * waves) {
        const int k = X.cand[row + c];
        const double s = wave_l1_score(qw, qv, nq, D.bw + (size_t)k * D.maxw, D.bv + (size_t)k * D.maxw, D.bn[k]);
        if (lane_id() == 0) X.si[row + k] = (float)s;
    }
}

// The scratch fields of keyframe n as the reference sees them after this query's word counting.
struct PostState {
    bool is_query;   // mn*Query == query id
    int words;
    float score;
};

// m*Score of keyframe n before query q of the batch: written by the latest earlier query that scored it
// (:135 / :361), else the value at batch start.  Relocalisation reads it for neighbours that share too
// few words to be scored by this query (:384-387).
__device__ float score_before(int kind, int n, int q, const QueryIn& Q, const QScratch& X, const StateDev& St, int S) {
    if (kind != KIND_COVIS)
        for (int i = q - 1; i >= 0; --i) {
            const size_t r = (size_t)i * S;
            const int c = X.cnt[r + n];
            if (kf_pushed(kind, c, St.q[n] == Q.id[i], excl_at(X, r + n)) && c > X.meta[i * 4 + 1]) return X.si[r + n];
        }
    return St.s[n];
}

__device__ __forceinline__ PostState post_state(int kind, int n, int q, const QueryIn& Q, const StateDev& St, const QScratch& X,
                                                int S, int minCommon) {
    const unsigned long long id = Q.id[q];
    const size_t row = (size_t)q * S;
    const int c = X.cnt[row + n];
    const bool stale = St.q[n] == id;
    const bool ex = excl_at(X, row + n);
    PostState p;
    if (stale) {
        p.is_query = true;
        p.words = St.w[n] + c;
        p.score = St.s[n];
    } else if (kf_pushed(kind, c, false, ex)) {
        p.is_query = true;
        p.words = c;
        p.score = (kind != KIND_COVIS && c > minCommon) ? X.si[row + n] : score_before(kind, n, q, Q, X, St, S);
    } else {
        p.is_query = false;
        p.words = 0;
        p.score = 0.f;
    }
    return p;
}

__global__ __launch_bounds__(256) void k_kfdb_accum(DbDev D, QueryIn Q, QScratch X, StateDev St, int kind, int32_t* __restrict__ out,
                                                    int out_stride, int32_t* __restrict__ out_n, int32_t* __restrict__ status) {
    __shared__ unsigned long long key[kKfdbMaxRetained];
    __shared__ int rbest[kKfdbMaxRetained];
    __shared__ int sbest[kKfdbMaxRetained];
    __shared__ uint8_t keep[kKfdbMaxRetained];
    __shared__ float s_part[256 / kWave];
    __shared__ int s_nr, s_tmp[256 / kWave + 1];
    const int q = blockIdx.x;
    const int T = blockDim.x;
    const size_t row = (size_t)q * D.S;
    const int minCommon = X.meta[q * 4 + 1];
    const int nc = X.meta[q * 4 + 2];
    const float minScore = Q.min_score ? Q.min_score[q] : 0.f;
    const float init = kind == KIND_RELOC ? 0.f : minScore;

    // accumulate by covisibility (:148-173 / :264-287 / :373-398); bestAcc: strict > from init = max
    float part = init;
    for (int c = threadIdx.x; c < nc; c += T) {
        const int k = X.cand[row + c];
        const float si = X.si[row + k];
        if (kind != KIND_RELOC && !(si >= minScore)) {
            X.acc[row + c] = 0.f;
            X.best[row + c] = -1;
            continue;
        }
        float best = si, acc = si;
        int bk = k;
        for (int j = 0; j < kKfdbCovis; ++j) {
            const int n = D.covis[(size_t)k * kKfdbCovis + j];
            if (n < 0) break;
            const PostState p = post_state(kind, n, q, Q, St, X, D.S, minCommon);
            if (!p.is_query) continue;
            if (kind != KIND_RELOC && !(p.words > minCommon)) continue;
            acc = __fadd_rn(acc, p.score);
            if (p.score > best) {
                bk = n;
                best = p.score;
            }
        }
        X.acc[row + c] = acc;
        X.best[row + c] = bk;
        if (acc > part) part = acc;
    }
    // wave then block max with the same strict rule (partials are never NaN)
    for (int o = 32; o > 0; o >>= 1) {
        const float t = __shfl_xor(part, o, kWave);
        if (t > part) part = t;
    }
    if (lane_id() == 0) s_part[threadIdx.x / kWave] = part;
    if (threadIdx.x == 0) s_nr = 0;
    __syncthreads();
    float bestAcc = s_part[0];
    for (int w = 1; w < T / kWave; ++w)
        if (s_part[w] > bestAcc) bestAcc = s_part[w];
    const float minRetain = 0.75f * bestAcc;

    // retained candidates with the reference's list key (first shared query word, add order)
    for (int c = threadIdx.x; c < nc; c += T) {
        if (X.best[row + c] < 0) continue;
        if (!(X.acc[row + c] > minRetain)) continue;
        const int r = atomicAdd(&s_nr, 1);
        if (r >= kKfdbMaxRetained) continue;
        const int k = X.cand[row + c];
        key[r] = ((unsigned long long)(uint32_t)X.first[row + k] << 44) | ((unsigned long long)D.seq[k] << 12) |
                 (unsigned long long)r;
        rbest[r] = X.best[row + c];
    }
    __syncthreads();
    int R = s_nr;
    if (R > kKfdbMaxRetained) {
        if (threadIdx.x == 0) atomicOr(status, 2);
        R = kKfdbMaxRetained;
    }
    int P2 = 1;
    while (P2 < R) P2 <<= 1;
    for (int i = R + threadIdx.x; i < P2; i += T) key[i] = ~0ull;
    __syncthreads();
    block_bitonic_u64(key, P2);
    // sbest[pos] = best keyframe in list order; then sort (best, pos) to find first occurrences
    for (int i = threadIdx.x; i < R; i += T) sbest[i] = rbest[key[i] & 0xFFF];
    __syncthreads();
    for (int i = threadIdx.x; i < P2; i += T) {
        key[i] = i < R ? (((unsigned long long)(uint32_t)sbest[i] << 12) | (unsigned long long)i) : ~0ull;
        if (i < R) keep[i] = 0;
    }
    __syncthreads();
    block_bitonic_u64(key, P2);
    for (int i = threadIdx.x; i < R; i += T)
        if (i == 0 || (key[i] >> 12) != (key[i - 1] >> 12)) keep[key[i] & 0xFFF] = 1;
    __syncthreads();
    // ordered compaction of the kept positions
    int written = 0;
    for (int base = 0; base < R; base += T) {
        const int i = base + threadIdx.x;
        const int f = (i < R) ? keep[i] : 0;
        int total;
        const int pos = block_excl_scan(f, s_tmp, &total) + written;
        if (f && pos < out_stride) out[(size_t)q * out_stride + pos] = sbest[i];
        written += total;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out_n[q] = min(written, out_stride);
        if (written > out_stride) atomicOr(status, 2);
    }
}

// Apply the batch's updates to the scratch fields in query order (:93-102 / :220-227 / :325-331,
// scores :135 / :361) and flag a batch whose queries see one another's updates in a way the batched
// kernels do not model: query j assumes the query id and word count of a slot are as at batch start
// whenever the id equals its own (stale fields, repeated ids).  Scores written by earlier queries of the
// batch are modelled (score_before).
__global__ __launch_bounds__(256) void k_kfdb_state(DbDev D, QueryIn Q, QScratch X, StateDev St, int kind, int nq,
                                                    int32_t* __restrict__ status) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= D.S) return;
    const unsigned long long q0 = St.q[k];
    unsigned long long qf = q0;
    int wf = St.w[k];
    float sf = St.s[k];
    bool touched = false;
    for (int j = 0; j < nq; ++j) {
        const unsigned long long id = Q.id[j];
        if (touched && (q0 == id || qf == id)) atomicOr(status, 1);
        const size_t row = (size_t)j * D.S;
        const int c = X.cnt[row + k];
        if (c == 0) continue;                            // COVIS-ignored slots were never counted
        const bool ex = excl_at(X, row + k);
        touched = true;
        if (qf == id) {
            wf += c;
        } else if (kind == KIND_LOOP && ex) {
            wf = 1;
        } else {
            qf = id;
            wf = c;
            if (kind != KIND_COVIS && X.meta[j * 4 + 0] > 0 && c > X.meta[j * 4 + 1]) sf = X.si[row + k];
        }
    }
    if (touched) {
        St.q[k] = qf;
        St.w[k] = wf;
        St.s[k] = sf;
    }
}

__global__ __launch_bounds__(256) void k_kfdb_score_pairs(DbDev D, const int32_t* __restrict__ pairs, int n, double* __restrict__ out) {
    const int p = blockIdx.x * (blockDim.x / kWave) + (int)(threadIdx.x / kWave);
    if (p >= n) return;
    const int a = pairs[2 * p], b = pairs[2 * p + 1];
    if (a < 0 || a >= D.S || b < 0 || b >= D.S) {
        if (lane_id() == 0) out[p] = 0.0;
        return;
    }
    const double s = wave_l1_score(D.bw + (size_t)a * D.maxw, D.bv + (size_t)a * D.maxw, D.bn[a], D.bw + (size_t)b * D.maxw,
                                   D.bv + (size_t)b * D.maxw, D.bn[b]);
    if (lane_id() == 0) out[p] = s;
}

}  // namespace orbx

using namespace orbx;

#ifndef ORBX_KFDB_STAGES
#define ORBX_KFDB_STAGES 16      // 4 throttled the bench host to the keyframe stream (1.54 of 2.1 ms per step blocked here)
#endif
constexpr int kKfdbStages = ORBX_KFDB_STAGES;

struct orbx_kfdb {
    int device = 0;
    hipStream_t stream = nullptr;      // lazy: own() on first host-API use
    std::once_flag stream_once;
    hipStream_t own() { return lazy_stream(stream, stream_once, device); }
    int n_vocab = 0, S = 0, maxw = 0;
    uint32_t* d_bw = nullptr;
    double* d_bv = nullptr;
    int32_t* d_bn = nullptr;
    int32_t* d_covis = nullptr;
    uint32_t* d_seq = nullptr;
    int32_t* d_if_off = nullptr;
    int32_t* d_if_cur = nullptr;
    int32_t* d_if_slot = nullptr;
    int32_t* d_scan = nullptr;
    int32_t* d_members = nullptr;
    unsigned long long* d_q[3] = {nullptr, nullptr, nullptr};
    int32_t* d_w[3] = {nullptr, nullptr, nullptr};
    float* d_s[3] = {nullptr, nullptr, nullptr};
    void* scratch = nullptr;       // per-query rows + host-form staging
    size_t scratch_bytes = 0;
    uint32_t* d_wmap = nullptr;    // word x slot bit matrix (k_kfdb_wmap_count), kept by every set_bow; NULL above
    int wmap_dw = 0;               // kWmapMaxSlots slots or a 1 GB matrix
    uint32_t* d_qbits = nullptr;   // per-query vocabulary bitmaps of the pairwise intersection: all zero between
    size_t qbits_bytes = 0;        // operations (each batch clears the words it set, k_kfdb_select)
    // Thread and stream contract (KeyFrameDatabase.cc:42,50,84,210,316 lock mMutex in add / erase / every Detect*):
    // every entry point holds 'mtx' while it runs, and every one that enqueues device work on the database's state
    // (BowVectors, membership, inverted file, scratch fields, 'scratch') first makes its stream wait for 'last_op' and
    // re-records it after -- so operations take effect in the order their calls took the lock, whatever threads and
    // streams they come from (DbOp below).
    std::recursive_mutex mtx;
    hipEvent_t last_op = nullptr;        // the last enqueue on database state, on its caller's stream
    bool last_op_set = false;            // last_op recorded after the previous operation (multi-stream mode)
    bool have_last = false, multi = false;
    hipStream_t last_stream = nullptr;   // the previous operation's stream
    void* score_stage = nullptr;   // orbx_kfdb_score's own staging (never shared with a detect in flight elsewhere)
    size_t score_stage_bytes = 0;
    std::vector<uint32_t> seq;     // host mirror of membership (add order)
    std::vector<int32_t> members;
    uint32_t* h_stage = nullptr;   // kKfdbStages pinned staging buffers of seq + members (membership uploads never
    hipEvent_t stage_done[kKfdbStages] = {};   // stall on a pageable copy; each is reused kKfdbStages uploads later,
                                               // so the host may run that many uploads ahead of the stream)
    int stage_next = 0;
    uint32_t next_seq = 0;
    bool dirty = true;             // inverted file stale (membership or a member's BowVector changed)
    bool seq_dirty = true;         // device membership (d_seq, d_members) stale
    int strategy = ORBX_KFDB_AUTO;
};

namespace {

// One database operation: the lock for its duration; its stream (if any) ordered after the previous operation.  A
// database driven from one stream needs only stream order, so nothing is enqueued for it; the first operation from a
// second stream drains the device once and switches to events ('multi': every operation records last_op, the next
// one on another stream waits for it) -- the per-call path pays no barrier or marker packet.
struct DbOp {
    orbx_kfdb* db;
    hipStream_t s;
    bool on_stream;
    std::unique_lock<std::recursive_mutex> lk;
    hipError_t err = hipSuccess;
    DbOp(orbx_kfdb* d, hipStream_t st, bool uses_stream) : db(d), s(st), on_stream(uses_stream), lk(d->mtx) {
        if (!on_stream || !db->have_last || db->last_stream == s) return;
        if (!db->multi) {
            err = ::orbx::device_sync();
            db->multi = true;
        } else if (db->last_op_set) {
            err = hipStreamWaitEvent(s, db->last_op, 0);
        }
    }
    ~DbOp() {
        if (!on_stream) return;
        if (db->multi) db->last_op_set = hipEventRecord(db->last_op, s) == hipSuccess;
        db->last_stream = s;
        db->have_last = true;
    }
};
#define ORBX_DBOP(db, stream)                                                                                          \
    DbOp op_((db), (stream), true);                                                                                  \
    ORBX_HIP(op_.err)
#define ORBX_DBLOCK(db) std::lock_guard<std::recursive_mutex> lock_((db)->mtx)

DbDev dev_view(const orbx_kfdb* db) {
    return DbDev{db->d_bw, db->d_bv, db->d_bn, db->d_covis, db->d_seq, db->d_if_off, db->d_if_slot, db->S, db->maxw, db->n_vocab,
                 db->d_wmap, db->wmap_dw};
}

int grow_scratch(orbx_kfdb* db, size_t bytes) {
    if (bytes <= db->scratch_bytes) return ORBX_OK;
    if (db->scratch) {
        // earlier operations may have run on callers' streams: every stream drained before the buffer goes away
        ::orbx::LegacyLock legacy_;
        ORBX_HIP(::orbx::device_sync());
        ORBX_HIP(hipFree(db->scratch));
        db->scratch = nullptr;
        db->scratch_bytes = 0;
    }
    ORBX_HIP(hipMalloc(&db->scratch, bytes));
    db->scratch_bytes = bytes;
    return ORBX_OK;
}

size_t align_up(size_t v) { return (v + 255) & ~(size_t)255; }

// Row layout of the query scratch for nq queries over S slots.
size_t qscratch_layout(int nq, int S, unsigned char* base, QScratch* X) {
    const size_t r = (size_t)nq * S;
    size_t o = 0;
    auto take = [&](size_t bytes) { unsigned char* p = base ? base + o : nullptr; o += align_up(bytes); return p; };
    QScratch x;
    x.cnt = (int32_t*)take(4 * r);
    x.first = (int32_t*)take(4 * r);
    x.excl = (uint8_t*)take(r);
    x.si = (float*)take(4 * r);
    x.cand = (int32_t*)take(4 * r);
    x.acc = (float*)take(4 * r);
    x.best = (int32_t*)take(4 * r);
    x.meta = (int32_t*)take(16 * (size_t)nq);
    if (X) *X = x;
    return o;
}

int upload_membership(orbx_kfdb* db, hipStream_t s) {
    if (!db->seq_dirty) return ORBX_OK;
    const int nm = (int)db->members.size();
    const int b = db->stage_next;
    db->stage_next = (b + 1) % kKfdbStages;
    uint32_t* stage = db->h_stage + (size_t)b * 2 * db->S;
    ORBX_HIP(hipEventSynchronize(db->stage_done[b]));       // the upload before last has left this buffer
    std::memcpy(stage, db->seq.data(), sizeof(uint32_t) * db->S);
    if (nm) std::memcpy(stage + db->S, db->members.data(), sizeof(int32_t) * nm);
    ORBX_HIP(hipMemcpyAsync(db->d_seq, stage, sizeof(uint32_t) * db->S, hipMemcpyHostToDevice, s));
    if (nm) ORBX_HIP(hipMemcpyAsync(db->d_members, stage + db->S, sizeof(int32_t) * nm, hipMemcpyHostToDevice, s));
    ORBX_HIP(hipEventRecord(db->stage_done[b], s));
    db->seq_dirty = false;
    return ORBX_OK;
}

int rebuild_inverted_file(orbx_kfdb* db, hipStream_t s) {
    int st = upload_membership(db, s);
    if (st) return st;
    if (!db->dirty) return ORBX_OK;
    const int nm = (int)db->members.size();
    const int n = db->n_vocab + 1;
    ORBX_HIP(hipMemsetAsync(db->d_if_off, 0, sizeof(int32_t) * n, s));
    DbDev D = dev_view(db);
    if (nm) hipLaunchKernelGGL(k_if_count, dim3(nm), dim3(256), 0, s, D, db->d_members, db->d_if_off);
    const int nb = (n + kScanChunk - 1) / kScanChunk;
    hipLaunchKernelGGL(k_scan_chunks, dim3(nb), dim3(1024), 0, s, db->d_if_off, n, db->d_scan);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(1024), 0, s, db->d_scan, nb);
    hipLaunchKernelGGL(k_scan_apply, dim3(nb), dim3(1024), 0, s, db->d_if_off, n, db->d_scan, db->d_if_cur);
    if (nm) hipLaunchKernelGGL(k_if_scatter, dim3(nm), dim3(256), 0, s, D, db->d_members, db->d_if_cur, db->d_if_slot);
    ORBX_HIP(hipGetLastError());
    db->dirty = false;
    return ORBX_OK;
}

// auto strategy: up to this many members, intersect pairwise (no inverted file); ORBX_KFDB_PAIRWISE_MAX overrides
// (diagnostics: A/B of the two strategies at a given ring size)
// ORBX_KFDB_WORDMAP=0 (diagnostics): no word map, AUTO falls back to the pairwise / inverted-file rule
static bool wmap_enabled() {
    static const bool v = [] { const char* e = std::getenv("ORBX_KFDB_WORDMAP"); return !e || std::atoi(e) != 0; }();
    return v;
}

static int pairwise_max_members() {
    static const int v = [] { const char* e = std::getenv("ORBX_KFDB_PAIRWISE_MAX"); return e ? std::atoi(e) : 2048; }();
    return v;
}


// The query batch on stream s; d_* are device pointers.  Scratch rows at 'base' (nq x S).
int detect_batch(orbx_kfdb* db, int kind, const QueryIn& Q, int nq, unsigned char* base, int32_t* d_out, int out_stride,
                 int32_t* d_out_n, int32_t* d_status, hipStream_t s) {
    const bool wordmap = db->d_wmap && (db->strategy == ORBX_KFDB_WORDMAP || db->strategy == ORBX_KFDB_AUTO);
    const bool pairwise = !wordmap && (db->strategy == ORBX_KFDB_PAIRWISE ||
                                       (db->strategy == ORBX_KFDB_AUTO && (int)db->members.size() <= pairwise_max_members()));
    int st = (pairwise || wordmap) ? upload_membership(db, s) : rebuild_inverted_file(db, s);
    if (st) return st;
    QScratch X;
    qscratch_layout(nq, db->S, base, &X);
    const size_t r = (size_t)nq * db->S;
    if (!Q.excl_off) X.excl = nullptr;
    DbDev D = dev_view(db);
    StateDev St{db->d_q[kind], db->d_w[kind], db->d_s[kind]};
    if (X.excl) {
        ORBX_HIP(hipMemsetAsync(X.excl, 0, r, s));
        hipLaunchKernelGGL(k_kfdb_mark_excl, dim3(nq), dim3(256), 0, s, Q, X, db->S);
    }
    const size_t lds = (size_t)db->maxw * (sizeof(double) + sizeof(uint32_t));
    const int nbw = (db->n_vocab + 31) / 32;
    uint32_t* qbits = nullptr;
    if (wordmap) {
        const size_t wl = (size_t)db->S * 8 + (size_t)db->maxw * 4;
        hipLaunchKernelGGL(k_kfdb_wmap_count, dim3(nq), dim3(256), wl, s, D, Q, X, kind);
    } else if (pairwise) {
        const size_t need = (size_t)4 * nbw * nq;
        if (need > db->qbits_bytes) {
            if (db->d_qbits) {
                ::orbx::LegacyLock legacy_;
                ORBX_HIP(::orbx::device_sync());
                ORBX_HIP(hipFree(db->d_qbits));
                db->d_qbits = nullptr;
                db->qbits_bytes = 0;
            }
            ORBX_HIP(hipMalloc((void**)&db->d_qbits, need));
            ORBX_HIP(hipMemsetAsync(db->d_qbits, 0, need, s));
            db->qbits_bytes = need;
        }
        qbits = db->d_qbits;
        hipLaunchKernelGGL(k_kfdb_bits, dim3(nq), dim3(256), 0, s, D, Q, qbits, nbw);
        const int gx = std::max(1, std::min((db->S + 15) / 16, 128));   // ~4 slots per wave
        hipLaunchKernelGGL(k_kfdb_pairwise_gb, dim3(kXcds * xcd_chunk(gx * nq)), dim3(256), 0, s, D, Q, X, kind, qbits,
                           nbw, nq, gx);
    } else {
        ORBX_HIP(hipMemsetAsync(X.cnt, 0, 4 * r, s));
        ORBX_HIP(hipMemsetAsync(X.first, 0x7f, 4 * r, s));
        hipLaunchKernelGGL(k_kfdb_share, dim3((db->maxw + 255) / 256, nq), dim3(256), 0, s, D, Q, X, kind);
    }
    hipLaunchKernelGGL(k_kfdb_select, dim3(nq), dim3(1024), 0, s, D, Q, X, St, kind, qbits, nbw);
    hipLaunchKernelGGL(k_kfdb_score, dim3(32, nq), dim3(256), lds, s, D, Q, X);   // the minCommonWords candidates
    hipLaunchKernelGGL(k_kfdb_accum, dim3(nq), dim3(256), 0, s, D, Q, X, St, kind, d_out, out_stride, d_out_n, d_status);
    hipLaunchKernelGGL(k_kfdb_state, dim3((db->S + 255) / 256), dim3(256), 0, s, D, Q, X, St, kind, nq, d_status);
    const hipError_t le = hipGetLastError();
    if (le != hipSuccess && qbits) {
        // the bitmaps must be all zero between batches (k_kfdb_select clears what k_kfdb_bits set): if a launch of this
        // batch failed, clear them all so the next batch does not count words it does not share
        (void)hipMemsetAsync(qbits, 0, db->qbits_bytes, s);
    }
    ORBX_HIP(le);
    return ORBX_OK;
}

}  // namespace

extern "C" {

int orbx_kfdb_create(int n_vocab_words, int max_slots, int max_words, int device, orbx_kfdb** out) {
    ORBX_REQUIRE(out, ORBX_ERR_ARG, "out is NULL");
    *out = nullptr;
    ORBX_REQUIRE(n_vocab_words >= 1 && max_slots >= 1 && max_slots <= (1 << 20), ORBX_ERR_ARG,
                 "bad sizes (n_vocab_words %d, max_slots %d)", n_vocab_words, max_slots);
    ORBX_REQUIRE(max_words >= 1 && max_words <= kKfdbMaxWords, ORBX_ERR_UNSUPPORTED, "max_words %d outside [1, %d]", max_words,
                 kKfdbMaxWords);
    int ndev = 0;
    ORBX_HIP(hipGetDeviceCount(&ndev));
    ORBX_REQUIRE(device >= 0 && device < ndev, ORBX_ERR_ARG, "device %d out of range (%d devices)", device, ndev);
    orbx_kfdb* db = new orbx_kfdb();
    db->device = device;
    db->n_vocab = n_vocab_words;
    db->S = max_slots;
    db->maxw = max_words;
    db->seq.assign(max_slots, kNoSeq);
    const size_t S = max_slots, W = max_words;
    hipError_t e = hipSetDevice(device);
    ::orbx::LegacyLock legacy_;
    auto alloc = [&](void** p, size_t bytes) {
        if (e == hipSuccess) e = hipMalloc(p, bytes);
        if (e == hipSuccess) e = hipMemset(*p, 0, bytes);
    };
    alloc((void**)&db->d_bw, 4 * S * W);
    alloc((void**)&db->d_bv, 8 * S * W);
    alloc((void**)&db->d_bn, 4 * S);
    alloc((void**)&db->d_covis, 4 * S * kKfdbCovis);
    if (e == hipSuccess) e = hipMemset(db->d_covis, 0xff, 4 * S * kKfdbCovis);
    alloc((void**)&db->d_seq, 4 * S);
    alloc((void**)&db->d_if_off, 4 * ((size_t)n_vocab_words + 1));
    alloc((void**)&db->d_if_cur, 4 * ((size_t)n_vocab_words + 1));
    alloc((void**)&db->d_if_slot, 4 * S * W);
    alloc((void**)&db->d_scan, 4 * ((size_t)(n_vocab_words + 1 + kScanChunk - 1) / kScanChunk + 1));
    alloc((void**)&db->d_members, 4 * S);
    if (e == hipSuccess && wmap_enabled() && max_slots <= kWmapMaxSlots) {
        // optional: a database whose word map does not fit in device memory works without it (pairwise / inverted file)
        const size_t dw = ((size_t)max_slots + 31) / 32, bytes = (size_t)n_vocab_words * dw * 4;
        if (bytes <= ((size_t)1 << 30) && hipMalloc((void**)&db->d_wmap, bytes) == hipSuccess) {
            if (hipMemset(db->d_wmap, 0, bytes) == hipSuccess) {
                db->wmap_dw = (int)dw;
            } else {
                (void)hipFree(db->d_wmap);
                db->d_wmap = nullptr;
            }
        }
        (void)hipGetLastError();                     // a refused allocation leaves no sticky error behind
    }
    for (int k = 0; k < 3; ++k) {
        alloc((void**)&db->d_q[k], 8 * S);
        alloc((void**)&db->d_w[k], 4 * S);
        alloc((void**)&db->d_s[k], 4 * S);
    }
    if (e == hipSuccess) e = init_done();   // the null-stream memsets above, before any kernel on a caller's stream
    if (e == hipSuccess) e = hipEventCreateWithFlags(&db->last_op, hipEventDisableTiming);
    if (e == hipSuccess) e = hipHostMalloc((void**)&db->h_stage, 8 * (size_t)kKfdbStages * S, hipHostMallocDefault);
    for (int b = 0; b < kKfdbStages; ++b) {
        if (e == hipSuccess) e = hipEventCreateWithFlags(&db->stage_done[b], hipEventDisableTiming);
    }
    if (e != hipSuccess) {
        set_error("kfdb create: %s", hipGetErrorString(e));
        orbx_kfdb_destroy(db);
        return ORBX_ERR_HIP;
    }
    *out = db;
    return ORBX_OK;
}

int orbx_kfdb_destroy(orbx_kfdb* db) {
    if (!db) return ORBX_OK;
    (void)hipSetDevice(db->device);
    (void)::orbx::device_sync();              // operations on callers' streams read the database's buffers
    void* bufs[] = {db->d_bw, db->d_bv, db->d_bn, db->d_covis, db->d_seq, db->d_if_off, db->d_if_cur, db->d_if_slot,
                    db->d_scan, db->d_members, db->scratch, db->score_stage, db->d_qbits, db->d_wmap};
    ::orbx::LegacyLock legacy_;
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    for (int k = 0; k < 3; ++k) {
        if (db->d_q[k]) (void)hipFree(db->d_q[k]);
        if (db->d_w[k]) (void)hipFree(db->d_w[k]);
        if (db->d_s[k]) (void)hipFree(db->d_s[k]);
    }
    for (int b = 0; b < kKfdbStages; ++b)
        if (db->stage_done[b]) {
            (void)hipEventSynchronize(db->stage_done[b]);
            (void)hipEventDestroy(db->stage_done[b]);
        }
    if (db->last_op) (void)hipEventDestroy(db->last_op);
    if (db->h_stage) (void)hipHostFree(db->h_stage);
    if (db->stream) (void)hipStreamDestroy(db->stream);
    delete db;
    return ORBX_OK;
}

int orbx_kfdb_info(const orbx_kfdb* db, int* n_vocab_words, int* max_slots, int* max_words, int* n_members) {
    ORBX_REQUIRE(db, ORBX_ERR_ARG, "db is NULL");
    ORBX_DBLOCK(const_cast<orbx_kfdb*>(db));
    if (n_vocab_words) *n_vocab_words = db->n_vocab;
    if (max_slots) *max_slots = db->S;
    if (max_words) *max_words = db->maxw;
    if (n_members) *n_members = (int)db->members.size();
    return ORBX_OK;
}

int orbx_kfdb_set_strategy(orbx_kfdb* db, int strategy) {
    ORBX_REQUIRE(db && strategy >= ORBX_KFDB_AUTO && strategy <= ORBX_KFDB_WORDMAP, ORBX_ERR_ARG, "bad strategy");
    ORBX_DBLOCK(db);
    ORBX_REQUIRE(strategy != ORBX_KFDB_WORDMAP || db->d_wmap, ORBX_ERR_UNSUPPORTED,
                 "no word map for this database (%d slots, %d words)", db->S, db->n_vocab);
    db->strategy = strategy;
    return ORBX_OK;
}

int orbx_kfdb_set_bow(orbx_kfdb* db, int slot, const uint32_t* words, const double* values, int n) {
    ORBX_REQUIRE(db && slot >= 0 && slot < db->S && n >= 0 && n <= db->maxw && (n == 0 || (words && values)), ORBX_ERR_ARG,
                 "bad argument (slot %d, n %d)", slot, n);
    for (int i = 0; i < n; ++i) {
        ORBX_REQUIRE(words[i] < (uint32_t)db->n_vocab, ORBX_ERR_ARG, "word id %u >= vocabulary size %d", words[i], db->n_vocab);
        ORBX_REQUIRE(i == 0 || words[i] > words[i - 1], ORBX_ERR_ARG, "BowVector word ids must ascend");
    }
    ORBX_HIP(hipSetDevice(db->device));
    ORBX_DBOP(db, db->own());
    const size_t o = (size_t)slot * db->maxw;
    DbDev D = dev_view(db);
    if (db->d_wmap) hipLaunchKernelGGL(k_wmap_slot, dim3(1), dim3(256), 0, db->own(), D, slot, false);
    if (n) {
        ORBX_HIP(hipMemcpyAsync(db->d_bw + o, words, 4 * (size_t)n, hipMemcpyHostToDevice, db->own()));
        ORBX_HIP(hipMemcpyAsync(db->d_bv + o, values, 8 * (size_t)n, hipMemcpyHostToDevice, db->own()));
    }
    ORBX_HIP(hipMemcpyAsync(db->d_bn + slot, &n, 4, hipMemcpyHostToDevice, db->own()));
    if (db->d_wmap) hipLaunchKernelGGL(k_wmap_slot, dim3(1), dim3(256), 0, db->own(), D, slot, true);
    ORBX_HIP(hipGetLastError());
    ORBX_HIP(hipStreamSynchronize(db->own()));
    if (db->seq[slot] != kNoSeq) db->dirty = true;
    return ORBX_OK;
}

int orbx_kfdb_set_bow_device(orbx_kfdb* db, const int32_t* d_slots, int n, const uint32_t* d_words, long long word_stride,
                             const double* d_values, long long value_stride, const int32_t* d_n_words, long long n_stride,
                             void* stream) {
    ORBX_REQUIRE(db && n >= 0 && (n == 0 || (d_slots && d_words && d_values && d_n_words)) && word_stride >= 0 &&
                     value_stride >= 0 && n_stride >= 0, ORBX_ERR_ARG, "bad argument");
    if (n == 0) return ORBX_OK;
    ORBX_HIP(hipSetDevice(db->device));
    ORBX_DBOP(db, (hipStream_t)stream);
    DbDev D = dev_view(db);
    hipLaunchKernelGGL(k_set_bow, dim3(n), dim3(256), 0, (hipStream_t)stream, D, db->d_bw, db->d_bv, db->d_bn, d_slots, d_words,
                       word_stride, d_values, value_stride, d_n_words, n_stride);
    ORBX_HIP(hipGetLastError());
    db->dirty = true;
    return ORBX_OK;
}

int orbx_kfdb_candidate_pairs_device(const int32_t* d_cand, int cand_stride, const int32_t* d_n_cand, const int32_t* d_query_slots,
                                     int nq, const int32_t* d_slot_group, const int32_t* d_query_group, int k, int32_t* d_pairs,
                                     void* stream) {
    ORBX_REQUIRE(nq >= 0 && k >= 0 && cand_stride >= 0, ORBX_ERR_ARG, "bad argument");
    if (nq == 0 || k == 0) return ORBX_OK;
    ORBX_REQUIRE(d_cand && d_n_cand && d_query_slots && d_pairs, ORBX_ERR_ARG, "null buffers");
    hipLaunchKernelGGL(k_kfdb_pairs, dim3((nq + 63) / 64), dim3(64), 0, (hipStream_t)stream, d_cand, cand_stride, d_n_cand,
                       d_query_slots, nq, d_slot_group, d_query_group, k, d_pairs);
    ORBX_HIP(hipGetLastError());
    return ORBX_OK;
}

int orbx_kfdb_set_covisibility(orbx_kfdb* db, const int32_t* slots, int n, const int32_t* best) {
    ORBX_REQUIRE(db && n >= 0 && (n == 0 || (slots && best)), ORBX_ERR_ARG, "bad argument");
    ORBX_HIP(hipSetDevice(db->device));
    ORBX_DBOP(db, db->own());
    for (int i = 0; i < n; ++i) {
        ORBX_REQUIRE(slots[i] >= 0 && slots[i] < db->S, ORBX_ERR_ARG, "slot %d out of range", slots[i]);
        for (int j = 0; j < kKfdbCovis; ++j)
            ORBX_REQUIRE(best[i * kKfdbCovis + j] >= -1 && best[i * kKfdbCovis + j] < db->S, ORBX_ERR_ARG,
                         "covisible slot %d out of range", best[i * kKfdbCovis + j]);
        ORBX_HIP(hipMemcpyAsync(db->d_covis + (size_t)slots[i] * kKfdbCovis, best + (size_t)i * kKfdbCovis,
                                4 * kKfdbCovis, hipMemcpyHostToDevice, db->own()));
    }
    ORBX_HIP(hipStreamSynchronize(db->own()));
    return ORBX_OK;
}

int orbx_kfdb_add(orbx_kfdb* db, const int32_t* slots, int n) {
    ORBX_REQUIRE(db && n >= 0 && (n == 0 || slots), ORBX_ERR_ARG, "bad argument");
    ORBX_DBLOCK(db);   // membership: host mirror only, uploaded by the next detect on that detect's stream
    for (int i = 0; i < n; ++i) {
        const int k = slots[i];
        ORBX_REQUIRE(k >= 0 && k < db->S, ORBX_ERR_ARG, "slot %d out of range", k);
        ORBX_REQUIRE(db->seq[k] == kNoSeq, ORBX_ERR_ARG, "slot %d is already in the database", k);
        ORBX_REQUIRE(db->next_seq < kNoSeq, ORBX_ERR_CAPACITY, "add sequence exhausted");
        db->seq[k] = db->next_seq++;
        db->members.push_back(k);
    }
    if (n) db->dirty = db->seq_dirty = true;
    return ORBX_OK;
}

int orbx_kfdb_erase(orbx_kfdb* db, const int32_t* slots, int n) {
    ORBX_REQUIRE(db && n >= 0 && (n == 0 || slots), ORBX_ERR_ARG, "bad argument");
    ORBX_DBLOCK(db);
    bool any = false;
    for (int i = 0; i < n; ++i) {
        const int k = slots[i];
        ORBX_REQUIRE(k >= 0 && k < db->S, ORBX_ERR_ARG, "slot %d out of range", k);
        if (db->seq[k] == kNoSeq) continue;      // not in the database: the reference's erase finds nothing
        db->seq[k] = kNoSeq;
        db->members.erase(std::find(db->members.begin(), db->members.end(), k));
        any = true;
    }
    if (any) db->dirty = db->seq_dirty = true;
    return ORBX_OK;
}

int orbx_kfdb_clear(orbx_kfdb* db) {
    ORBX_REQUIRE(db, ORBX_ERR_ARG, "db is NULL");
    ORBX_DBLOCK(db);
    std::fill(db->seq.begin(), db->seq.end(), kNoSeq);
    db->members.clear();
    db->dirty = db->seq_dirty = true;
    return ORBX_OK;
}

int orbx_kfdb_get_state(orbx_kfdb* db, int kind, uint64_t* query, int32_t* words, float* score) {
    ORBX_REQUIRE(db && kind >= 0 && kind <= 2 && query && words && score, ORBX_ERR_ARG, "bad argument");
    ORBX_HIP(hipSetDevice(db->device));
    ORBX_DBOP(db, db->own());
    ORBX_HIP(hipMemcpyAsync(query, db->d_q[kind], 8 * (size_t)db->S, hipMemcpyDeviceToHost, db->own()));
    ORBX_HIP(hipMemcpyAsync(words, db->d_w[kind], 4 * (size_t)db->S, hipMemcpyDeviceToHost, db->own()));
    ORBX_HIP(hipMemcpyAsync(score, db->d_s[kind], 4 * (size_t)db->S, hipMemcpyDeviceToHost, db->own()));
    ORBX_HIP(hipStreamSynchronize(db->own()));
    return ORBX_OK;
}

int orbx_kfdb_set_state(orbx_kfdb* db, int kind, const uint64_t* query, const int32_t* words, const float* score) {
    ORBX_REQUIRE(db && kind >= 0 && kind <= 2 && query && words && score, ORBX_ERR_ARG, "bad argument");
    ORBX_HIP(hipSetDevice(db->device));
    ORBX_DBOP(db, db->own());
    ORBX_HIP(hipMemcpyAsync(db->d_q[kind], query, 8 * (size_t)db->S, hipMemcpyHostToDevice, db->own()));
    ORBX_HIP(hipMemcpyAsync(db->d_w[kind], words, 4 * (size_t)db->S, hipMemcpyHostToDevice, db->own()));
    ORBX_HIP(hipMemcpyAsync(db->d_s[kind], score, 4 * (size_t)db->S, hipMemcpyHostToDevice, db->own()));
    ORBX_HIP(hipStreamSynchronize(db->own()));
    return ORBX_OK;
}

int orbx_kfdb_score_device(orbx_kfdb* db, const int32_t* d_pairs, int n, double* d_scores, void* stream) {
    ORBX_REQUIRE(db && n >= 0 && (n == 0 || (d_pairs && d_scores)), ORBX_ERR_ARG, "bad argument");
    if (n == 0) return ORBX_OK;
    ORBX_HIP(hipSetDevice(db->device));
    ORBX_DBOP(db, (hipStream_t)stream);
    hipLaunchKernelGGL(k_kfdb_score_pairs, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, dev_view(db), d_pairs, n,
                       d_scores);
    ORBX_HIP(hipGetLastError());
    return ORBX_OK;
}

int orbx_kfdb_score(orbx_kfdb* db, const int32_t* pairs, int n, double* scores) {
    ORBX_REQUIRE(db && n >= 0 && (n == 0 || (pairs && scores)), ORBX_ERR_ARG, "bad argument");
    if (n == 0) return ORBX_OK;
    ORBX_HIP(hipSetDevice(db->device));
    ORBX_DBOP(db, db->own());
    const size_t need = align_up(8 * (size_t)n) + align_up(8 * (size_t)n);
    if (need > db->score_stage_bytes) {          // the db's own stream is the only user of this buffer
        ::orbx::LegacyLock legacy_;
        ORBX_HIP(::orbx::device_sync());
        if (db->score_stage) ORBX_HIP(hipFree(db->score_stage));
        db->score_stage = nullptr;
        db->score_stage_bytes = 0;
        ORBX_HIP(hipMalloc(&db->score_stage, need));
        db->score_stage_bytes = need;
    }
    int st;
    int32_t* d_pairs = (int32_t*)db->score_stage;
    double* d_out = (double*)((unsigned char*)d_pairs + align_up(8 * (size_t)n));
    ORBX_HIP(hipMemcpyAsync(d_pairs, pairs, 8 * (size_t)n, hipMemcpyHostToDevice, db->own()));
    st = orbx_kfdb_score_device(db, d_pairs, n, d_out, db->own());
    if (st) return st;
    ORBX_HIP(hipMemcpyAsync(scores, d_out, 8 * (size_t)n, hipMemcpyDeviceToHost, db->own()));
    ORBX_HIP(hipStreamSynchronize(db->own()));
    return ORBX_OK;
}

}  // extern "C"

namespace {

int detect_device_impl(orbx_kfdb* db, int kind, const int32_t* d_query_slots, const uint64_t* d_query_ids,
                       const float* d_min_scores, int nq, const int32_t* d_excl_offsets, const int32_t* d_excl_slots,
                       int32_t* d_out, int out_stride, int32_t* d_out_n, int32_t* d_status, void* stream, int seq_bounded) {
    ORBX_REQUIRE(db && kind >= 0 && kind <= 2 && nq >= 0 && out_stride >= 0, ORBX_ERR_ARG, "bad argument");
    ORBX_REQUIRE(nq == 0 || (d_query_slots && d_query_ids && d_out && d_out_n && d_status), ORBX_ERR_ARG, "null buffers");
    ORBX_REQUIRE(kind == ORBX_KFDB_RELOC || nq == 0 || d_min_scores, ORBX_ERR_ARG, "min scores required for this query kind");
    if (nq == 0) return ORBX_OK;
    ORBX_HIP(hipSetDevice(db->device));
    ORBX_DBOP(db, (hipStream_t)stream);
    const size_t qb = qscratch_layout(nq, db->S, nullptr, nullptr);
    int st = grow_scratch(db, qb);
    if (st) return st;
    QueryIn Q{d_query_slots, (const unsigned long long*)d_query_ids, d_min_scores, d_excl_offsets, d_excl_slots, seq_bounded};
    return detect_batch(db, kind, Q, nq, (unsigned char*)db->scratch, d_out, out_stride, d_out_n, d_status,
                        (hipStream_t)stream);
}

}  // namespace

extern "C" {

int orbx_kfdb_detect_device(orbx_kfdb* db, int kind, const int32_t* d_query_slots, const uint64_t* d_query_ids,
                            const float* d_min_scores, int nq, const int32_t* d_excl_offsets, const int32_t* d_excl_slots,
                            int32_t* d_out, int out_stride, int32_t* d_out_n, int32_t* d_status, void* stream) {
    return detect_device_impl(db, kind, d_query_slots, d_query_ids, d_min_scores, nq, d_excl_offsets, d_excl_slots, d_out,
                              out_stride, d_out_n, d_status, stream, 0);
}

int orbx_kfdb_detect_sequential_device(orbx_kfdb* db, int kind, const int32_t* d_query_slots, const uint64_t* d_query_ids,
                                       const float* d_min_scores, int nq, const int32_t* d_excl_offsets,
                                       const int32_t* d_excl_slots, int32_t* d_out, int out_stride, int32_t* d_out_n,
                                       int32_t* d_status, void* stream) {
    return detect_device_impl(db, kind, d_query_slots, d_query_ids, d_min_scores, nq, d_excl_offsets, d_excl_slots, d_out,
                              out_stride, d_out_n, d_status, stream, 1);
}

}  // extern "C"

namespace {

int detect_host_impl(orbx_kfdb* db, int kind, const int32_t* query_slots, const uint64_t* query_ids, const float* min_scores,
                     int nq, const int32_t* excl_offsets, const int32_t* excl_slots, int32_t* out_offsets, int32_t* out,
                     int out_cap, int seq_bounded) {
    ORBX_REQUIRE(db && kind >= 0 && kind <= 2 && nq >= 0 && out_cap >= 0, ORBX_ERR_ARG, "bad argument");
    ORBX_REQUIRE(nq == 0 || (query_slots && query_ids && out_offsets), ORBX_ERR_ARG, "null buffers");
    ORBX_REQUIRE(kind == ORBX_KFDB_RELOC || nq == 0 || min_scores, ORBX_ERR_ARG, "min scores required for this query kind");
    if (out_offsets) out_offsets[0] = 0;
    if (nq == 0) return ORBX_OK;
    for (int q = 0; q < nq; ++q)
        ORBX_REQUIRE(query_slots[q] >= 0 && query_slots[q] < db->S, ORBX_ERR_ARG, "query slot %d out of range", query_slots[q]);
    const int n_excl = excl_offsets ? excl_offsets[nq] : 0;
    ORBX_REQUIRE(!excl_offsets || (excl_offsets[0] == 0 && (n_excl == 0 || excl_slots)), ORBX_ERR_ARG, "bad exclusion lists");
    ORBX_HIP(hipSetDevice(db->device));
    ORBX_DBOP(db, db->own());
    const int S = db->S;
    // device staging: [query scratch][slots][ids][min][excl_off][excl][out nq x S][out_n][status][state snapshot]
    const size_t qb = qscratch_layout(nq, S, nullptr, nullptr);
    size_t o = qb;
    const size_t o_slot = o; o += align_up(4 * (size_t)nq);
    const size_t o_id = o; o += align_up(8 * (size_t)nq);
    const size_t o_min = o; o += align_up(4 * (size_t)nq);
    const size_t o_eoff = o; o += align_up(4 * (size_t)(nq + 1));
    const size_t o_excl = o; o += align_up(4 * (size_t)std::max(n_excl, 1));
    const size_t o_out = o; o += align_up(4 * (size_t)nq * S);
    const size_t o_outn = o; o += align_up(4 * (size_t)nq);
    const size_t o_stat = o; o += align_up(4);
    const size_t o_snap = o; o += align_up(16 * (size_t)S);
    int st = grow_scratch(db, o);
    if (st) return st;
    unsigned char* b = (unsigned char*)db->scratch;
    hipStream_t s = db->own();
    ORBX_HIP(hipMemcpyAsync(b + o_slot, query_slots, 4 * (size_t)nq, hipMemcpyHostToDevice, s));
    ORBX_HIP(hipMemcpyAsync(b + o_id, query_ids, 8 * (size_t)nq, hipMemcpyHostToDevice, s));
    if (min_scores) ORBX_HIP(hipMemcpyAsync(b + o_min, min_scores, 4 * (size_t)nq, hipMemcpyHostToDevice, s));
    if (excl_offsets) {
        ORBX_HIP(hipMemcpyAsync(b + o_eoff, excl_offsets, 4 * (size_t)(nq + 1), hipMemcpyHostToDevice, s));
        if (n_excl) ORBX_HIP(hipMemcpyAsync(b + o_excl, excl_slots, 4 * (size_t)n_excl, hipMemcpyHostToDevice, s));
    }
    // snapshot of this kind's scratch fields, restored if the batch has to be re-run one query at a time
    ORBX_HIP(hipMemcpyAsync(b + o_snap, db->d_q[kind], 8 * (size_t)S, hipMemcpyDeviceToDevice, s));
    ORBX_HIP(hipMemcpyAsync(b + o_snap + 8 * (size_t)S, db->d_w[kind], 4 * (size_t)S, hipMemcpyDeviceToDevice, s));
    ORBX_HIP(hipMemcpyAsync(b + o_snap + 12 * (size_t)S, db->d_s[kind], 4 * (size_t)S, hipMemcpyDeviceToDevice, s));
    int32_t* d_status = (int32_t*)(b + o_stat);
    ORBX_HIP(hipMemsetAsync(d_status, 0, 4, s));
    QueryIn Q{(const int32_t*)(b + o_slot), (const unsigned long long*)(b + o_id), min_scores ? (const float*)(b + o_min) : nullptr,
              excl_offsets ? (const int32_t*)(b + o_eoff) : nullptr, (const int32_t*)(b + o_excl), seq_bounded};
    st = detect_batch(db, kind, Q, nq, b, (int32_t*)(b + o_out), S, (int32_t*)(b + o_outn), d_status, s);
    if (st) return st;
    int32_t status = 0;
    ORBX_HIP(hipMemcpyAsync(&status, d_status, 4, hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipStreamSynchronize(s));
    if ((status & 1) && nq > 1) {
        // the queries interact through the scratch fields: restore them and run in order, one by one
        ORBX_HIP(hipMemcpyAsync(db->d_q[kind], b + o_snap, 8 * (size_t)S, hipMemcpyDeviceToDevice, s));
        ORBX_HIP(hipMemcpyAsync(db->d_w[kind], b + o_snap + 8 * (size_t)S, 4 * (size_t)S, hipMemcpyDeviceToDevice, s));
        ORBX_HIP(hipMemcpyAsync(db->d_s[kind], b + o_snap + 12 * (size_t)S, 4 * (size_t)S, hipMemcpyDeviceToDevice, s));
        ORBX_HIP(hipMemsetAsync(d_status, 0, 4, s));
        for (int q = 0; q < nq; ++q) {
            QueryIn Q1{Q.slot + q, Q.id + q, Q.min_score ? Q.min_score + q : nullptr, Q.excl_off ? Q.excl_off + q : nullptr,
                       Q.excl, seq_bounded};
            st = detect_batch(db, kind, Q1, 1, b, (int32_t*)(b + o_out) + (size_t)q * S, S, (int32_t*)(b + o_outn) + q, d_status,
                              s);
            if (st) return st;
        }
        ORBX_HIP(hipMemcpyAsync(&status, d_status, 4, hipMemcpyDeviceToHost, s));
        ORBX_HIP(hipStreamSynchronize(s));
        status &= ~1;
    }
    ORBX_REQUIRE(!(status & 2), ORBX_ERR_CAPACITY, "more than %d retained candidates in one query", kKfdbMaxRetained);
    std::vector<int32_t> cnt(nq);
    ORBX_HIP(hipMemcpyAsync(cnt.data(), b + o_outn, 4 * (size_t)nq, hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipStreamSynchronize(s));
    int total = 0;
    for (int q = 0; q < nq; ++q) {
        out_offsets[q + 1] = out_offsets[q] + cnt[q];
        total += cnt[q];
    }
    if (total > out_cap) {
        set_error("output capacity %d < %d candidates", out_cap, total);
        return ORBX_ERR_CAPACITY;
    }
    for (int q = 0; q < nq; ++q)
        if (cnt[q]) ORBX_HIP(hipMemcpyAsync(out + out_offsets[q], (int32_t*)(b + o_out) + (size_t)q * S, 4 * (size_t)cnt[q],
                                            hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipStreamSynchronize(s));
    return ORBX_OK;
}

}  // namespace

extern "C" {

int orbx_kfdb_detect(orbx_kfdb* db, int kind, const int32_t* query_slots, const uint64_t* query_ids, const float* min_scores,
                     int nq, const int32_t* excl_offsets, const int32_t* excl_slots, int32_t* out_offsets, int32_t* out,
                     int out_cap) {
    return detect_host_impl(db, kind, query_slots, query_ids, min_scores, nq, excl_offsets, excl_slots, out_offsets, out,
                            out_cap, 0);
}

int orbx_kfdb_detect_sequential(orbx_kfdb* db, int kind, const int32_t* query_slots, const uint64_t* query_ids,
                                const float* min_scores, int nq, const int32_t* excl_offsets, const int32_t* excl_slots,
                                int32_t* out_offsets, int32_t* out, int out_cap) {
    return detect_host_impl(db, kind, query_slots, query_ids, min_scores, nq, excl_offsets, excl_slots, out_offsets, out,
                            out_cap, 1);
}

}  // extern "C"
