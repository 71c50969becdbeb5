// =====================================================================================================
// orbx_vocab.hip — DBoW2 vocabulary transform on gfx950: descriptors -> BowVector + FeatureVector.
//
// Replaces TemplatedVocabulary<FORB>::transform(features, BowVector&, FeatureVector&, levelsup)
// (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1125-1187, per-feature descent :1218-1259), called by
// Frame::ComputeBoW / KeyFrame::ComputeBoW with levelsup = 4 (src/Frame.cc:395-402).  Its FeatureVector
// is what ORBmatcher::SearchByBoW buckets on.
//
//   k_vocab_words      one thread per descriptor: descend the k-ary tree, at each level the child with
//                      the smallest Hamming distance (first minimum, strict <, :1244), record the node
//                      at level L - levelsup, return the leaf's word id and weight.
//   k_vocab_aggregate  two workgroups per descriptor set: FeatureVector = (node, feature) pairs sorted
//                      (bitonic, LDS) and run-length grouped; BowVector = (word) sorted, TF-IDF weights
//                      accumulated in feature order per word (BowVector::addWeight), L1 norm summed
//                      sequentially in word order (BowVector::normalize) so doubles match bit for bit.
// Only TF_IDF / TF weighting with L1 scoring (ORBvoc.txt: "10 6 0 0") and IDF / BINARY (addIfNotExist)
// are supported; features whose word weight is 0 are skipped, as in :1153-1157.
// =====================================================================================================
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "orbx_common.h"

namespace orbx {

enum { W_TF_IDF = 0, W_TF = 1, W_IDF = 2, W_BINARY = 3 };      // DBoW2 WeightingType
enum { S_L1 = 0, S_L2 = 1 };                                  // DBoW2 ScoringType (L1_NORM, L2_NORM, ...)
constexpr int kVocabAggThreads = 1024;
constexpr int kVocabMaxSet = 4096;                            // descriptors per set in one workgroup

struct VocabDev {
    const uint4* desc;        // [n_nodes][2]
    const int32_t* child_off; // [n_nodes + 1] CSR of children
    const int32_t* child;     // children ids
    const double* weight;     // [n_nodes]
    const int32_t* word_id;   // [n_nodes] (-1 for inner nodes)
    int n_nodes;
};

__global__ __launch_bounds__(256) void k_vocab_words(VocabDev V, const uint8_t* __restrict__ desc, const int32_t* __restrict__ counts,
                                                     int n_fixed, int stride, int nid_level, int32_t* __restrict__ word,
                                                     double* __restrict__ wgt, int32_t* __restrict__ node) {
    const int img = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = counts ? counts[img] : n_fixed;
    if (i >= n) return;
    const size_t o = (size_t)img * stride + i;
    const uint4* dp = reinterpret_cast<const uint4*>(desc + 32 * o);
    const uint4 a0 = dp[0], a1 = dp[1];
    int cur = 0, level = 0, nid = 0;
    while (V.child_off[cur + 1] > V.child_off[cur]) {          // !isLeaf
        ++level;
        const int c0 = V.child_off[cur], c1 = V.child_off[cur + 1];
        int best = V.child[c0];
        int bd = hamming256(a0, a1, V.desc[2 * best], V.desc[2 * best + 1]);
        for (int c = c0 + 1; c < c1; ++c) {
            const int id = V.child[c];
            const int d = hamming256(a0, a1, V.desc[2 * id], V.desc[2 * id + 1]);
            if (d < bd) { bd = d; best = id; }
        }
        cur = best;
        if (level == nid_level) nid = cur;
    }
    word[o] = V.word_id[cur];
    wgt[o] = V.weight[cur];
    node[o] = nid;
}

// The same descent with 16 lanes per descriptor (4 per wave; branching factor k <= 16): lane j of a group scores
// child j, and the group's (distance, j) minimum -- the first minimum, as the sequential strict '<' -- picks the
// next node.  One level costs one round of independent loads (CSR row, child id, child descriptor) instead of k
// dependent ones.
__device__ __forceinline__ uint32_t group16_min(uint32_t v) {
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0xB1, 0xF, 0xF, false));   // quad_perm 1,0,3,2
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x4E, 0xF, 0xF, false));   // quad_perm 2,3,0,1
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x141, 0xF, 0xF, false));  // row_half_mirror
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x140, 0xF, 0xF, false));  // row_mirror
    return v;
}

__global__ __launch_bounds__(256) void k_vocab_words16(VocabDev V, const uint8_t* __restrict__ desc,
                                                       const int32_t* __restrict__ counts, int n_fixed, int stride,
                                                       int nid_level, int32_t* __restrict__ word, double* __restrict__ wgt,
                                                       int32_t* __restrict__ node) {
    const int img = blockIdx.y;
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x) >> 4, j = (int)threadIdx.x & 15;
    const int n = counts ? counts[img] : n_fixed;
    if (__builtin_amdgcn_read_exec() == 0) return;
    const bool live = i < n;
    const size_t o = (size_t)img * stride + (live ? i : 0);
    const uint4* dp = reinterpret_cast<const uint4*>(desc + 32 * o);
    const uint4 a0 = dp[0], a1 = dp[1];
    int cur = 0, level = 0, nid = 0;
    // every group of the wave walks the same number of levels only if the tree is balanced; groups that reached a
    // leaf idle (their lanes keep the wave's DPP reductions well defined)
    bool done = !live;
    for (;;) {
        int c0 = 0, c1 = 0;
        if (!done) { c0 = V.child_off[cur]; c1 = V.child_off[cur + 1]; }
        if (!done && c1 <= c0) done = true;                      // isLeaf
        if (__builtin_amdgcn_read_exec() == __ballot(done)) break;
        uint32_t key = 0xffffffffu;
        int id = 0;
        if (!done && c0 + j < c1) {
            id = V.child[c0 + j];
            key = ((uint32_t)hamming256(a0, a1, V.desc[2 * id], V.desc[2 * id + 1]) << 8) | (uint32_t)j;
        }
        const uint32_t best = group16_min(key);
        const int bj = (int)(best & 0xff);
        const int bid = __builtin_amdgcn_ds_bpermute(((int)(threadIdx.x & ~15u) + bj) << 2, id);
        if (!done) {
            ++level;
            cur = bid;
            if (level == nid_level) nid = cur;
        }
    }
    if (live && j == 0) {
        word[o] = V.word_id[cur];
        wgt[o] = V.weight[cur];
        node[o] = nid;
    }
}

struct BowOut {
    uint32_t* words; double* values; int32_t* n_words;
    uint32_t* fv_nodes; int32_t* fv_off; int32_t* fv_idx; int32_t* n_fv;
};

// kT threads, sets of <= kMaxSet descriptors: <1024, 4096> (49 KB of LDS) or, for sets of <= 2048, <256, 2048> (24 KB)
// -- a workgroup the size of a FAST band's, so the keyframe batch's 2 x 25 workgroups find CU room beside the front
// end instead of waiting for a CU with 1024 free lanes and 49 KB of LDS.
template <int kT, int kMaxSet>
__global__ __launch_bounds__(kT) void k_vocab_aggregate(const int32_t* __restrict__ counts, int n_fixed, int stride,
                                                                      const int32_t* __restrict__ word, const double* __restrict__ wgt,
                                                                      const int32_t* __restrict__ node, int weighting, int scoring,
                                                                      BowOut out) {
    // blockIdx.y = 0: FeatureVector of set blockIdx.x; 1: its BowVector (independent, so two workgroups per set)
    __shared__ unsigned long long key[kMaxSet];
    __shared__ int flag[kMaxSet + 1];
    __shared__ int tmp[64];
    const int img = blockIdx.x, tid = threadIdx.x, T = blockDim.x;
    const int n = min(counts ? counts[img] : n_fixed, kMaxSet);
    const size_t o = (size_t)img * stride;
    int P2 = 1;
    while (P2 < n) P2 <<= 1;
    const bool fv = blockIdx.y == 0;
    // (node or word, feature) for features whose word is not stopped (w > 0)
    const int32_t* kv = fv ? node : word;
    for (int i = tid; i < P2; i += T)
        key[i] = (i < n && wgt[o + i] > 0) ? ((unsigned long long)(uint32_t)kv[o + i] << 32) | (uint32_t)i : ~0ull;
    __syncthreads();
    block_bitonic_u64(key, P2);
    for (int i = tid; i < P2; i += T) flag[i] = (key[i] != ~0ull && (i == 0 || (key[i] >> 32) != (key[i - 1] >> 32))) ? 1 : 0;
    __syncthreads();
    int nv = 0;   // number of valid entries
    for (int i = tid; i < P2; i += T) nv += key[i] != ~0ull;
    nv = wave_sum(nv);
    if (lane_id() == 0) tmp[32 + (tid >> 6)] = nv;
    __syncthreads();
    nv = 0;
    for (int wv = 0; wv < (T >> 6); ++wv) nv += tmp[32 + wv];
    __syncthreads();
    if (fv) {
        // ---- FeatureVector: node groups of the sorted (node, feature) list
        const int nnodes = block_scan_array(flag, P2, tmp);   // flag[i] = index of i's group if it starts one
        for (int i = tid; i < nv; i += T) {
            out.fv_idx[o + i] = (int32_t)(key[i] & 0xffffffffu);
            const bool start = (i == 0) || (key[i] >> 32) != (key[i - 1] >> 32);
            if (start) {
                out.fv_nodes[o + flag[i]] = (uint32_t)(key[i] >> 32);
                out.fv_off[o + img + flag[i]] = i;   // offsets array has stride + 1 per image: index o + img
            }
        }
        if (tid == 0) {
            out.fv_off[o + img + nnodes] = nv;
            out.n_fv[img] = nnodes;
        }
        return;
    }
    // ---- BowVector: one value per word of the sorted (word, feature) list
    const int nwords = block_scan_array(flag, P2, tmp);
    // per word: its weight accumulated in feature order (addWeight: one += per further occurrence), kept in
    // registers until every thread is done reading key[], then written over key[] as doubles
    constexpr int kPer = kMaxSet / kT;
    double myv[kPer];
    int myslot[kPer];
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
        const int i = tid + r * T;
        myslot[r] = -1;
        if (i >= nv) continue;
        const bool start = (i == 0) || (key[i] >> 32) != (key[i - 1] >> 32);
        if (!start) continue;
        const double w = wgt[o + (key[i] & 0xffffffffu)];
        double v = w;
        if (weighting == W_TF_IDF || weighting == W_TF) {
            for (int k = i + 1; k < nv && (key[k] >> 32) == (key[i] >> 32); ++k) v += w;
        }                                                        // IDF / BINARY: addIfNotExist keeps w
        out.words[o + flag[i]] = (uint32_t)(key[i] >> 32);
        myv[r] = v;
        myslot[r] = flag[i];
    }
    __syncthreads();
    double* vals = reinterpret_cast<double*>(key);
#pragma unroll
    for (int r = 0; r < kPer; ++r)
        if (myslot[r] >= 0) vals[myslot[r]] = myv[r];
    __syncthreads();
    // BowVector::normalize: the norm is a sequential sum in word order (bit-exact), read from LDS
    __shared__ double norm_sh;
    if (tid == 0) {
        double norm = 0.0;
        int k = 0;
        if (scoring == S_L1) {
            for (; k + 8 <= nwords; k += 8) {
                double x[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) x[u] = vals[k + u];
#pragma unroll
                for (int u = 0; u < 8; ++u) norm += fabs(x[u]);
            }
            for (; k < nwords; ++k) norm += fabs(vals[k]);
        } else {
            for (; k + 8 <= nwords; k += 8) {
                double x[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) x[u] = vals[k + u];
#pragma unroll
                for (int u = 0; u < 8; ++u) norm += x[u] * x[u];
            }
            for (; k < nwords; ++k) norm += vals[k] * vals[k];
            norm = sqrt(norm);
        }
        norm_sh = norm;
        out.n_words[img] = nwords;
    }
    __syncthreads();
    const double norm = norm_sh;
    for (int k = tid; k < nwords; k += T) out.values[o + k] = norm > 0.0 ? vals[k] / norm : vals[k];
}

struct Vocab {
    int k = 0, L = 0, scoring = 0, weighting = 0, device = 0;
    int n_nodes = 0, n_words = 0;
    int max_children = 0;              // the descent uses 16-lane groups when every node has <= 16 children
    hipStream_t stream = nullptr;      // lazy: own() on first host-API use
    std::once_flag stream_once;
    hipStream_t own() { return lazy_stream(stream, stream_once, device); }
    void* mem = nullptr;
    VocabDev dev{};
    // scratch for the host API
    void* scratch = nullptr;
    size_t scratch_bytes = 0;
};

static int vocab_build(Vocab* v, int n_lines, const int32_t* parent, const uint8_t* is_leaf, const uint8_t* desc,
                       const double* weight) {
    // node 0 = root; line i (0-based) = node i + 1, exactly as loadFromTextFile numbers nodes
    const int N = n_lines + 1;
    std::vector<std::vector<int>> children(N);
    std::vector<int32_t> word(N, -1);
    std::vector<double> w(N, 0.0);
    std::vector<uint8_t> d((size_t)N * 32, 0);
    int nw = 0;
    for (int i = 0; i < n_lines; ++i) {
        const int id = i + 1;
        ORBX_REQUIRE(parent[i] >= 0 && parent[i] < id, ORBX_ERR_ARG, "vocab node %d: bad parent %d", id, parent[i]);
        children[parent[i]].push_back(id);
        std::memcpy(&d[(size_t)id * 32], desc + (size_t)i * 32, 32);
        w[id] = weight[i];
        if (is_leaf[i]) word[id] = nw++;
    }
    for (int id = 0; id < N; ++id)
        ORBX_REQUIRE(!children[id].empty() || word[id] >= 0 || id == 0, ORBX_ERR_ARG,
                     "vocab node %d is neither a leaf nor has children", id);
    std::vector<int32_t> off(N + 1, 0), ch;
    for (int id = 0; id < N; ++id) {
        off[id] = (int)ch.size();
        ch.insert(ch.end(), children[id].begin(), children[id].end());
    }
    off[N] = (int)ch.size();
    v->max_children = 0;
    for (int id = 0; id < N; ++id) v->max_children = std::max(v->max_children, (int)children[id].size());
    const size_t bd = (size_t)N * 32, bo = 4 * ((size_t)N + 1), bc = 4 * std::max<size_t>(ch.size(), 1), bw = 8 * (size_t)N,
                 bwi = 4 * (size_t)N;
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t total = al(bd) + al(bo) + al(bc) + al(bw) + al(bwi);
    ORBX_HIP(hipSetDevice(v->device));
    ::orbx::LegacyLock legacy_;
    ORBX_HIP(hipMalloc(&v->mem, total));
    uint8_t* p = (uint8_t*)v->mem;
    v->dev.desc = (const uint4*)p;             ORBX_HIP(hipMemcpy(p, d.data(), bd, hipMemcpyHostToDevice)); p += al(bd);
    v->dev.child_off = (const int32_t*)p;      ORBX_HIP(hipMemcpy(p, off.data(), bo, hipMemcpyHostToDevice)); p += al(bo);
    v->dev.child = (const int32_t*)p;          if (!ch.empty()) ORBX_HIP(hipMemcpy(p, ch.data(), 4 * ch.size(), hipMemcpyHostToDevice)); p += al(bc);
    v->dev.weight = (const double*)p;          ORBX_HIP(hipMemcpy(p, w.data(), bw, hipMemcpyHostToDevice)); p += al(bw);
    v->dev.word_id = (const int32_t*)p;        ORBX_HIP(hipMemcpy(p, word.data(), bwi, hipMemcpyHostToDevice));
    v->dev.n_nodes = N;
    v->n_nodes = N;
    v->n_words = nw;
    return ORBX_OK;
}

}  // namespace orbx

using namespace orbx;
struct orbx_vocab : public orbx::Vocab {};

static int vocab_new(int k, int L, int scoring, int weighting, int device, orbx_vocab** out) {
    ORBX_REQUIRE(out, ORBX_ERR_ARG, "out is NULL");
    *out = nullptr;
    ORBX_REQUIRE(k >= 2 && k <= 20 && L >= 1 && L <= 10 && scoring >= 0 && scoring <= 5 && weighting >= 0 && weighting <= 3,
                 ORBX_ERR_ARG, "bad vocabulary header %d %d %d %d", k, L, scoring, weighting);
    ORBX_REQUIRE(scoring == S_L1 || scoring == S_L2, ORBX_ERR_UNSUPPORTED, "only L1/L2 scoring is supported");
    int ndev = 0;
    ORBX_HIP(hipGetDeviceCount(&ndev));
    ORBX_REQUIRE(device >= 0 && device < ndev, ORBX_ERR_ARG, "device %d out of range", device);
    orbx_vocab* v = new orbx_vocab();
    v->k = k; v->L = L; v->scoring = scoring; v->weighting = weighting; v->device = device;
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) {
        set_error("stream create: %s", hipGetErrorString(e));
        delete v;
        return ORBX_ERR_HIP;
    }
    *out = v;
    return ORBX_OK;
}

static size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

static int vocab_launch(orbx_vocab* v, const uint8_t* d_desc, const int32_t* d_counts, int n_fixed, int batch, int stride,
                        int levelsup, int32_t* d_word, double* d_wgt, int32_t* d_node, BowOut out, hipStream_t s, bool aggregate) {
    const int nid_level = v->L - levelsup;   // nid_level <= 0 -> root (node 0), as :1226
    if (v->max_children <= 16)
        hipLaunchKernelGGL(k_vocab_words16, dim3((stride + 15) / 16, batch), dim3(256), 0, s, v->dev, d_desc, d_counts, n_fixed,
                           stride, nid_level > 0 ? nid_level : -1, d_word, d_wgt, d_node);
    else
        hipLaunchKernelGGL(k_vocab_words, dim3((stride + 255) / 256, batch), dim3(256), 0, s, v->dev, d_desc, d_counts, n_fixed,
                           stride, nid_level > 0 ? nid_level : -1, d_word, d_wgt, d_node);
    if (aggregate)
    {
        const bool small = stride <= 2048;
        auto kagg = small ? k_vocab_aggregate<256, 2048> : k_vocab_aggregate<kVocabAggThreads, kVocabMaxSet>;
        hipLaunchKernelGGL(kagg, dim3(batch, 2), dim3(small ? 256 : kVocabAggThreads), 0, s, d_counts, n_fixed, stride, d_word,
                           d_wgt, d_node, v->weighting, v->scoring, out);
    }
    ORBX_HIP(hipGetLastError());
    return ORBX_OK;
}

extern "C" {

int orbx_vocab_create(int k, int L, int scoring, int weighting, int n_lines, const int32_t* parent, const uint8_t* is_leaf,
                      const uint8_t* desc, const double* weight, int device, orbx_vocab** out) {
    ORBX_REQUIRE(n_lines >= 1 && parent && is_leaf && desc && weight, ORBX_ERR_ARG, "bad vocabulary arrays");
    int st = vocab_new(k, L, scoring, weighting, device, out);
    if (st) return st;
    st = vocab_build(*out, n_lines, parent, is_leaf, desc, weight);
    if (st) {
        orbx_vocab_destroy(*out);
        *out = nullptr;
    }
    return st;
}

// TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1338-1424): header "k L scoring weighting",
// then one line per node "parent isLeaf d0 .. d31 weight" (node ids = line order, root = 0).
int orbx_vocab_load_text(const char* path, int device, orbx_vocab** out) {
    ORBX_REQUIRE(path && out, ORBX_ERR_ARG, "null argument");
    *out = nullptr;
    std::ifstream f(path);
    ORBX_REQUIRE(f.good(), ORBX_ERR_ARG, "cannot open %s", path);
    std::string line;
    std::getline(f, line);
    std::stringstream hs(line);
    int k = -1, L = -1, n1 = -1, n2 = -1;
    hs >> k >> L >> n1 >> n2;
    ORBX_REQUIRE(!(k < 0 || k > 20 || L < 1 || L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3), ORBX_ERR_ARG,
                 "Vocabulary loading failure: This is not a correct text file!");
    std::vector<int32_t> parent;
    std::vector<uint8_t> leaf, desc;
    std::vector<double> weight;
    while (std::getline(f, line)) {
        std::stringstream ss(line);
        int pid, isleaf;
        if (!(ss >> pid)) continue;   // blank trailing line
        ss >> isleaf;
        uint8_t d[32] = {0};
        for (int i = 0; i < 32; ++i) {
            int x;
            if (ss >> x) d[i] = (uint8_t)x;
        }
        double w = 0;
        ss >> w;
        parent.push_back(pid);
        leaf.push_back(isleaf > 0);
        desc.insert(desc.end(), d, d + 32);
        weight.push_back(w);
    }
    ORBX_REQUIRE(!parent.empty(), ORBX_ERR_ARG, "vocabulary %s has no nodes", path);
    return orbx_vocab_create(k, L, n1, n2, (int)parent.size(), parent.data(), leaf.data(), desc.data(), weight.data(), device,
                             out);
}

int orbx_vocab_destroy(orbx_vocab* v) {
    if (!v) return ORBX_OK;
    (void)hipSetDevice(v->device);
    ::orbx::LegacyLock legacy_;
    (void)::orbx::device_sync();              // device calls on callers' streams read the tree and the scratch
    if (v->mem) (void)hipFree(v->mem);
    if (v->scratch) (void)hipFree(v->scratch);
    if (v->stream) (void)hipStreamDestroy(v->stream);
    delete v;
    return ORBX_OK;
}

int orbx_vocab_info(const orbx_vocab* v, int* k, int* L, int* n_nodes, int* n_words) {
    ORBX_REQUIRE(v, ORBX_ERR_ARG, "null vocabulary");
    if (k) *k = v->k;
    if (L) *L = v->L;
    if (n_nodes) *n_nodes = v->n_nodes;
    if (n_words) *n_words = v->n_words;
    return ORBX_OK;
}

int orbx_vocab_words_device(orbx_vocab* v, const uint8_t* d_desc, int n, int levelsup, int32_t* d_word, double* d_weight,
                            int32_t* d_node, void* stream) {
    ORBX_REQUIRE(v && n >= 0 && (n == 0 || (d_desc && d_word && d_weight && d_node)), ORBX_ERR_ARG, "bad argument");
    if (n == 0) return ORBX_OK;
    ORBX_HIP(hipSetDevice(v->device));
    return vocab_launch(v, d_desc, nullptr, n, 1, n, levelsup, d_word, d_weight, d_node, BowOut{}, (hipStream_t)stream, false);
}

int orbx_vocab_transform_batch_device(orbx_vocab* v, const uint8_t* d_desc, const int32_t* d_counts, int batch, int capacity,
                                      int levelsup, int32_t* d_word, double* d_weight, int32_t* d_node, uint32_t* d_bow_words,
                                      double* d_bow_values, int32_t* d_n_words, uint32_t* d_fv_nodes, int32_t* d_fv_offsets,
                                      int32_t* d_fv_indices, int32_t* d_n_fv_nodes, void* stream) {
    ORBX_REQUIRE(v && d_desc && d_counts && batch > 0 && capacity > 0 && d_word && d_weight && d_node && d_bow_words &&
                     d_bow_values && d_n_words && d_fv_nodes && d_fv_offsets && d_fv_indices && d_n_fv_nodes,
                 ORBX_ERR_ARG, "bad argument");
    ORBX_REQUIRE(capacity <= kVocabMaxSet, ORBX_ERR_UNSUPPORTED, "capacity %d > %d", capacity, kVocabMaxSet);
    ORBX_HIP(hipSetDevice(v->device));
    BowOut out{d_bow_words, d_bow_values, d_n_words, d_fv_nodes, d_fv_offsets, d_fv_indices, d_n_fv_nodes};
    return vocab_launch(v, d_desc, d_counts, 0, batch, capacity, levelsup, d_word, d_weight, d_node, out, (hipStream_t)stream, true);
}

// Host form of TemplatedVocabulary::transform(features, BowVector&, FeatureVector&, levelsup).
int orbx_vocab_transform(orbx_vocab* v, const uint8_t* desc, int n, int levelsup, uint32_t* bow_words, double* bow_values,
                         int* n_words, uint32_t* fv_nodes, int32_t* fv_offsets, int32_t* fv_indices, int* n_fv_nodes) {
    ORBX_REQUIRE(v && n_words && n_fv_nodes && n >= 0, ORBX_ERR_ARG, "bad argument");
    *n_words = 0;
    *n_fv_nodes = 0;
    if (n == 0) {
        if (fv_offsets) fv_offsets[0] = 0;
        return ORBX_OK;
    }
    ORBX_REQUIRE(desc && bow_words && bow_values && fv_nodes && fv_offsets && fv_indices, ORBX_ERR_ARG, "null output");
    ORBX_REQUIRE(n <= kVocabMaxSet, ORBX_ERR_UNSUPPORTED, "more than %d descriptors", kVocabMaxSet);
    ORBX_HIP(hipSetDevice(v->device));
    const size_t N = (size_t)n;
    const size_t bytes = al256(32 * N) + 3 * al256(4 * N) + 2 * al256(8 * N) + 3 * al256(4 * (N + 1)) + al256(64);
    if (bytes > v->scratch_bytes) {
        if (v->scratch) {
            ::orbx::LegacyLock legacy_;
            ORBX_HIP(::orbx::device_sync());      // an earlier call on any stream may still read the old buffer
            (void)hipFree(v->scratch);
        }
        v->scratch = nullptr;
        ORBX_HIP(hipMalloc(&v->scratch, bytes));
        v->scratch_bytes = bytes;
    }
    uint8_t* p = (uint8_t*)v->scratch;
    auto take = [&](size_t b) { uint8_t* q = p; p += al256(b); return q; };
    uint8_t* dd = take(32 * N);
    int32_t* dwd = (int32_t*)take(4 * N);
    double* dwt = (double*)take(8 * N);
    int32_t* dnd = (int32_t*)take(4 * N);
    uint32_t* dbw = (uint32_t*)take(4 * (N + 1));
    double* dbv = (double*)take(8 * N);
    uint32_t* dfn = (uint32_t*)take(4 * (N + 1));
    int32_t* dfo = (int32_t*)take(4 * (N + 1));
    int32_t* dfi = (int32_t*)take(4 * N);
    int32_t* dcnt = (int32_t*)take(64);
    hipStream_t s = v->own();
    int32_t hn[3] = {n, 0, 0};
    ORBX_HIP(hipMemcpyAsync(dd, desc, 32 * N, hipMemcpyHostToDevice, s));
    ORBX_HIP(hipMemcpyAsync(dcnt, hn, 4, hipMemcpyHostToDevice, s));
    BowOut out{dbw, dbv, dcnt + 1, dfn, dfo, dfi, dcnt + 2};
    int st = vocab_launch(v, dd, dcnt, 0, 1, n, levelsup, dwd, dwt, dnd, out, s, true);
    if (st) return st;
    ORBX_HIP(hipMemcpyAsync(hn, dcnt, 12, hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipStreamSynchronize(s));
    *n_words = hn[1];
    *n_fv_nodes = hn[2];
    ORBX_HIP(hipMemcpyAsync(bow_words, dbw, 4 * (size_t)hn[1], hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipMemcpyAsync(bow_values, dbv, 8 * (size_t)hn[1], hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipMemcpyAsync(fv_nodes, dfn, 4 * (size_t)hn[2], hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipMemcpyAsync(fv_offsets, dfo, 4 * ((size_t)hn[2] + 1), hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipMemcpyAsync(fv_indices, dfi, 4 * N, hipMemcpyDeviceToHost, s));
    ORBX_HIP(hipStreamSynchronize(s));
    return ORBX_OK;
}

}  // extern "C"
