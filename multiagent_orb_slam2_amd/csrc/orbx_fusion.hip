// =====================================================================================================
// orbx_fusion.hip — the keyframe path of one agent into MapFusion, as one native object (include/orbx.h,
// "Keyframe fusion").  Replaces what the reference does per keyframe between LoopClosing and MapFusion:
//
//   KeyFrame::ComputeBoW (src/KeyFrame.cc, DBoW2 transform)          -> orbx_vocab_transform_batch_device
//   LoopClosing::Run -> MultiAgentServer::InsertKeyFrame -> MapFusion::InsertKeyFrame
//                       (src/LoopClosing.cc:83-94, src/MapFusion.cc:83-88: a KeyFrame* queue)
//                                                                     -> fixed-size packets in a device ring,
//                                                                        all-gathered across agents
//   MapFusion::DetectFusionCandidates: KeyFrameDatabase::DetectLoopCandidates (src/MapFusion.cc:133), drop
//                       same-map candidates (:136-144), then add the keyframe to the database (:149 / :222)
//                                                                     -> orbx_kfdb_detect_sequential_device +
//                                                                        orbx_kfdb_candidate_pairs_device
//   MapFusion::ComputeSim3: ORBmatcher(0.75, true).SearchByBoW(curKF, candKF) and the 20-match gate (:275-281)
//                                                                     -> orbx_search_by_bow_kfkf_pairs_device
//
// A step is two device phases around the (optional) exchange: pack (gather the keyframe rows of an extractor
// batch, BoW, packets) and commit (ring slots, database, queries, SearchByBoW).  With one agent the packets are
// written straight into the ring; with several, the caller all-gathers them into the ring region that
// orbx_fusion_pack_device returns (RCCL over xGMI through torch.distributed, or orbx_exchange below).  Every
// host-side decision (ring position, membership) is O(keyframes) bookkeeping; nothing is synchronised.
//
// orbx_exchange: an RCCL communicator opened by dlopen of the process's librccl (the copy torch.distributed
// already loaded, when there is one), for callers without torch -- the reference's MultiAgentServer in C++.
// =====================================================================================================
#include <hip/hip_runtime.h>
#include <dlfcn.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "orbx_common.h"

namespace orbx {

constexpr int kPacketHeader = 32;

static size_t a16(size_t x) { return (x + 15) & ~(size_t)15; }

// Byte layout of one keyframe packet (multiagent.py PacketLayout is the same; checked by tests/test_capi.py):
// header 32 | kps cap*28 | desc cap*32 | fv_nodes cap*4 | fv_offsets (cap+1)*4 | fv_indices cap*4 | valid cap |
// bow_words cap*4 | bow_values cap*8, every field 16-byte aligned.  Header: int32 count, agent, frame, n_fv, n_words.
struct PacketLayout {
    size_t kps, desc, fv_nodes, fv_offsets, fv_indices, valid, bow_words, bow_values, bytes;
    explicit PacketLayout(int cap) {
        size_t o = kPacketHeader;
        auto take = [&](size_t sz) { const size_t r = o; o = a16(o + sz); return r; };
        kps = take((size_t)cap * 28);
        desc = take((size_t)cap * 32);
        fv_nodes = take((size_t)cap * 4);
        fv_offsets = take(((size_t)cap + 1) * 4);
        fv_indices = take((size_t)cap * 4);
        valid = take((size_t)cap);
        bow_words = take((size_t)cap * 4);
        bow_values = take((size_t)cap * 8);
        bytes = o;
    }
};

struct PackArgs {
    const orbx_keypoint* kps; const uint8_t* desc; const int32_t* counts;   // extractor batch layout
    const float* depth; const uint8_t* valid;                              // MapPoint-valid source (one of them)
    int first_row, row_step, capacity;
    long long frame_base; int frame_step;
    int agent;
    // vocabulary outputs of the gathered rows (set j at j * capacity)
    const uint32_t* fv_nodes; const int32_t* fv_offsets; const int32_t* fv_indices; const int32_t* n_fv;
    const uint32_t* bow_words; const double* bow_values; const int32_t* n_words;
    uint8_t* out; size_t P;
    size_t o_kps, o_desc, o_fvn, o_fvo, o_fvi, o_valid, o_bw, o_bv;
};

// Rows of the extractor batch -> contiguous descriptor sets + counts for the vocabulary transform.
__global__ __launch_bounds__(256) void k_fusion_gather(const uint8_t* __restrict__ desc, const int32_t* __restrict__ counts,
                                                       int first_row, int row_step, int capacity, uint4* __restrict__ out_desc,
                                                       int32_t* __restrict__ out_counts) {
    const int j = blockIdx.y;
    const size_t row = (size_t)first_row + (size_t)j * row_step;
    const int n = min(max(counts[row], 0), capacity);
    const uint4* src = reinterpret_cast<const uint4*>(desc + row * capacity * 32);
    uint4* dst = out_desc + (size_t)j * capacity * 2;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < 2 * n; i += gridDim.x * blockDim.x) dst[i] = src[i];
    if (blockIdx.x == 0 && threadIdx.x == 0) out_counts[j] = n;
}

// One workgroup per keyframe: header, keypoints, descriptors, MapPoint-valid flags, FeatureVector, BowVector.
__global__ __launch_bounds__(256) void k_fusion_pack(PackArgs A) {
    const int j = blockIdx.x, t = threadIdx.x, T = blockDim.x;
    const size_t row = (size_t)A.first_row + (size_t)j * A.row_step;
    const int cap = A.capacity;
    const int n = min(max(A.counts[row], 0), cap);
    uint8_t* P = A.out + (size_t)j * A.P;
    const int nfv = A.n_fv[j], nw = A.n_words[j];
    if (t < 8) {
        int32_t h = 0;
        if (t == 0) h = n;
        else if (t == 1) h = A.agent;
        else if (t == 2) h = (int32_t)(A.frame_base + (long long)j * A.frame_step);
        else if (t == 3) h = nfv;
        else if (t == 4) h = nw;
        reinterpret_cast<int32_t*>(P)[t] = h;
    }
    const uint32_t* ks = reinterpret_cast<const uint32_t*>(A.kps + row * cap);
    uint32_t* kd = reinterpret_cast<uint32_t*>(P + A.o_kps);
    for (int i = t; i < 7 * cap; i += T) kd[i] = ks[i];
    const uint4* ds = reinterpret_cast<const uint4*>(A.desc + row * cap * 32);
    uint4* dd = reinterpret_cast<uint4*>(P + A.o_desc);
    for (int i = t; i < 2 * cap; i += T) dd[i] = ds[i];
    for (int i = t; i < cap; i += T) {
        uint8_t v = 0;
        if (i < n) v = A.valid ? (A.valid[row * cap + i] != 0) : (A.depth ? (A.depth[row * cap + i] > 0.0f) : 1);
        P[A.o_valid + i] = v;
    }
    const size_t s = (size_t)j * cap;
    uint32_t* fvn = reinterpret_cast<uint32_t*>(P + A.o_fvn);
    int32_t* fvo = reinterpret_cast<int32_t*>(P + A.o_fvo);
    int32_t* fvi = reinterpret_cast<int32_t*>(P + A.o_fvi);
    uint32_t* bw = reinterpret_cast<uint32_t*>(P + A.o_bw);
    double* bv = reinterpret_cast<double*>(P + A.o_bv);
    const int nidx = nfv > 0 ? A.fv_offsets[(size_t)j * (cap + 1) + nfv] : 0;
    for (int i = t; i < nfv; i += T) fvn[i] = A.fv_nodes[s + i];
    for (int i = t; i <= nfv; i += T) fvo[i] = A.fv_offsets[(size_t)j * (cap + 1) + i];
    for (int i = t; i < nidx; i += T) fvi[i] = A.fv_indices[s + i];
    for (int i = t; i < nw; i += T) {
        bw[i] = A.bow_words[s + i];
        bv[i] = A.bow_values[s + i];
    }
}

// Per-step device tables: the new ring slots in processing order, this agent's query slots and keyframe ids, the
// zero minimum scores, and the map (agent) of every new slot and query.
__global__ __launch_bounds__(256) void k_fusion_prep(int first_slot, int n_new, int n, int mine_first, long long id0, int world,
                                                     int agent, int32_t* __restrict__ new_slots, int32_t* __restrict__ qslots,
                                                     unsigned long long* __restrict__ ids, float* __restrict__ zeros,
                                                     int32_t* __restrict__ slot_group, int32_t* __restrict__ qgroup) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_new) {
        new_slots[i] = first_slot + i;
        slot_group[first_slot + i] = world > 1 ? i / n : agent;
    }
    if (i < n) {
        qslots[i] = mine_first + i;
        ids[i] = (unsigned long long)(id0 + i);
        zeros[i] = 0.0f;
        qgroup[i] = agent;
    }
}

__global__ __launch_bounds__(256) void k_fusion_gate(const int32_t* __restrict__ nm, int n, int min_matches,
                                                     unsigned long long* __restrict__ total) {
    int c = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) c += nm[i] >= min_matches;
    c = wave_sum(c);
    if (lane_id() == 0 && c) atomicAdd(total, (unsigned long long)c);
}

}  // namespace orbx

using namespace orbx;

struct orbx_fusion {
    int device = 0;
    orbx_vocab* vocab = nullptr;      // not owned
    orbx_matcher* matcher = nullptr;  // not owned
    orbx_kfdb* db = nullptr;          // owned
    int capacity = 0, slots = 0, k = 16, levelsup = 4, min_matches = 20, agent = 0, world = 1, max_n = 0;
    int max_fv_nodes = 1;
    PacketLayout lay{1};
    uint8_t* ring = nullptr;          // slots x packet bytes
    uint8_t* send = nullptr;          // max_n packets (world > 1)
    // vocabulary scratch for max_n sets
    uint8_t* g_desc = nullptr; int32_t* g_counts = nullptr;
    int32_t* v_word = nullptr; double* v_weight = nullptr; int32_t* v_node = nullptr;
    uint32_t* v_bw = nullptr; double* v_bv = nullptr; int32_t* v_nw = nullptr;
    uint32_t* v_fvn = nullptr; int32_t* v_fvo = nullptr; int32_t* v_fvi = nullptr; int32_t* v_nfv = nullptr;
    // per-step tables and outputs
    int32_t* new_slots = nullptr; int32_t* qslots = nullptr; unsigned long long* ids = nullptr; float* zeros = nullptr;
    int32_t* slot_group = nullptr; int32_t* qgroup = nullptr;
    int32_t* cand = nullptr; int32_t* ncand = nullptr; int32_t* status = nullptr;
    int32_t* pairs = nullptr; int32_t* m12 = nullptr; int32_t* nm = nullptr;
    unsigned long long* gate = nullptr;
    // host bookkeeping
    int pos = 0;
    long long next_id = 1;
    std::vector<int32_t> agent_of;     // per slot, -1 empty
    int pending_first = -1, pending_n = 0, pending_total = 0;   // between pack and commit
    int last_first = 0, last_total = 0, last_mine = 0, last_n = 0;
};

namespace {

template <typename T>
int falloc(T** p, size_t count) {
    ORBX_HIP(hipMalloc((void**)p, std::max<size_t>(count, 1) * sizeof(T)));
    return ORBX_OK;
}

orbx_kf_store ring_store(const orbx_fusion* f) {
    orbx_kf_store S{};
    const size_t P = f->lay.bytes;
    S.desc = f->ring + f->lay.desc; S.desc_stride = P;
    S.kps = (const orbx_keypoint*)(f->ring + f->lay.kps); S.kps_stride = P;
    S.valid = f->ring + f->lay.valid; S.valid_stride = P;
    S.fv_nodes = (const uint32_t*)(f->ring + f->lay.fv_nodes); S.fv_nodes_stride = P;
    S.fv_offsets = (const int32_t*)(f->ring + f->lay.fv_offsets); S.fv_offsets_stride = P;
    S.fv_indices = (const int32_t*)(f->ring + f->lay.fv_indices); S.fv_indices_stride = P;
    S.n_fv = (const int32_t*)(f->ring + 12); S.n_fv_stride = P;
    S.capacity = f->capacity;
    return S;
}

}  // namespace

extern "C" {

int orbx_packet_layout(int capacity, size_t* offsets, size_t* bytes) {
    ORBX_REQUIRE(capacity > 0 && offsets && bytes, ORBX_ERR_ARG, "bad argument");
    const PacketLayout L(capacity);
    const size_t o[8] = {L.kps, L.desc, L.fv_nodes, L.fv_offsets, L.fv_indices, L.valid, L.bow_words, L.bow_values};
    std::memcpy(offsets, o, sizeof(o));
    *bytes = L.bytes;
    return ORBX_OK;
}

int orbx_fusion_create(orbx_vocab* vocab, orbx_matcher* matcher, int capacity, int slots, int max_keyframes, int candidates,
                       int levelsup, int min_matches, int agent, int world, int device, orbx_fusion** out) {
    ORBX_REQUIRE(out, ORBX_ERR_ARG, "out is NULL");
    *out = nullptr;
    ORBX_REQUIRE(vocab && matcher && capacity > 0 && capacity <= 4096 && max_keyframes > 0 && world >= 1 && agent >= 0 &&
                     agent < world && candidates >= 0 && levelsup >= 0,
                 ORBX_ERR_ARG, "bad fusion parameters");
    ORBX_REQUIRE(slots >= world * max_keyframes, ORBX_ERR_ARG, "ring of %d slots cannot hold one exchange of %d x %d keyframes",
                 slots, world, max_keyframes);
    ORBX_REQUIRE(matcher_device(matcher) == device, ORBX_ERR_ARG, "matcher is bound to device %d, not %d",
                 matcher_device(matcher), device);
    int vk = 0, vL = 0, vnodes = 0, vwords = 0;
    int st = orbx_vocab_info(vocab, &vk, &vL, &vnodes, &vwords);
    if (st) return st;
    orbx_fusion* f = new orbx_fusion();
    f->device = device; f->vocab = vocab; f->matcher = matcher;
    f->capacity = capacity; f->slots = slots; f->k = candidates; f->levelsup = levelsup; f->min_matches = min_matches;
    f->agent = agent; f->world = world; f->max_n = max_keyframes;
    int w = 1;
    for (int l = 0; l < std::max(vL - levelsup, 0); ++l) w = std::min(w * vk, capacity);
    f->max_fv_nodes = std::min(capacity, w + 1);   // launch width hint of the batched SearchByBoW
    f->lay = PacketLayout(capacity);
    f->agent_of.assign(slots, -1);
    auto fail = [&](int code) { orbx_fusion_destroy(f); return code; };
    if (hipSetDevice(device) != hipSuccess) { set_error("hipSetDevice(%d) failed", device); return fail(ORBX_ERR_HIP); }
    if ((st = orbx_kfdb_create(vwords, slots, std::min(capacity, 4096), device, &f->db))) return fail(st);
    const size_t N = (size_t)max_keyframes, C = (size_t)capacity, S = (size_t)slots;
    if ((st = falloc(&f->ring, S * f->lay.bytes)) || (st = falloc(&f->send, N * f->lay.bytes)) ||
        (st = falloc(&f->g_desc, N * C * 32)) || (st = falloc(&f->g_counts, N)) || (st = falloc(&f->v_word, N * C)) ||
        (st = falloc(&f->v_weight, N * C)) || (st = falloc(&f->v_node, N * C)) || (st = falloc(&f->v_bw, N * C)) ||
        (st = falloc(&f->v_bv, N * C)) || (st = falloc(&f->v_nw, N)) || (st = falloc(&f->v_fvn, N * C)) ||
        (st = falloc(&f->v_fvo, N * (C + 1))) || (st = falloc(&f->v_fvi, N * C)) || (st = falloc(&f->v_nfv, N)) ||
        (st = falloc(&f->new_slots, (size_t)world * N)) || (st = falloc(&f->qslots, N)) || (st = falloc(&f->ids, N)) ||
        (st = falloc(&f->zeros, N)) || (st = falloc(&f->slot_group, S)) || (st = falloc(&f->qgroup, N)) ||
        (st = falloc(&f->cand, N * S)) || (st = falloc(&f->ncand, N)) || (st = falloc(&f->status, 1)) ||
        (st = falloc(&f->pairs, 2 * N * std::max(candidates, 1))) || (st = falloc(&f->m12, N * std::max(candidates, 1) * C)) ||
        (st = falloc(&f->nm, N * std::max(candidates, 1))) || (st = falloc(&f->gate, 1)))
        return fail(st);
    ::orbx::LegacyLock legacy_;
    if (hipMemset(f->ring, 0, S * f->lay.bytes) != hipSuccess || hipMemset(f->slot_group, 0xff, 4 * S) != hipSuccess ||
        hipMemset(f->status, 0, 4) != hipSuccess || hipMemset(f->gate, 0, 8) != hipSuccess ||
        init_done() != hipSuccess) {   // complete before the first kernel on a caller's (non-blocking) stream
        set_error("fusion init memset failed");
        return fail(ORBX_ERR_HIP);
    }
    *out = f;
    return ORBX_OK;
}

int orbx_fusion_destroy(orbx_fusion* f) {
    if (!f) return ORBX_OK;
    (void)hipSetDevice(f->device);
    (void)::orbx::device_sync();
    if (f->db) orbx_kfdb_destroy(f->db);
    void* bufs[] = {f->ring, f->send, f->g_desc, f->g_counts, f->v_word, f->v_weight, f->v_node, f->v_bw, f->v_bv, f->v_nw,
                    f->v_fvn, f->v_fvo, f->v_fvi, f->v_nfv, f->new_slots, f->qslots, f->ids, f->zeros, f->slot_group,
                    f->qgroup, f->cand, f->ncand, f->status, f->pairs, f->m12, f->nm, f->gate};
    ::orbx::LegacyLock legacy_;
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    delete f;
    return ORBX_OK;
}

int orbx_fusion_info(const orbx_fusion* f, size_t* packet_bytes, int* slots, void** d_ring, orbx_kf_store* store) {
    ORBX_REQUIRE(f, ORBX_ERR_ARG, "null fusion");
    if (packet_bytes) *packet_bytes = f->lay.bytes;
    if (slots) *slots = f->slots;
    if (d_ring) *d_ring = f->ring;
    if (store) *store = ring_store(f);
    return ORBX_OK;
}

int orbx_fusion_pack_device(orbx_fusion* f, const orbx_keypoint* d_kps, const uint8_t* d_desc, const int32_t* d_counts,
                            const float* d_depth, const uint8_t* d_valid, int capacity, int first_row, int row_step, int n,
                            long long frame_base, int frame_step, void* d_send_out, void** d_exchange_dst, void** d_send,
                            void* stream) {
    ORBX_REQUIRE(f && d_kps && d_desc && d_counts && capacity == f->capacity && first_row >= 0 && row_step >= 1 && n >= 1 &&
                     n <= f->max_n,
                 ORBX_ERR_ARG, "bad pack arguments (capacity %d vs %d, n %d of at most %d)", capacity, f->capacity, n, f->max_n);
    ORBX_REQUIRE(f->pending_first < 0, ORBX_ERR_ARG, "pack called twice without commit");
    ORBX_HIP(hipSetDevice(f->device));
    hipStream_t s = (hipStream_t)stream;
    const int C = f->capacity;
    // ring slots of this exchange (rank-major), as DeviceKeyframeStore._reserve
    const int total = f->world * n;
    if (f->pos + total > f->slots) f->pos = 0;
    const int first = f->pos;
    f->pos += total;
    // BoW of the keyframe rows
    dim3 gg((2 * C + 255) / 256, n);
    hipLaunchKernelGGL(k_fusion_gather, gg, dim3(256), 0, s, d_desc, d_counts, first_row, row_step, C, (uint4*)f->g_desc,
                       f->g_counts);
    int st = orbx_vocab_transform_batch_device(f->vocab, f->g_desc, f->g_counts, n, C, f->levelsup, f->v_word, f->v_weight,
                                               f->v_node, f->v_bw, f->v_bv, f->v_nw, f->v_fvn, f->v_fvo, f->v_fvi, f->v_nfv, s);
    if (st) return st;
    PackArgs A{};
    A.kps = d_kps; A.desc = d_desc; A.counts = d_counts; A.depth = d_depth; A.valid = d_valid;
    A.first_row = first_row; A.row_step = row_step; A.capacity = C; A.frame_base = frame_base; A.frame_step = frame_step;
    A.agent = f->agent;
    A.fv_nodes = f->v_fvn; A.fv_offsets = f->v_fvo; A.fv_indices = f->v_fvi; A.n_fv = f->v_nfv;
    A.bow_words = f->v_bw; A.bow_values = f->v_bv; A.n_words = f->v_nw;
    // one agent: straight into the ring; several: into the send buffer the exchange gathers from (the caller's
    // when given)
    uint8_t* send = d_send_out ? (uint8_t*)d_send_out : f->send;
    A.out = f->world > 1 ? send : f->ring + (size_t)first * f->lay.bytes;
    A.P = f->lay.bytes;
    A.o_kps = f->lay.kps; A.o_desc = f->lay.desc; A.o_fvn = f->lay.fv_nodes; A.o_fvo = f->lay.fv_offsets;
    A.o_fvi = f->lay.fv_indices; A.o_valid = f->lay.valid; A.o_bw = f->lay.bow_words; A.o_bv = f->lay.bow_values;
    hipLaunchKernelGGL(k_fusion_pack, dim3(n), dim3(256), 0, s, A);
    ORBX_HIP(hipGetLastError());
    f->pending_first = first;
    f->pending_n = n;
    f->pending_total = total;
    if (d_exchange_dst) *d_exchange_dst = f->ring + (size_t)first * f->lay.bytes;
    if (d_send) *d_send = A.out;
    return ORBX_OK;
}

int orbx_fusion_commit_device(orbx_fusion* f, const void* d_exchanged, int32_t* d_pairs, int32_t* d_match12, int32_t* d_nmatches,
                              void* stream) {
    ORBX_REQUIRE(f && f->pending_first >= 0, ORBX_ERR_ARG, "commit without pack");
    ORBX_HIP(hipSetDevice(f->device));
    hipStream_t s = (hipStream_t)stream;
    const int first = f->pending_first, n = f->pending_n, total = f->pending_total;
    f->pending_first = -1;
    if (d_exchanged)   // the caller gathered the packets elsewhere: into this exchange's ring slots
        ORBX_HIP(hipMemcpyAsync(f->ring + (size_t)first * f->lay.bytes, d_exchanged, (size_t)total * f->lay.bytes,
                                hipMemcpyDeviceToDevice, s));
    const int mine = first + f->agent * n;
    const size_t P = f->lay.bytes;
    for (int i = 0; i < total; ++i) f->agent_of[first + i] = f->world > 1 ? i / n : f->agent;
    const long long id0 = f->next_id + (mine - first);   // global keyframe ids in processing order (KeyFrame::mnId)
    f->next_id += total;
    hipLaunchKernelGGL(k_fusion_prep, dim3((total + 255) / 256), dim3(256), 0, s, first, total, n, mine, id0, f->world,
                       f->agent, f->new_slots, f->qslots, f->ids, f->zeros, f->slot_group, f->qgroup);
    ORBX_HIP(hipGetLastError());
    // the ring overwrote these slots: they leave the database, take the new BowVectors and join it in processing
    // order; the sequential detect answers each query as if it ran right before its own add
    std::vector<int32_t> nl(total);
    for (int i = 0; i < total; ++i) nl[i] = first + i;
    int st;
    if ((st = orbx_kfdb_erase(f->db, nl.data(), total))) return st;
    uint8_t* rows = f->ring + (size_t)first * P;
    if ((st = orbx_kfdb_set_bow_device(f->db, f->new_slots, total, (const uint32_t*)(rows + f->lay.bow_words), (long long)(P / 4),
                                       (const double*)(rows + f->lay.bow_values), (long long)(P / 8), (const int32_t*)(rows + 16),
                                       (long long)(P / 4), s)))
        return st;
    if ((st = orbx_kfdb_add(f->db, nl.data(), total))) return st;
    if ((st = orbx_kfdb_detect_sequential_device(f->db, ORBX_KFDB_LOOP, f->qslots, (const uint64_t*)f->ids, f->zeros, n, nullptr,
                                                 nullptr, f->cand, f->slots, f->ncand, f->status, s)))
        return st;
    const bool multi = f->world > 1;
    if ((st = orbx_kfdb_candidate_pairs_device(f->cand, f->slots, f->ncand, f->qslots, n, multi ? f->slot_group : nullptr,
                                               multi ? f->qgroup : nullptr, f->k, f->pairs, s)))
        return st;
    if (d_pairs && n * f->k > 0)
        ORBX_HIP(hipMemcpyAsync(d_pairs, f->pairs, 8 * (size_t)n * f->k, hipMemcpyDeviceToDevice, s));
    int32_t* m12 = d_match12 ? d_match12 : f->m12;
    int32_t* nm = d_nmatches ? d_nmatches : f->nm;
    const orbx_kf_store S = ring_store(f);
    if ((st = orbx_search_by_bow_kfkf_pairs_device(f->matcher, &S, f->pairs, n * f->k, f->max_fv_nodes, m12, nm, s)))
        return st;
    if (n * f->k > 0) hipLaunchKernelGGL(k_fusion_gate, dim3(1), dim3(256), 0, s, nm, n * f->k, f->min_matches, f->gate);
    ORBX_HIP(hipGetLastError());
    f->last_first = first; f->last_total = total; f->last_mine = mine; f->last_n = n;
    return ORBX_OK;
}

int orbx_fusion_read_ring(orbx_fusion* f, uint8_t* host_dst) {
    ORBX_REQUIRE(f && host_dst, ORBX_ERR_ARG, "bad argument");
    ORBX_HIP(hipSetDevice(f->device));
    ::orbx::LegacyLock legacy_;
    ORBX_HIP(::orbx::device_sync());
    ORBX_HIP(hipMemcpy(host_dst, f->ring, (size_t)f->slots * f->lay.bytes, hipMemcpyDeviceToHost));
    return ORBX_OK;
}

int orbx_fusion_last_step(const orbx_fusion* f, int* first_slot, int* n_new, int* query_first, int* n_queries) {
    ORBX_REQUIRE(f, ORBX_ERR_ARG, "null fusion");
    if (first_slot) *first_slot = f->last_first;
    if (n_new) *n_new = f->last_total;
    if (query_first) *query_first = f->last_mine;
    if (n_queries) *n_queries = f->last_n;
    return ORBX_OK;
}

int orbx_fusion_stats(orbx_fusion* f, long long* gate_passed, int* status) {
    ORBX_REQUIRE(f, ORBX_ERR_ARG, "null fusion");
    ORBX_HIP(hipSetDevice(f->device));
    ::orbx::LegacyLock legacy_;
    ORBX_HIP(::orbx::device_sync());
    unsigned long long g = 0;
    int s = 0;
    ORBX_HIP(hipMemcpy(&g, f->gate, 8, hipMemcpyDeviceToHost));
    ORBX_HIP(hipMemcpy(&s, f->status, 4, hipMemcpyDeviceToHost));
    if (gate_passed) *gate_passed = (long long)g;
    if (status) *status = s;
    return ORBX_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------------------
// orbx_exchange: RCCL all-gather of keyframe packets (the MapFusion ingress, src/MapFusion.cc:83-88, as one
// collective over xGMI).  librccl is opened at run time (dlopen "librccl.so.1": the copy already in the process
// when torch.distributed loaded one), so liborbx has no link-time RCCL dependency.
// ---------------------------------------------------------------------------------------------------------
namespace {

typedef struct { char internal[128]; } RcclUniqueId;
typedef void* RcclComm;
typedef int (*FnGetUniqueId)(RcclUniqueId*);
typedef int (*FnCommInitRank)(RcclComm*, int, RcclUniqueId, int);
typedef int (*FnAllGather)(const void*, void*, size_t, int, RcclComm, hipStream_t);
typedef int (*FnCommDestroy)(RcclComm);
typedef const char* (*FnGetErrorString)(int);

struct Rccl {
    void* so = nullptr;
    FnGetUniqueId get_unique_id = nullptr;
    FnCommInitRank comm_init_rank = nullptr;
    FnAllGather all_gather = nullptr;
    FnCommDestroy comm_destroy = nullptr;
    FnGetErrorString error_string = nullptr;
};

int rccl_load(Rccl* r) {
    if (r->so) return ORBX_OK;
    const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    for (const char* n : names)
        if ((r->so = dlopen(n, RTLD_NOW | RTLD_GLOBAL))) break;
    ORBX_REQUIRE(r->so, ORBX_ERR_UNSUPPORTED, "librccl not found (%s)", dlerror());
    r->get_unique_id = (FnGetUniqueId)dlsym(r->so, "ncclGetUniqueId");
    r->comm_init_rank = (FnCommInitRank)dlsym(r->so, "ncclCommInitRank");
    r->all_gather = (FnAllGather)dlsym(r->so, "ncclAllGather");
    r->comm_destroy = (FnCommDestroy)dlsym(r->so, "ncclCommDestroy");
    r->error_string = (FnGetErrorString)dlsym(r->so, "ncclGetErrorString");
    ORBX_REQUIRE(r->get_unique_id && r->comm_init_rank && r->all_gather && r->comm_destroy, ORBX_ERR_UNSUPPORTED,
                 "librccl misses symbols");
    return ORBX_OK;
}

Rccl g_rccl;

}  // namespace

struct orbx_exchange {
    int device = 0, world = 1, rank = 0;
    RcclComm comm = nullptr;
};

extern "C" {

int orbx_exchange_unique_id(void* id128) {
    ORBX_REQUIRE(id128, ORBX_ERR_ARG, "null id buffer");
    int st = rccl_load(&g_rccl);
    if (st) return st;
    RcclUniqueId id;
    const int e = g_rccl.get_unique_id(&id);
    ORBX_REQUIRE(e == 0, ORBX_ERR_HIP, "ncclGetUniqueId: %s", g_rccl.error_string ? g_rccl.error_string(e) : "error");
    std::memcpy(id128, &id, sizeof(id));
    return ORBX_OK;
}

int orbx_exchange_create(const void* id128, int world, int rank, int device, orbx_exchange** out) {
    ORBX_REQUIRE(id128 && out && world >= 1 && rank >= 0 && rank < world, ORBX_ERR_ARG, "bad exchange arguments");
    *out = nullptr;
    int st = rccl_load(&g_rccl);
    if (st) return st;
    ORBX_HIP(hipSetDevice(device));
    RcclUniqueId id;
    std::memcpy(&id, id128, sizeof(id));
    orbx_exchange* x = new orbx_exchange();
    x->device = device; x->world = world; x->rank = rank;
    const int e = g_rccl.comm_init_rank(&x->comm, world, id, rank);
    if (e != 0) {
        set_error("ncclCommInitRank: %s", g_rccl.error_string ? g_rccl.error_string(e) : "error");
        delete x;
        return ORBX_ERR_HIP;
    }
    *out = x;
    return ORBX_OK;
}

int orbx_exchange_destroy(orbx_exchange* x) {
    if (!x) return ORBX_OK;
    if (x->comm && g_rccl.comm_destroy) g_rccl.comm_destroy(x->comm);
    delete x;
    return ORBX_OK;
}

int orbx_exchange_allgather_device(orbx_exchange* x, const void* d_send, size_t bytes, void* d_recv, void* stream) {
    ORBX_REQUIRE(x && x->comm && d_send && d_recv, ORBX_ERR_ARG, "bad all-gather arguments");
    if (bytes == 0) return ORBX_OK;
    ORBX_HIP(hipSetDevice(x->device));
    const int ncclUint8 = 1;   // ncclDataType_t ncclUint8
    const int e = g_rccl.all_gather(d_send, d_recv, bytes, ncclUint8, x->comm, (hipStream_t)stream);
    ORBX_REQUIRE(e == 0, ORBX_ERR_HIP, "ncclAllGather: %s", g_rccl.error_string ? g_rccl.error_string(e) : "error");
    return ORBX_OK;
}

int orbx_fusion_step_device(orbx_fusion* f, orbx_exchange* x, const orbx_keypoint* d_kps, const uint8_t* d_desc,
                            const int32_t* d_counts, const float* d_depth, const uint8_t* d_valid, int capacity, int first_row,
                            int row_step, int n, long long frame_base, int frame_step, int32_t* d_pairs, int32_t* d_match12,
                            int32_t* d_nmatches, void* stream) {
    ORBX_REQUIRE(f, ORBX_ERR_ARG, "null fusion");
    ORBX_REQUIRE((f->world > 1) == (x != nullptr) && (!x || (x->world == f->world && x->rank == f->agent)), ORBX_ERR_ARG,
                 "exchange does not match the fusion's world / agent");
    void* dst = nullptr;
    void* send = nullptr;
    int st = orbx_fusion_pack_device(f, d_kps, d_desc, d_counts, d_depth, d_valid, capacity, first_row, row_step, n, frame_base,
                                     frame_step, nullptr, &dst, &send, stream);
    if (st) return st;
    if (x && (st = orbx_exchange_allgather_device(x, send, (size_t)n * f->lay.bytes, dst, stream))) {
        f->pending_first = -1;
        return st;
    }
    return orbx_fusion_commit_device(f, nullptr, d_pairs, d_match12, d_nmatches, stream);
}

}  // extern "C"
