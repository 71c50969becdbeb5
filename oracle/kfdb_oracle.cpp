// =====================================================================================================
// kfdb_oracle.cpp — TEST INFRASTRUCTURE ONLY (the checker; never on the product path).
//
// Scalar restatement of the keyframe database query that precedes every cross-agent match
// (SURVEY §8f row 4), in the reference's own sequential order, with the per-keyframe scratch fields
// the reference keeps on KeyFrame (include/KeyFrame.h:155-163) held in a table indexed by slot:
//   KeyFrameDatabase::add / erase / clear                 src/KeyFrameDatabase.cc:40-73
//   KeyFrameDatabase::DetectLoopCandidates                src/KeyFrameDatabase.cc:76-197
//     (LoopClosing::DetectLoop, src/LoopClosing.cc:164; MapFusion::DetectFusion, src/MapFusion.cc:133)
//   KeyFrameDatabase::DetectCovisibilityCandidates        src/KeyFrameDatabase.cc:199-308
//     (MapFusion covisibility discovery, src/MapFusion.cc:820)
//   KeyFrameDatabase::DetectRelocalizationCandidates      src/KeyFrameDatabase.cc:310-420
//     (Tracking::Relocalization, src/Tracking.cc:1366)
//   L1Scoring::score (ORBvoc.txt scoring)                 Thirdparty/DBoW2/DBoW2/ScoringObject.cpp:23-66
// The inverted file is a std::list per word in add order, as in the reference; BowVectors are
// std::map<word, double> so score() walks them exactly as DBoW2 does (lower_bound skips).
// KeyFrame::GetBestCovisibilityKeyFrames(10) (src/KeyFrame.cc:189-197) and GetConnectedKeyFrames
// (:174-181) are inputs: a per-slot ordered list of at most 10 best covisible slots, and the
// per-query exclusion set (connected keyframes for loop queries, keyframes to ignore for covisibility
// queries).  mLoopScore / mCovisScore / mRelocScore are never initialised by the reference
// (src/KeyFrame.cc:34 initialises only the query ids and word counts); here they start at whatever
// the caller sets (orc_kfdb_set_state), 0 by default.
// Compiled with -ffp-contract=off (oracle/Makefile).
// =====================================================================================================
#include <cmath>
#include <cstdint>
#include <list>
#include <map>
#include <set>
#include <utility>
#include <vector>

namespace {

enum { KIND_LOOP = 0, KIND_COVIS = 1, KIND_RELOC = 2 };

struct KfState {   // KeyFrame.h:155-163, one triple per query kind
    uint64_t query[3] = {0, 0, 0};
    int words[3] = {0, 0, 0};
    float score[3] = {0.f, 0.f, 0.f};
};

struct Db {
    std::vector<std::list<int>> inverted;          // mvInvertedFile (KeyFrameDatabase.h), slot ids
    std::vector<std::map<uint32_t, double>> bow;   // KeyFrame::mBowVec per slot
    std::vector<std::vector<int>> covis;           // GetBestCovisibilityKeyFrames(10) per slot
    std::vector<KfState> st;
};

// DBoW2 L1Scoring::score (ScoringObject.cpp:23-66): sum over common words in ascending id order of
// |v-w| - |v| - |w|, then -score/2.
double l1_score(const std::map<uint32_t, double>& v1, const std::map<uint32_t, double>& v2) {
    auto a = v1.begin(), b = v2.begin();
    double score = 0;
    while (a != v1.end() && b != v2.end()) {
        const double vi = a->second, wi = b->second;
        if (a->first == b->first) {
            score += std::fabs(vi - wi) - std::fabs(vi) - std::fabs(wi);
            ++a;
            ++b;
        } else if (a->first < b->first) {
            a = v1.lower_bound(b->first);
        } else {
            b = v2.lower_bound(a->first);
        }
    }
    return -score / 2.0;
}

// The three Detect* functions share one skeleton; 'kind' selects the differences the reference has:
//   LOOP : excluded (connected) keyframes reset their word count but never enter the list (:93-102);
//          scores written to mLoopScore (:135); keep si >= minScore (:136); neighbour needs
//          words > minCommon (:159); bestAcc starts at minScore (:145).
//   COVIS: excluded (ignored) keyframes are skipped entirely (:220); scores are not stored; the
//          neighbour test reads mCovisScore, which nothing assigns (:275); otherwise as LOOP.
//   RELOC: no exclusions; mRelocScore written (:361); no minScore filter; neighbour needs only the
//          query id (:384); bestAcc starts at 0 (:370).
std::vector<int> detect(Db& db, int kind, int qslot, uint64_t qid, float minScore, const std::set<int>& excl) {
    std::list<int> sharing;
    for (const auto& wv : db.bow[qslot]) {
        for (int k : db.inverted[wv.first]) {
            KfState& s = db.st[k];
            if (kind == KIND_COVIS) {
                if (excl.count(k)) continue;
                if (s.query[kind] != qid) {
                    s.words[kind] = 0;
                    s.query[kind] = qid;
                    sharing.push_back(k);
                }
            } else {
                if (s.query[kind] != qid) {
                    s.words[kind] = 0;
                    if (kind == KIND_RELOC || !excl.count(k)) {
                        s.query[kind] = qid;
                        sharing.push_back(k);
                    }
                }
            }
            s.words[kind]++;
        }
    }
    if (sharing.empty()) return {};

    int maxCommon = 0;
    for (int k : sharing)
        if (db.st[k].words[kind] > maxCommon) maxCommon = db.st[k].words[kind];
    const int minCommon = maxCommon * 0.8f;

    std::list<std::pair<float, int>> scored;
    for (int k : sharing) {
        if (db.st[k].words[kind] > minCommon) {
            const float si = (float)l1_score(db.bow[qslot], db.bow[k]);
            if (kind != KIND_COVIS) db.st[k].score[kind] = si;
            if (kind == KIND_RELOC || si >= minScore) scored.push_back({si, k});
        }
    }
    if (scored.empty()) return {};

    std::list<std::pair<float, int>> acc_list;
    float bestAcc = kind == KIND_RELOC ? 0.f : minScore;
    for (const auto& sm : scored) {
        float best = sm.first, acc = sm.first;
        int bestKf = sm.second;
        for (int n : db.covis[sm.second]) {
            const KfState& t = db.st[n];
            if (t.query[kind] != qid) continue;
            if (kind != KIND_RELOC && !(t.words[kind] > minCommon)) continue;
            acc += t.score[kind];
            if (t.score[kind] > best) {
                bestKf = n;
                best = t.score[kind];
            }
        }
        acc_list.push_back({acc, bestKf});
        if (acc > bestAcc) bestAcc = acc;
    }

    const float minRetain = 0.75f * bestAcc;
    std::set<int> added;
    std::vector<int> out;
    for (const auto& am : acc_list) {
        if (am.first > minRetain && !added.count(am.second)) {
            out.push_back(am.second);
            added.insert(am.second);
        }
    }
    return out;
}

}  // namespace

extern "C" {

void* orc_kfdb_create(int n_vocab_words, int n_slots) {
    Db* db = new Db;
    db->inverted.resize(n_vocab_words);
    db->bow.resize(n_slots);
    db->covis.resize(n_slots);
    db->st.resize(n_slots);
    return db;
}

void orc_kfdb_destroy(void* h) { delete static_cast<Db*>(h); }

void orc_kfdb_set_bow(void* h, int slot, const uint32_t* words, const double* values, int n) {
    Db& db = *static_cast<Db*>(h);
    db.bow[slot].clear();
    for (int i = 0; i < n; ++i) db.bow[slot][words[i]] = values[i];
}

void orc_kfdb_set_covis(void* h, int slot, const int32_t* best, int n) {
    Db& db = *static_cast<Db*>(h);
    db.covis[slot].assign(best, best + n);
}

void orc_kfdb_add(void* h, int slot) {   // KeyFrameDatabase::add (:40-46)
    Db& db = *static_cast<Db*>(h);
    for (const auto& wv : db.bow[slot]) db.inverted[wv.first].push_back(slot);
}

void orc_kfdb_erase(void* h, int slot) {   // KeyFrameDatabase::erase (:48-67): first occurrence per word
    Db& db = *static_cast<Db*>(h);
    for (const auto& wv : db.bow[slot]) {
        auto& l = db.inverted[wv.first];
        for (auto it = l.begin(); it != l.end(); ++it)
            if (*it == slot) {
                l.erase(it);
                break;
            }
    }
}

void orc_kfdb_clear(void* h) {   // KeyFrameDatabase::clear (:69-73)
    Db& db = *static_cast<Db*>(h);
    for (auto& l : db.inverted) l.clear();
}

void orc_kfdb_set_state(void* h, int kind, const uint64_t* q, const int32_t* w, const float* s) {
    Db& db = *static_cast<Db*>(h);
    for (size_t k = 0; k < db.st.size(); ++k) {
        db.st[k].query[kind] = q[k];
        db.st[k].words[kind] = w[k];
        db.st[k].score[kind] = s[k];
    }
}

void orc_kfdb_get_state(void* h, int kind, uint64_t* q, int32_t* w, float* s) {
    const Db& db = *static_cast<Db*>(h);
    for (size_t k = 0; k < db.st.size(); ++k) {
        q[k] = db.st[k].query[kind];
        w[k] = db.st[k].words[kind];
        s[k] = db.st[k].score[kind];
    }
}

double orc_kfdb_score(void* h, int a, int b) {   // ORBVocabulary::score(a.mBowVec, b.mBowVec)
    const Db& db = *static_cast<Db*>(h);
    return l1_score(db.bow[a], db.bow[b]);
}

// Returns the number of candidates written to out (or -needed when cap is too small).
int orc_kfdb_detect(void* h, int kind, int qslot, uint64_t qid, float minScore, const int32_t* excl, int n_excl,
                    int32_t* out, int cap) {
    Db& db = *static_cast<Db*>(h);
    const std::set<int> ex(excl, excl + n_excl);
    const std::vector<int> r = detect(db, kind, qslot, qid, minScore, ex);
    if ((int)r.size() > cap) return -(int)r.size();
    for (size_t i = 0; i < r.size(); ++i) out[i] = r[i];
    return (int)r.size();
}

}  // extern "C"
