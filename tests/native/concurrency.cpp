// Native concurrency check of the C-ABI (the reference's threading: Frame.cc:78-81 runs the left and right
// ORBextractor::operator() on two std::threads; Tracking, LocalMapping, LoopClosing and MapFusion call ORBmatcher from
// their own threads).  Two extractors on two threads and four matchers on four threads, three agents' stereo Frames on
// three threads, fresh extractors' first calls racing, and the KeyFrameDatabase's threads, each repeating its call and comparing every result with its
// single-threaded first result (bit-exact).  Plain build: build/concurrency (make; tests/test_gpu_native_concurrency.py);
// with ThreadSanitizer on the host code: make tsan, scripts/tsan_gpu.sh.  Exit status = number of mismatches.
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/orbx.h"

namespace {

// Deterministic textured image: gradient + rectangles + LCG noise (structured FAST corners, like synthetic.py).
std::vector<uint8_t> make_image(int rows, int cols, uint32_t seed) {
    std::vector<uint8_t> im((size_t)rows * cols);
    uint32_t s = seed * 2654435761u + 1u;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return s >> 8; };
    for (int y = 0; y < rows; ++y)
        for (int x = 0; x < cols; ++x) im[(size_t)y * cols + x] = (uint8_t)(60 + (x * 37 + y * 11) / 64 % 120);
    for (int k = 0; k < 300; ++k) {
        const int x0 = (int)(rnd() % cols), y0 = (int)(rnd() % rows), w = 4 + (int)(rnd() % 60), h = 4 + (int)(rnd() % 40);
        const uint8_t v = (uint8_t)(rnd() % 256);
        for (int y = y0; y < y0 + h && y < rows; ++y)
            for (int x = x0; x < x0 + w && x < cols; ++x) im[(size_t)y * cols + x] = v;
    }
    for (auto& p : im) p = (uint8_t)std::min(255, std::max(0, (int)p + (int)(rnd() % 9) - 4));
    return im;
}

struct Extraction {
    std::vector<orbx_keypoint> kps;
    std::vector<uint8_t> desc;
    int n = 0;
};

int extract(orbx_extractor* ex, const std::vector<uint8_t>& im, int rows, int cols, Extraction& out) {
    const int cap = orbx_extractor_max_keypoints(ex, rows, cols);
    if (cap < 0) return cap;
    out.kps.assign(cap, orbx_keypoint{});
    out.desc.assign((size_t)cap * 32, 0);
    return orbx_extract(ex, im.data(), rows, cols, (size_t)cols, out.kps.data(), out.desc.data(), cap, &out.n);
}

bool same(const Extraction& a, const Extraction& b) {
    return a.n == b.n && std::memcmp(a.kps.data(), b.kps.data(), sizeof(orbx_keypoint) * a.n) == 0 &&
           std::memcmp(a.desc.data(), b.desc.data(), (size_t)a.n * 32) == 0;
}

// ---- KeyFrameDatabase: one database shared by the reference's threads (KeyFrameDatabase.cc:42-316 lock mMutex).
// Tracking's relocalisation queries (Tracking.cc:1366), LoopClosing's detect-then-add (LoopClosing.cc:164,169) and
// KeyFrame::SetBadFlag's erase (KeyFrame.cc:564) each run on their own thread; a test-side ticket lock records the
// order in which the calls reached the library, a fourth thread reads (info, score) without it.  The log is replayed
// on a second database single-threaded: every candidate list must match.
struct KfdbSetup {
    int n_vocab = 4000, S = 160;
    std::vector<std::vector<uint32_t>> words;
    std::vector<std::vector<double>> values;
    std::vector<std::vector<int32_t>> covis;
};

KfdbSetup make_kfdb(uint32_t seed) {
    KfdbSetup k;
    uint32_t s = seed * 2654435761u + 7u;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return s >> 8; };
    k.words.resize(k.S); k.values.resize(k.S); k.covis.resize(k.S);
    for (int i = 0; i < k.S; ++i) {
        const int place = i % 8;
        std::vector<uint32_t> w;
        const int m = 60 + (int)(rnd() % 120);
        for (int j = 0; j < m; ++j) w.push_back(rnd() % 3 ? (uint32_t)(place * 400 + rnd() % 400) : (uint32_t)(rnd() % k.n_vocab));
        std::sort(w.begin(), w.end());
        w.erase(std::unique(w.begin(), w.end()), w.end());
        std::vector<double> v(w.size());
        double t = 0;
        for (auto& x : v) { x = 1.0 + (rnd() % 1000); t += x; }
        for (auto& x : v) x /= t;
        k.words[i] = w; k.values[i] = v;
        for (int j = 1; j <= 10; ++j) k.covis[i].push_back((i + 8 * j) % k.S);
    }
    return k;
}

int kfdb_init(orbx_kfdb** db, const KfdbSetup& k) {
    int st = orbx_kfdb_create(k.n_vocab, k.S, 512, 0, db);
    for (int i = 0; i < k.S && !st; ++i) st = orbx_kfdb_set_bow(*db, i, k.words[i].data(), k.values[i].data(), (int)k.words[i].size());
    std::vector<int32_t> slots(k.S), best((size_t)k.S * 10);
    for (int i = 0; i < k.S; ++i) { slots[i] = i; std::copy(k.covis[i].begin(), k.covis[i].end(), best.begin() + 10 * i); }
    if (!st) st = orbx_kfdb_set_covisibility(*db, slots.data(), k.S, best.data());
    std::vector<int32_t> init;
    for (int i = 0; i < 80; ++i) init.push_back(i);
    if (!st) st = orbx_kfdb_add(*db, init.data(), (int)init.size());
    return st;
}

struct KfOp { int kind, slot; uint64_t id; float min_score; std::vector<int32_t> excl, result; };  // kind -1 add, -2 erase

int kfdb_apply(orbx_kfdb* db, KfOp& op) {
    if (op.kind == -1) return orbx_kfdb_add(db, &op.slot, 1);
    if (op.kind == -2) return orbx_kfdb_erase(db, &op.slot, 1);
    int32_t eo[2] = {0, (int32_t)op.excl.size()}, oo[2] = {0, 0};
    std::vector<int32_t> out(160);
    const int st = orbx_kfdb_detect(db, op.kind, &op.slot, &op.id, op.kind == ORBX_KFDB_RELOC ? nullptr : &op.min_score, 1,
                                    op.kind == ORBX_KFDB_RELOC ? nullptr : eo, op.excl.empty() ? nullptr : op.excl.data(), oo,
                                    out.data(), (int)out.size());
    op.result.assign(out.begin(), out.begin() + oo[1]);
    return st;
}

int kfdb_concurrency(int reps) {
    const KfdbSetup k = make_kfdb(11);
    orbx_kfdb *db = nullptr, *db2 = nullptr;
    if (kfdb_init(&db, k) || kfdb_init(&db2, k)) { std::fprintf(stderr, "%s\n", orbx_last_error()); return 100; }
    std::mutex ticket;
    std::vector<KfOp> log;
    int errors = 0;
    auto run = [&](KfOp op) {
        std::lock_guard<std::mutex> g(ticket);
        if (kfdb_apply(db, op)) ++errors;
        log.push_back(std::move(op));
    };
    std::vector<std::pair<int32_t, int32_t>> pairs;
    for (int i = 0; i < 64; ++i) pairs.push_back({i, (i * 7 + 3) % k.S});
    std::vector<double> sref(pairs.size());
    if (orbx_kfdb_score(db2, &pairs[0].first, (int)pairs.size(), sref.data())) return 100;
    std::atomic<bool> stop{false};
    int reader_bad = 0;
    std::vector<std::thread> th;
    th.emplace_back([&] {   // Tracking: relocalisation queries from frames (spare slots 150..159)
        for (int r = 0; r < 4 * reps; ++r) run(KfOp{ORBX_KFDB_RELOC, 150 + r % 10, 1000000ull + r, 0.f, {}, {}});
    });
    th.emplace_back([&] {   // LoopClosing: DetectLoopCandidates, then the keyframe joins the database
        for (int i = 0; i < 40; ++i) {
            const int slot = 80 + i;
            run(KfOp{ORBX_KFDB_LOOP, slot, 2000000ull + i, 0.01f, k.covis[slot], {}});
            run(KfOp{-1, slot, 0, 0.f, {}, {}});
        }
    });
    th.emplace_back([&] {   // KeyFrame::SetBadFlag: erase
        for (int i = 0; i < 30; ++i) { run(KfOp{-2, i, 0, 0.f, {}, {}}); std::this_thread::yield(); }
    });
    std::thread reader([&] {   // no ticket: the database's own lock orders these against the writers
        std::vector<double> sc(pairs.size());
        while (!stop.load()) {
            int nm = 0;
            if (orbx_kfdb_info(db, nullptr, nullptr, nullptr, &nm) || nm < 0 || nm > k.S) ++reader_bad;
            if (orbx_kfdb_score(db, &pairs[0].first, (int)pairs.size(), sc.data()) || sc != sref) ++reader_bad;
        }
    });
    for (auto& t : th) t.join();
    stop = true;
    reader.join();
    int mismatch = 0;
    for (auto& op : log) {   // single-threaded replay in ticket order
        KfOp r = op;
        if (kfdb_apply(db2, r)) ++errors;
        if (r.result != op.result) ++mismatch;
    }
    int nres = 0;
    for (auto& op : log) nres += (int)op.result.size();
    std::printf("kfdb concurrency: %zu operations on 3 threads + reader, %d candidates, %d replay mismatches, %d errors, %d reader "
                "errors\n", log.size(), nres, mismatch, errors, reader_bad);
    orbx_kfdb_destroy(db);
    orbx_kfdb_destroy(db2);
    return mismatch + errors + reader_bad;
}

// ---- First calls racing: fresh extractors used for the first time by several threads at once (the first stereo frame,
// Frame.cc:78-81, and agents starting together): one thread's configuration must not break another's host-graph
// capture.  Every first and second result must equal a warm extractor's.
int first_calls_concurrency(int trials, int rows, int cols) {
    constexpr int kThreads = 6;
    std::vector<uint8_t> im[2] = {make_image(rows, cols, 31), make_image(rows, cols, 32)};
    Extraction warm[2];
    {
        orbx_extractor* w = nullptr;
        if (orbx_extractor_create(2000, 1.2f, 8, 20, 7, 0, &w) || extract(w, im[0], rows, cols, warm[0]) ||
            extract(w, im[1], rows, cols, warm[1])) {
            std::fprintf(stderr, "first calls setup: %s\n", orbx_last_error());
            return 1;
        }
        orbx_extractor_destroy(w);
    }
    int bad = 0;
    for (int t = 0; t < trials; ++t) {
        orbx_extractor* ex[kThreads] = {};
        for (auto& e : ex)
            if (orbx_extractor_create(2000, 1.2f, 8, 20, 7, 0, &e)) return 1;
        std::atomic<int> ready{0};
        int fails[kThreads] = {};
        std::vector<std::thread> th;
        for (int k = 0; k < kThreads; ++k)
            th.emplace_back([&, k] {
                ready.fetch_add(1);
                while (ready.load() < kThreads) std::this_thread::yield();   // all first calls at once
                for (int r = 0; r < 2; ++r) {
                    Extraction e;
                    if (extract(ex[k], im[k & 1], rows, cols, e) || !same(e, warm[k & 1])) ++fails[k];
                }
            });
        for (auto& x : th) x.join();
        for (int k = 0; k < kThreads; ++k) bad += fails[k];
        for (auto& e : ex) orbx_extractor_destroy(e);
    }
    std::printf("first calls: %d trials x %d fresh extractors on %d threads, %d mismatches\n", trials, kThreads, kThreads, bad);
    return bad;
}

// ---- Stereo frames of several agents at once: each agent's Tracking thread builds its stereo Frames (Frame.cc:61-117,
// the two extractions of :78-81 and ComputeStereoMatches :101) with its own left / right extractors and matcher, the
// multi-agent system running one Tracking per agent in one process.  Agent a alternates orbx_stereo_frame with
// orbx_extract_pair + orbx_compute_stereo_matches on its own images; every result must equal its first one.
struct StereoOut {
    Extraction l, r;
    std::vector<float> ur, dp;
    int ns = 0;
};

int stereo_frame_concurrency(int reps, int rows, int cols) {
    constexpr int kAgents = 3;
    orbx_extractor* ex[kAgents][2] = {};
    orbx_matcher* mt[kAgents] = {};
    std::vector<uint8_t> im[kAgents][2];
    const float bf = 386.1448f, b = 0.537166f;   // KITTI 00-02 stereo baseline x fx, baseline (m)
    int st = 0;
    for (int a = 0; a < kAgents && !st; ++a) {
        for (int s = 0; s < 2 && !st; ++s) {
            st = orbx_extractor_create(2000, 1.2f, 8, 20, 7, 0, &ex[a][s]);
        }
        // the right view: the left one shifted by a disparity of 6 + 3a px (right x = left x - d)
        im[a][0] = make_image(rows, cols, 10 + a);
        im[a][1] = im[a][0];
        const int d = 6 + 3 * a;
        for (int y = 0; y < rows; ++y)
            for (int x = 0; x < cols; ++x) im[a][1][(size_t)y * cols + x] = im[a][0][(size_t)y * cols + std::min(x + d, cols - 1)];
        if (!st) st = orbx_matcher_create(0.6f, 1, 0, &mt[a]);
    }
    auto run = [&](int a, bool one_call, StereoOut& o) {
        const int cap = orbx_extractor_max_keypoints(ex[a][0], rows, cols);
        if (cap < 0) return cap;
        o.l.kps.assign(cap, orbx_keypoint{}); o.l.desc.assign((size_t)cap * 32, 0);
        o.r.kps.assign(cap, orbx_keypoint{}); o.r.desc.assign((size_t)cap * 32, 0);
        o.ur.assign(cap, 0.f); o.dp.assign(cap, 0.f);
        if (one_call)
            return orbx_stereo_frame(mt[a], ex[a][0], ex[a][1], im[a][0].data(), (size_t)cols, im[a][1].data(), (size_t)cols,
                                     rows, cols, o.l.kps.data(), o.l.desc.data(), cap, &o.l.n, o.r.kps.data(),
                                     o.r.desc.data(), cap, &o.r.n, bf, b, o.ur.data(), o.dp.data(), &o.ns);
        int e = orbx_extract_pair(ex[a][0], ex[a][1], im[a][0].data(), (size_t)cols, im[a][1].data(), (size_t)cols, rows,
                                  cols, o.l.kps.data(), o.l.desc.data(), cap, &o.l.n, o.r.kps.data(), o.r.desc.data(), cap,
                                  &o.r.n);
        if (!e)
            e = orbx_compute_stereo_matches(mt[a], ex[a][0], ex[a][1], o.l.kps.data(), o.l.desc.data(), o.l.n,
                                            o.r.kps.data(), o.r.desc.data(), o.r.n, bf, b, o.ur.data(), o.dp.data(), &o.ns);
        return e;
    };
    auto equal = [](const StereoOut& x, const StereoOut& y) {
        return same(x.l, y.l) && same(x.r, y.r) && x.ns == y.ns &&
               std::memcmp(x.ur.data(), y.ur.data(), sizeof(float) * x.l.n) == 0 &&
               std::memcmp(x.dp.data(), y.dp.data(), sizeof(float) * x.l.n) == 0;
    };
    StereoOut ref[kAgents];
    for (int a = 0; a < kAgents && !st; ++a) st = run(a, true, ref[a]);
    int bad[kAgents] = {}, errors = 0;
    if (st) {
        std::fprintf(stderr, "stereo frame setup: %s\n", orbx_last_error());
        errors = 1;
    } else {
        std::vector<std::thread> th;
        for (int a = 0; a < kAgents; ++a)
            th.emplace_back([&, a] {
                for (int r = 0; r < reps; ++r) {
                    StereoOut o;
                    if (run(a, r & 1, o) || !equal(o, ref[a])) ++bad[a];
                }
            });
        for (auto& t : th) t.join();
    }
    int total = errors;
    for (int a = 0; a < kAgents; ++a) total += bad[a];
    std::printf("stereo frames: %d agents x %d frames on %d threads (%d / %d / %d stereo matches), %d mismatches\n", kAgents,
                reps, kAgents, ref[0].ns, ref[1].ns, ref[2].ns, total);
    for (auto& m : mt) orbx_matcher_destroy(m);
    for (auto& p : ex)
        for (auto& e : p) orbx_extractor_destroy(e);
    return total;
}

}  // namespace

int main(int argc, char** argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 20;
    if (orbx_device_count() < 1) {
        std::fprintf(stderr, "no HIP device\n");
        return 2;
    }
    const int rows = 375, cols = 1242;
    const std::vector<uint8_t> left = make_image(rows, cols, 1), right = make_image(rows, cols, 2);
    orbx_extractor* ex[2] = {};
    for (auto& e : ex)
        if (orbx_extractor_create(2000, 1.2f, 8, 20, 7, 0, &e)) { std::fprintf(stderr, "%s\n", orbx_last_error()); return 2; }
    Extraction ref[2];
    if (extract(ex[0], left, rows, cols, ref[0]) || extract(ex[1], right, rows, cols, ref[1])) {
        std::fprintf(stderr, "%s\n", orbx_last_error());
        return 2;
    }
    // matcher problems: left descriptors against right descriptors (and the reverse), four matchers
    orbx_matcher* mt[4] = {};
    for (auto& m : mt)
        if (orbx_matcher_create(0.6f, 1, 0, &m)) { std::fprintf(stderr, "%s\n", orbx_last_error()); return 2; }
    struct Bf { std::vector<int32_t> bi, bd, sd; };
    auto bf = [&](orbx_matcher* m, int k, Bf& o) {
        const Extraction& q = ref[k & 1];
        const Extraction& t = ref[(k + 1) & 1];
        o.bi.assign(q.n, 0); o.bd.assign(q.n, 0); o.sd.assign(q.n, 0);
        return orbx_bf_match(m, q.desc.data(), q.n, t.desc.data(), t.n, o.bi.data(), o.bd.data(), o.sd.data());
    };
    Bf bref[4];
    for (int k = 0; k < 4; ++k)
        if (bf(mt[k], k, bref[k])) { std::fprintf(stderr, "%s\n", orbx_last_error()); return 2; }
    int bad[6] = {};
    std::vector<std::thread> th;
    for (int k = 0; k < 2; ++k)
        th.emplace_back([&, k] {
            for (int r = 0; r < reps; ++r) {
                Extraction e;
                if (extract(ex[k], k ? right : left, rows, cols, e) || !same(e, ref[k])) ++bad[k];
            }
        });
    for (int k = 0; k < 4; ++k)
        th.emplace_back([&, k] {
            for (int r = 0; r < reps; ++r) {
                Bf o;
                if (bf(mt[k], k, o) || o.bi != bref[k].bi || o.bd != bref[k].bd || o.sd != bref[k].sd) ++bad[2 + k];
            }
        });
    for (auto& t : th) t.join();
    int total = 0;
    for (int k = 0; k < 6; ++k) total += bad[k];
    std::printf("concurrency: %d extractions (%d, %d keypoints) and %d all-pairs matches on 6 threads, %d mismatches\n",
                2 * reps, ref[0].n, ref[1].n, 4 * reps, total);
    for (auto& m : mt) orbx_matcher_destroy(m);
    for (auto& e : ex) orbx_extractor_destroy(e);
    return total + stereo_frame_concurrency(reps, rows, cols) + first_calls_concurrency(std::max(2, reps / 2), rows, cols) +
           kfdb_concurrency(reps);
}
