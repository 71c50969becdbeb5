// Native concurrency check of the C-ABI (the reference's threading: Frame.cc:78-81 runs the left and right
// ORBextractor::operator() on two std::threads; Tracking, LocalMapping, LoopClosing and MapFusion call ORBmatcher from
// their own threads).  Two extractors on two threads and four matchers on four threads, each repeating its call and
// comparing every result with its single-threaded first result (bit-exact).  Built with ThreadSanitizer on the host
// code (make tsan; scripts/tsan_gpu.sh runs it on the GPU box); exit status = number of mismatches.
#include <cstdint>
#include <cstdio>
#include <cstring>
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
    return total;
}
