// Native latency of the per-call drop-in path (what an unchanged Frame constructor pays):
// orbx_extract(left) and orbx_extract(right) on two std::threads (Frame.cc:78-81), then orbx_compute_stereo_matches,
// host buffers in and out, one stereo frame per call.  The library is dlopen'ed from a path so that builds of older
// commits can be timed by the same driver (bisecting a latency change); only the stable host-API symbols are used.
//
//   host_api_bench <liborbx.so> [frames=300] [rows=375] [cols=1242] [nfeatures=2000]
//
// Prints one JSON line: frames/s from the mean, and median / p95 / max of the frame, left-extract, right-extract
// and stereo phases (ms); "pair": the same frames through orbx_extract_pair from one thread; "stereo_frame": through
// orbx_stereo_frame (extractions + stereo search in one call).
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "../../include/orbx.h"

namespace {

std::vector<uint8_t> make_image(int rows, int cols, uint32_t seed) {   // as tests/native/concurrency.cpp
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

std::vector<uint8_t> shift_right(const std::vector<uint8_t>& l, int rows, int cols, int d) {
    std::vector<uint8_t> r(l.size());
    for (int y = 0; y < rows; ++y)
        for (int x = 0; x < cols; ++x) r[(size_t)y * cols + x] = l[(size_t)y * cols + std::min(cols - 1, x + d)];
    return r;
}

using clk = std::chrono::steady_clock;
double ms_since(clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); }

struct Stats { double med, p95, max, mean; };
Stats stats(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    double m = 0;
    for (double x : v) m += x;
    const size_t n = v.size();
    return {v[n / 2], v[std::min(n - 1, (size_t)(0.95 * (double)n))], v.back(), m / (double)n};
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: %s liborbx.so [frames rows cols nfeatures]\n", argv[0]); return 2; }
    const int frames = argc > 2 ? std::atoi(argv[2]) : 300;
    const int rows = argc > 3 ? std::atoi(argv[3]) : 375, cols = argc > 4 ? std::atoi(argv[4]) : 1242;
    const int nf = argc > 5 ? std::atoi(argv[5]) : 2000;
    void* h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
    if (!h) { std::fprintf(stderr, "dlopen: %s\n", dlerror()); return 2; }
#define SYM(name) auto name = (decltype(&::name))dlsym(h, #name); if (!name) { std::fprintf(stderr, "no %s\n", #name); return 2; }
    SYM(orbx_extractor_create) SYM(orbx_extractor_destroy) SYM(orbx_extract) SYM(orbx_matcher_create)
    SYM(orbx_matcher_destroy) SYM(orbx_compute_stereo_matches) SYM(orbx_last_error)
#undef SYM
    orbx_extractor *exl = nullptr, *exr = nullptr;
    orbx_matcher* m = nullptr;
    if (orbx_extractor_create(nf, 1.2f, 8, 20, 7, 0, &exl) || orbx_extractor_create(nf, 1.2f, 8, 20, 7, 0, &exr) ||
        orbx_matcher_create(0.75f, 1, 0, &m)) {
        std::fprintf(stderr, "create: %s\n", orbx_last_error());
        return 1;
    }
    constexpr int kDistinct = 8;
    std::vector<std::vector<uint8_t>> L, R;
    for (int i = 0; i < kDistinct; ++i) {
        L.push_back(make_image(rows, cols, 100 + i));
        R.push_back(shift_right(L.back(), rows, cols, 3 + i));
    }
    const int cap = 4 * nf + 64;
    std::vector<orbx_keypoint> kl(cap), kr(cap);
    std::vector<uint8_t> dl((size_t)cap * 32), dr((size_t)cap * 32);
    std::vector<float> ur(cap), depth(cap);
    const float fx = 718.856f, bf = 386.1448f;
    std::vector<double> t_frame, t_left, t_right, t_stereo;
    int bad = 0;
    double warm_max = 0;                                          // 10 untimed frames (one-time runtime set-up)
    for (int f = -10; f < frames; ++f) {
        const int k = (f + kDistinct * 4) % kDistinct;
        int nl = 0, nr = 0, ns = 0, str = 0;
        double tr = 0;
        const auto t0 = clk::now();
        std::thread th([&] {
            const auto a = clk::now();
            str = orbx_extract(exr, R[k].data(), rows, cols, (size_t)cols, kr.data(), dr.data(), cap, &nr);
            tr = ms_since(a);
        });
        const int stl = orbx_extract(exl, L[k].data(), rows, cols, (size_t)cols, kl.data(), dl.data(), cap, &nl);
        const double tl = ms_since(t0);
        th.join();
        const auto t1 = clk::now();
        const int sts = orbx_compute_stereo_matches(m, exl, exr, kl.data(), dl.data(), nl, kr.data(), dr.data(), nr, bf,
                                                    bf / fx, ur.data(), depth.data(), &ns);
        const double tsm = ms_since(t1), tf = ms_since(t0);
        if (stl || str || sts) { ++bad; std::fprintf(stderr, "frame %d: %s\n", f, orbx_last_error()); }
        if (f < 0) { warm_max = std::max(warm_max, tf); continue; }
        t_frame.push_back(tf); t_left.push_back(tl); t_right.push_back(tr); t_stereo.push_back(tsm);
    }
    // the same frames through orbx_extract_pair from this one thread (both extractions enqueued before either is waited
    // for), when the library has it
    std::string pair = "null";
    if (auto ep = (decltype(&::orbx_extract_pair))dlsym(h, "orbx_extract_pair")) {
        std::vector<double> t_pair;
        for (int f = -10; f < frames; ++f) {
            const int k = (f + kDistinct * 4) % kDistinct;
            int nl = 0, nr = 0, ns = 0;
            const auto t0 = clk::now();
            const int st = ep(exl, exr, L[k].data(), (size_t)cols, R[k].data(), (size_t)cols, rows, cols, kl.data(), dl.data(), cap,
                              &nl, kr.data(), dr.data(), cap, &nr);
            const int sts = orbx_compute_stereo_matches(m, exl, exr, kl.data(), dl.data(), nl, kr.data(), dr.data(), nr, bf,
                                                        bf / fx, ur.data(), depth.data(), &ns);
            if (st || sts) { ++bad; std::fprintf(stderr, "pair frame %d: %s\n", f, orbx_last_error()); }
            if (f >= 0) t_pair.push_back(ms_since(t0));
        }
        const Stats P = stats(t_pair);
        char buf[256];
        std::snprintf(buf, sizeof buf, "{\"frames_per_s\": %.1f, \"frame_ms\": {\"median\": %.4f, \"p95\": %.4f, \"max\": %.4f, "
                      "\"mean\": %.4f}}", 1e3 / P.mean, P.med, P.p95, P.max, P.mean);
        pair = buf;
    }
    // ... and through orbx_stereo_frame (both extractions and the stereo search in one call), when the library has it
    std::string sframe = "null";
    if (auto sf = (decltype(&::orbx_stereo_frame))dlsym(h, "orbx_stereo_frame")) {
        std::vector<double> t_sf;
        for (int f = -10; f < frames; ++f) {
            const int k = (f + kDistinct * 4) % kDistinct;
            int nl = 0, nr = 0, ns = 0;
            const auto t0 = clk::now();
            const int st = sf(m, exl, exr, L[k].data(), (size_t)cols, R[k].data(), (size_t)cols, rows, cols, kl.data(), dl.data(),
                              cap, &nl, kr.data(), dr.data(), cap, &nr, bf, bf / fx, ur.data(), depth.data(), &ns);
            if (st) { ++bad; std::fprintf(stderr, "stereo_frame %d: %s\n", f, orbx_last_error()); }
            if (f >= 0) t_sf.push_back(ms_since(t0));
        }
        const Stats P = stats(t_sf);
        char buf[256];
        std::snprintf(buf, sizeof buf, "{\"frames_per_s\": %.1f, \"frame_ms\": {\"median\": %.4f, \"p95\": %.4f, \"max\": %.4f, "
                      "\"mean\": %.4f}}", 1e3 / P.mean, P.med, P.p95, P.max, P.mean);
        sframe = buf;
    }
    const Stats F = stats(t_frame), A = stats(t_left), B = stats(t_right), S = stats(t_stereo);
    std::vector<int> order(t_frame.size());                      // the slowest frames, for outlier attribution
    for (size_t i = 0; i < order.size(); ++i) order[i] = (int)i;
    std::sort(order.begin(), order.end(), [&](int a, int b) { return t_frame[a] > t_frame[b]; });
    std::string slow;
    for (size_t i = 0; i < std::min<size_t>(3, order.size()); ++i)
        slow += (i ? ", " : "") + std::string("[") + std::to_string(order[i]) + ", " + std::to_string(t_frame[order[i]]) + ", " +
                std::to_string(t_left[order[i]]) + ", " + std::to_string(t_right[order[i]]) + ", " + std::to_string(t_stereo[order[i]]) + "]";
    std::printf("{\"lib\": \"%s\", \"frames\": %d, \"frames_per_s\": %.1f, \"frame_ms\": {\"median\": %.4f, \"p95\": %.4f, "
                "\"max\": %.4f, \"mean\": %.4f}, \"extract_left_ms\": {\"median\": %.4f, \"p95\": %.4f}, "
                "\"extract_right_ms\": {\"median\": %.4f, \"p95\": %.4f}, \"stereo_ms\": {\"median\": %.4f, \"p95\": %.4f}, "
                "\"errors\": %d, \"slowest\": [%s], \"warmup_frames\": 10, \"warmup_ms_max\": %.4f, \"pair\": %s, "
                "\"stereo_frame\": %s}\n",
                argv[1], frames, 1e3 / F.mean, F.med, F.p95, F.max, F.mean, A.med, A.p95, B.med, B.p95, S.med, S.p95, bad, slow.c_str(), warm_max,
                pair.c_str(), sframe.c_str());
    orbx_matcher_destroy(m);
    orbx_extractor_destroy(exl);
    orbx_extractor_destroy(exr);
    return bad ? 1 : 0;
}
