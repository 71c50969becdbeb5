// =====================================================================================================
//  orb_oracle.cpp — TEST INFRASTRUCTURE ONLY (never linked into, loaded by, or called from the product).
//
//  Scalar CPU restatement of the ORB front-end and Hamming matchers of andresenwc/MultiAgent_ORB_SLAM2,
//  written from a reading of the reference (citations are file:line under the reference root).  It is
//  the parity checker for the HIP path in multiagent_orb_slam2_amd/csrc and the "port" CPU baseline
//  timed by bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
//
//  PARITY STATUS: "parity unpinned".  The reference cannot be built in this image (it needs OpenCV,
//  Eigen3 and Pangolin, CMakeLists.txt:31-40; the task forbids stand-in headers), and it ships no tests,
//  golden vectors or known-answer data for this path.  The reference's own control flow (cell grid,
//  quadtree, IC angle, rBRIEF, matcher loops) is restated line by line; the OpenCV primitives it calls
//  are pinned to one documented interpretation:
//    * resize INTER_LINEAR 8U  — OpenCV 3.2 generic fixed-point path (11-bit coefficients, no SIMD).
//    * FAST-9 (TYPE_9_16)+NMS  — OpenCV 3.2 scalar FAST_t / cornerScore<16>.
//    * GaussianBlur 7x7 s=2 8U — OpenCV 3.2 integer separable path, kernel {18,34,49,55,49,34,18}
//                                (float kernel x256 rounded), column pass (acc + 2^15) >> 16, REFLECT_101.
//    * fastAtan2               — OpenCV 3.2 scalar polynomial (degrees).
//    * cos/sin of the BRIEF angle — correctly rounded float: (float)cos((double)angle).
//    * cvRound                 — round-half-even;  no FMA contraction anywhere (-ffp-contract=off).
//    * DistributeOctTree phase-2 tie between equal-size nodes — the reference breaks it by heap address
//      (ORBextractor.cc:681-684, allocator dependent); pinned here to creation order (later created =
//      larger key), i.e. a stable sort by size.
// =====================================================================================================
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <list>
#include <map>
#include <vector>

#include "../multiagent_orb_slam2_amd/csrc/orbx_pattern.h"

namespace {

struct Kp {  // cv::KeyPoint layout (28 B)
    float x, y, size, angle, response;
    int32_t octave, class_id;
};

inline int round_even_d(double v) { return (int)std::nearbyint(v); }
inline int round_even_f(float v) { return (int)std::nearbyintf(v); }
inline int floor_i(double v) { return (int)std::floor(v); }
inline int ceil_i(double v) { return (int)std::ceil(v); }

// ---------------------------------------------------------------------------------------------------
// Extractor tables — ORBextractor::ORBextractor (src/ORBextractor.cc:410-470)
// ---------------------------------------------------------------------------------------------------
struct Tables {
    int nfeatures, nlevels, iniTh, minTh;
    double scaleFactor;  // a double member initialised from the float argument (ORBextractor.h:98)
    std::vector<float> scale, invScale, sigma2, invSigma2;
    std::vector<int> nPerLevel;
    int umax[16];
};

Tables make_tables(int nfeatures, float scaleFactorF, int nlevels, int iniTh, int minTh) {
    Tables t;
    t.nfeatures = nfeatures; t.nlevels = nlevels; t.iniTh = iniTh; t.minTh = minTh;
    t.scaleFactor = (double)scaleFactorF;
    t.scale.assign(nlevels, 1.0f); t.sigma2.assign(nlevels, 1.0f);
    for (int i = 1; i < nlevels; ++i) {                        // :419-423
        t.scale[i] = (float)((double)t.scale[i - 1] * t.scaleFactor);
        t.sigma2[i] = t.scale[i] * t.scale[i];
    }
    t.invScale.resize(nlevels); t.invSigma2.resize(nlevels);
    for (int i = 0; i < nlevels; ++i) {                        // :427-431
        t.invScale[i] = 1.0f / t.scale[i];
        t.invSigma2[i] = 1.0f / t.sigma2[i];
    }
    // features per level: geometric series (:435-446)
    float factor = (float)(1.0f / t.scaleFactor);
    float want = (float)nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nlevels));
    t.nPerLevel.assign(nlevels, 0);
    int acc = 0;
    for (int l = 0; l < nlevels - 1; ++l) {
        t.nPerLevel[l] = round_even_f(want);
        acc += t.nPerLevel[l];
        want *= factor;
    }
    t.nPerLevel[nlevels - 1] = std::max(nfeatures - acc, 0);
    // circular patch half-widths (:454-469)
    const int R = 15;
    int vmax = (int)std::floor(R * std::sqrt(2.f) / 2 + 1);
    int vmin = (int)std::ceil(R * std::sqrt(2.f) / 2);
    const double r2 = (double)R * R;
    for (int v = 0; v <= vmax; ++v) t.umax[v] = round_even_d(std::sqrt(r2 - v * v));
    for (int v = R, v0 = 0; v >= vmin; --v) {
        while (t.umax[v0] == t.umax[v0 + 1]) ++v0;
        t.umax[v] = v0;
        ++v0;
    }
    return t;
}

// ---------------------------------------------------------------------------------------------------
// Image container (row-major, arbitrary stride)
// ---------------------------------------------------------------------------------------------------
struct Img {
    int w = 0, h = 0;
    std::vector<uint8_t> px;
    uint8_t at(int y, int x) const { return px[(size_t)y * w + x]; }
    const uint8_t* row(int y) const { return px.data() + (size_t)y * w; }
};

// resize(src, dst, dsize, 0, 0, INTER_LINEAR) for 8U — ComputePyramid (:1120); OpenCV 3.2 generic
// fixed-point semantics (coefficients x 2048, vertical (a*b0 + b*b1 + 2^21) >> 22).
Img resize_linear(const Img& s, int dw, int dh) {
    Img d; d.w = dw; d.h = dh; d.px.assign((size_t)dw * dh, 0);
    const double sxs = 1.0 / ((double)dw / s.w), sys = 1.0 / ((double)dh / s.h);
    std::vector<int> xo(dw), a0(dw), a1(dw);
    int xlim = dw;
    for (int x = 0; x < dw; ++x) {
        float fx = (float)((x + 0.5) * sxs - 0.5);
        int ix = floor_i(fx);
        fx -= ix;
        if (ix < 0) { fx = 0; ix = 0; }
        if (ix + 1 >= s.w) {
            xlim = std::min(xlim, x);
            if (ix >= s.w - 1) { fx = 0; ix = s.w - 1; }
        }
        xo[x] = ix;
        a0[x] = std::min(std::max(round_even_f((1.f - fx) * 2048), -32768), 32767);
        a1[x] = std::min(std::max(round_even_f(fx * 2048), -32768), 32767);
    }
    std::vector<int> r0(dw), r1(dw);
    auto hpass = [&](int sy, std::vector<int>& out) {
        const uint8_t* S = s.row(sy);
        for (int x = 0; x < dw; ++x)
            out[x] = (x < xlim) ? (int)S[xo[x]] * a0[x] + (int)S[xo[x] + 1] * a1[x] : (int)S[xo[x]] * 2048;
    };
    for (int y = 0; y < dh; ++y) {
        float fy = (float)((y + 0.5) * sys - 0.5);
        int iy = floor_i(fy);
        fy -= iy;
        int b0 = std::min(std::max(round_even_f((1.f - fy) * 2048), -32768), 32767);
        int b1 = std::min(std::max(round_even_f(fy * 2048), -32768), 32767);
        int ya = std::min(std::max(iy, 0), s.h - 1), yb = std::min(std::max(iy + 1, 0), s.h - 1);
        hpass(ya, r0);
        hpass(yb, r1);
        uint8_t* D = d.px.data() + (size_t)y * dw;
        for (int x = 0; x < dw; ++x) {
            int v = (r0[x] * b0 + r1[x] * b1 + (1 << 21)) >> 22;
            D[x] = (uint8_t)std::min(std::max(v, 0), 255);
        }
    }
    return d;
}

std::vector<Img> build_pyramid(const Tables& t, const Img& im) {  // :1107-1132
    std::vector<Img> pyr(t.nlevels);
    pyr[0] = im;
    for (int l = 1; l < t.nlevels; ++l) {
        int w = round_even_f((float)im.w * t.invScale[l]);
        int h = round_even_f((float)im.h * t.invScale[l]);
        pyr[l] = resize_linear(pyr[l - 1], w, h);
    }
    return pyr;
}

// ---------------------------------------------------------------------------------------------------
// FAST-9/16 with 3x3 non-max suppression over one ROI (OpenCV FAST_t<16> + cornerScore<16>);
// called per grid cell at ORBextractor.cc:809-816.  Returns ROI-relative keypoints, row-major.
// ---------------------------------------------------------------------------------------------------
const int kCircle[16][2] = {{0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2}, {1, -3},
                            {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};

int corner_score16(const uint8_t* p, const int* off, int thr) {
    int d[25];
    const int v = p[0];
    for (int k = 0; k < 25; ++k) d[k] = v - p[off[k]];
    int a0 = thr;
    for (int k = 0; k < 16; k += 2) {
        int a = std::min(d[k + 1], std::min(d[k + 2], d[k + 3]));
        if (a <= a0) continue;
        for (int m = 4; m <= 8; ++m) a = std::min(a, d[k + m]);
        a0 = std::max(a0, std::min(a, d[k]));
        a0 = std::max(a0, std::min(a, d[k + 9]));
    }
    int b0 = -a0;
    for (int k = 0; k < 16; k += 2) {
        int b = std::max(std::max(d[k + 1], d[k + 2]), std::max(d[k + 3], std::max(d[k + 4], d[k + 5])));
        if (b >= b0) continue;
        for (int m = 6; m <= 8; ++m) b = std::max(b, d[k + m]);
        b0 = std::min(b0, std::max(b, d[k]));
        b0 = std::min(b0, std::max(b, d[k + 9]));
    }
    return -b0 - 1;
}

void fast_roi(const Img& L, int x0, int y0, int x1, int y1, int thr, std::vector<Kp>& out) {
    out.clear();
    const int W = x1 - x0, H = y1 - y0, step = L.w;
    if (W <= 0 || H <= 0) return;
    thr = std::min(std::max(thr, 0), 255);
    int off[25];
    for (int k = 0; k < 16; ++k) off[k] = kCircle[k][0] + kCircle[k][1] * step;
    for (int k = 16; k < 25; ++k) off[k] = off[k - 16];
    uint8_t tab[512];
    for (int i = -255; i <= 255; ++i) tab[i + 255] = (uint8_t)(i < -thr ? 1 : i > thr ? 2 : 0);
    // three rolling score rows + corner positions, like FAST_t
    std::vector<uint8_t> sbuf[3];
    std::vector<int> cpos[3];
    for (int k = 0; k < 3; ++k) { sbuf[k].assign(W, 0); cpos[k].clear(); }
    for (int i = 3; i < H - 2; ++i) {
        uint8_t* cur = sbuf[(i - 3) % 3].data();
        std::vector<int>& cp = cpos[(i - 3) % 3];
        std::memset(cur, 0, W);
        cp.clear();
        if (i < H - 3) {
            const uint8_t* rowp = L.row(y0 + i) + x0;
            for (int j = 3; j < W - 3; ++j) {
                const uint8_t* p = rowp + j;
                const int v = p[0];
                const uint8_t* tb = tab - v + 255;
                int dd = tb[p[off[0]]] | tb[p[off[8]]];
                if (!dd) continue;
                dd &= tb[p[off[2]]] | tb[p[off[10]]];
                dd &= tb[p[off[4]]] | tb[p[off[12]]];
                dd &= tb[p[off[6]]] | tb[p[off[14]]];
                if (!dd) continue;
                dd &= tb[p[off[1]]] | tb[p[off[9]]];
                dd &= tb[p[off[3]]] | tb[p[off[11]]];
                dd &= tb[p[off[5]]] | tb[p[off[13]]];
                dd &= tb[p[off[7]]] | tb[p[off[15]]];
                for (int pol = 1; pol <= 2; ++pol) {
                    if (!(dd & pol)) continue;
                    int run = 0;
                    for (int k = 0; k < 25; ++k) {
                        int x = p[off[k]];
                        bool hit = (pol == 1) ? (x < v - thr) : (x > v + thr);
                        if (hit) {
                            if (++run > 8) {
                                cp.push_back(j);
                                cur[j] = (uint8_t)corner_score16(p, off, thr);
                                break;
                            }
                        } else {
                            run = 0;
                        }
                    }
                }
            }
        }
        if (i == 3) continue;
        const uint8_t* prev = sbuf[(i - 4 + 3) % 3].data();
        const uint8_t* pprev = sbuf[(i - 5 + 3) % 3].data();
        const std::vector<int>& pcp = cpos[(i - 4 + 3) % 3];
        for (int j : pcp) {
            int s = prev[j];
            if (s > prev[j + 1] && s > prev[j - 1] && s > pprev[j - 1] && s > pprev[j] && s > pprev[j + 1] &&
                s > cur[j - 1] && s > cur[j] && s > cur[j + 1]) {
                Kp k{(float)j, (float)(i - 1), 7.f, -1.f, (float)s, 0, -1};
                out.push_back(k);
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------------
// Quadtree distribution — ORBextractor::DistributeOctTree (:539-763) + ExtractorNode::DivideNode (:481-537)
// ---------------------------------------------------------------------------------------------------
struct QNode {
    std::vector<Kp> keys;
    int x0, x1, y0, y1;  // UL.x, UR.x, UL.y, BL.y
    bool leaf = false;   // bNoMore
    long seq = 0;        // creation order (pinned tie-break for the phase-2 sort)
};

void split4(const QNode& n, QNode c[4]) {
    const int hx = (int)std::ceil((float)(n.x1 - n.x0) / 2);
    const int hy = (int)std::ceil((float)(n.y1 - n.y0) / 2);
    const int mx = n.x0 + hx, my = n.y0 + hy;
    c[0].x0 = n.x0; c[0].x1 = mx;   c[0].y0 = n.y0; c[0].y1 = my;
    c[1].x0 = mx;   c[1].x1 = n.x1; c[1].y0 = n.y0; c[1].y1 = my;
    c[2].x0 = n.x0; c[2].x1 = mx;   c[2].y0 = my;   c[2].y1 = n.y1;
    c[3].x0 = mx;   c[3].x1 = n.x1; c[3].y0 = my;   c[3].y1 = n.y1;
    for (int q = 0; q < 4; ++q) { c[q].keys.clear(); c[q].keys.reserve(n.keys.size()); c[q].leaf = false; }
    for (const Kp& k : n.keys) {
        const int q = (k.x < (float)mx ? 0 : 1) + (k.y < (float)my ? 0 : 2);
        c[q].keys.push_back(k);
    }
    for (int q = 0; q < 4; ++q)
        if (c[q].keys.size() == 1) c[q].leaf = true;
}

// Phase-2 tie study: the reference orders equal-size nodes by heap address (:681-684), i.e. an
// allocator-dependent permutation of each tie group.  tie_mode 0 is the pinned rule (creation order, later-created
// first, as the HIP path); 1 = earlier-created first; 2 = a seeded pseudo-random permutation of every tie group.
// The counters record how often a phase-2 pass splits equal-size nodes and how often its >=N break falls inside
// a run of equal sizes (only then can the keypoint SET depend on the tie order).
struct TieStats {
    long levels = 0, levels_phase2 = 0, passes_phase2 = 0, passes_with_tie_split = 0, breaks_inside_tie = 0;
};
static thread_local int g_tie_mode = 0;
static thread_local unsigned g_tie_salt = 0;
static thread_local TieStats g_tie_stats;

static unsigned tie_hash(long seq) {
    unsigned x = (unsigned)seq * 2654435761u ^ g_tie_salt;
    x ^= x >> 15; x *= 2246822519u; x ^= x >> 13; x *= 3266489917u; x ^= x >> 16;
    return x;
}

std::vector<Kp> distribute_octtree(const std::vector<Kp>& cand, int minX, int maxX, int minY, int maxY, int N) {
    // A level whose detection window is empty has no candidates; the reference would divide by zero
    // here (undefined behaviour) — both this oracle and the HIP path return no keypoints.
    if (maxX - minX <= 0 || maxY - minY <= 0 || cand.empty()) return {};
    // nIni = 0 (window more than twice as tall as wide) indexes an empty vector in the reference (UB);
    // pinned to one root node here and in the HIP path.
    const int nIni = std::max(1, (int)std::round((float)(maxX - minX) / (maxY - minY)));
    const float hX = (float)(maxX - minX) / nIni;
    std::list<QNode> nodes;
    std::vector<QNode*> roots(nIni);
    long seq = 0;
    for (int i = 0; i < nIni; ++i) {
        QNode n;
        n.x0 = (int)(hX * (float)i);
        n.x1 = (int)(hX * (float)(i + 1));
        n.y0 = 0;
        n.y1 = maxY - minY;
        n.seq = seq++;
        nodes.push_back(n);
        roots[i] = &nodes.back();
    }
    for (const Kp& k : cand) roots[(size_t)(k.x / hX)]->keys.push_back(k);
    for (auto it = nodes.begin(); it != nodes.end();) {
        if (it->keys.size() == 1) { it->leaf = true; ++it; }
        else if (it->keys.empty()) it = nodes.erase(it);
        else ++it;
    }

    // a child is pushed to the list front if non-empty; expandable children are remembered with their size
    typedef std::pair<std::pair<size_t, long>, std::list<QNode>::iterator> Expandable;
    std::vector<Expandable> expandable;
    auto emit_children = [&](QNode c[4], std::vector<Expandable>* rec) {
        int grown = 0;
        for (int q = 0; q < 4; ++q) {
            if (c[q].keys.empty()) continue;
            c[q].seq = seq++;
            nodes.push_front(c[q]);
            if (c[q].keys.size() > 1) {
                ++grown;
                if (rec) rec->push_back(Expandable({c[q].keys.size(), c[q].seq}, nodes.begin()));
            }
        }
        return grown;
    };

    bool done = false;
    bool level_phase2 = false;
    g_tie_stats.levels++;
    while (!done) {
        const int before = (int)nodes.size();
        int nToExpand = 0;
        expandable.clear();
        for (auto it = nodes.begin(); it != nodes.end();) {   // phase 1: split every expandable node
            if (it->leaf) { ++it; continue; }
            QNode c[4];
            split4(*it, c);
            nToExpand += emit_children(c, &expandable);
            it = nodes.erase(it);
        }
        if ((int)nodes.size() >= N || (int)nodes.size() == before) {
            done = true;
        } else if ((int)nodes.size() + nToExpand * 3 > N) {
            while (!done) {                                    // phase 2: largest nodes first
                const int before2 = (int)nodes.size();
                std::vector<Expandable> prev = expandable;
                expandable.clear();
                if (g_tie_mode == 0) {
                    std::sort(prev.begin(), prev.end(),
                              [](const Expandable& a, const Expandable& b) { return a.first < b.first; });
                } else {
                    std::sort(prev.begin(), prev.end(), [](const Expandable& a, const Expandable& b) {
                        if (a.first.first != b.first.first) return a.first.first < b.first.first;
                        if (g_tie_mode == 1) return a.first.second > b.first.second;
                        return tie_hash(a.first.second) < tie_hash(b.first.second);
                    });
                }
                if (!level_phase2) { level_phase2 = true; g_tie_stats.levels_phase2++; }
                g_tie_stats.passes_phase2++;
                int j_last = -1;
                for (int j = (int)prev.size() - 1; j >= 0; --j) {
                    QNode c[4];
                    split4(*prev[j].second, c);
                    emit_children(c, &expandable);
                    nodes.erase(prev[j].second);
                    j_last = j;
                    if ((int)nodes.size() >= N) break;
                }
                bool tie_split = false;
                for (int j = (int)prev.size() - 1; j > j_last && j > 0; --j)
                    if (prev[j].first.first == prev[j - 1].first.first && j - 1 >= j_last) tie_split = true;
                if (tie_split) g_tie_stats.passes_with_tie_split++;
                if (j_last > 0 && prev[j_last].first.first == prev[j_last - 1].first.first) g_tie_stats.breaks_inside_tie++;
                if ((int)nodes.size() >= N || (int)nodes.size() == before2) done = true;
            }
        }
    }

    std::vector<Kp> best;
    best.reserve(nodes.size());
    for (const QNode& n : nodes) {                             // :742-760 first max response per node
        const Kp* b = &n.keys[0];
        for (size_t k = 1; k < n.keys.size(); ++k)
            if (n.keys[k].response > b->response) b = &n.keys[k];
        best.push_back(*b);
    }
    return best;
}

// ---------------------------------------------------------------------------------------------------
// Orientation — IC_Angle (:77-104) + OpenCV fastAtan2 (degrees)
// ---------------------------------------------------------------------------------------------------
float fast_atan2_deg(float y, float x) {
    const float k = (float)(180 / M_PI);
    const float p1 = 0.9997878412794807f * k, p3 = -0.3258083974640975f * k;
    const float p5 = 0.1555786518463281f * k, p7 = -0.04432655554792128f * k;
    const float eps = (float)2.2204460492503131e-016;
    float ax = std::fabs(x), ay = std::fabs(y), a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + eps);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + eps);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

float ic_angle(const Img& L, float px, float py, const int* umax) {
    const int cx = round_even_f(px), cy = round_even_f(py);
    int m01 = 0, m10 = 0;
    for (int u = -15; u <= 15; ++u) m10 += u * L.at(cy, cx + u);
    for (int v = 1; v <= 15; ++v) {
        int vs = 0;
        const int d = umax[v];
        for (int u = -d; u <= d; ++u) {
            int hi = L.at(cy + v, cx + u), lo = L.at(cy - v, cx + u);
            vs += hi - lo;
            m10 += u * (hi + lo);
        }
        m01 += v * vs;
    }
    return fast_atan2_deg((float)m01, (float)m10);
}

// ---------------------------------------------------------------------------------------------------
// GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101) on the level clone (:1085-1086), integer path.
// ---------------------------------------------------------------------------------------------------
void gauss_taps(int taps[7]) {
    float k[7];
    double s = 0;
    for (int i = 0; i < 7; ++i) {
        double x = i - 3.0;
        k[i] = (float)std::exp(-0.5 / (2.0 * 2.0) * x * x);
        s += k[i];
    }
    s = 1. / s;
    for (int i = 0; i < 7; ++i) {
        k[i] = (float)(k[i] * s);
        taps[i] = round_even_d((double)k[i] * 256.0);
    }
}

inline int reflect101(int i, int n) {
    if (n == 1) return 0;
    while (i < 0 || i >= n) i = (i < 0) ? -i : 2 * n - 2 - i;
    return i;
}

Img blur7(const Img& s) {
    int taps[7];
    gauss_taps(taps);
    Img d; d.w = s.w; d.h = s.h; d.px.assign(s.px.size(), 0);
    std::vector<int> rowsum((size_t)s.w * s.h);
    for (int y = 0; y < s.h; ++y)
        for (int x = 0; x < s.w; ++x) {
            int acc = 0;
            for (int k = -3; k <= 3; ++k) acc += taps[k + 3] * s.at(y, reflect101(x + k, s.w));
            rowsum[(size_t)y * s.w + x] = acc;
        }
    for (int y = 0; y < s.h; ++y)
        for (int x = 0; x < s.w; ++x) {
            int acc = 0;
            for (int k = -3; k <= 3; ++k) acc += taps[k + 3] * rowsum[(size_t)reflect101(y + k, s.h) * s.w + x];
            int v = (acc + (1 << 15)) >> 16;
            d.px[(size_t)y * s.w + x] = (uint8_t)std::min(std::max(v, 0), 255);
        }
    return d;
}

// ---------------------------------------------------------------------------------------------------
// Steered BRIEF — computeOrbDescriptor (:108-147)
// ---------------------------------------------------------------------------------------------------
void rbrief(const Img& B, const Kp& k, uint8_t* desc) {
    const float toRad = (float)(M_PI / 180.f);
    const float ang = k.angle * toRad;
    const float a = (float)std::cos((double)ang), b = (float)std::sin((double)ang);
    const int cx = round_even_f(k.x), cy = round_even_f(k.y);
    const uint8_t* c = B.px.data() + (size_t)cy * B.w + cx;
    const int step = B.w;
    auto sample = [&](int px, int py) {
        const float fx = (float)px, fy = (float)py;
        float ry = fx * b;  ry = ry + fy * a;
        float rx = fx * a;  rx = rx - fy * b;
        return (int)c[round_even_f(ry) * step + round_even_f(rx)];
    };
    for (int i = 0; i < 32; ++i) {
        int byte = 0;
        for (int bit = 0; bit < 8; ++bit) {
            const signed char* p = ORBX_PATTERN + (i * 8 + bit) * 4;
            byte |= (sample(p[0], p[1]) < sample(p[2], p[3])) << bit;
        }
        desc[i] = (uint8_t)byte;
    }
}

// ---------------------------------------------------------------------------------------------------
// ORBextractor::operator() (:1043-1105) + ComputeKeyPointsOctTree (:765-853)
// ---------------------------------------------------------------------------------------------------
struct Extraction {
    std::vector<Kp> kps;
    std::vector<uint8_t> desc;
    std::vector<Img> pyr;
    std::vector<int> ncand;  // FAST candidates per level (diagnostic)
};

Extraction extract(const Tables& t, const Img& im) {
    Extraction ex;
    if (im.w == 0 || im.h == 0) return ex;
    ex.pyr = build_pyramid(t, im);
    const int EDGE = 19;
    const float Wc = 30;
    std::vector<std::vector<Kp>> perLevel(t.nlevels);
    ex.ncand.assign(t.nlevels, 0);
    std::vector<Kp> cell;
    for (int l = 0; l < t.nlevels; ++l) {
        const Img& L = ex.pyr[l];
        const int minBX = EDGE - 3, minBY = minBX, maxBX = L.w - EDGE + 3, maxBY = L.h - EDGE + 3;
        const float width = (float)(maxBX - minBX), height = (float)(maxBY - minBY);
        const int nCols = (int)(width / Wc), nRows = (int)(height / Wc);
        const int wCell = nCols > 0 ? (int)std::ceil(width / nCols) : 0;
        const int hCell = nRows > 0 ? (int)std::ceil(height / nRows) : 0;
        std::vector<Kp> cand;
        for (int i = 0; i < nRows; ++i) {
            const float iniY = (float)(minBY + i * hCell);
            float maxY = iniY + hCell + 6;
            if (iniY >= maxBY - 3) continue;
            if (maxY > maxBY) maxY = (float)maxBY;
            for (int j = 0; j < nCols; ++j) {
                const float iniX = (float)(minBX + j * wCell);
                float maxX = iniX + wCell + 6;
                if (iniX >= maxBX - 6) continue;
                if (maxX > maxBX) maxX = (float)maxBX;
                fast_roi(L, (int)iniX, (int)iniY, (int)maxX, (int)maxY, t.iniTh, cell);
                if (cell.empty()) fast_roi(L, (int)iniX, (int)iniY, (int)maxX, (int)maxY, t.minTh, cell);
                for (Kp k : cell) {
                    k.x += j * wCell;
                    k.y += i * hCell;
                    cand.push_back(k);
                }
            }
        }
        ex.ncand[l] = (int)cand.size();
        std::vector<Kp> kps = distribute_octtree(cand, minBX, maxBX, minBY, maxBY, t.nPerLevel[l]);
        const int patch = (int)(31 * t.scale[l]);
        for (Kp& k : kps) {
            k.x += minBX;
            k.y += minBY;
            k.octave = l;
            k.size = (float)patch;
        }
        for (Kp& k : kps) k.angle = ic_angle(L, k.x, k.y, t.umax);
        perLevel[l] = kps;
    }
    size_t total = 0;
    for (auto& v : perLevel) total += v.size();
    ex.desc.assign(total * 32, 0);
    ex.kps.reserve(total);
    size_t row = 0;
    for (int l = 0; l < t.nlevels; ++l) {
        if (perLevel[l].empty()) continue;
        Img B = blur7(ex.pyr[l]);
        for (Kp& k : perLevel[l]) {
            rbrief(B, k, ex.desc.data() + row * 32);
            ++row;
        }
        if (l != 0) {
            const float s = t.scale[l];
            for (Kp& k : perLevel[l]) { k.x = k.x * s; k.y = k.y * s; }
        }
        ex.kps.insert(ex.kps.end(), perLevel[l].begin(), perLevel[l].end());
    }
    return ex;
}

// ---------------------------------------------------------------------------------------------------
// Matchers
// ---------------------------------------------------------------------------------------------------
int hamming(const uint8_t* a, const uint8_t* b) {   // ORBmatcher::DescriptorDistance (ORBmatcher.cc:1649-1665)
    int d = 0;
    for (int i = 0; i < 8; ++i) {
        uint32_t x, y;
        std::memcpy(&x, a + 4 * i, 4);
        std::memcpy(&y, b + 4 * i, 4);
        uint32_t v = x ^ y;
        v = v - ((v >> 1) & 0x55555555u);
        v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
        d += (int)((((v + (v >> 4)) & 0x0F0F0F0Fu) * 0x01010101u) >> 24);
    }
    return d;
}

// ORBmatcher::ComputeThreeMaxima (ORBmatcher.cc:1603-1644)
void three_maxima(const int* h, int L, int& i1, int& i2, int& i3) {
    int m1 = 0, m2 = 0, m3 = 0;
    i1 = i2 = i3 = -1;
    for (int i = 0; i < L; ++i) {
        const int s = h[i];
        if (s > m1) { m3 = m2; m2 = m1; m1 = s; i3 = i2; i2 = i1; i1 = i; }
        else if (s > m2) { m3 = m2; m2 = s; i3 = i2; i2 = i; }
        else if (s > m3) { m3 = s; i3 = i; }
    }
    if (m2 < 0.1f * (float)m1) { i2 = -1; i3 = -1; }
    else if (m3 < 0.1f * (float)m1) { i3 = -1; }
}

int rot_bin(float a1, float a2) {   // ORBmatcher.cc:609-614 (factor = 1/HISTO_LENGTH)
    float rot = a1 - a2;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)std::round(rot * (1.0f / 30));
    if (bin == 30) bin = 0;
    return bin;
}

// Apply the rotation-consistency filter given per-query bins; drops matches outside the 3 top bins.
int rot_filter(std::vector<int>& match, const std::vector<int>& bin, int nmatches) {
    std::vector<int> hist(30, 0);
    for (size_t i = 0; i < match.size(); ++i)
        if (match[i] >= 0) hist[bin[i]]++;
    int a, b, c;
    three_maxima(hist.data(), 30, a, b, c);
    for (size_t i = 0; i < match.size(); ++i) {
        if (match[i] < 0) continue;
        const int k = bin[i];
        if (k == a || k == b || k == c) continue;
        match[i] = -1;
        --nmatches;
    }
    return nmatches;
}

}  // namespace

// =====================================================================================================
// C ABI for the test harness (ctypes)
// =====================================================================================================
extern "C" {

struct orc_kp { float x, y, size, angle, response; int32_t octave, class_id; };

int orc_tables(int nfeatures, float scaleFactor, int nlevels, int iniTh, int minTh, float* scale,
               float* invScale, float* sigma2, float* invSigma2, int* nPerLevel, int* umax) {
    Tables t = make_tables(nfeatures, scaleFactor, nlevels, iniTh, minTh);
    for (int l = 0; l < nlevels; ++l) {
        scale[l] = t.scale[l]; invScale[l] = t.invScale[l];
        sigma2[l] = t.sigma2[l]; invSigma2[l] = t.invSigma2[l];
        nPerLevel[l] = t.nPerLevel[l];
    }
    for (int v = 0; v < 16; ++v) umax[v] = t.umax[v];
    return 0;
}

// Full extraction.  kps/desc capacity 'cap'; returns count (or -needed if cap too small).
// pyr_out (optional): concatenated unpadded levels; ncand (optional): FAST candidates per level.
int orc_extract(int nfeatures, float scaleFactor, int nlevels, int iniTh, int minTh, const uint8_t* img,
                int rows, int cols, int step, orc_kp* kps, uint8_t* desc, int cap, uint8_t* pyr_out,
                int* ncand) {
    Tables t = make_tables(nfeatures, scaleFactor, nlevels, iniTh, minTh);
    Img im;
    im.w = cols; im.h = rows; im.px.resize((size_t)rows * cols);
    for (int y = 0; y < rows; ++y) std::memcpy(im.px.data() + (size_t)y * cols, img + (size_t)y * step, cols);
    Extraction ex = extract(t, im);
    if (pyr_out) {
        size_t o = 0;
        for (auto& L : ex.pyr) { std::memcpy(pyr_out + o, L.px.data(), L.px.size()); o += L.px.size(); }
    }
    if (ncand) for (int l = 0; l < nlevels; ++l) ncand[l] = ex.ncand.empty() ? 0 : ex.ncand[l];
    const int n = (int)ex.kps.size();
    if (n > cap) return -n;
    std::memcpy(kps, ex.kps.data(), sizeof(Kp) * n);
    std::memcpy(desc, ex.desc.data(), (size_t)n * 32);
    return n;
}


// Per-level FAST candidates in reference order (input of DistributeOctTree), window-relative coords.
// Returns the total count (or -needed); per_level[l] = candidates of level l.
int orc_level_candidates(int nfeatures, float scaleFactor, int nlevels, int iniTh, int minTh, const uint8_t* img,
                         int rows, int cols, float* xyr, int cap, int* per_level) {
    Tables t = make_tables(nfeatures, scaleFactor, nlevels, iniTh, minTh);
    Img im;
    im.w = cols; im.h = rows; im.px.assign(img, img + (size_t)rows * cols);
    std::vector<Img> pyr = build_pyramid(t, im);
    std::vector<Kp> cell, all;
    for (int l = 0; l < nlevels; ++l) {
        const Img& L = pyr[l];
        const int minBX = 16, minBY = 16, maxBX = L.w - 16, maxBY = L.h - 16;
        const float width = (float)(maxBX - minBX), height = (float)(maxBY - minBY);
        const int nCols = (int)(width / 30), nRows = (int)(height / 30);
        const int wCell = nCols > 0 ? (int)std::ceil(width / nCols) : 0;
        const int hCell = nRows > 0 ? (int)std::ceil(height / nRows) : 0;
        int before = (int)all.size();
        for (int i = 0; i < nRows; ++i) {
            const float iniY = (float)(minBY + i * hCell);
            float maxY = iniY + hCell + 6;
            if (iniY >= maxBY - 3) continue;
            if (maxY > maxBY) maxY = (float)maxBY;
            for (int j = 0; j < nCols; ++j) {
                const float iniX = (float)(minBX + j * wCell);
                float maxX = iniX + wCell + 6;
                if (iniX >= maxBX - 6) continue;
                if (maxX > maxBX) maxX = (float)maxBX;
                fast_roi(L, (int)iniX, (int)iniY, (int)maxX, (int)maxY, t.iniTh, cell);
                if (cell.empty()) fast_roi(L, (int)iniX, (int)iniY, (int)maxX, (int)maxY, t.minTh, cell);
                for (Kp k : cell) { k.x += j * wCell; k.y += i * hCell; k.octave = l; all.push_back(k); }
            }
        }
        per_level[l] = (int)all.size() - before;
    }
    const int n = (int)all.size();
    if (n > cap) return -n;
    for (int i = 0; i < n; ++i) { xyr[3 * i] = all[i].x; xyr[3 * i + 1] = all[i].y; xyr[3 * i + 2] = all[i].response; }
    return n;
}

// DistributeOctTree on given window-relative candidates (x, y, response) — returns kept count and the
// kept keys (x, y, response) in list order.
// Tie-rule study hooks (test infrastructure): set the phase-2 tie mode of this thread, read / reset its counters.
void orc_set_tie_mode(int mode, unsigned salt) { g_tie_mode = mode; g_tie_salt = salt; }
void orc_tie_stats(long* out5) {
    out5[0] = g_tie_stats.levels; out5[1] = g_tie_stats.levels_phase2; out5[2] = g_tie_stats.passes_phase2;
    out5[3] = g_tie_stats.passes_with_tie_split; out5[4] = g_tie_stats.breaks_inside_tie;
    g_tie_stats = TieStats();
}

int orc_distribute(const float* xyr, int n, int minX, int maxX, int minY, int maxY, int N, float* out, int cap) {
    std::vector<Kp> cand(n);
    for (int i = 0; i < n; ++i) cand[i] = Kp{xyr[3 * i], xyr[3 * i + 1], 7.f, -1.f, xyr[3 * i + 2], 0, -1};
    std::vector<Kp> r = distribute_octtree(cand, minX, maxX, minY, maxY, N);
    const int m = (int)r.size();
    if (m > cap) return -m;
    for (int i = 0; i < m; ++i) { out[3 * i] = r[i].x; out[3 * i + 1] = r[i].y; out[3 * i + 2] = r[i].response; }
    return m;
}

int orc_resize(const uint8_t* src, int sw, int sh, uint8_t* dst, int dw, int dh) {
    Img s; s.w = sw; s.h = sh; s.px.assign(src, src + (size_t)sw * sh);
    Img d = resize_linear(s, dw, dh);
    std::memcpy(dst, d.px.data(), d.px.size());
    return 0;
}

int orc_blur7(const uint8_t* src, int w, int h, uint8_t* dst) {
    Img s; s.w = w; s.h = h; s.px.assign(src, src + (size_t)w * h);
    Img d = blur7(s);
    std::memcpy(dst, d.px.data(), d.px.size());
    return 0;
}

float orc_fast_atan2(float y, float x) { return fast_atan2_deg(y, x); }

int orc_descriptor_distance(const uint8_t* a, const uint8_t* b) { return hamming(a, b); }

// MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:246-311) per MapPoint p over its observed descriptors
// desc[offsets[p] .. offsets[p+1]): float distance table, each row copied into a vector<int>, sorted, element
// 0.5*(N-1) (converted to size_t) as the median; the first row with a strictly smaller median wins.  best[p] = -1
// when p has no descriptors (the reference returns early).
void orc_distinctive(const uint8_t* desc, const int32_t* offsets, int M, int32_t* best) {
    for (int p = 0; p < M; ++p) {
        const size_t N = (size_t)(offsets[p + 1] - offsets[p]);
        const uint8_t* d = desc + 32 * (size_t)offsets[p];
        if (N == 0) { best[p] = -1; continue; }
        std::vector<float> D(N * N);
        for (size_t i = 0; i < N; i++) {
            D[i * N + i] = 0;
            for (size_t j = i + 1; j < N; j++) {
                const int dij = hamming(d + 32 * i, d + 32 * j);
                D[i * N + j] = (float)dij;
                D[j * N + i] = (float)dij;
            }
        }
        int bestMedian = INT_MAX, bestIdx = 0;
        for (size_t i = 0; i < N; i++) {
            std::vector<int> v(D.begin() + i * N, D.begin() + (i + 1) * N);
            std::sort(v.begin(), v.end());
            const int median = v[(size_t)(0.5 * (double)(N - 1))];
            if (median < bestMedian) { bestMedian = median; bestIdx = (int)i; }
        }
        best[p] = bestIdx;
    }
}

// Brute force: per query, min distance, lowest index achieving it, second smallest distance (multiset),
// with the reference's "init 256, strict <" update rule (ORBmatcher.cc:568-598).
int orc_bf_match(const uint8_t* q, int nq, const uint8_t* t, int nt, int32_t* best_idx, int32_t* best,
                 int32_t* second) {
    for (int i = 0; i < nq; ++i) {
        int b1 = 256, b2 = 256, bi = -1;
        for (int j = 0; j < nt; ++j) {
            const int d = hamming(q + 32 * (size_t)i, t + 32 * (size_t)j);
            if (d < b1) { b2 = b1; b1 = d; bi = j; }
            else if (d < b2) { b2 = d; }
        }
        best_idx[i] = bi; best[i] = b1; second[i] = b2;
    }
    return 0;
}

// Frame::ComputeStereoMatches descriptor part (src/Frame.cc:466-552): per left keypoint the right
// index with the smallest distance (init TH_HIGH=100, strict <, candidates in ascending right index
// within row (int)vL's band, octave within +-1, uR in [uL - bf/b, uL]); accepted when < 75.
int orc_stereo_match(const orc_kp* kl, const uint8_t* dl, int nl, const orc_kp* kr, const uint8_t* dr, int nr,
                     const float* scale, int rows, float bf, float b, int32_t* best_idx, int32_t* best_dist) {
    std::vector<std::vector<int>> rowIdx(rows);
    for (int r = 0; r < nr; ++r) {
        const float rad = 2.0f * scale[kr[r].octave];
        const int maxr = (int)std::ceil(kr[r].y + rad), minr = (int)std::floor(kr[r].y - rad);
        for (int y = minr; y <= maxr; ++y)
            if (y >= 0 && y < rows) rowIdx[y].push_back(r);
    }
    const float minZ = b, minD = 0, maxD = bf / minZ;
    int n = 0;
    for (int l = 0; l < nl; ++l) {
        best_idx[l] = -1; best_dist[l] = 100;
        const int lev = kl[l].octave;
        const float vL = kl[l].y, uL = kl[l].x;
        const int vrow = (int)vL;
        if (vrow < 0 || vrow >= rows) continue;
        const std::vector<int>& cand = rowIdx[vrow];
        if (cand.empty()) continue;
        const float minU = uL - maxD, maxU = uL - minD;
        if (maxU < 0) continue;
        int bd = 100, bi = -1;
        for (int r : cand) {
            if (kr[r].octave < lev - 1 || kr[r].octave > lev + 1) continue;
            const float uR = kr[r].x;
            if (uR >= minU && uR <= maxU) {
                const int d = hamming(dl + 32 * (size_t)l, dr + 32 * (size_t)r);
                if (d < bd) { bd = d; bi = r; }
            }
        }
        best_dist[l] = bd;
        best_idx[l] = (bd < 75) ? bi : -1;
        if (bd < 75) ++n;
    }
    return n;
}

// Frame::ComputeStereoMatches sub-pixel part (src/Frame.cc:554-639), after the descriptor search above:
// for each left keypoint with an accepted right match, an 11x11 SAD window (centre-subtracted, exact
// integer arithmetic as the float Mats hold small integers) slid over +-5 px on the left keypoint's
// pyramid level, parabola fit, disparity check, then the median-distance outlier rejection.  Level l of
// the left/right pyramids: lvl*[l] with row step step*[l] and size rows*[l] x cols*[l].  Bounds of the left
// window and of the right window's low side are not checked by the reference (cv::Mat::colRange would
// assert); extractor keypoints never reach them, here such keypoints get no depth.  An empty accepted set
// skips the median step (the reference indexes vDistIdx[0] of an empty vector).
int orc_stereo_refine(const orc_kp* kl, int nl, const orc_kp* kr, const int32_t* best_idx, const float* scale,
                      const float* inv_scale, const uint8_t* const* lvlL, const int* stepL, const int* rowsL,
                      const int* colsL, const uint8_t* const* lvlR, const int* stepR, const int* rowsR, const int* colsR,
                      float bf, float b, float* uright, float* depth, int32_t* sad) {
    const float minZ = b, minD = 0, maxD = bf / minZ;
    std::vector<std::pair<int, int>> distIdx;
    for (int l = 0; l < nl; ++l) {
        uright[l] = -1.0f; depth[l] = -1.0f; sad[l] = -1;
        if (best_idx[l] < 0) continue;
        const int oct = kl[l].octave;
        const float uL = kl[l].x;
        const float uR0 = kr[best_idx[l]].x;
        const float sf = inv_scale[oct];
        const float suL = std::round(kl[l].x * sf), svL = std::round(kl[l].y * sf), suR0 = std::round(uR0 * sf);
        const int w = 5, L = 5;
        const int iuL = (int)suL, ivL = (int)svL, iuR0 = (int)suR0;
        if (ivL - w < 0 || ivL + w >= rowsL[oct] || iuL - w < 0 || iuL + w >= colsL[oct] || ivL + w >= rowsR[oct] ||
            iuR0 - L - w < 0)
            continue;
        const float iniu = suR0 + L - w, endu = suR0 + L + w + 1;
        if (iniu < 0 || endu >= colsR[oct]) continue;
        const uint8_t* IL = lvlL[oct] + (size_t)(ivL - w) * stepL[oct] + (iuL - w);
        const int cL = IL[(size_t)w * stepL[oct] + w];
        int bestDist = 0x7fffffff, bestInc = 0;
        int dists[11];
        for (int inc = -L; inc <= L; ++inc) {
            const uint8_t* IR = lvlR[oct] + (size_t)(ivL - w) * stepR[oct] + (iuR0 + inc - w);
            const int cR = IR[(size_t)w * stepR[oct] + w];
            int d = 0;
            for (int y = 0; y < 2 * w + 1; ++y)
                for (int x = 0; x < 2 * w + 1; ++x)
                    d += std::abs((IL[(size_t)y * stepL[oct] + x] - cL) - (IR[(size_t)y * stepR[oct] + x] - cR));
            if ((float)d < (float)bestDist) { bestDist = d; bestInc = inc; }
            dists[L + inc] = d;
        }
        if (bestInc == -L || bestInc == L) continue;
        const float d1 = (float)dists[L + bestInc - 1], d2 = (float)dists[L + bestInc], d3 = (float)dists[L + bestInc + 1];
        const float deltaR = (d1 - d3) / (2.0f * (d1 + d3 - 2.0f * d2));
        if (deltaR < -1 || deltaR > 1) continue;
        float bestuR = scale[oct] * ((float)suR0 + (float)bestInc + deltaR);
        float disparity = uL - bestuR;
        if (disparity >= minD && disparity < maxD) {
            if (disparity <= 0) {
                disparity = 0.01;
                bestuR = uL - 0.01;
            }
            depth[l] = bf / disparity;
            uright[l] = bestuR;
            sad[l] = bestDist;
            distIdx.push_back({bestDist, l});
        }
    }
    if (distIdx.empty()) return 0;
    std::sort(distIdx.begin(), distIdx.end());
    const float median = distIdx[distIdx.size() / 2].first;
    const float thDist = 1.5f * 1.4f * median;
    int n = (int)distIdx.size();
    for (int i = (int)distIdx.size() - 1; i >= 0; --i) {
        if (distIdx[i].first < thDist) break;
        uright[distIdx[i].second] = -1;
        depth[distIdx[i].second] = -1;
        --n;
    }
    return n;
}

// FeatureVector as CSR: node ids ascending, offsets[n_nodes+1], feature indices.
struct orc_fv { const uint32_t* node; const int32_t* off; int n_nodes; const int32_t* idx; };

// ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*, ...) (ORBmatcher.cc:524-657).  valid1/valid2 = the
// keypoint has a non-bad MapPoint.  match12[i] = index in KF2 or -1.  Returns nmatches.
int orc_search_by_bow_kfkf(const uint8_t* d1, const float* ang1, const uint8_t* valid1, int n1, orc_fv f1,
                           const uint8_t* d2, const float* ang2, const uint8_t* valid2, int n2, orc_fv f2,
                           float nnratio, int checkOri, int32_t* match12) {
    std::vector<int> m(n1, -1), bins(n1, 0);
    std::vector<char> taken(n2, 0);
    int nm = 0;
    int a = 0, b = 0;
    while (a < f1.n_nodes && b < f2.n_nodes) {
        if (f1.node[a] == f2.node[b]) {
            for (int p = f1.off[a]; p < f1.off[a + 1]; ++p) {
                const int i1 = f1.idx[p];
                if (!valid1[i1]) continue;
                int b1 = 256, b2 = 256, bi = -1;
                for (int q = f2.off[b]; q < f2.off[b + 1]; ++q) {
                    const int i2 = f2.idx[q];
                    if (taken[i2] || !valid2[i2]) continue;
                    const int d = hamming(d1 + 32 * (size_t)i1, d2 + 32 * (size_t)i2);
                    if (d < b1) { b2 = b1; b1 = d; bi = i2; }
                    else if (d < b2) b2 = d;
                }
                if (b1 < 50 && (float)b1 < nnratio * (float)b2) {
                    m[i1] = bi;
                    taken[bi] = 1;
                    if (checkOri) bins[i1] = rot_bin(ang1[i1], ang2[bi]);
                    ++nm;
                }
            }
            ++a; ++b;
        } else if (f1.node[a] < f2.node[b]) {
            while (a < f1.n_nodes && f1.node[a] < f2.node[b]) ++a;   // lower_bound
        } else {
            while (b < f2.n_nodes && f2.node[b] < f1.node[a]) ++b;
        }
    }
    if (checkOri) nm = rot_filter(m, bins, nm);
    std::memcpy(match12, m.data(), sizeof(int) * n1);
    return nm;
}

// ORBmatcher::SearchByBoW(KeyFrame*, Frame&, ...) (ORBmatcher.cc:161-290).  validKF = KF keypoint has
// a non-bad MapPoint.  matchF[iF] = KF index assigned to frame keypoint iF, or -1.
int orc_search_by_bow_kff(const uint8_t* dk, const float* angk, const uint8_t* validk, int /*nk*/, orc_fv fk,
                          const uint8_t* df, const float* angf, int nf, orc_fv ff, float nnratio, int checkOri,
                          int32_t* matchF) {
    std::vector<int> m(nf, -1), bins(nf, 0);
    int nm = 0, a = 0, b = 0;
    while (a < fk.n_nodes && b < ff.n_nodes) {
        if (fk.node[a] == ff.node[b]) {
            for (int p = fk.off[a]; p < fk.off[a + 1]; ++p) {
                const int ik = fk.idx[p];
                if (!validk[ik]) continue;
                int b1 = 256, b2 = 256, bi = -1;
                for (int q = ff.off[b]; q < ff.off[b + 1]; ++q) {
                    const int jf = ff.idx[q];
                    if (m[jf] >= 0) continue;
                    const int d = hamming(dk + 32 * (size_t)ik, df + 32 * (size_t)jf);
                    if (d < b1) { b2 = b1; b1 = d; bi = jf; }
                    else if (d < b2) b2 = d;
                }
                if (b1 <= 50 && (float)b1 < nnratio * (float)b2) {
                    m[bi] = ik;
                    if (checkOri) bins[bi] = rot_bin(angk[ik], angf[bi]);
                    ++nm;
                }
            }
            ++a; ++b;
        } else if (fk.node[a] < ff.node[b]) {
            while (a < fk.n_nodes && fk.node[a] < ff.node[b]) ++a;
        } else {
            while (b < ff.n_nodes && ff.node[b] < fk.node[a]) ++b;
        }
    }
    if (checkOri) nm = rot_filter(m, bins, nm);
    std::memcpy(matchF, m.data(), sizeof(int) * nf);
    return nm;
}

// ORBmatcher::SearchForTriangulation (ORBmatcher.cc:659-825) + CheckDistEpipolarLine (:142-159).
// has_mp: keypoint already has a MapPoint (skipped); uright >= 0 marks stereo keypoints.
// F12 row-major 3x3 float; sigma2/scale2 = KF2 level tables; (ex, ey) = epipole in KF2.
int orc_search_for_triangulation(const uint8_t* d1, const orc_kp* k1, const uint8_t* has_mp1, const float* uright1,
                                 int n1, orc_fv f1, const uint8_t* d2, const orc_kp* k2, const uint8_t* has_mp2,
                                 const float* uright2, int n2, orc_fv f2, const float* F12, const float* sigma2,
                                 const float* scale2, float ex, float ey, int onlyStereo, int checkOri,
                                 int32_t* match12) {
    (void)n2;
    std::vector<int> m(n1, -1), bins(n1, 0);
    int nm = 0, a = 0, b = 0;
    auto F = [&](int r, int c) { return F12[r * 3 + c]; };
    while (a < f1.n_nodes && b < f2.n_nodes) {
        if (f1.node[a] == f2.node[b]) {
            for (int p = f1.off[a]; p < f1.off[a + 1]; ++p) {
                const int i1 = f1.idx[p];
                if (has_mp1[i1]) continue;
                const bool st1 = uright1[i1] >= 0;
                if (onlyStereo && !st1) continue;
                const orc_kp& kp1 = k1[i1];
                int bd = 50, bi = -1;
                for (int q = f2.off[b]; q < f2.off[b + 1]; ++q) {
                    const int i2 = f2.idx[q];
                    if (has_mp2[i2]) continue;   // vbMatched2 is never set by the reference (:679,727)
                    const bool st2 = uright2[i2] >= 0;
                    if (onlyStereo && !st2) continue;
                    const int d = hamming(d1 + 32 * (size_t)i1, d2 + 32 * (size_t)i2);
                    if (d > 50 || d > bd) continue;
                    const orc_kp& kp2 = k2[i2];
                    if (!st1 && !st2) {
                        const float dx = ex - kp2.x, dy = ey - kp2.y;
                        if (dx * dx + dy * dy < 100 * scale2[kp2.octave]) continue;
                    }
                    const float la = kp1.x * F(0, 0) + kp1.y * F(1, 0) + F(2, 0);
                    const float lb = kp1.x * F(0, 1) + kp1.y * F(1, 1) + F(2, 1);
                    const float lc = kp1.x * F(0, 2) + kp1.y * F(1, 2) + F(2, 2);
                    const float num = la * kp2.x + lb * kp2.y + lc;
                    const float den = la * la + lb * lb;
                    if (den == 0) continue;
                    const float dsqr = num * num / den;
                    if (dsqr < 3.84 * sigma2[kp2.octave]) { bi = i2; bd = d; }
                }
                if (bi >= 0) {
                    m[i1] = bi;
                    ++nm;
                    if (checkOri) bins[i1] = rot_bin(kp1.angle, k2[bi].angle);
                }
            }
            ++a; ++b;
        } else if (f1.node[a] < f2.node[b]) {
            while (a < f1.n_nodes && f1.node[a] < f2.node[b]) ++a;
        } else {
            while (b < f2.n_nodes && f2.node[b] < f1.node[a]) ++b;
        }
    }
    if (checkOri) nm = rot_filter(m, bins, nm);
    std::memcpy(match12, m.data(), sizeof(int) * n1);
    return nm;
}

// ---------------------------------------------------------------------------------------------------
// DBoW2 TemplatedVocabulary<FORB>::transform (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1125-1187,
// :1218-1259): std::map BowVector / FeatureVector exactly as DBoW2 builds them.  Node numbering as in
// loadFromTextFile (:1338-1424): line i = node i + 1, root 0.
// ---------------------------------------------------------------------------------------------------
struct OrcVocab {
    int L, scoring, weighting;
    std::vector<std::vector<int>> children;
    std::vector<int> word;
    std::vector<double> w;
    std::vector<uint8_t> desc;   // node id - 1
};

// TemplatedVocabulary::loadFromTextFile's tree (TemplatedVocabulary.h:1338-1424), built once.
void* orc_vocab_new(int L, int scoring, int weighting, int n_lines, const int32_t* parent, const uint8_t* is_leaf,
                    const uint8_t* vdesc, const double* vweight) {
    OrcVocab* v = new OrcVocab();
    v->L = L; v->scoring = scoring; v->weighting = weighting;
    const int N = n_lines + 1;
    v->children.assign(N, {});
    v->word.assign(N, -1);
    v->w.assign(N, 0.0);
    v->desc.assign(vdesc, vdesc + 32 * (size_t)n_lines);
    int nw = 0;
    for (int i = 0; i < n_lines; ++i) {
        v->children[parent[i]].push_back(i + 1);
        v->w[i + 1] = vweight[i];
        if (is_leaf[i]) v->word[i + 1] = nw++;
    }
    return v;
}

void orc_vocab_free(void* h) { delete static_cast<OrcVocab*>(h); }

// TemplatedVocabulary::transform(features, BowVector&, FeatureVector&, levelsup) (:1125-1187, :1218-1259).
int orc_vocab_apply(void* h, const uint8_t* feats, int n, int levelsup, uint32_t* bow_words, double* bow_values, int* n_words,
                    uint32_t* fv_nodes, int32_t* fv_off, int32_t* fv_idx, int* n_fv) {
    const OrcVocab& V = *static_cast<OrcVocab*>(h);
    std::map<uint32_t, double> bow;
    std::map<uint32_t, std::vector<unsigned>> fv;
    const int nid_level = V.L - levelsup;
    for (int f = 0; f < n; ++f) {
        const uint8_t* x = feats + 32 * (size_t)f;
        unsigned nid = 0, final_id = 0;
        int level = 0;
        do {
            ++level;
            const std::vector<int>& nodes = V.children[final_id];
            final_id = nodes[0];
            double best_d = hamming(x, V.desc.data() + 32 * (size_t)(final_id - 1));
            for (size_t c = 1; c < nodes.size(); ++c) {
                const double d = hamming(x, V.desc.data() + 32 * (size_t)(nodes[c] - 1));
                if (d < best_d) { best_d = d; final_id = nodes[c]; }
            }
            if (level == nid_level) nid = final_id;
        } while (!V.children[final_id].empty());
        const double wt = V.w[final_id];
        if (wt > 0) {
            const uint32_t id = (uint32_t)V.word[final_id];
            if (V.weighting == 0 || V.weighting == 1) {   // TF_IDF, TF: addWeight
                auto it = bow.find(id);
                if (it != bow.end()) it->second += wt; else bow.emplace(id, wt);
            } else {                                      // IDF, BINARY: addIfNotExist
                bow.emplace(id, wt);
            }
            fv[nid].push_back((unsigned)f);
        }
    }
    double norm = 0.0;                                    // BowVector::normalize (L1 or L2)
    if (V.scoring == 0) { for (auto& kv : bow) norm += std::fabs(kv.second); }
    else { for (auto& kv : bow) norm += kv.second * kv.second; norm = std::sqrt(norm); }
    if (norm > 0.0) for (auto& kv : bow) kv.second /= norm;
    int i = 0;
    for (auto& kv : bow) { bow_words[i] = kv.first; bow_values[i] = kv.second; ++i; }
    *n_words = i;
    int j = 0, o = 0;
    for (auto& kv : fv) {
        fv_nodes[j] = kv.first;
        fv_off[j] = o;
        for (unsigned idx : kv.second) fv_idx[o++] = (int32_t)idx;
        ++j;
    }
    fv_off[j] = o;
    *n_fv = j;
    return 0;
}

int orc_vocab_transform(int /*k*/, int L, int scoring, int weighting, int n_lines, const int32_t* parent,
                        const uint8_t* is_leaf, const uint8_t* vdesc, const double* vweight, const uint8_t* feats, int n,
                        int levelsup, uint32_t* bow_words, double* bow_values, int* n_words, uint32_t* fv_nodes,
                        int32_t* fv_off, int32_t* fv_idx, int* n_fv) {
    void* h = orc_vocab_new(L, scoring, weighting, n_lines, parent, is_leaf, vdesc, vweight);
    const int r = orc_vocab_apply(h, feats, n, levelsup, bow_words, bow_values, n_words, fv_nodes, fv_off, fv_idx, n_fv);
    orc_vocab_free(h);
    return r;
}

}  // extern "C"
