// =====================================================================================================
// proj_oracle.cpp — TEST INFRASTRUCTURE ONLY (the checker; never on the product path).
//
// Scalar restatement of the keypoint grid and the projection / radius matchers of the reference
// (SURVEY §8f row 2), line by line in the reference's loop order, over flat arrays:
//   Frame::AssignFeaturesToGrid / PosInGrid           src/Frame.cc:230-245, :382-392
//   Frame::GetFeaturesInArea                          src/Frame.cc:327-380
//   KeyFrame::GetFeaturesInArea                       src/KeyFrame.cc:589-628
//   ORBmatcher::SearchByProjection(Frame&, vpMapPoints, th)            src/ORBmatcher.cc:45-131
//   ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono)    src/ORBmatcher.cc:1330-1472
//   ORBmatcher::SearchByProjection(Frame&, KeyFrame*, set, th, ORBdist) src/ORBmatcher.cc:1474-1601
//   ORBmatcher::SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th) src/ORBmatcher.cc:292-405
//   ORBmatcher::Fuse(KeyFrame*, vpMapPoints, th) — the search   src/ORBmatcher.cc:894-951
//   ORBmatcher::Fuse(KeyFrame*, Scw, ...) — the search          src/ORBmatcher.cc:1053-1081
//   ORBmatcher::SearchBySim3 — each direction's search          src/ORBmatcher.cc:1193-1226, 1273-1306
//   ORBmatcher::SearchForInitialization                         src/ORBmatcher.cc:407-522
// A query carries the window the reference passes to GetFeaturesInArea and the values its inner loop tests; the
// projection arithmetic that produces it (cv::Mat products, isInFrustum, PredictScale) is restated by orc_project,
// and the MapPoints of a stereo frame (UnprojectStereo + the Frame form of the MapPoint constructor) by
// orc_stereo_mappoints.
// Struct layouts are identical to orbx_grid / orbx_proj_query / orbx_proj_params (include/orbx.h).
// Compiled with -ffp-contract=off (oracle/Makefile): float expressions evaluate as written.
// =====================================================================================================
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <utility>
#include <vector>

namespace {

struct Kp { float x, y, size, angle, response; int32_t octave, class_id; };   // cv::KeyPoint (28 B)

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

void three_maxima(const int* h, int L, int& i1, int& i2, int& i3) {   // ORBmatcher.cc:1603-1644
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

int rot_bin(float a1, float a2) {   // e.g. ORBmatcher.cc:1435-1440 (factor = 1/HISTO_LENGTH)
    float rot = a1 - a2;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)std::round(rot * (1.0f / 30));
    if (bin == 30) bin = 0;
    return bin;
}

}  // namespace

extern "C" {

struct orc_grid { float min_x, min_y, max_x, max_y, inv_w, inv_h; int32_t cols, rows; };
struct orc_proj_query {
    float x, y, r;                 // GetFeaturesInArea(x, y, r, min_level, max_level)
    int32_t min_level, max_level;
    float ur, ur_tol, angle;       // stereo right coordinate + tolerance, query keypoint angle
    int32_t level, flags;
};
struct orc_proj_params {
    int32_t mode, accept_max;
    float nnratio;
    int32_t check_ori, nlevels;
    float inv_sigma2[32];
};
enum { ORC_PROJ_MAPPOINTS = 0, ORC_PROJ_LASTFRAME, ORC_PROJ_KEYFRAME, ORC_PROJ_SIM3, ORC_PROJ_FUSE, ORC_PROJ_BEST,
       ORC_PROJ_INIT };
enum { ORC_QF_SKIP = 1, ORC_QF_BLOCKS = 2 };

// The projection step before the searches (include/orbx.h orbx_proj_project): one MapPoint -> one query, in the
// reference's operation order for each caller.  float expressions evaluate as written (-ffp-contract=off); the
// cv::Mat pieces are pinned as DESIGN §2 states: Rcw * X + tcw as float products summed left to right; cv::norm and
// Mat::dot of 3-vectors as double products accumulated in double (orc_norm2); PredictScale's log in double.
struct orc_map_point {
    float x, y, z, nx, ny, nz, min_dist, max_dist, angle;
    int32_t octave, flags, pad;
};
struct orc_view {
    float R[9], t[3], Ow[3];
    float fx, fy, cx, cy, bf;
    float min_x, max_x, min_y, max_y;
    float th, view_cos_limit;
    int32_t level_mode, pad;
};

// cv::norm(3x1 CV_32F) in OpenCV 3.2's generic path: normL2_32f -> normL2Sqr<float, double>: each element widened to
// double, squared and summed left to right in double, then std::sqrt (stat.cpp).  Mat::dot likewise (dotProd_32f ->
// dotProd_<float>: (double)a[i] * b[i] summed in double; the SSE block loop does not run for 3 elements).
static double orc_norm2(float x, float y, float z) {
    double s = 0.0;
    s += (double)x * x;
    s += (double)y * y;
    s += (double)z * z;
    return s;
}

static int orc_predict_scale(float max_dist, float dist, float log_sf, int nlevels) {   // MapPoint.cc:389-421
    const float ratio = max_dist / dist;
    int n = (int)std::ceil(std::log((double)ratio) / (double)log_sf);
    if (n < 0) n = 0;
    else if (n >= nlevels) n = nlevels - 1;
    return n;
}

int orc_project(int mode, const orc_map_point* P, int n, const orc_view* V, const float* scale, int nlevels, float log_sf,
                orc_proj_query* out) {
    int kept = 0;
    for (int i = 0; i < n; ++i) {
        const orc_map_point& p = P[i];
        orc_proj_query q{};
        q.min_level = -1;
        q.max_level = -1;
        q.ur = 0.0f;
        q.ur_tol = -1.0f;
        q.level = -1;
        q.flags = ORC_QF_SKIP;
        out[i] = q;
        if (p.flags & ORC_QF_SKIP) continue;
        // x3Dc = Rcw * x3Dw + tcw (:1363-1364, Frame.cc:277, :855)
        const float xc = V->R[0] * p.x + V->R[1] * p.y + V->R[2] * p.z + V->t[0];
        const float yc = V->R[3] * p.x + V->R[4] * p.y + V->R[5] * p.z + V->t[1];
        const float zc = V->R[6] * p.x + V->R[7] * p.y + V->R[8] * p.z + V->t[2];
        if (mode == ORC_PROJ_LASTFRAME) {
            const float invzc = (float)(1.0 / (double)zc);                               // :1368
            if (invzc < 0) continue;
            const float u = V->fx * xc * invzc + V->cx;                                  // :1373-1374
            const float v = V->fy * yc * invzc + V->cy;
            if (u < V->min_x || u > V->max_x) continue;
            if (v < V->min_y || v > V->max_y) continue;
            const int oct = p.octave;
            const float radius = V->th * scale[oct];                                     // :1384
            q.x = u; q.y = v; q.r = radius;
            if (V->level_mode > 0) { q.min_level = oct; q.max_level = -1; }              // :1388-1393
            else if (V->level_mode < 0) { q.min_level = 0; q.max_level = oct; }
            else { q.min_level = oct - 1; q.max_level = oct + 1; }
            q.ur = u - V->bf * invzc;                                                    // :1418-1426
            q.ur_tol = radius;
            q.angle = p.angle;
            q.level = oct;
        } else {
            float u, v, invz;
            if (mode == ORC_PROJ_MAPPOINTS) {                                            // Frame::isInFrustum
                if (zc < 0.0f) continue;
                invz = 1.0f / zc;
                u = V->fx * xc * invz + V->cx;
                v = V->fy * yc * invz + V->cy;
                if (u < V->min_x || u > V->max_x) continue;
                if (v < V->min_y || v > V->max_y) continue;
            } else {                                                                     // Fuse :857-871
                if (zc < 0.0f) continue;
                invz = 1 / zc;
                const float x = xc * invz, y = yc * invz;
                u = V->fx * x + V->cx;
                v = V->fy * y + V->cy;
                if (!(u >= V->min_x && u < V->max_x && v >= V->min_y && v < V->max_y)) continue;   // KeyFrame::IsInImage
            }
            const float maxD = 1.2f * p.max_dist, minD = 0.8f * p.min_dist;            // MapPoint.cc:377-387
            const float POx = p.x - V->Ow[0], POy = p.y - V->Ow[1], POz = p.z - V->Ow[2];
            const float dist = (float)std::sqrt(orc_norm2(POx, POy, POz));              // cv::norm
            if (dist < minD || dist > maxD) continue;
            double dot = 0.0;                                                            // PO.dot(Pn): dotProd_
            dot += (double)POx * p.nx;
            dot += (double)POy * p.ny;
            dot += (double)POz * p.nz;
            const int pred = orc_predict_scale(p.max_dist, dist, log_sf, nlevels);
            if (mode == ORC_PROJ_MAPPOINTS) {
                const float viewCos = (float)(dot / (double)dist);                       // Frame.cc:308-311
                if (viewCos < V->view_cos_limit) continue;
                float r = (double)viewCos > 0.998 ? 2.5f : 4.0f;                         // RadiusByViewingCos :133-139
                if (V->th != 1.0f) r *= V->th;                                           // :65-68
                q.x = u; q.y = v; q.r = r * scale[pred];                                 // :70-71
                q.min_level = pred - 1; q.max_level = pred;
                q.ur = u - V->bf * invz;                                                 // mTrackProjXR (Frame.cc:319)
                q.ur_tol = r * scale[pred];                                              // :92-98
            } else {
                if (dot < 0.5 * (double)dist) continue;                                  // :887-888
                q.x = u; q.y = v; q.r = V->th * scale[pred];                             // :890-893
                q.min_level = pred - 1; q.max_level = pred;                              // :915-918
                q.ur = u - V->bf * invz;                                                 // :873
            }
            q.level = pred;
        }
        q.flags = p.flags & ~ORC_QF_SKIP;
        out[i] = q;
        ++kept;
    }
    return kept;
}

// MapPoints of one stereo frame: Frame::UnprojectStereo (src/Frame.cc:666-680) + MapPoint::MapPoint(Pos, pMap, pFrame,
// idxF) (src/MapPoint.cc:47-68).  twc = Rwc (9, row-major) then Ow (3); camera = fx, fy, cx, cy.
int orc_stereo_mappoints(const Kp* k, const float* depth, int n, const float* twc, const float* camera, const float* scale,
                         int nlevels, int flags, orc_map_point* out) {
    const float invfx = 1.0f / camera[0], invfy = 1.0f / camera[1];     // Frame.cc:94-95
    int made = 0;
    for (int i = 0; i < n; ++i) {
        orc_map_point p{};
        p.octave = k[i].octave;
        p.angle = k[i].angle;
        p.flags = ORC_QF_SKIP;
        const float z = depth[i];
        if (z > 0) {
            const float u = k[i].x, v = k[i].y;
            const float x = (u - camera[2]) * z * invfx;
            const float y = (v - camera[3]) * z * invfy;
            p.x = twc[0] * x + twc[1] * y + twc[2] * z + twc[9];               // mRwc * x3Dc + mOw
            p.y = twc[3] * x + twc[4] * y + twc[5] * z + twc[10];
            p.z = twc[6] * x + twc[7] * y + twc[8] * z + twc[11];
            const float dx = p.x - twc[9], dy = p.y - twc[10], dz = p.z - twc[11];
            const double nrm = std::sqrt(orc_norm2(dx, dy, dz));                 // cv::norm
            const float inv = (float)(1.0 / nrm);                              // mNormalVector / cv::norm(...)
            p.nx = dx * inv; p.ny = dy * inv; p.nz = dz * inv;
            const float dist = (float)nrm;
            p.max_dist = dist * scale[k[i].octave];                            // MapPoint.cc:60-64
            p.min_dist = p.max_dist / scale[nlevels - 1];
            p.flags = flags & ~ORC_QF_SKIP;
            ++made;
        }
        out[i] = p;
    }
    return made;
}

// Frame::AssignFeaturesToGrid with PosInGrid: cell (ix, iy) -> CSR row ix * rows + iy; indices ascending
// inside a cell (push_back in index order).  Returns the number of keypoints placed.
int orc_grid_assign(const Kp* k, int n, orc_grid g, int32_t* cell_start, int32_t* cell_idx) {
    std::vector<std::vector<int>> cells((size_t)g.cols * g.rows);
    for (int i = 0; i < n; ++i) {
        const int px = (int)std::round((k[i].x - g.min_x) * g.inv_w);
        const int py = (int)std::round((k[i].y - g.min_y) * g.inv_h);
        if (px < 0 || px >= g.cols || py < 0 || py >= g.rows) continue;
        cells[(size_t)px * g.rows + py].push_back(i);
    }
    int o = 0;
    for (size_t c = 0; c < cells.size(); ++c) {
        cell_start[c] = o;
        for (int i : cells[c]) cell_idx[o++] = i;
    }
    cell_start[cells.size()] = o;
    return o;
}

}  // extern "C"

namespace {

// Frame::GetFeaturesInArea; the KeyFrame version walks the same cells without a level test, and its callers
// test the level inside their own loop (same candidate order), so they pass their level range here.
void features_in_area(const Kp* k, const int32_t* cs, const int32_t* ci, const orc_grid& g, float x, float y, float r,
                      int minLevel, int maxLevel, std::vector<int>& out) {
    out.clear();
    const int nMinCellX = std::max(0, (int)std::floor((x - g.min_x - r) * g.inv_w));
    if (nMinCellX >= g.cols) return;
    const int nMaxCellX = std::min(g.cols - 1, (int)std::ceil((x - g.min_x + r) * g.inv_w));
    if (nMaxCellX < 0) return;
    const int nMinCellY = std::max(0, (int)std::floor((y - g.min_y - r) * g.inv_h));
    if (nMinCellY >= g.rows) return;
    const int nMaxCellY = std::min(g.rows - 1, (int)std::ceil((y - g.min_y + r) * g.inv_h));
    if (nMaxCellY < 0) return;
    const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    for (int ix = nMinCellX; ix <= nMaxCellX; ++ix)
        for (int iy = nMinCellY; iy <= nMaxCellY; ++iy) {
            const int c = ix * g.rows + iy;
            for (int j = cs[c]; j < cs[c + 1]; ++j) {
                const Kp& kp = k[ci[j]];
                if (bCheckLevels) {
                    if (kp.octave < minLevel) continue;
                    if (maxLevel >= 0 && kp.octave > maxLevel) continue;
                }
                const float distx = kp.x - x, disty = kp.y - y;
                if (std::fabs(distx) < r && std::fabs(disty) < r) out.push_back(ci[j]);
            }
        }
}

}  // namespace

extern "C" {

int orc_features_in_area(const Kp* k, const int32_t* cs, const int32_t* ci, orc_grid g, float x, float y, float r,
                         int minLevel, int maxLevel, int32_t* out, int cap) {
    std::vector<int> v;
    features_in_area(k, cs, ci, g, x, y, r, minLevel, maxLevel, v);
    for (size_t i = 0; i < v.size() && (int)i < cap; ++i) out[i] = v[i];
    return (int)v.size();
}

// All modes as one sequential walk over the queries in order.  blocked0[idx] != 0: the target keypoint
// already holds a MapPoint that excludes it (MAPPOINTS/LASTFRAME: Observations() > 0; KEYFRAME: any MapPoint;
// SIM3: vpMatched[idx]).  A query with ORC_QF_BLOCKS excludes the keypoint it is assigned to from later
// queries (MAPPOINTS/LASTFRAME: the assigned MapPoint has observations; KEYFRAME/SIM3: always).
// Outputs: q_idx/q_dist per query (accepted candidate, -1 if none; INIT: vnMatches12 after stealing and the
// rotation filter); owner[idx] (modes MAPPOINTS..SIM3): -1 untouched, q = MapPoint of query q (last
// writer), -2 = set to NULL by the rotation filter.  Returns nmatches as the reference counts it.
int orc_proj_search(orc_proj_params P, const orc_proj_query* Q, const uint8_t* qd, int nq, const Kp* k,
                    const uint8_t* kd, const float* uright, const uint8_t* blocked0, int n, orc_grid g,
                    const int32_t* cs, const int32_t* ci, int32_t* q_idx, int32_t* q_dist, int32_t* owner) {
    const int mode = P.mode;
    const bool assigning = mode <= ORC_PROJ_SIM3;
    const bool rot_mode = P.check_ori && (mode == ORC_PROJ_LASTFRAME || mode == ORC_PROJ_KEYFRAME || mode == ORC_PROJ_INIT);
    std::vector<int> own(n, -1), ownBlocks(n, 0), matchedDist(n, INT_MAX), m21(n, -1);
    std::vector<int> cand;
    std::vector<std::pair<int, int>> rot;   // (bin, entry): rotHist[bin].push_back(entry) in acceptance order
    int nm = 0;
    for (int q = 0; q < nq; ++q) {
        q_idx[q] = -1;
        q_dist[q] = -1;
    }
    for (int q = 0; q < nq; ++q) {
        const orc_proj_query& Qq = Q[q];
        if (Qq.flags & ORC_QF_SKIP) continue;
        features_in_area(k, cs, ci, g, Qq.x, Qq.y, Qq.r, Qq.min_level, Qq.max_level, cand);
        if (cand.empty()) continue;
        const uint8_t* d = qd + 32 * (size_t)q;
        int bestDist = 256, bestIdx = -1, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1;
        if (mode == ORC_PROJ_INIT || mode == ORC_PROJ_BEST) bestDist = bestDist2 = INT_MAX;
        for (int idx : cand) {
            const Kp& kp = k[idx];
            if (assigning) {
                if (blocked0 && blocked0[idx]) continue;
                if (own[idx] >= 0 && ownBlocks[idx]) continue;
            }
            if ((mode == ORC_PROJ_MAPPOINTS || mode == ORC_PROJ_LASTFRAME) && uright && Qq.ur_tol >= 0 && uright[idx] > 0) {
                const float er = std::fabs(Qq.ur - uright[idx]);   // :93-97, :1409-1415
                if (er > Qq.ur_tol) continue;
            }
            if (mode == ORC_PROJ_FUSE) {                           // :916-940
                const float ex = Qq.x - kp.x, ey = Qq.y - kp.y;
                if (uright && uright[idx] >= 0) {
                    const float er = Qq.ur - uright[idx];
                    const float e2 = ex * ex + ey * ey + er * er;
                    if (e2 * P.inv_sigma2[kp.octave] > 7.8) continue;
                } else {
                    const float e2 = ex * ex + ey * ey;
                    if (e2 * P.inv_sigma2[kp.octave] > 5.99) continue;
                }
            }
            const int dist = hamming(d, kd + 32 * (size_t)idx);
            if (mode == ORC_PROJ_INIT && matchedDist[idx] <= dist) continue;   // :446-447
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestLevel2 = bestLevel;
                bestDist = dist;
                bestLevel = kp.octave;
                bestIdx = idx;
            } else if (dist < bestDist2) {
                bestLevel2 = kp.octave;
                bestDist2 = dist;
            }
        }
        if (bestIdx < 0 || bestDist > P.accept_max) continue;
        if (mode == ORC_PROJ_MAPPOINTS && bestLevel == bestLevel2 && (float)bestDist > P.nnratio * (float)bestDist2) continue;
        if (mode == ORC_PROJ_INIT && !((float)bestDist < (float)bestDist2 * P.nnratio)) continue;
        q_idx[q] = bestIdx;
        q_dist[q] = bestDist;
        ++nm;
        if (assigning) {
            own[bestIdx] = q;
            ownBlocks[bestIdx] = (Qq.flags & ORC_QF_BLOCKS) ? 1 : 0;
        }
        if (mode == ORC_PROJ_INIT) {                               // :465-473
            if (m21[bestIdx] >= 0) {
                q_idx[m21[bestIdx]] = -1;
                --nm;
            }
            m21[bestIdx] = q;
            matchedDist[bestIdx] = bestDist;
        }
        if (rot_mode) rot.push_back({rot_bin(Qq.angle, k[bestIdx].angle), mode == ORC_PROJ_INIT ? q : bestIdx});
    }
    if (rot_mode) {                                                // :1449-1469, :1579-1598, :491-514
        int hist[30] = {0};
        for (auto& e : rot) hist[e.first]++;
        int i1, i2, i3;
        three_maxima(hist, 30, i1, i2, i3);
        for (int b = 0; b < 30; ++b) {
            if (b == i1 || b == i2 || b == i3) continue;
            for (auto& e : rot) {
                if (e.first != b) continue;
                if (mode == ORC_PROJ_INIT) {
                    if (q_idx[e.second] >= 0) {
                        q_idx[e.second] = -1;
                        --nm;
                    }
                } else {
                    own[e.second] = -2;                            // CurrentFrame.mvpMapPoints[...] = NULL
                    --nm;
                }
            }
        }
    }
    for (int q = 0; q < nq; ++q)
        if (q_idx[q] < 0) q_dist[q] = -1;   // stolen (INIT) or filtered entries carry no distance
    if (owner)
        for (int i = 0; i < n; ++i) owner[i] = own[i];
    return nm;
}


// Frame::UndistortKeyPoints / ComputeImageBounds (src/Frame.cc:404-464) via OpenCV 3.2 cvUndistortPoints(src, dst, K,
// D, R = I, P = K) restated: double precision, 5 fixed iterations (test infrastructure; -ffp-contract=off).
void orc_undistort_points(const float* xy, int n, const float* K, const float* dist, int n_dist, float* out) {
    double k[14] = {0};
    for (int i = 0; i < n_dist; ++i) k[i] = dist[i];
    const double fx = K[0], fy = K[4], cx = K[2], cy = K[5], ifx = 1. / fx, ify = 1. / fy;
    double RR[3][3];
    for (int i = 0; i < 9; ++i) RR[i / 3][i % 3] = K[i];
    const bool copy = n_dist == 0 || dist[0] == 0.0f;
    for (int i = 0; i < n; ++i) {
        if (copy) { out[2 * i] = xy[2 * i]; out[2 * i + 1] = xy[2 * i + 1]; continue; }
        double x = xy[2 * i], y = xy[2 * i + 1];
        x = (x - cx) * ifx;
        y = (y - cy) * ify;
        const double x0 = x, y0 = y;
        for (int j = 0; j < 5; j++) {
            double r2 = x * x + y * y;
            double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
            double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
            double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
            x = (x0 - deltaX) * icdist;
            y = (y0 - deltaY) * icdist;
        }
        double xx = RR[0][0] * x + RR[0][1] * y + RR[0][2];
        double yy = RR[1][0] * x + RR[1][1] * y + RR[1][2];
        double ww = 1. / (RR[2][0] * x + RR[2][1] * y + RR[2][2]);
        out[2 * i] = (float)(xx * ww);
        out[2 * i + 1] = (float)(yy * ww);
    }
}

}  // extern "C"
