/*
 * crt_light_bins.cpp — light bins (crt_layout.h DLightBin): per light, the
 * candidate lists its shadow rays walk instead of the BVH (crt_bvh.h
 * lbin_first_hit).  Built once per scene at the first shadow-ray frame: the
 * lights and triangles do not move with the camera.
 *
 * Why a ray's list holds every triangle it can hit within the light.  A
 * shadow ray o + d t (crt_renderer.cpp:81-96: o = p + n bias, d towards the
 * light L) has its hits the reference's test accepts at t in [0, lim]
 * (fl(t * t) <= r2), and the exact point q = o + d t of such a hit lies in
 * the triangle's hull (crt_scene_build.cpp, "pruned-walk structures"; for
 * |o|_inf <= prune_origin_max).  The walk takes a ray only when its line
 * passes L at a distance e <= e_max and its end o + d lim lies within R0 of
 * L.  Let c be the line's closest point to L:
 *   - past c (towards the end) every point is within max(e, |end - L|) < R0
 *     of L, so a hull holding q comes within R0: the near list;
 *   - before c, |q - L| <= |w| (w = o - L) and q - L, w lie in one plane
 *     with L and the line, on the same side of c: the angle between them is
 *     at most asin(e / |q - L|).  A hull that stays R0 away (not near) is
 *     hit only at |q - L| >= R0, so q - L is within theta = asin(e_max / R0)
 *     of w.
 * w's cube face (axis k: its largest component) puts w within
 * acos(1/sqrt 3) + theta of the axis, q too, so s (q_k - L_k) >=
 * |q - L| cos(54.74 deg + theta) >= 0.45 dist(L, hull) (theta <= 0.1), and
 * along the arc from w to q the face coordinate u_j = x_j / x_k moves by at
 * most theta / cos^2(54.74 deg + theta) (its gradient on the unit sphere is
 * at most 1 / x_k^2).  A hull dist >= R0 away is hit only at
 * |q - L| >= dist, so its own theta_t = asin(e_max / dist) bounds the
 * angle for it: far triangles get narrow margins.  A hull is listed in every cell of a face whose
 * u-range — the extremes of a / m over the box part with
 * m = s (x_k - L_k) >= 0.45 dist, a = x_j - L_j (corner values, m > 0) —
 * widened by that margin and 1e-9, meets the cell.  dmin = dist(L, hull)
 * rounded down: a hit before c has dist <= |q - L| <= |w|, so a sorted list
 * ends at the first dmin > |w|.
 *
 * Per light R0 is the largest of 64, 32, 16 e_max whose near list holds at
 * most kLightNearCap hulls (unbounded hulls are always near); a light with
 * none, or lists past kLightRecCap records in all, takes the BVH.
 */
#include <algorithm>
#include <cmath>
#include <thread>
#include <vector>

#include "crt_bins.h"
#include "crt_host.h"

namespace crt_amd {

namespace {

constexpr int kLightNearCap = 32;
constexpr int64_t kLightRecCap = int64_t(1) << 24;

struct Rect {
    int face, u0, u1, v0, v1;
};

/* The cells of one hull for one light (dist: its distance from L). */
void hull_cells(const double lo[3], const double hi[3], const double L[3], double dist, double margin, int N,
                std::vector<Rect> &out) {
    out.clear();
    const double h = 0.5 * N;
    for (int face = 0; face < 6; ++face) {
        const int k = face >> 1;
        const bool neg = face & 1;
        double m_lo = neg ? L[k] - hi[k] : lo[k] - L[k];
        const double m_hi = neg ? L[k] - lo[k] : hi[k] - L[k];
        const double m0 = 0.45 * dist;
        if (!(m_hi >= m0) || !(m0 > 0.0)) continue;
        m_lo = std::max(m_lo, m0);
        const int j1 = k == 0 ? 1 : 0, j2 = k == 2 ? 1 : 2;
        int c0[2], c1[2];
        bool ok = true;
        for (int q = 0; q < 2 && ok; ++q) {
            const int j = q == 0 ? j1 : j2;
            const double a_lo = lo[j] - L[j], a_hi = hi[j] - L[j];
            const double ulo = a_lo / (a_lo < 0.0 ? m_lo : m_hi) - margin;
            const double uhi = a_hi / (a_hi > 0.0 ? m_lo : m_hi) + margin;
            if (uhi < -1.0 || ulo > 1.0) {
                ok = false;
                break;
            }
            c0[q] = std::max(0, (int)std::floor((ulo + 1.0) * h));
            c1[q] = std::min(N - 1, (int)std::floor((uhi + 1.0) * h));
            if (c0[q] > c1[q]) ok = false;
        }
        if (ok) out.push_back(Rect{face, c0[0], c1[0], c0[1], c1[1]});
    }
}

struct OneLight {
    DLightBin par{};
    std::vector<int32_t> off;     /* 6 N^2 + 2, relative to recs */
    std::vector<LightCand> recs;
};

void build_one(const CamCand *tpl, int nt, const DLight &lt, double e_max, int N, OneLight &out) {
    const double L[3] = {lt.px, lt.py, lt.pz};
    out.par.lx = L[0];
    out.par.ly = L[1];
    out.par.lz = L[2];
    out.par.on = 0;
    if (!std::isfinite(L[0]) || !std::isfinite(L[1]) || !std::isfinite(L[2])) return;
    std::vector<double> dist((size_t)nt);
    int unbounded = 0;
    for (int t = 0; t < nt; ++t) {
        const CamCand &c = tpl[t];
        const double lo[3] = {c.lo_x, c.lo_y, c.lo_z}, hi[3] = {c.hi_x, c.hi_y, c.hi_z};
        bool fin = true;
        double s = 0.0;
        for (int j = 0; j < 3; ++j) {
            fin = fin && std::isfinite(lo[j]) && std::isfinite(hi[j]);
            const double g = std::max(0.0, std::max(lo[j] - L[j], L[j] - hi[j]));
            s += g * g;
        }
        dist[(size_t)t] = fin ? std::sqrt(s) * (1.0 - 1e-12) : -1.0;   /* -1: unbounded, always near */
        if (!fin) ++unbounded;
    }
    if (unbounded > kLightNearCap) return;
    double R0 = 0.0;
    for (double f : {64.0, 32.0, 16.0}) {
        const double r = f * e_max;
        int near = 0;
        for (int t = 0; t < nt; ++t) near += dist[(size_t)t] <= r * (1.0 + 1e-9) ? 1 : 0;
        if (near <= kLightNearCap) {
            R0 = r;
            break;
        }
    }
    if (!(R0 > 0.0)) return;
    /* a hull dist away is hit only at |q - L| >= dist: its margin is that of
     * theta_t = asin(e_max / dist) <= asin(e_max / R0) */
    auto margin_of = [&](double dist) {
        const double theta = std::asin(e_max / std::max(dist, R0));
        const double ca = std::cos(std::acos(1.0 / std::sqrt(3.0)) + theta);
        return theta / (ca * ca) * (1.0 + 1e-6) + 1e-9;
    };
    const int64_t ncell = 6 * (int64_t)N * N;
    std::vector<int64_t> cnt((size_t)ncell + 1, 0);
    std::vector<Rect> rects;
    int64_t total = 0, near_n = 0;
    auto near_of = [&](int t) { return dist[(size_t)t] <= R0 * (1.0 + 1e-9); };
    for (int t = 0; t < nt; ++t) {
        if (near_of(t)) {
            ++near_n;
            continue;
        }
        const CamCand &c = tpl[t];
        const double lo[3] = {c.lo_x, c.lo_y, c.lo_z}, hi[3] = {c.hi_x, c.hi_y, c.hi_z};
        hull_cells(lo, hi, L, dist[(size_t)t], margin_of(dist[(size_t)t]), N, rects);
        for (const Rect &r : rects)
            for (int v = r.v0; v <= r.v1; ++v)
                for (int u = r.u0; u <= r.u1; ++u) ++cnt[(size_t)((r.face * N + v) * N + u)];
        for (const Rect &r : rects) total += (int64_t)(r.u1 - r.u0 + 1) * (r.v1 - r.v0 + 1);
        if (total > kLightRecCap) return;
    }
    out.off.assign((size_t)ncell + 2, 0);
    out.off[1] = (int32_t)near_n;
    for (int64_t c = 0; c < ncell; ++c) out.off[(size_t)c + 2] = out.off[(size_t)c + 1] + (int32_t)cnt[(size_t)c];
    out.recs.resize((size_t)(near_n + total));
    std::vector<int32_t> fill(out.off.begin(), out.off.end() - 1);
    auto rec = [&](int t) {
        LightCand r{};
        r.dmin = dist[(size_t)t] < 0.0 ? 0.0f : round_down(dist[(size_t)t]);
        r.id = tpl[t].id;
        r.g = tpl[t].g;
        return r;
    };
    for (int t = 0; t < nt; ++t) {
        if (near_of(t)) {
            out.recs[(size_t)fill[0]++] = rec(t);
            continue;
        }
        const CamCand &c = tpl[t];
        const double lo[3] = {c.lo_x, c.lo_y, c.lo_z}, hi[3] = {c.hi_x, c.hi_y, c.hi_z};
        hull_cells(lo, hi, L, dist[(size_t)t], margin_of(dist[(size_t)t]), N, rects);
        const LightCand r = rec(t);
        for (const Rect &q : rects)
            for (int v = q.v0; v <= q.v1; ++v)
                for (int u = q.u0; u <= q.u1; ++u) out.recs[(size_t)fill[(size_t)1 + (q.face * N + v) * N + u]++] = r;
    }
    /* each list by (dmin, triangle id) */
    for (size_t c = 0; c + 1 < out.off.size(); ++c)
        std::sort(out.recs.begin() + out.off[c], out.recs.begin() + out.off[c + 1],
                  [](const LightCand &a, const LightCand &b) {
                      return a.dmin < b.dmin || (a.dmin == b.dmin && (a.id & 0x7fffffff) < (b.id & 0x7fffffff));
                  });
    out.par.r0_sq = R0 * R0;
    out.par.e_sq = e_max * e_max;
    out.par.on = 1;
}

}  // namespace

bool build_light_bins(const CamCand *tpl, int nt, const DLight *lights, int nl, double e_max, int N,
                      LightBinsHost &out) {
    out = LightBinsHost{};
    if (nt <= 0 || nl <= 0 || !(e_max > 0.0) || N < 1) return false;
    std::vector<OneLight> per((size_t)nl);
    const int nth = std::max(1, std::min(nl, 8));
    std::vector<std::thread> pool;
    for (int k = 0; k < nth; ++k)
        pool.emplace_back([&, k]() {
            for (int l = k; l < nl; l += nth) build_one(tpl, nt, lights[l], e_max, N, per[(size_t)l]);
        });
    for (auto &th : pool) th.join();
    const int64_t stride = 6 * (int64_t)N * N + 2;
    out.n = N;
    out.par.resize((size_t)nl);
    out.off.assign((size_t)(stride * nl), 0);
    int64_t base = 0;
    bool any = false;
    for (int l = 0; l < nl; ++l) {
        OneLight &o = per[(size_t)l];
        out.par[(size_t)l] = o.par;
        out.par[(size_t)l].base = (int32_t)(stride * l);
        if (!o.par.on || base + (int64_t)o.recs.size() > kLightRecCap) {
            out.par[(size_t)l].on = 0;
            continue;
        }
        for (int64_t c = 0; c < stride; ++c) out.off[(size_t)(stride * l + c)] = (int32_t)(base + o.off[(size_t)c]);
        out.recs.insert(out.recs.end(), o.recs.begin(), o.recs.end());
        base += (int64_t)o.recs.size();
        any = true;
    }
    if (!any) out = LightBinsHost{};
    return any;
}

}  // namespace crt_amd
