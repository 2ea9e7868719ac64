/*
 * crt_bins.h — the per-triangle and per-cell arithmetic of the camera bins
 * (crt_layout.h CamCand, crt_bvh.h walk_bins), shared by the host checker
 * (crt_bvh_build.cpp build_camera_bins) and the device binning that runs in
 * every camera frame (crt_bins.hip).  Plain double arithmetic in a fixed
 * order with correctly rounded sqrt / divide on both sides (crt_device.h
 * sqrt_rn, div_rn; -ffp-contract=off), so host and device agree bit for bit.
 *
 * Why a cell's list holds every triangle its camera rays can hit.  The
 * reference accepts a hit at t only when the exact point q = o + d t lies in
 * the triangle's hull (the hull margins, crt_scene_build.cpp "pruned-walk
 * structures"; they hold for |o|_inf <= prune_origin_max, checked by
 * bin_camera).  A hull entirely in front of the camera projects into the
 * rectangle of its eight projected corners, and q projects to the point of
 * the image plane its camera ray passes: pixel x's ray passes X = x + 1/2
 * exactly up to the fp32 rounding of Camera::generate_ray (crt_camera.cpp:
 * 7-35: a few ulps of the direction, ~1e-3 px at 1920 wide), far inside the
 * 2-pixel margin added on every side.  Hulls not strictly in front of the
 * camera (or unbounded) are listed in every cell ("everywhere").
 *
 * Why dmin bounds t from below.  t = |q - o| / |d| >= dist(o, hull) / |d|,
 * and |d| of the normalised fp32 direction is 1 within a few ulps: dist is
 * computed in double from the fp32 box and scaled by 1 - 2^-20 before it is
 * rounded down.
 *
 * Lists: a cell's candidates sorted by (dmin, triangle id) — the host's
 * stable sort by dmin over triangles in id order.  A cell with more than
 * kBinCellCap candidates keeps no list: its pixels take the BVH walk (the
 * same answer, crt_bvh.h).  No bins at all (every pixel on the BVH) when
 * more than kBinMaxEverywhere hulls are everywhere or the lists would hold
 * more than kBinMeanCap candidates per cell on average.
 */
#pragma once
#include <math.h>
#include <stdint.h>

#include "crt_device.h"

namespace crt_amd {

constexpr int kBinMaxEverywhere = 64;   /* hulls listed in every cell */
constexpr int kBinCellCap = 512;        /* candidates of one cell (more: that cell walks the BVH) */
constexpr int64_t kBinMeanCap = 32;     /* mean candidates per cell */
constexpr double kBinMargin = 2.0;      /* pixels */
constexpr int kBinsMedium = 16;         /* cells with this many candidates are dispatched early (crt_bins.hip) */

/* Per-scene constants of the projection (host: bin_camera). */
struct BinCamera {
    double o[3];          /* camera location */
    double Mi[3][3];      /* inverse of the camera rotation (crt_matrix.h row vector convention) */
    double sx, sy;        /* aspect * tan(fov/2), tan(fov/2) */
    int32_t W, H;         /* image size */
    int32_t tx, ty;       /* 8x8 cells a row, rows */
};

/* A triangle's place in the frame: the pixel rectangle whose centres lie within
 * the margin of its hull's projection (px0 > px1: none), or everywhere. */
struct alignas(16) BinItem {
    int32_t px0, px1, py0, py1;
    float dmin;
    int32_t every;
    int32_t pad0, pad1;
};

/* One corner q (0..7) of a hull box projected: false if it is not strictly
 * in front of the camera (or not finite), else its image-plane X, Y. */
CRT_HD bool bin_corner(const double lo[3], const double hi[3], int q, const BinCamera &cam, double &X, double &Y) {
    const double p[3] = {(q & 1) ? hi[0] : lo[0], (q & 2) ? hi[1] : lo[1], (q & 4) ? hi[2] : lo[2]};
    const double w[3] = {p[0] - cam.o[0], p[1] - cam.o[1], p[2] - cam.o[2]};
    double cv[3];
    for (int j = 0; j < 3; ++j) cv[j] = w[0] * cam.Mi[0][j] + w[1] * cam.Mi[1][j] + w[2] * cam.Mi[2][j];
    const double wn = sqrt_rn(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    if (!isfinite(wn) || !isfinite(cv[0]) || !isfinite(cv[1]) || !isfinite(cv[2]) || !(cv[2] < -1e-9 * wn))
        return false;
    X = (div_rn(div_rn(cv[0], -cv[2]), cam.sx) + 1.0) * 0.5 * cam.W;
    Y = (1.0 - div_rn(div_rn(cv[1], -cv[2]), cam.sy)) * 0.5 * cam.H;
    return true;
}

/* dmin of a hull box: its distance from the camera, scaled by 1 - 2^-20,
 * rounded down (0 if not finite). */
CRT_HD float bin_dmin(const double lo[3], const double hi[3], const BinCamera &cam) {
    double d2 = 0.0;
    for (int k = 0; k < 3; ++k) {
        const double e = fmax(fmax(lo[k] - cam.o[k], cam.o[k] - hi[k]), 0.0);
        d2 += e * e;
    }
    const double dist = sqrt_rn(d2) * (1.0 - 0x1p-20);
    return isfinite(dist) ? round_down(dist) : 0.0f;
}

/* The item from the corners' bounds (every: some corner not in front).  The
 * bounds are exact minima / maxima, so any order of the corners gives them. */
CRT_HD BinItem bin_finish(bool every, double X0, double X1, double Y0, double Y1, float dmin, const BinCamera &cam) {
    BinItem it;
    it.every = 0;
    it.pad0 = it.pad1 = 0;
    it.dmin = dmin;
    if (every) {
        it.every = 1;
        it.px0 = 0;
        it.px1 = cam.W - 1;
        it.py0 = 0;
        it.py1 = cam.H - 1;
        it.dmin = 0.0f;
        return it;
    }
    /* pixels whose centre X = x + 1/2 lies within the margin of [X0, X1] */
    const double px0 = ceil(X0 - 0.5 - kBinMargin), px1 = floor(X1 - 0.5 + kBinMargin);
    const double py0 = ceil(Y0 - 0.5 - kBinMargin), py1 = floor(Y1 - 0.5 + kBinMargin);
    if (px1 < 0.0 || py1 < 0.0 || px0 > cam.W - 1 || py0 > cam.H - 1 || px0 > px1 || py0 > py1) {
        it.px0 = 1;
        it.px1 = 0;
        it.py0 = 1;
        it.py1 = 0;
        return it;
    }
    it.px0 = (int32_t)fmax(0.0, px0);
    it.px1 = (int32_t)fmin((double)(cam.W - 1), px1);
    it.py0 = (int32_t)fmax(0.0, py0);
    it.py1 = (int32_t)fmin((double)(cam.H - 1), py1);
    return it;
}

CRT_HD BinItem bin_project(const float blo[3], const float bhi[3], const BinCamera &cam) {
    const double lo[3] = {blo[0], blo[1], blo[2]}, hi[3] = {bhi[0], bhi[1], bhi[2]};
    bool every = false;
    double X0 = INFINITY, X1 = -INFINITY, Y0 = INFINITY, Y1 = -INFINITY;
    for (int q = 0; q < 8 && !every; ++q) {
        double X, Y;
        if (!bin_corner(lo, hi, q, cam, X, Y)) {
            every = true;
            break;
        }
        X0 = fmin(X0, X);
        X1 = fmax(X1, X);
        Y0 = fmin(Y0, Y);
        Y1 = fmax(Y1, Y);
    }
    return bin_finish(every, X0, X1, Y0, Y1, bin_dmin(lo, hi, cam), cam);
}

/* The pixels of cell (cx, cy) inside the item's rectangle (bit 8 y + x). */
CRT_HD uint64_t bin_mask(const BinItem &it, int cx, int cy) {
    const int x0 = it.px0 > 8 * cx ? it.px0 : 8 * cx, x1 = it.px1 < 8 * cx + 7 ? it.px1 : 8 * cx + 7;
    const int y0 = it.py0 > 8 * cy ? it.py0 : 8 * cy, y1 = it.py1 < 8 * cy + 7 ? it.py1 : 8 * cy + 7;
    if (x0 > x1 || y0 > y1) return 0ull;
    const uint64_t row = ((1ull << (x1 - x0 + 1)) - 1ull) << (x0 - 8 * cx);
    uint64_t m = 0ull;
    for (int y = y0; y <= y1; ++y) m |= row << (8 * (y - 8 * cy));
    return m;
}

/* Sort key of a cell's candidate: (dmin, triangle id), dmin >= 0. */
CRT_HD uint64_t bin_key(float dmin, int32_t t) {
    union { float f; uint32_t u; } b;
    b.f = dmin;
    return ((uint64_t)b.u << 32) | (uint32_t)t;
}

}  // namespace crt_amd
