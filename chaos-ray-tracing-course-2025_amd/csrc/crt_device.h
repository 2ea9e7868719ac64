/*
 * crt_device.h — per-ray math of the hot path for gfx950, written in the
 * reference's exact fp32 operation order so results are bit-identical
 * (build with -ffp-contract=off; fp32 '/' and sqrtf stay correctly rounded,
 * HIP's default).  Reference lines are cited per function.
 */
#pragma once
#include <math.h>
#include <stdint.h>

#include "crt_layout.h"

#if defined(__HIPCC__)
#define CRT_HD __host__ __device__ __forceinline__
#else
#define CRT_HD inline
#endif

namespace crt_amd {

struct Vec { float x, y, z; };

CRT_HD Vec vec(float x, float y, float z) { Vec r; r.x = x; r.y = y; r.z = z; return r; }
CRT_HD Vec vadd(Vec a, Vec b) { return vec(a.x + b.x, a.y + b.y, a.z + b.z); }
CRT_HD Vec vsub(Vec a, Vec b) { return vec(a.x - b.x, a.y - b.y, a.z - b.z); }
CRT_HD Vec vneg(Vec a) { return vec(-a.x, -a.y, -a.z); }
CRT_HD Vec vscale(Vec a, float s) { return vec(a.x * s, a.y * s, a.z * s); }
CRT_HD Vec vdiv(Vec a, float s) { return vec(a.x / s, a.y / s, a.z / s); }
/* crt_vector.h:76-78: Vector*Vector multiplies the y component twice. */
CRT_HD Vec vmul_quirk(Vec a, Vec b) { return vec(a.x * b.x, a.y * b.y * a.y, a.z * b.z); }
CRT_HD float vdot(Vec a, Vec b) { return a.x * b.x + a.y * b.y + a.z * b.z; }          /* crt_vector.h:115-117 */
CRT_HD Vec vcross(Vec a, Vec b) {                                                        /* crt_vector.h:107-113 */
    return vec(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
CRT_HD float vlen_sq(Vec a) { return a.x * a.x + a.y * a.y + a.z * a.z; }               /* crt_vector.h:13-15 */
CRT_HD float vlen(Vec a) { return sqrtf(vlen_sq(a)); }                                   /* crt_vector.cpp:7-9 */
CRT_HD Vec vnormalize(Vec a) { return vdiv(a, vlen(a)); }                                /* crt_vector.h:98-101 */

/* crt_matrix.h:66-74: row vector times row-major 3x3, each column summed from 0.0f. */
CRT_HD Vec vec_mat(Vec v, const float m[9]) {
    float r0 = 0.0f, r1 = 0.0f, r2 = 0.0f;
    r0 += v.x * m[0]; r0 += v.y * m[3]; r0 += v.z * m[6];
    r1 += v.x * m[1]; r1 += v.y * m[4]; r1 += v.z * m[7];
    r2 += v.x * m[2]; r2 += v.y * m[5]; r2 += v.z * m[8];
    return vec(r0, r1, r2);
}

/* Node record fields (crt_layout.h): interior b = -(depth+1), a = skip;
 * leaf a = count | depth << 24, b = first slot. */
CRT_HD int node_leaf_count(const DNode &n) { return n.a & 0xffffff; }
CRT_HD int node_depth(const DNode &n) { return n.b < 0 ? -n.b - 1 : (int)((unsigned)n.a >> 24); }

/* Camera::generate_ray (crt_camera.cpp:7-35). aspect and tan_half_fov are the
 * per-frame constants float(W)/H and std::tan(fov*0.5f), computed on the host. */
CRT_HD void camera_ray(const DCamera &c, int x, int y, Vec &o, Vec &d) {
    float dx = x + 0.5f, dy = y + 0.5f;
    dx /= (float)c.width;
    dy /= (float)c.height;
    dx = (2.0f * dx) - 1.0f;
    dy = 1.0f - (2.0f * dy);
    dx *= c.aspect;
    dx *= c.tan_half_fov;
    dy *= c.tan_half_fov;
    o = vec(c.loc[0], c.loc[1], c.loc[2]);
    d = vnormalize(vec_mat(vec(dx, dy, -1.0f), c.rot));
}

/* ray_intersect_aabb_p (crt_intersection.cpp:14-45): for extent ∈ {min,max},
 * axis ∈ {x,y,z}: skip near-parallel axes and faces behind the origin, else
 * the hit point must lie in the face's other two slabs (inclusive).  The
 * function is a pure OR over the six faces, so evaluation order is free.
 *
 * t = (plane - o) / d is negative iff the two operands have opposite signs and
 * the quotient does not underflow to -0; for a nonzero numerator that needs
 * |d| >= 2 (the smallest denormal halved ties to zero), so while |d| < 2 the
 * sign test decides "behind" exactly and only faces in front pay the
 * correctly-rounded divide. */
CRT_HD bool opposite_signs(float a, float b) { return (a < 0.0f && b > 0.0f) || (a > 0.0f && b < 0.0f); }

CRT_HD bool box_face(float plane, float o_a, float d_a, float o_u, float d_u, float o_w, float d_w,
                     float lo_u, float hi_u, float lo_w, float hi_w) {
    if (fabsf(d_a) < 1e-6f) return false;
    const float num = plane - o_a;
    if (opposite_signs(num, d_a) && fabsf(d_a) < 2.0f) return false;
    const float t = num / d_a;
    if (t < 0.0f) return false;
    const float pu = o_u + d_u * t;
    const float pw = o_w + d_w * t;
    return pu >= lo_u && pu <= hi_u && pw >= lo_w && pw <= hi_w;
}

CRT_HD bool box_hit(Vec o, Vec d, const DNode &n) {
    /* faces min.x, min.y, min.z, max.x, max.y, max.z; (u,v) = (1,2),(2,0),(0,1) */
    return box_face(n.lo_x, o.x, d.x, o.y, d.y, o.z, d.z, n.lo_y, n.hi_y, n.lo_z, n.hi_z) ||
           box_face(n.lo_y, o.y, d.y, o.z, d.z, o.x, d.x, n.lo_z, n.hi_z, n.lo_x, n.hi_x) ||
           box_face(n.lo_z, o.z, d.z, o.x, d.x, o.y, d.y, n.lo_x, n.hi_x, n.lo_y, n.hi_y) ||
           box_face(n.hi_x, o.x, d.x, o.y, d.y, o.z, d.z, n.lo_y, n.hi_y, n.lo_z, n.hi_z) ||
           box_face(n.hi_y, o.y, d.y, o.z, d.z, o.x, d.x, n.lo_z, n.hi_z, n.lo_x, n.hi_x) ||
           box_face(n.hi_z, o.z, d.z, o.x, d.x, o.y, d.y, n.lo_x, n.hi_x, n.lo_y, n.hi_y);
}

/* Branch-free form of the same predicate: all six faces evaluated, OR-ed
 * without short-circuit (no exec-mask branches; more VALU, no SALU). */
CRT_HD int box_face_bf(float plane, float o_a, float d_a, float o_u, float d_u, float o_w, float d_w,
                        float lo_u, float hi_u, float lo_w, float hi_w) {
    const float num = plane - o_a;
    const float t = num / d_a;
    const float pu = o_u + d_u * t;
    const float pw = o_w + d_w * t;
    return (int)!(fabsf(d_a) < 1e-6f) & (int)!(t < 0.0f) & (int)(pu >= lo_u) & (int)(pu <= hi_u) &
           (int)(pw >= lo_w) & (int)(pw <= hi_w);
}

CRT_HD bool box_hit_bf(Vec o, Vec d, const DNode &n) {
    return 0 != (box_face_bf(n.lo_x, o.x, d.x, o.y, d.y, o.z, d.z, n.lo_y, n.hi_y, n.lo_z, n.hi_z) |
           box_face_bf(n.lo_y, o.y, d.y, o.z, d.z, o.x, d.x, n.lo_z, n.hi_z, n.lo_x, n.hi_x) |
           box_face_bf(n.lo_z, o.z, d.z, o.x, d.x, o.y, d.y, n.lo_x, n.hi_x, n.lo_y, n.hi_y) |
           box_face_bf(n.hi_x, o.x, d.x, o.y, d.y, o.z, d.z, n.lo_y, n.hi_y, n.lo_z, n.hi_z) |
           box_face_bf(n.hi_y, o.y, d.y, o.z, d.z, o.x, d.x, n.lo_z, n.hi_z, n.lo_x, n.hi_x) |
           box_face_bf(n.hi_z, o.z, d.z, o.x, d.x, o.y, d.y, n.lo_x, n.hi_x, n.lo_y, n.hi_y));
}

/* ---- per-ray hoisted division ---------------------------------------- */
/* hipcc lowers fp32 a/b to (LLVM AMDGPU LowerFDIV32):
 *   y0 = rcp(b'); y1 = fma(fma(-b', y0, 1), y0, y0); q0 = a'*y1;
 *   q1 = fma(fma(-b', q0, a'), y1, q0); q = div_fmas(fma(-b', q1, a'), y1, q1); div_fixup
 * with a', b' = div_scale(a, b).  div_scale leaves both operands unchanged and
 * div_fmas is a plain fma unless |exp(a) - exp(b)| approaches 96, b is
 * denormal or a is near the denormal range; div_fixup only rewrites special
 * values.  So for |b| in [2^-20, 2^20] and |a| in [2^-64, 2^64] the sequence
 * below, with the b-only part (y1) computed once per ray and axis, returns
 * the same bits as '/', i.e. the correctly rounded quotient.  Anything outside
 * that window takes the compiler's '/'. */
struct RayRcp {
    float y1[3];     /* refined 1/d; NaN where |d| < 1e-6 discards the axis' faces (every quotient and
                      * hit point of those faces is then NaN, and NaN fails each of the face's compares) */
    bool fast;       /* every box-face quotient of this ray is inside the exact window */
};

CRT_HD float rcp_refined(float b) {
#if defined(__HIP_DEVICE_COMPILE__)
    const float y0 = __builtin_amdgcn_rcpf(b);
#else
    const float y0 = 1.0f / b;   /* host builds of this header never take the fast path */
#endif
    return fmaf(fmaf(-b, y0, 1.0f), y0, y0);
}

/* 0, or a magnitude in [2^-40, 2^62].  If every box plane p and every origin
 * component o satisfies this, each numerator a = p - o is 0 or has
 * |a| in [2^-63, 2^63]: two such nonzero floats are multiples of ulp(2^-40) =
 * 2^-63, and |p| + |o| <= 2^63.  A zero numerator gives a zero quotient whose
 * sign may differ from '/', which no face test can observe (t < 0 is false
 * for both zeros and o + d*(+-0) compares equal).  Faces with |d| < 1e-6 are
 * discarded before their quotient is used, and |d| >= 1e-6 > 2^-20; so with
 * |d| <= 2^20 every quotient a face test reads is the correctly rounded one. */
CRT_HD bool coord_ok(float x) {
    const float m = fabsf(x);
    return x == 0.0f || (m >= 9.094947017729282e-13f && m <= 4.611686018427388e18f);
}

CRT_HD RayRcp make_ray_rcp(Vec o, Vec d, bool planes_ok) {
    RayRcp r;
#if defined(__HIP_DEVICE_COMPILE__)
    r.fast = planes_ok && coord_ok(o.x) && coord_ok(o.y) && coord_ok(o.z) && fabsf(d.x) <= 1048576.0f &&
             fabsf(d.y) <= 1048576.0f && fabsf(d.z) <= 1048576.0f;
#else
    (void)o;
    (void)planes_ok;
    r.fast = false;
#endif
    r.y1[0] = fabsf(d.x) < 1e-6f ? NAN : rcp_refined(d.x);
    r.y1[1] = fabsf(d.y) < 1e-6f ? NAN : rcp_refined(d.y);
    r.y1[2] = fabsf(d.z) < 1e-6f ? NAN : rcp_refined(d.z);
    return r;
}

CRT_HD float div_fast(float a, float b, float y1) {
    const float q0 = a * y1;
    const float q1 = fmaf(fmaf(-b, q0, a), y1, q0);
    return fmaf(fmaf(-b, q1, a), y1, q1);
}

CRT_HD bool face_ok(float t, float d_a, float o_u, float d_u, float o_w, float d_w, float lo_u, float hi_u,
                    float lo_w, float hi_w) {
    const float pu = o_u + d_u * t;
    const float pw = o_w + d_w * t;
    return !(fabsf(d_a) < 1e-6f) & !(t < 0.0f) & (pu >= lo_u) & (pu <= hi_u) & (pw >= lo_w) & (pw <= hi_w);
}

/* Fast-ray form of the face test.  For a fast ray every term of a tested
 * face is finite (|t| <= 2^63 / 1e-6, |d| <= 2^20, |o|, |plane| <= 2^62).
 * The two faces of an axis share d and the refined reciprocal, so their
 * quotients and hit points are computed as float pairs
 * (v_pk_mul/fma/add_f32); each range check is one med3 and a compare. */
typedef float f2 __attribute__((ext_vector_type(2)));

CRT_HD f2 div_fast2(f2 a, float b, float y1) {
    const f2 B = b, Y = y1;
    const f2 q0 = a * Y;
    const f2 q1 = __builtin_elementwise_fma(__builtin_elementwise_fma(-B, q0, a), Y, q0);
    return __builtin_elementwise_fma(__builtin_elementwise_fma(-B, q1, a), Y, q1);
}

/* lo <= p <= hi for a finite p and ordered planes (lo <= hi: part of the
 * planes_ok condition): a med3 returns one of its operands, so it equals p
 * exactly when p lies in the closed range (-0 and +0 compare equal, as the
 * reference's >= / <= do). */
CRT_HD bool in_slab(float p, float lo, float hi) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_fmed3f(p, lo, hi) == p;
#else
    return (p >= lo) & (p <= hi);
#endif
}

/* The two faces of axis a (planes pl = lo, hi) for a fast ray: quotients and
 * hit points as float pairs.  The face's t >= 0 test (!(t < 0): t of a fast
 * ray is finite or, on a discarded axis, NaN) is folded into pu, which is
 * NaN for a face that fails it, so the face passes iff both hit-point
 * coordinates are in range (axis_pass). */
CRT_HD void axis_points(f2 pl, float o_a, float d_a, float y1, float o_u, float d_u, float o_w, float d_w, f2 &pu,
                        f2 &pw) {
    const f2 t = div_fast2(pl - o_a, d_a, y1);
    pu = o_u + d_u * t;
    pw = o_w + d_w * t;
    pu.x = t.x >= 0.0f ? pu.x : NAN;
    pu.y = t.y >= 0.0f ? pu.y : NAN;
}

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wbitwise-instead-of-logical"   /* no short-circuit: branch-free ORs */
CRT_HD bool axis_pass(f2 pu, f2 pw, float lo_u, float hi_u, float lo_w, float hi_w) {
    return (in_slab(pu.x, lo_u, hi_u) & in_slab(pw.x, lo_w, hi_w)) |
           (in_slab(pu.y, lo_u, hi_u) & in_slab(pw.y, lo_w, hi_w));
}

/* ray_intersect_aabb_p (crt_intersection.cpp:14-45), branch-free over the six
 * faces, with the per-ray hoisted divisions (see coord_ok for when they are
 * exact; other rays take the compiler's '/' and the plain compares). */
/* The fast-ray form alone (caller guarantees r.fast for every lane it uses). */
CRT_HD bool box_hit_fast(Vec o, Vec d, const RayRcp &r, const DNode n) {
    f2 px, qx, py, qy, pz, qz;
    axis_points((f2){n.lo_x, n.hi_x}, o.x, d.x, r.y1[0], o.y, d.y, o.z, d.z, px, qx);
    axis_points((f2){n.lo_y, n.hi_y}, o.y, d.y, r.y1[1], o.z, d.z, o.x, d.x, py, qy);
    axis_points((f2){n.lo_z, n.hi_z}, o.z, d.z, r.y1[2], o.x, d.x, o.y, d.y, pz, qz);
    return axis_pass(px, qx, n.lo_y, n.hi_y, n.lo_z, n.hi_z) | axis_pass(py, qy, n.lo_z, n.hi_z, n.lo_x, n.hi_x) |
           axis_pass(pz, qz, n.lo_x, n.hi_x, n.lo_y, n.hi_y);
}

CRT_HD bool box_hit_r(Vec o, Vec d, const RayRcp &r, const DNode n) {
    if (r.fast) return box_hit_fast(o, d, r, n);
    const float t0 = (n.lo_x - o.x) / d.x, t1 = (n.lo_y - o.y) / d.y, t2 = (n.lo_z - o.z) / d.z;
    const float t3 = (n.hi_x - o.x) / d.x, t4 = (n.hi_y - o.y) / d.y, t5 = (n.hi_z - o.z) / d.z;
    return face_ok(t0, d.x, o.y, d.y, o.z, d.z, n.lo_y, n.hi_y, n.lo_z, n.hi_z) |
           face_ok(t1, d.y, o.z, d.z, o.x, d.x, n.lo_z, n.hi_z, n.lo_x, n.hi_x) |
           face_ok(t2, d.z, o.x, d.x, o.y, d.y, n.lo_x, n.hi_x, n.lo_y, n.hi_y) |
           face_ok(t3, d.x, o.y, d.y, o.z, d.z, n.lo_y, n.hi_y, n.lo_z, n.hi_z) |
           face_ok(t4, d.y, o.z, d.z, o.x, d.x, n.lo_z, n.hi_z, n.lo_x, n.hi_x) |
           face_ok(t5, d.z, o.x, d.x, o.y, d.y, n.lo_x, n.hi_x, n.lo_y, n.hi_y);
}
#pragma clang diagnostic pop

/* ---- pruned walks ------------------------------------------------------ */
/* Hull slab test of a PNode (crt_layout.h).  The hull is conservative by a
 * margin (crt_scene_build.cpp) far above this test's own rounding, so `alive`
 * is false only when no triangle in the subtree can produce a hit with
 * t <= lim.  The slab distance of plane P on axis a is one fma,
 * P * (1/d_a) + c_a with c_a = -o_a * (1/d_a) rounded once per ray: a
 * reciprocal with ~1 ulp error and two roundings put it within a few ulps of
 * |o_a| + |P - o_a| (over |d_a|) of the exact distance, the same order as the
 * (P - o) * (1/d) form and far inside the margin's 2^-13 G.  An axis whose
 * reciprocal is so large that a product could overflow (|1/d_a| G > 2^100,
 * d_a = 0 included) gets 1/d_a = NaN: its slab distances are NaN, which
 * fminf/fmaxf drop, so that axis stops restricting the test — the test stays
 * conservative.  The final tests are negated so a NaN bound keeps the subtree. */
struct PruneRay {
    float ix, iy, iz;      /* ~1/d, or NaN (see above) */
    float cx, cy, cz;      /* -o * ix */
    bool on;               /* |o|_inf <= prune_origin_max: the margins hold for this ray */
};

CRT_HD float rcp_any(float b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcpf(b);
#else
    return 1.0f / b;
#endif
}

CRT_HD float prune_rcp(float d, float omax) {
    const float i = rcp_any(d);
    return fabsf(i) * fmaxf(omax, 1.0f) <= 0x1p100f ? i : NAN;
}

CRT_HD PruneRay make_prune_ray(Vec o, Vec d, float omax) {
    PruneRay p;
    p.ix = prune_rcp(d.x, omax);
    p.iy = prune_rcp(d.y, omax);
    p.iz = prune_rcp(d.z, omax);
    p.cx = -o.x * p.ix;
    p.cy = -o.y * p.iy;
    p.cz = -o.z * p.iz;
    p.on = fmaxf(fabsf(o.x), fmaxf(fabsf(o.y), fabsf(o.z))) <= omax;
    return p;
}

CRT_HD bool hull_alive(const PNode &n, const PruneRay &p, float lim) {
    const float t0x = fmaf(n.tlo_x, p.ix, p.cx), t1x = fmaf(n.thi_x, p.ix, p.cx);
    const float t0y = fmaf(n.tlo_y, p.iy, p.cy), t1y = fmaf(n.thi_y, p.iy, p.cy);
    const float t0z = fmaf(n.tlo_z, p.iz, p.cz), t1z = fmaf(n.thi_z, p.iz, p.cz);
    const float tin = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
    const float tout = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
    return !p.on || (!(tin > lim) && !(tin > tout) && !(tout < 0.0f));
}

/* ---- hull margins (derivation: crt_scene_build.cpp) — host and device build */
CRT_HD float round_down(double v) {
    float f = (float)v;
    if ((double)f > v) f = nextafterf(f, -INFINITY);
    return f;
}
CRT_HD float round_up(double v) {
    float f = (float)v;
    if ((double)f < v) f = nextafterf(f, INFINITY);
    return f;
}

struct HullD { double lo[3], hi[3]; };

/* correctly rounded double sqrt / divide on both sides (the GPU's default
 * f64 sqrt is not guaranteed to be), so host and device builds agree bit for bit */
CRT_HD double sqrt_rn(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __dsqrt_rn(x);
#else
    return sqrt(x);
#endif
}
CRT_HD double div_rn(double a, double b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __ddiv_rn(a, b);
#else
    return a / b;
#endif
}

/* Box of one triangle widened by 2^-14 (diam * kappa + 2 G); unbounded for a
 * non-finite normal or vertex or a zero-area triangle.  Plain double
 * arithmetic in a fixed order (no contraction), identical on host and GPU. */
CRT_HD HullD triangle_hull(const float *a, const float *b, const float *c, const float *fn, double G) {
    HullD h;
    for (int k = 0; k < 3; ++k) { h.lo[k] = -(double)INFINITY; h.hi[k] = (double)INFINITY; }
    bool finite = isfinite(fn[0]) && isfinite(fn[1]) && isfinite(fn[2]);
    for (int k = 0; k < 3; ++k) finite = finite && isfinite(a[k]) && isfinite(b[k]) && isfinite(c[k]);
    if (!finite) return h;
    double e[3][3];
    for (int k = 0; k < 3; ++k) {
        e[0][k] = (double)b[k] - (double)a[k];
        e[1][k] = (double)c[k] - (double)b[k];
        e[2][k] = (double)a[k] - (double)c[k];
    }
    double len[3];
    for (int i = 0; i < 3; ++i) len[i] = sqrt_rn(e[i][0] * e[i][0] + e[i][1] * e[i][1] + e[i][2] * e[i][2]);
    const double cx = e[0][1] * (-e[2][2]) - e[0][2] * (-e[2][1]);
    const double cy = e[0][2] * (-e[2][0]) - e[0][0] * (-e[2][2]);
    const double cz = e[0][0] * (-e[2][1]) - e[0][1] * (-e[2][0]);
    const double area2 = sqrt_rn(cx * cx + cy * cy + cz * cz);   /* 2 * area */
    const double perim = len[0] + len[1] + len[2];
    if (!(area2 > 0.0) || !(perim > 0.0)) return h;
    const double inradius = div_rn(area2, perim);
    const double diam = fmax(len[0], fmax(len[1], len[2]));
    const double kappa = div_rn(diam, inradius);
    const double eta = ldexp(diam * kappa + 2.0 * G, -14);
    if (!isfinite(eta)) return h;
    for (int k = 0; k < 3; ++k) {
        const double lo = fmin((double)a[k], fmin((double)b[k], (double)c[k]));
        const double hi = fmax((double)a[k], fmax((double)b[k], (double)c[k]));
        h.lo[k] = lo - eta;
        h.hi[k] = hi + eta;
    }
    return h;
}

CRT_HD DNode cell_of(const PNode &p) {
    DNode n;
    n.lo_x = p.lo_x; n.lo_y = p.lo_y; n.lo_z = p.lo_z;
    n.hi_x = p.hi_x; n.hi_y = p.hi_y; n.hi_z = p.hi_z;
    n.a = p.a; n.b = p.b;
    return n;
}
/* Octant `oct`'s node order: each order holds node_count records plus one
 * zero record, so a walk may load the successors i+1 and skip(i) of any node
 * without a bounds check. */
CRT_HD const PNode *pnode_order(const PNode *base, int node_count, int oct) {
    return base + (size_t)oct * (size_t)(node_count + 1);
}
CRT_HD int pnode_leaf_count(const PNode &n) { return n.count; }
CRT_HD int pnode_depth(const PNode &n) { return n.depth; }

/* direction octant: bit k set iff d[k] < 0 (crt_layout.h PNode orders) */
CRT_HD int ray_octant(Vec d) { return (d.x < 0.0f ? 1 : 0) | (d.y < 0.0f ? 2 : 0) | (d.z < 0.0f ? 4 : 0); }

/* (t, slot) beats the best so far: the reference keeps the first hit found
 * with strict '<' while visiting slots in increasing order
 * (crt_intersection.cpp:100,122-125), i.e. the minimum of the key (t, slot);
 * a walk in another order reproduces it with the slot as tie-break. */
CRT_HD bool key_better(float t, int slot, float best_t, int best) {
    return best < 0 || t < best_t || (t == best_t && slot < best);
}

/* ray_intersect_triangle (crt_intersection.cpp:47-93), branch-free. */
CRT_HD bool tri_hit_bf(Vec o, Vec d, const DTriGeo &g, bool cull, float &t_out) {
    const Vec N = vec(g.nx, g.ny, g.nz);
    const Vec v0 = vec(g.v0x, g.v0y, g.v0z), v1 = vec(g.v1x, g.v1y, g.v1z), v2 = vec(g.v2x, g.v2y, g.v2z);
    const float rn = vdot(N, d);
    const float op = vdot(N, vsub(v0, o));
    const float t = op / rn;
    const Vec e0 = vsub(v1, v0), e1 = vsub(v2, v1), e2 = vsub(v0, v2);
    const Vec p = vadd(o, vscale(d, t));
    const Vec v0p = vsub(p, v0), v1p = vsub(p, v1), v2p = vsub(p, v2);
    const int ok = (int)!(fabsf(rn) < 1e-6f) & (int)((op < 0.0f) | !cull) & (int)!(t < 0.0f) &
                   (int)(vdot(N, vcross(e0, v0p)) >= 0.0f) & (int)(vdot(N, vcross(e1, v1p)) >= 0.0f) &
                   (int)(vdot(N, vcross(e2, v2p)) >= 0.0f);
    t_out = t;
    return ok != 0;
}

/* tri_hit_bf split in two: the plane stage (crt_intersection.cpp:49-63:
 * parallel, culling and behind tests, t = op / rn) and the edge stage
 * (:65-69: p = o + d*t and the three inside tests), same operations. */
CRT_HD bool tri_plane(Vec o, Vec d, const DTriGeo &g, bool cull, float &t_out) {
    const Vec N = vec(g.nx, g.ny, g.nz);
    const Vec v0 = vec(g.v0x, g.v0y, g.v0z);
    const float rn = vdot(N, d);
    const float op = vdot(N, vsub(v0, o));
    const float t = op / rn;
    t_out = t;
    return ((int)!(fabsf(rn) < 1e-6f) & (int)((op < 0.0f) | !cull) & (int)!(t < 0.0f)) != 0;
}
CRT_HD bool tri_edges(Vec o, Vec d, const DTriGeo &g, float t) {
    const Vec N = vec(g.nx, g.ny, g.nz);
    const Vec v0 = vec(g.v0x, g.v0y, g.v0z), v1 = vec(g.v1x, g.v1y, g.v1z), v2 = vec(g.v2x, g.v2y, g.v2z);
    const Vec e0 = vsub(v1, v0), e1 = vsub(v2, v1), e2 = vsub(v0, v2);
    const Vec p = vadd(o, vscale(d, t));
    const Vec v0p = vsub(p, v0), v1p = vsub(p, v1), v2p = vsub(p, v2);
    return ((int)(vdot(N, vcross(e0, v0p)) >= 0.0f) & (int)(vdot(N, vcross(e1, v1p)) >= 0.0f) &
            (int)(vdot(N, vcross(e2, v2p)) >= 0.0f)) != 0;
}

/* ray_intersect_triangle (crt_intersection.cpp:47-93), distance only.  The
 * back_face_culling flag is read (from *cull) only for back-facing candidates. */
CRT_HD bool tri_hit(Vec o, Vec d, const DTriGeo &g, const uint8_t *cull, float &t_out) {
    const Vec N = vec(g.nx, g.ny, g.nz);
    const float rn = vdot(N, d);
    if (fabsf(rn) < 1e-6f) return false;
    const Vec v0 = vec(g.v0x, g.v0y, g.v0z);
    const float op = vdot(N, vsub(v0, o));
    if (!(op < 0.0f) && *cull) return false;
    if (opposite_signs(op, rn) && fabsf(rn) < 2.0f) return false;
    const float t = op / rn;
    if (t < 0.0f) return false;
    const Vec v1 = vec(g.v1x, g.v1y, g.v1z), v2 = vec(g.v2x, g.v2y, g.v2z);
    const Vec e0 = vsub(v1, v0), e1 = vsub(v2, v1), e2 = vsub(v0, v2);
    const Vec p = vadd(o, vscale(d, t));
    const Vec v0p = vsub(p, v0), v1p = vsub(p, v1), v2p = vsub(p, v2);
    if (vdot(N, vcross(e0, v0p)) >= 0.0f && vdot(N, vcross(e1, v1p)) >= 0.0f &&
        vdot(N, vcross(e2, v2p)) >= 0.0f) {
        t_out = t;
        return true;
    }
    return false;
}

/* Per-ray pruned walk (stackless) over one octant's PNode order: a node is
 * entered iff its hull is alive for the best key so far and the reference's
 * six-face test passes on its cell — the same eligibility rule as
 * crt_intersection.cpp:116-133, so every leaf copy the reference could pick
 * and that can still win is tested.  Returns the winning slot (-1: miss). */
struct WalkCounts { uint32_t nodes, tris; };

template <bool COUNT>
CRT_HD int walk_pruned(const PNode *nodes, int n, const DTriGeo *slots, const uint8_t *cull, Vec o, Vec d,
                       const RayRcp &rr, const PruneRay &pr, float &best_t, WalkCounts &c) {
    int best = -1;
    float lim = INFINITY;
    best_t = 0.0f;
    int i = 0;
    while (i < n) {
        const PNode nd = nodes[i];
        bool pass = false;
        if (hull_alive(nd, pr, lim)) {
            pass = box_hit_r(o, d, rr, cell_of(nd));
            if (COUNT) ++c.nodes;
        }
        if (nd.b < 0) {
            i = pass ? i + 1 : nd.a;
            continue;
        }
        if (pass) {
            const int cnt = pnode_leaf_count(nd);
            for (int k = 0; k < cnt; ++k) {
                const int slot = nd.b + k;
                float t;
                if (COUNT) ++c.tris;
                if (tri_hit(o, d, slots[slot], cull + slot, t) && key_better(t, slot, best_t, best)) {
                    best_t = t;
                    best = slot;
                    lim = t;
                }
            }
        }
        ++i;
    }
    return best;
}

/* Full Intersection record of the winning triangle (crt_intersection.cpp:71-88):
 * recomputed from (ray, triangle, t) with the same operations, so it equals the
 * record the reference built when it first found this hit. */
struct HitRec {
    float t;
    Vec p, n, uv;
    float bu, bv;
    int32_t mat;
};

CRT_HD void hit_record(Vec o, Vec d, float t, const DTriGeo &g, const DTriAttr &at, const DVec4 &n0,
                       const DVec4 &n1, const DVec4 &n2, const DVec4 &t0, const DVec4 &t1, const DVec4 &t2,
                       HitRec &h) {
    const Vec v0 = vec(g.v0x, g.v0y, g.v0z), v1 = vec(g.v1x, g.v1y, g.v1z), v2 = vec(g.v2x, g.v2y, g.v2z);
    const Vec e0 = vsub(v1, v0), e2 = vsub(v0, v2);
    const Vec p = vadd(o, vscale(d, t));
    const Vec v0p = vsub(p, v0);
    const Vec v0v1 = e0, v0v2 = vneg(e2);
    const float bu = vlen(vcross(v0p, v0v2)) / vlen(vcross(v0v1, v0v2));
    const float bv = vlen(vcross(v0v1, v0p)) / vlen(vcross(v0v1, v0v2));
    h.t = t;
    h.p = p;
    if (at.mat_flags < 0) {   /* smooth shading bit */
        const Vec a = vscale(vec(n1.x, n1.y, n1.z), bu);
        const Vec b = vscale(vec(n2.x, n2.y, n2.z), bv);
        const Vec c = vscale(vec(n0.x, n0.y, n0.z), 1 - bu - bv);
        h.n = vadd(vadd(a, b), c);
    } else {
        h.n = vec(g.nx, g.ny, g.nz);
    }
    h.uv = vadd(vadd(vscale(vec(t1.x, t1.y, t1.z), bu), vscale(vec(t2.x, t2.y, t2.z), bv)),
                vscale(vec(t0.x, t0.y, t0.z), 1.0f - bu - bv));
    h.bu = bu;
    h.bv = bv;
    h.mat = at.mat_flags & 0x7fffffff;
}

/* PCG32 (crt_random.h:10-43) */
struct Pcg32 {
    uint64_t state, inc;
    CRT_HD uint32_t next() {
        const uint64_t old = state;
        state = old * 6364136223846793005ULL + inc;
        const uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        const uint32_t rot = (uint32_t)(old >> 59u);
        return (xs >> rot) | (xs << ((0u - rot) & 31u));
    }
};
CRT_HD Pcg32 make_pcg(uint32_t x, uint32_t y) {
    const uint64_t seed = ((uint64_t)x << 32) | y;
    Pcg32 g;
    g.state = 0;
    g.inc = (seed << 1) | 1;
    (void)g.next();
    g.state += seed;
    (void)g.next();
    return g;
}
/* uniform() = bits(0x3f800000 | r>>9) - 1.0f = (r>>9) * 2^-23 exactly: the
 * mantissa index m = r >> 9 addresses the host-computed sin/cos tables. */

/* x86 cvttss2si semantics for the reference's static_cast<int>(float)
 * (out of range / NaN → INT_MIN) */
CRT_HD int trunc_x86(float f) {
    if (f >= -2147483648.0f && f < 2147483648.0f) return (int)f;
    return (int)0x80000000;
}

/* Texture::sample (crt_texture.cpp:9-49) */
CRT_HD Vec sample_texture(const DTexture &tx, const DVec4 *texels, Vec uv, float bu, float bv) {
    switch (tx.type) {
    case 0: return vec(tx.c0x, tx.c0y, tx.c0z);
    case 1:
        if (bu <= tx.scalar || bv <= tx.scalar || (1.0f - bu - bv) <= tx.scalar) return vec(tx.c0x, tx.c0y, tx.c0z);
        return vec(tx.c1x, tx.c1y, tx.c1z);
    case 2: {
        const int row = trunc_x86(uv.x / tx.scalar);
        const int col = trunc_x86(uv.y / tx.scalar);
        return ((row + col) & 1) ? vec(tx.c1x, tx.c1y, tx.c1z) : vec(tx.c0x, tx.c0y, tx.c0z);
    }
    default: {
        int rx = trunc_x86(uv.x * tx.w) % tx.w;
        int ry = trunc_x86((1.0f - uv.y) * tx.h) % tx.h;
        if (rx < 0) rx += tx.w;   /* the reference indexes out of bounds here (UB) */
        if (ry < 0) ry += tx.h;
        const DVec4 t = texels[tx.texel_offset + (int64_t)ry * tx.w + rx];
        return vec(t.x, t.y, t.z);
    }
    }
}

}  // namespace crt_amd
