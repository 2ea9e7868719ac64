/*
 * crt_bvh_build.cpp — host build of the secondary-ray BVH (crt_bvh.h,
 * crt_layout.h BNode).
 *
 * The BVH is an acceleration structure of our own, next to the reference's
 * tree, not a replacement of it: scattered rays find their closest triangle
 * through it and then prove on the reference's tree that the reference
 * reaches that triangle (crt_bvh.h).  So its shape is free and only its
 * boxes carry the exactness argument: every box is the union, rounded
 * outwards, of the conservative hulls of the triangles below it
 * (crt_device.h triangle_hull, the same hulls as the pruned kd walks'), so a
 * box the ray misses before `lim` holds no triangle the reference's test
 * could accept at t <= lim.
 *
 * Shape: binned SAH (16 bins over triangle centroids, surface areas of the
 * triangles' own boxes), leaves of at most kLeafMax triangles; every triangle
 * once.  Stored once per direction octant (8 orders) in preorder with the
 * near child first along the node's split axis, with skip links, so the walk
 * is stackless.
 */
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <limits>
#include <thread>
#include <vector>

#include "crt_bins.h"
#include "crt_bvh.h"
#include "crt_device.h"
#include "crt_host.h"

namespace crt_amd {

namespace {

constexpr int kLeafMax = 2;     /* triangles per leaf (15-01/scene2 GI rays: ~15 box + ~3.3 triangle tests) */
constexpr int kBins = 16;
constexpr int kMaxDepth = 48;   /* deeper subtrees are split at the median index */

struct Aabb {
    float lo[3], hi[3];
};

Aabb aabb_empty() {
    const float inf = std::numeric_limits<float>::infinity();
    return Aabb{{inf, inf, inf}, {-inf, -inf, -inf}};
}

void grow(Aabb &a, const Aabb &b) {
    for (int k = 0; k < 3; ++k) {
        a.lo[k] = std::min(a.lo[k], b.lo[k]);
        a.hi[k] = std::max(a.hi[k], b.hi[k]);
    }
}

double area(const Aabb &a) {
    const double dx = (double)a.hi[0] - a.lo[0], dy = (double)a.hi[1] - a.lo[1], dz = (double)a.hi[2] - a.lo[2];
    if (!(dx >= 0.0) || !(dy >= 0.0) || !(dz >= 0.0)) return 0.0;
    return 2.0 * (dx * dy + dy * dz + dz * dx);
}

struct Build {
    int32_t left = -1, right = -1;   /* children (build numbering) */
    int32_t axis = 0;
    int32_t first = 0, count = 0;    /* leaf: range of `order` */
    HullD hull;
};

}  // namespace

int build_bvh(HostScene &hs) {
    hs.bnodes.clear();
    hs.btri.clear();
    hs.btri_id.clear();
    const int32_t nt = (int32_t)hs.tri_attr.size();
    if (nt == 0) return CRT_OK;
    const double G = hs.prune_G;

    std::vector<Aabb> box((size_t)nt);
    std::vector<float> cen((size_t)nt * 3);
    std::vector<HullD> hull((size_t)nt);
    for (int32_t t = 0; t < nt; ++t) {
        const DTriAttr &at = hs.tri_attr[t];
        const float *v[3] = {&hs.vpos[3 * (size_t)at.i0], &hs.vpos[3 * (size_t)at.i1], &hs.vpos[3 * (size_t)at.i2]};
        Aabb b = aabb_empty();
        bool finite = true;
        for (int k = 0; k < 3; ++k)
            for (int j = 0; j < 3; ++j) {
                finite = finite && std::isfinite(v[j][k]);
                b.lo[k] = std::min(b.lo[k], v[j][k]);
                b.hi[k] = std::max(b.hi[k], v[j][k]);
            }
        if (!finite) b = Aabb{{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};   /* shape only; its hull is unbounded */
        box[t] = b;
        for (int k = 0; k < 3; ++k) cen[3 * (size_t)t + k] = 0.5f * (b.lo[k] + b.hi[k]);
        hull[t] = triangle_hull(v[0], v[1], v[2], &hs.face_normal[3 * (size_t)t], G);
    }

    std::vector<int32_t> order((size_t)nt);
    for (int32_t t = 0; t < nt; ++t) order[t] = t;
    std::vector<Build> nodes;
    nodes.reserve((size_t)nt * 2 / kLeafMax + 2);
    struct Work { int32_t node, lo, hi, depth; };
    std::vector<Work> st;
    nodes.push_back(Build{});
    st.push_back(Work{0, 0, nt, 0});
    while (!st.empty()) {
        const Work w = st.back();
        st.pop_back();
        const int32_t cnt = w.hi - w.lo;
        Aabb cb = aabb_empty();
        for (int32_t i = w.lo; i < w.hi; ++i) {
            const int32_t t = order[i];
            Aabb c{{cen[3 * t], cen[3 * t + 1], cen[3 * t + 2]}, {cen[3 * t], cen[3 * t + 1], cen[3 * t + 2]}};
            grow(cb, c);
        }
        if (cnt <= kLeafMax) {
            nodes[w.node].first = w.lo;
            nodes[w.node].count = cnt;
            continue;
        }
        int best_axis = -1, best_split = -1;
        double best_cost = std::numeric_limits<double>::infinity();
        if (w.depth < kMaxDepth) {
            for (int ax = 0; ax < 3; ++ax) {
                const float ext = cb.hi[ax] - cb.lo[ax];
                if (!(ext > 0.f)) continue;
                Aabb bins[kBins];
                int32_t bc[kBins] = {0};
                for (auto &b : bins) b = aabb_empty();
                for (int32_t i = w.lo; i < w.hi; ++i) {
                    const int32_t t = order[i];
                    const int k = std::min(kBins - 1, (int)((cen[3 * t + ax] - cb.lo[ax]) / ext * kBins));
                    ++bc[k];
                    grow(bins[k], box[t]);
                }
                for (int s = 1; s < kBins; ++s) {
                    Aabb l = aabb_empty(), r = aabb_empty();
                    int32_t nl = 0, nr = 0;
                    for (int k = 0; k < s; ++k) { grow(l, bins[k]); nl += bc[k]; }
                    for (int k = s; k < kBins; ++k) { grow(r, bins[k]); nr += bc[k]; }
                    if (nl == 0 || nr == 0) continue;
                    const double c = area(l) * nl + area(r) * nr;
                    if (c < best_cost) {
                        best_cost = c;
                        best_axis = ax;
                        best_split = s;
                    }
                }
            }
        }
        int32_t mid;
        int axis = 0;
        if (best_axis >= 0) {
            axis = best_axis;
            const float ext = cb.hi[axis] - cb.lo[axis];
            const auto it = std::stable_partition(order.begin() + w.lo, order.begin() + w.hi, [&](int32_t t) {
                return std::min(kBins - 1, (int)((cen[3 * t + axis] - cb.lo[axis]) / ext * kBins)) < best_split;
            });
            mid = (int32_t)(it - order.begin());
        } else {
            /* coincident centroids (or too deep): halves by index along the widest axis */
            for (int k = 1; k < 3; ++k)
                if (cb.hi[k] - cb.lo[k] > cb.hi[axis] - cb.lo[axis]) axis = k;
            mid = w.lo + cnt / 2;
            std::stable_sort(order.begin() + w.lo, order.begin() + w.hi,
                             [&](int32_t a, int32_t b) { return cen[3 * a + axis] < cen[3 * b + axis]; });
        }
        if (mid <= w.lo || mid >= w.hi) mid = w.lo + cnt / 2;
        const int32_t l = (int32_t)nodes.size(), r = l + 1;
        nodes.push_back(Build{});
        nodes.push_back(Build{});
        nodes[w.node].left = l;
        nodes[w.node].right = r;
        nodes[w.node].axis = axis;
        st.push_back(Work{r, mid, w.hi, w.depth + 1});
        st.push_back(Work{l, w.lo, mid, w.depth + 1});
    }
    const int32_t n = (int32_t)nodes.size();
    if ((int64_t)nt * 16 >= (int64_t)std::numeric_limits<int32_t>::max())
        return set_error(CRT_E_UNSUPPORTED, "too many triangles for the BVH leaf record");

    /* hulls bottom up: children are numbered after their parent */
    const double inf = std::numeric_limits<double>::infinity();
    for (int32_t x = n - 1; x >= 0; --x) {
        HullD h{{inf, inf, inf}, {-inf, -inf, -inf}};
        auto merge = [&](const HullD &o) {
            for (int k = 0; k < 3; ++k) {
                h.lo[k] = std::min(h.lo[k], o.lo[k]);
                h.hi[k] = std::max(h.hi[k], o.hi[k]);
            }
        };
        if (nodes[x].left < 0) {
            for (int32_t i = 0; i < nodes[x].count; ++i) merge(hull[order[nodes[x].first + i]]);
        } else {
            merge(nodes[nodes[x].left].hull);
            merge(nodes[nodes[x].right].hull);
        }
        nodes[x].hull = h;
    }
    std::vector<int32_t> subtree((size_t)n, 1);
    for (int32_t x = n - 1; x >= 0; --x)
        if (nodes[x].left >= 0) subtree[x] += subtree[nodes[x].left] + subtree[nodes[x].right];

    /* triangles in leaf order, geometry exactly as the leaf slots hold it */
    hs.btri.resize((size_t)nt);
    hs.btri_id.resize((size_t)nt);
    for (int32_t i = 0; i < nt; ++i) {
        const int32_t t = order[i];
        const DTriAttr &at = hs.tri_attr[t];
        DTriGeo g;
        g.v0x = hs.vpos[3 * (size_t)at.i0]; g.v0y = hs.vpos[3 * (size_t)at.i0 + 1]; g.v0z = hs.vpos[3 * (size_t)at.i0 + 2];
        g.v1x = hs.vpos[3 * (size_t)at.i1]; g.v1y = hs.vpos[3 * (size_t)at.i1 + 1]; g.v1z = hs.vpos[3 * (size_t)at.i1 + 2];
        g.v2x = hs.vpos[3 * (size_t)at.i2]; g.v2y = hs.vpos[3 * (size_t)at.i2 + 1]; g.v2z = hs.vpos[3 * (size_t)at.i2 + 2];
        g.nx = hs.face_normal[3 * (size_t)t]; g.ny = hs.face_normal[3 * (size_t)t + 1]; g.nz = hs.face_normal[3 * (size_t)t + 2];
        hs.btri[i] = g;
        hs.btri_id[i] = t | (hs.tri_cull[t] ? (int32_t)0x80000000 : 0);
    }

    hs.bnodes.assign((size_t)8 * (n + 1), BNode{});   /* + one zero record per order */
    std::vector<int32_t> st2;
    for (int oct = 0; oct < 8; ++oct) {
        BNode *out = hs.bnodes.data() + (size_t)oct * (n + 1);
        int32_t k = 0;
        st2.assign(1, 0);
        while (!st2.empty()) {
            const int32_t x = st2.back();
            st2.pop_back();
            const Build &b = nodes[x];
            BNode &o = out[k];
            o.lo_x = round_down(b.hull.lo[0]); o.lo_y = round_down(b.hull.lo[1]); o.lo_z = round_down(b.hull.lo[2]);
            o.hi_x = round_up(b.hull.hi[0]); o.hi_y = round_up(b.hull.hi[1]); o.hi_z = round_up(b.hull.hi[2]);
            o.skip = k + subtree[x];
            if (b.left < 0) {
                o.leaf = b.first * 16 + b.count;
            } else {
                o.leaf = 0;
                /* near child first: the right child holds the larger centroids
                 * along the split axis, entered first by a ray going down it */
                const bool neg = ((oct >> b.axis) & 1) != 0;
                st2.push_back(neg ? b.left : b.right);
                st2.push_back(neg ? b.right : b.left);
            }
            ++k;
        }
    }
    hs.bnode_count = n;
    return CRT_OK;
}

/* Topology records of the proof (crt_layout.h KTopo) over the flattened
 * reference-order tree (interior node i: first child i + 1, second child, if
 * any, where the first one's subtree ends, before skip(i) = a).  Each child's
 * cell is checked to be its parent's half as verify_topo recomputes it. */
int build_proof_tables(HostScene &hs) {
    const std::vector<DNode> &nodes = hs.nodes;
    const int32_t n = (int32_t)nodes.size();
    hs.ktopo.assign((size_t)n, KTopo{0, 0});
    for (int32_t i = 0; i < n; ++i) {
        const DNode &nd = nodes[(size_t)i];
        KTopo &t = hs.ktopo[(size_t)i];
        if (nd.b >= 0) {
            t.a = node_leaf_count(nd);
            t.b = nd.b;
            continue;
        }
        const int32_t c1 = i + 1;
        if (c1 >= nd.a) {   /* childless interior node (the empty scene's root): a leaf without copies */
            t.a = 0;
            t.b = 0;
            continue;
        }
        const DNode &n1 = nodes[(size_t)c1];
        const int32_t c2 = n1.b < 0 ? n1.a : c1 + 1;
        const int axis = node_depth(nd) % 3;
        DNode lo_half = nd, hi_half = nd;
        topo_halves(nd, axis, lo_half, hi_half);
        const bool first_lo = cell_equal(n1, lo_half);
        bool ok = first_lo || cell_equal(n1, hi_half);
        if (c2 < nd.a) ok = ok && cell_equal(nodes[(size_t)c2], first_lo ? hi_half : lo_half);
        if (!ok) {
            hs.ktopo.clear();   /* not the reference's halving: the proof descends the nodes (verify_kd) */
            hs.ktopo2.clear();
            return CRT_OK;
        }
        t.a = c2 < nd.a ? c2 : -1;
        t.b = first_lo ? -1 : -2;
    }
    /* two levels a record (crt_layout.h KTopo2) */
    hs.ktopo2.assign((size_t)n, KTopo2{});
    for (int32_t i = 0; i < n; ++i) {
        int32_t idx[8];
        idx[1] = i;
        for (int q = 2; q < 8; ++q) {
            const int32_t par = idx[q >> 1];
            int32_t c = -1;
            if (par >= 0 && hs.ktopo[(size_t)par].b < 0) c = (q & 1) ? hs.ktopo[(size_t)par].a : par + 1;
            idx[q] = c;
            hs.ktopo2[(size_t)i].t[q - 2] = c >= 0 ? hs.ktopo[(size_t)c] : KTopo{0, 0};
        }
    }
    return CRT_OK;
}

/* Camera bins (crt_bins.h): the host restatement of the device binning
 * (crt_bins.hip), used as its checker and by the CPU walk checks. */
bool bin_camera(const HostScene &hs, BinCamera &cam) {
    if (hs.tri_attr.empty()) return false;
    return bin_camera_of(host_camera(hs), hs.prune_origin_max, cam);
}

bool bin_camera_of(const DCamera &c, float prune_origin_max, BinCamera &cam) {
    const int W = c.width, H = c.height;
    if (W <= 0 || H <= 0) return false;
    for (int k = 0; k < 3; ++k) {
        cam.o[k] = c.loc[k];
        if (!(std::fabs(cam.o[k]) <= (double)prune_origin_max)) return false;
    }
    double M[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) M[i][j] = c.rot[3 * i + j];
    const double det = M[0][0] * (M[1][1] * M[2][2] - M[1][2] * M[2][1]) -
                       M[0][1] * (M[1][0] * M[2][2] - M[1][2] * M[2][0]) +
                       M[0][2] * (M[1][0] * M[2][1] - M[1][1] * M[2][0]);
    if (!std::isfinite(det) || !(std::fabs(det) > 1e-12)) return false;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            const int i1 = (j + 1) % 3, i2 = (j + 2) % 3, j1 = (i + 1) % 3, j2 = (i + 2) % 3;
            cam.Mi[i][j] = (M[i1][j1] * M[i2][j2] - M[i1][j2] * M[i2][j1]) / det;
        }
    cam.sx = (double)c.aspect * (double)c.tan_half_fov;
    cam.sy = c.tan_half_fov;
    if (!(cam.sx > 0.0) || !(cam.sy > 0.0) || !std::isfinite(cam.sx) || !std::isfinite(cam.sy)) return false;
    cam.W = W;
    cam.H = H;
    cam.tx = (W + 7) / 8;
    cam.ty = (H + 7) / 8;
    return true;
}

void bin_templates_range(const HostScene &hs, std::vector<CamCand> &tpl, int32_t t0, int32_t t1);

/* Per triangle: its hull box (crt_device.h triangle_hull, rounded outwards),
 * id | culling << 31 and geometry as the BVH's triangle arrays hold them; the
 * per-frame fields (dmin, mask, rest) zero. */
void bin_templates(const HostScene &hs, std::vector<CamCand> &tpl) {
    const int32_t nt = (int32_t)hs.tri_attr.size();
    tpl.assign((size_t)nt, CamCand{});
    /* independent per triangle: large scenes (C5: 1 M triangles, ~50 ms of
     * f64 hulls) on several threads */
    const int nth = nt < 65536 ? 1 : (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> pool;
    for (int k = 1; k < nth; ++k)
        pool.emplace_back([&, k]() { bin_templates_range(hs, tpl, (int32_t)((int64_t)nt * k / nth),
                                                         (int32_t)((int64_t)nt * (k + 1) / nth)); });
    bin_templates_range(hs, tpl, 0, (int32_t)((int64_t)nt / nth));
    for (auto &th : pool) th.join();
}

void bin_templates_range(const HostScene &hs, std::vector<CamCand> &tpl, int32_t t0, int32_t t1) {
    for (int32_t t = t0; t < t1; ++t) {
        const DTriAttr &at = hs.tri_attr[t];
        const float *v[3] = {&hs.vpos[3 * (size_t)at.i0], &hs.vpos[3 * (size_t)at.i1], &hs.vpos[3 * (size_t)at.i2]};
        const HullD hd = triangle_hull(v[0], v[1], v[2], &hs.face_normal[3 * (size_t)t], hs.prune_G);
        CamCand &c = tpl[(size_t)t];
        c.lo_x = round_down(hd.lo[0]); c.lo_y = round_down(hd.lo[1]); c.lo_z = round_down(hd.lo[2]);
        c.hi_x = round_up(hd.hi[0]); c.hi_y = round_up(hd.hi[1]); c.hi_z = round_up(hd.hi[2]);
        c.id = t | (hs.tri_cull[t] ? (int32_t)0x80000000 : 0);
        c.g.v0x = v[0][0]; c.g.v0y = v[0][1]; c.g.v0z = v[0][2];
        c.g.v1x = v[1][0]; c.g.v1y = v[1][1]; c.g.v1z = v[1][2];
        c.g.v2x = v[2][0]; c.g.v2y = v[2][1]; c.g.v2z = v[2][2];
        c.g.nx = hs.face_normal[3 * (size_t)t]; c.g.ny = hs.face_normal[3 * (size_t)t + 1];
        c.g.nz = hs.face_normal[3 * (size_t)t + 2];
    }
}

int build_camera_bins(const HostScene &hs, std::vector<CamCand> &bins, std::vector<int32_t> &off,
                      std::vector<uint8_t> *over) {
    bins.clear();
    off.clear();
    if (over) over->clear();
    BinCamera cam;
    if (!bin_camera(hs, cam)) return CRT_OK;
    const int32_t nt = (int32_t)hs.tri_attr.size();
    const int tx = cam.tx, ty = cam.ty;
    const int64_t ncell = (int64_t)tx * ty;
    std::vector<CamCand> tpl;
    bin_templates(hs, tpl);
    std::vector<BinItem> items((size_t)nt);
    int everywhere = 0;
    for (int32_t t = 0; t < nt; ++t) {
        const CamCand &c = tpl[(size_t)t];
        const float lo[3] = {c.lo_x, c.lo_y, c.lo_z}, hi[3] = {c.hi_x, c.hi_y, c.hi_z};
        items[(size_t)t] = bin_project(lo, hi, cam);
        if (items[(size_t)t].every && ++everywhere > kBinMaxEverywhere) return CRT_OK;
    }
    /* cell lists in triangle order, then a stable sort by dmin: ordered by (dmin, id) */
    std::vector<int64_t> cnt((size_t)ncell, 0);
    for (const BinItem &it : items)
        if (it.px0 <= it.px1)
            for (int32_t y = it.py0 / 8; y <= it.py1 / 8; ++y)
                for (int32_t x = it.px0 / 8; x <= it.px1 / 8; ++x) ++cnt[(size_t)y * tx + x];
    std::vector<uint8_t> ov((size_t)ncell, 0);
    int64_t total = 0;
    for (int64_t c = 0; c < ncell; ++c) {
        if (cnt[(size_t)c] > kBinCellCap) ov[(size_t)c] = 1;   /* this cell's pixels walk the BVH */
        else total += cnt[(size_t)c];
    }
    int64_t mean_cap = kBinMeanCap;   /* the device's cap (crt_api.hip; A/B builds: env CRT_BINS_MEAN_CAP) */
#ifdef CRT_AB_OPTIONS
    if (const char *e = std::getenv("CRT_BINS_MEAN_CAP")) mean_cap = std::max<int64_t>(1, std::atoll(e));
#endif
    if (total > mean_cap * ncell || total >= (int64_t)std::numeric_limits<int32_t>::max()) return CRT_OK;
    off.assign((size_t)ncell + 1, 0);
    for (int64_t c = 0; c < ncell; ++c) off[(size_t)c + 1] = off[(size_t)c] + (ov[(size_t)c] ? 0 : (int32_t)cnt[(size_t)c]);
    bins.resize((size_t)total);
    std::vector<int32_t> fill(off.begin(), off.end() - 1);
    for (int32_t t = 0; t < nt; ++t) {
        const BinItem &it = items[(size_t)t];
        if (it.px0 > it.px1) continue;
        for (int32_t y = it.py0 / 8; y <= it.py1 / 8; ++y)
            for (int32_t x = it.px0 / 8; x <= it.px1 / 8; ++x) {
                const size_t cell = (size_t)y * tx + x;
                if (ov[cell]) continue;
                CamCand &c = bins[(size_t)fill[cell]++];
                c = tpl[(size_t)t];
                c.dmin = it.dmin;
                c.mask = bin_mask(it, x, y);
            }
    }
    for (int64_t c = 0; c < ncell; ++c) {
        const auto b = bins.begin() + off[(size_t)c], e = bins.begin() + off[(size_t)c + 1];
        std::stable_sort(b, e, [](const CamCand &u, const CamCand &v) { return u.dmin < v.dmin; });
        uint64_t r = 0;
        for (auto q = e; q != b;) {
            --q;
            r |= q->mask;
            q->rest = r;
        }
    }
    if (over) over->swap(ov);
    return CRT_OK;
}

}  // namespace crt_amd
