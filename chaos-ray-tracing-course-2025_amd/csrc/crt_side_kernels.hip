/*
 * crt_side_kernels.hip — the small kernels around the render: the trace hook
 * (crt_hip_trace_batch), shard unpack, live-pixel mask of compact shards and
 * write_ppm's quantisation (crt_image_ppm.cpp:15-18).
 */
#define CRT_KERNEL_TU 1
#include "crt_kernels.h"
#include "crt_shade.h"

namespace crt_amd {

/* crt_hip_trace_batch: closest hit of arbitrary rays (a1–a4 KATs). */
__global__ __launch_bounds__(256) void k_trace_rays(DeviceScene s, const float *__restrict__ rays, int64_t n,
                                                    crt_hit *__restrict__ hits, int walk) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Vec o = vec(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]);
    const Vec d = vec(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
    LaneCounts cnt;
    float t;
    const int slot = walk == 2 && s.bnodes ? trace_lane_bvh<false>(s, true, o, d, t, cnt)
                     : walk >= 1 ? trace_lane_pruned<false>(s, true, o, d, t, cnt) : trace_closest<false>(s, o, d, t, cnt);
    crt_hit r;
    r.distance = 0.f;
    r.point[0] = r.point[1] = r.point[2] = 0.f;
    r.normal[0] = r.normal[1] = r.normal[2] = 0.f;
    r.uv[0] = r.uv[1] = r.uv[2] = 0.f;
    r.bary_u = r.bary_v = 0.f;
    r.material_index = 0;
    r.hit = 0;
    r.triangle_index = -1;
    if (slot >= 0) {
        HitRec h;
        int32_t tri;
        make_hit(s, o, d, t, slot, h, &tri);
        r.distance = h.t;
        r.point[0] = h.p.x; r.point[1] = h.p.y; r.point[2] = h.p.z;
        r.normal[0] = h.n.x; r.normal[1] = h.n.y; r.normal[2] = h.n.z;
        r.uv[0] = h.uv.x; r.uv[1] = h.uv.y; r.uv[2] = h.uv.z;
        r.bary_u = h.bu; r.bary_v = h.bv;
        r.material_index = h.mat;
        r.hit = 1;
        r.triangle_index = tri;
    }
    hits[i] = r;
}

/* Scatter gathered shard buffers back into the row-major frame (fp32 RGB or
 * the quantised 8-bit RGB of k_quantize). */
template <class T>
__global__ __launch_bounds__(256) void k_unpack(const UnpackBucket *__restrict__ buckets, const T *__restrict__ src,
                                                T *__restrict__ dst, int width, Rgb<T> bg) {
    const UnpackBucket b = buckets[blockIdx.x];
    const int npx = b.w * b.h;
    for (int p = (int)threadIdx.x; p < npx; p += (int)blockDim.x) {
        const int lx = p % b.w, ly = p / b.w;
        T *d = dst + 3 * ((int64_t)(b.y + ly) * width + (b.x + lx));
        if (b.src < 0) {   /* dead tile of a compact shard: the background (shade_ray's miss colour) */
            d[0] = bg.c[0];
            d[1] = bg.c[1];
            d[2] = bg.c[2];
        } else {
            const T *s = src + b.src + 3 * (int64_t)p;
            d[0] = s[0];
            d[1] = s[1];
            d[2] = s[2];
        }
    }
}

/* One device scene record into its ring slot (sync_device_record): the
 * record is this launch's by-value argument, so the write is ordered on the
 * launch's stream like any kernel. */
__global__ void k_put_record(DeviceScene *__restrict__ dst, DeviceScene v) {
    if (threadIdx.x == 0) *dst = v;
}

/* Live pixels for the compact shards: the camera ray passes the reference's
 * six-face test on the root cell (crt_intersection.cpp:14-45, node 0 popped
 * first, :114-121).  A ray that fails it is a miss, i.e. shade_ray returns the
 * background colour (crt_renderer.cpp:142-144) — so dead pixels need neither
 * rendering nor transport. */
__global__ __launch_bounds__(256) void k_live_pixels(const DeviceScene *__restrict__ scene, uint8_t *__restrict__ live) {
    const DeviceScene &s = *scene;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)s.cam.width * s.cam.height) return;
    const int x = (int)(i % s.cam.width), y = (int)(i / s.cam.width);
    Vec o, d;
    camera_ray(s.cam, x, y, o, d);
    bool hit = false;
    if (s.node_count > 0) {
        const RayRcp rr = make_ray_rcp(o, d, s.planes_ok != 0);
        hit = box_hit_r(o, d, rr, load_global(s.nodes, 0));
    }
    live[i] = hit ? 1 : 0;
}

/* write_ppm's per-component conversion (crt_image_ppm.cpp:15-18):
 * clamp(static_cast<int>(c * max), 0, max), with x86 cvttss2si semantics for
 * the cast (NaN / out of range -> INT_MIN -> 0).  Four components per thread:
 * 16-B loads, one 4-B store (HBM-bound: 5 B moved per component). */
__global__ __launch_bounds__(256) void k_quantize(const float *__restrict__ src, uint8_t *__restrict__ dst, int64_t n,
                                                  float maxf, int maxi) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t i = 4 * q;
    if (i >= n) return;
    auto cv = [&](float c) -> uint32_t {
        int v = trunc_x86(c * maxf);
        v = v < 0 ? 0 : (v > maxi ? maxi : v);
        return (uint32_t)v;
    };
    if (i + 4 <= n && ((reinterpret_cast<uintptr_t>(src + i) & 15u) == 0) &&
        ((reinterpret_cast<uintptr_t>(dst + i) & 3u) == 0)) {
        const float4 c = *reinterpret_cast<const float4 *>(src + i);
        const uint32_t w = cv(c.x) | (cv(c.y) << 8) | (cv(c.z) << 16) | (cv(c.w) << 24);
        *reinterpret_cast<uint32_t *>(dst + i) = w;
    } else {
        for (int64_t k = i; k < n && k < i + 4; ++k) dst[k] = (uint8_t)cv(src[k]);
    }
}

/* The compact image copy (crt_api.hip image_to_host), first kernel, one block
 * a row: the row's first and last pixel whose bits differ from the
 * background's, so every pixel outside [x0, x1) is the background bit for
 * bit, for every renderer (NaN included).  The span goes to the device list
 * (k_rows_to_host reads it) and to the row's pinned host record (the host
 * writes the background outside it once this kernel's end is signalled). */
__global__ __launch_bounds__(256) void k_row_spans(const float *__restrict__ img, int width, Rgb<uint32_t> bg,
                                                   int2 *__restrict__ spans, HostRow *__restrict__ rows) {
    __shared__ int lo, hi;
    if (threadIdx.x == 0) {
        lo = width;
        hi = -1;
    }
    __syncthreads();
    const int y = (int)blockIdx.x;
    const int64_t n = 3 * (int64_t)width;
    const uint32_t *row = reinterpret_cast<const uint32_t *>(img) + (int64_t)y * n;
    int mylo = width, myhi = -1;
    if ((n & 3) == 0) {   /* rows of whole 16-B words (hipMalloc'd image) */
        const uint4 *r4 = reinterpret_cast<const uint4 *>(row);
        for (int64_t q = threadIdx.x; q < n / 4; q += blockDim.x) {
            const uint4 v = r4[q];
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
            for (int k = 0; k < 4; ++k) {
                const int64_t i = 4 * q + k;
                if (w[k] != bg.c[i % 3]) {
                    const int px = (int)(i / 3);
                    mylo = min(mylo, px);
                    myhi = max(myhi, px);
                }
            }
        }
    } else {
        for (int64_t i = threadIdx.x; i < n; i += blockDim.x)
            if (row[i] != bg.c[i % 3]) {
                const int px = (int)(i / 3);
                mylo = min(mylo, px);
                myhi = max(myhi, px);
            }
    }
    for (int s = 32; s > 0; s >>= 1) {
        mylo = min(mylo, __shfl_xor(mylo, s));
        myhi = max(myhi, __shfl_xor(myhi, s));
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMin(&lo, mylo);
        atomicMax(&hi, myhi);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const int x0 = hi < 0 ? 0 : lo, x1 = hi < 0 ? 0 : hi + 1;
        spans[y] = make_int2(x0, x1);
        rows[y].x0 = x0;
        rows[y].x1 = x1;
    }
}

/* ... second kernel, one block a row: the row's span written straight into
 * host memory (`host`: the caller's pinned image or the pinned staging image,
 * same layout), widened to whole 16-B words of host memory (PCIe carries
 * 16-B stores far better than 4-B ones).  Any float the widening adds gets
 * its own correct value — the one the host writes there too if it writes it
 * at all (the background, outside a span) — so the order of the two writers
 * does not matter.  Only the spans cross PCIe. */
__global__ __launch_bounds__(256) void k_rows_to_host(const float *__restrict__ img, int width, int height, int y0,
                                                      const int2 *__restrict__ spans, float *__restrict__ host) {
    const int y = y0 + (int)blockIdx.x;   /* a launch takes a band of rows from y0 */
    const int2 sp = spans[y];
    if (sp.y <= sp.x) return;
    const int64_t n = 3 * (int64_t)width, total = n * (int64_t)height;
    int64_t a = (int64_t)y * n + 3 * (int64_t)sp.x, b = (int64_t)y * n + 3 * (int64_t)sp.y;
    if ((reinterpret_cast<uintptr_t>(host) & 15) == 0) {   /* host and img both 16-B aligned at multiples of 4 floats */
        a &= ~(int64_t)3;
        b = min((b + 3) & ~(int64_t)3, total);
        const int64_t q1 = b >> 2;
        const float4 *s4 = reinterpret_cast<const float4 *>(img);
        float4 *d4 = reinterpret_cast<float4 *>(host);
        for (int64_t q = (a >> 2) + threadIdx.x; q < q1; q += blockDim.x) d4[q] = s4[q];
        for (int64_t i = (q1 << 2) + threadIdx.x; i < b; i += blockDim.x) host[i] = img[i];
    } else {
        for (int64_t i = a + threadIdx.x; i < b; i += blockDim.x) host[i] = img[i];
    }
}

template __global__ void k_unpack<float>(const UnpackBucket *__restrict__, const float *__restrict__,
                                         float *__restrict__, int, Rgb<float>);
template __global__ void k_unpack<uint8_t>(const UnpackBucket *__restrict__, const uint8_t *__restrict__,
                                           uint8_t *__restrict__, int, Rgb<uint8_t>);

/* empty kernel: its launch at scene creation loads this TU's code object
 * (warm_code_objects) */
__global__ void k_warm_side() {}

}  // namespace crt_amd
