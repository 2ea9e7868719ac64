/*
 * crt_render_gi.hip — GI frames (15-01/scene2, C4): the per-lane state
 * machine over the BVH walk (crt_gi_machine.h, the default) and the older
 * frame-stack kernel with pixel refill over the cooperative walks (option
 * gi_machine 0, and settings beyond the machine's limits).  Built with its
 * own LLVM scheduling strategy (Makefile GI_SCHED).
 */
#define CRT_KERNEL_TU 1
#include "crt_kernels.h"
#include "crt_shade.h"
#include "crt_gi_machine.h"

namespace crt_amd {

/* Frame-stack kernel with pixel refill (GI frames, cooperative walk).  A
 * persistent grid of waves pulls pixels from the tile list in plan order
 * (one global counter, one atomic per wave and pass): a lane whose pixel is
 * finished takes the next one at the top of the following pass, so a wave no
 * longer waits for its tile's longest pixel with the other lanes idle.  Every
 * pixel runs exactly shade_pixel's sequence (camera ray, PCG seeded by (x, y),
 * the same passes), so the image bits do not depend on which lane or wave
 * renders it.  Lanes without a pixel stay in the walk calls as helpers (they
 * take donated pieces); the wave leaves when the list is exhausted and none
 * of its lanes holds a pixel. */
template <int MAXF, int TRAV, bool COUNT>
__global__ CRT_RENDER_BOUNDS __attribute__((amdgpu_waves_per_eu(MAXF == 4 ? (TRAV == 10 ? CRT_GI10_WAVES : CRT_GI_WAVES) : 1))) void k_render_refill(
    const DeviceScene *__restrict__ scene, DSettings st, const Tile *__restrict__ tiles, int ntiles,
    float *__restrict__ out, int32_t *__restrict__ next_px, unsigned long long *__restrict__ counters) {
    const int lane = (int)(threadIdx.x & 63);
    const DeviceScene &s = *scene;
    const int total = ntiles * 64;   /* pixel slots: tile k, lane j -> (j & 7, j >> 3) inside tile k */
    const unsigned long long lt = (1ull << lane) - 1ull;
    __shared__ CoopLds coop[kIsCoop<TRAV> ? 4 : 1];
    CoopLds *L = &coop[kIsCoop<TRAV> ? (threadIdx.x >> 6) : 0];
    LaneCounts cnt = {};
    bool has = false, dry = false;
    int64_t opx = 0;
    Vec o = vec(0.f, 0.f, 0.f), d = vec(0.f, 0.f, 1.f), col = vec(0.f, 0.f, 0.f);
    uint32_t depth = 0;
    Pcg32 rng = make_pcg(0u, 0u);
    Frame stack[MAXF];
    int sp = 0;
    for (;;) {
        /* ---- lanes without a pixel take the next slots of the list ---- */
        const unsigned long long need = __ballot(!has && !dry);
        if (need != 0ull) {
            const int leader = __ffsll((long long)need) - 1;
            int base = 0;
            if (lane == leader) base = atomicAdd(next_px, __popcll(need));
            base = __shfl(base, leader);
            if (!has && !dry) {
                const int k = base + __popcll(need & lt);
                if (k >= total) {
                    dry = true;
                } else {
                    const Tile tl = tiles[k >> 6];
                    const int lx = k & 7, ly = (k >> 3) & 7;
                    if (lx < tl.w && ly < tl.h) {   /* slots outside a partial tile: retry next pass */
                        has = true;
                        opx = tl.out_base + (int64_t)ly * tl.out_stride + lx;
                        camera_ray(s.cam, tl.x + lx, tl.y + ly, o, d);
                        depth = 0;
                        rng = make_pcg((uint32_t)(tl.x + lx), (uint32_t)(tl.y + ly));
                        sp = 0;
                    }
                }
            }
        }
        if (!__any(has)) {
            if (__any(!dry)) continue;
            break;
        }
        const bool more = shade_pass<true, MAXF, TRAV, TRAV, COUNT>(s, st, cnt, L, has, o, d, depth, rng, stack, sp,
                                                                     col);
        if (has && !more) {
            float *px = out + 3 * opx;
            px[0] = col.x;
            px[1] = col.y;
            px[2] = col.z;
            has = false;
        }
    }
    if (COUNT) {
        atomicAdd(&counters[0], (unsigned long long)cnt.traversals);
        atomicAdd(&counters[1], (unsigned long long)cnt.nodes);
        atomicAdd(&counters[2], (unsigned long long)cnt.tris);
        atomicAdd(&counters[3], (unsigned long long)cnt.hits);
    }
}

#define CRT_INST_REFILL(MAXF, T, C) template __global__ CRT_REFILL_SIG(MAXF, T, C)
#define CRT_INST_GIM(C) template __global__ CRT_GIM_SIG(C)
CRT_REFILL_INSTANCES(CRT_INST_REFILL)
CRT_GIM_INSTANCES(CRT_INST_GIM)

/* empty kernel: its launch at scene creation loads this TU's code object
 * (warm_code_objects) */
__global__ void k_warm_gi() {}

}  // namespace crt_amd
