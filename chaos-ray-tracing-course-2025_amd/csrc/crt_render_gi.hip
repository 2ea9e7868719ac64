/* GI refill kernels (k_render_refill) in a translation unit of their own, built
 * with -mllvm -amdgpu-sched-strategy=max-memory-clause (see crt_render.hip). */
#define CRT_SIDE_TU 1
#define CRT_GI_TU 1
#include "crt_render.hip"
