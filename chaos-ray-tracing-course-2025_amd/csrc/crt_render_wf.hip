/* Wavefront level kernels >= 1 (k_wf_level<SEC, false, *>) in a translation unit
 * of their own, built with their own LLVM scheduling strategy (see crt_render.hip). */
#define CRT_SIDE_TU 1
#define CRT_WF_TU 1
#include "crt_render.hip"
