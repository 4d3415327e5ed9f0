/*
 * bzr_debug.h -- test hooks of libbzr.so (not part of the drop-in boundary).
 */
#ifndef BZR_DEBUG_H
#define BZR_DEBUG_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
/* The culling boxes the BVH is built from, by patch index: boxes[6*i] = lo.xyz, hi.xyz of the region
 * where patch i's planar gate can pass for ray origins with |s|_inf <= *s_max.  Returns 0 on success. */
int32_t bzr_debug_gate_boxes(const void *patches, uint32_t n, uint32_t stride, float *boxes, float *s_max);
#ifdef __cplusplus
}
#endif
#endif
