/*
 * rt_oracle.h — TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference per-pixel render path.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and only
 * as the checker / CPU baseline.  The product (librt_hip.so) never links or calls it.
 *
 * Parity status: the reference (CUDA + cuRAND + Thrust) cannot be built in this image, and it ships no
 * tests, fixtures or golden images.  This restatement is pinned only by the survey-time probe values
 * recorded in SURVEY.md §8(c) (cuRAND XORWOW KAT for seed 1984; BASELINE config 1 pixels/checksum) — see
 * DESIGN.md "Oracle".  Where the reference leaves behaviour unspecified (argument evaluation order,
 * uninitialised values, int(NaN)) the choice made here is documented at the function.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include "../include/rt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_scene orc_scene;

/* cuRAND XORWOW restatement (curand_kernel.h, CUDA toolkit >= 12.0; not vendored in the reference). */
void orc_xorwow_seed(unsigned long long seed, unsigned int xor0, unsigned int xor1, unsigned int mul0,
                     unsigned int mul1, rt_curand_state* state);
void orc_curand_init(unsigned long long seed, rt_curand_state* state);
unsigned int orc_curand(rt_curand_state* state);
float orc_curand_uniform(rt_curand_state* state);

/* Philox4x32-10 (rocRAND philox4x32_10_engine / rocrand_uniform): ten rounds of the Random123 function, and
 * draw n of the sequential (seed, pixel, frame) stream; the perf-mode kernel (RT_FLAG_RNG_PHILOX) takes one
 * block of it per draw group (rt_oracle.c). */
void orc_philox4x32_10(const unsigned int ctr[4], const unsigned int key[2], unsigned int out[4]);
float orc_philox_uniform_at(unsigned long long seed, unsigned int pixel, unsigned int frame, unsigned int n);

/* Reference BVH (Hittable.cuh:303-385) over the scene's active hittables. */
orc_scene* orc_scene_build(const rt_scene_desc* desc);
void orc_scene_free(orc_scene* s);
int orc_scene_num_nodes(const orc_scene* s);
int orc_scene_depth(const orc_scene* s);
/* exact = 1: closest hit over all active primitives without the reference's AABB culling.  The reference's
 * slab test (AABB.cuh:30-50) on unpadded boxes can reject a box whose rectangle the rect test accepts
 * (hits within rounding of a box edge); this mode gives the geometric closest hit instead. */
void orc_scene_set_exact(orc_scene* s, int exact);

/* RenderInit (Kernel.cu:166-176) for the (floor-division) grid gx×gy of 16×16 blocks, or for every pixel
 * when full != 0. */
/* GetSphereUV's acos / atan2 (fixed binary32 sequences shared with the kernel, see rt_oracle.c). */
float orc_acos(float x);
float orc_atan2(float y, float x);

void orc_render_init(rt_curand_state* state, unsigned width, unsigned height, unsigned long long seed_base,
                     int full);

/* Counters: [0] rays (color() iterations, Kernel.cu:39), [1] AABB tests, [2] primitive tests, [3] primary,
 * [4] rectangle tests (the part of [2] that are XY/XZ/YZRect::Hit, Hittable.cuh:140-281; SURVEY §8(d) D4 prices
 * them at 12 FLOP against a sphere test's 23) */
typedef struct orc_counters {
    unsigned long long rays, box_tests, prim_tests, primary, rect_tests;
} orc_counters;

/* One frame of Kernel (Kernel.cu:102-158).  pos: W·H uint32 (row 0 = bottom); radiance: optional W·H·4
 * floats (col/spp, pre-gamma); accum: optional W·H·4 float running sum (rgb += Σ samples, w += spp; the
 * image then shows rgb / w — the renderer's RT_FLAG_ACCUMULATE, not a reference feature).  Only rows row_begin, row_begin + row_step, ... < row_end are rendered
 * (bounded CPU-baseline samples; row_step 0 = 1).
 * faithful_grid: skip pixels outside whole 16×16 blocks (Kernel.cu:184).  threads: OpenMP threads (0 =
 * default).  rius_order: 0 = left-to-right evaluation of Vec3(ξ,ξ,ξ) in Random() (Math.cuh:231-234),
 * 1 = right-to-left (what g++ emits for that constructor call).  philox != 0: every pixel draws from the
 * Philox stream (seed, global pixel index, frame) instead of its XORWOW state; `state` is not used and may
 * be NULL. */
void orc_render(const orc_scene* scene, unsigned int* pos, float* radiance, float* accum, unsigned width,
                unsigned height,
                unsigned spp, unsigned max_depth, rt_curand_state* state, const rt_input_struct* inputs,
                int faithful_grid, unsigned row_begin, unsigned row_end, unsigned row_step, int threads,
                int rius_order, int philox, unsigned long long seed, unsigned frame, orc_counters* counters);

/* Known-answer helpers. */
typedef struct orc_hit {
    int hit;
    float t, p[3], normal[3], u, v;
    int front_face;
} orc_hit;
int orc_hittable_hit(const rt_hittable_desc* h, const float o[3], const float d[3], float tmin, float tmax,
                     orc_hit* rec);
/* Scatter with a given RNG state: returns the Scatter() flag, fills scattered origin/dir and attenuation;
 * *draws = number of curand_uniform calls consumed. */
int orc_scatter(const rt_material_desc* m, const float o[3], const float d[3], const orc_hit* rec,
                rt_curand_state* state, float scattered_o[3], float scattered_d[3], float attenuation[3],
                int* draws, int rius_order);
unsigned int orc_rgb_to_int(float r, float g, float b);

#ifdef __cplusplus
}
#endif

#endif
