/*
 * rt_oracle.c — TEST INFRASTRUCTURE ONLY (see rt_oracle.h).  CPU restatement of the per-pixel path-trace
 * kernel of Trippasch/CudaRayTracer, written in plain C99 from the reference's behaviour; every function
 * cites the reference file:line it restates (paths relative to CudaRayTracer/src/).
 *
 * Arithmetic contract: compiled with -ffp-contract=off and without -ffast-math, so each +,-,*,/ and
 * sqrtf is one IEEE-754 binary32 operation, evaluated in the order the reference's C++ expressions
 * associate (left to right).  The reference's Release build used nvcc -use_fast_math
 * (CudaRayTracer/CMakeLists.txt:36) whose approximate rcp/rsqrt/transcendentals cannot be reproduced
 * without an NVIDIA GPU; the effective parity target is this restatement.
 *
 * Deviations where the reference is unspecified or undefined:
 *   - pow(1-cos, 5) in Schlick (Material.cuh:144) is evaluated as ((x·x)·(x·x))·x.
 *   - Dielectric with reflect_prob = 1 and ξ = 1.0 reads an uninitialised `refracted` (Material.cuh:113,
 *     131-134); here it is the zero vector.
 *   - int(NaN) in RgbToInt (Kernel.cu:18) is 0 (CUDA cvt.rzi semantics).
 *   - DiffuseLight/Lambertian/Metal with an unknown texture type (Material.cuh:48-60, 164-176) yield 0.
 */
#include "rt_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_PI 3.141592654f /* Math.cuh:9 */

/* ---------------------------------------------------------------------------------------------- */
/* Vec3 (Utils/Math.cuh:16-229)                                                                   */
/* ---------------------------------------------------------------------------------------------- */
typedef struct { float x, y, z; } v3;

static inline v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }           /* :117-120 */
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }           /* :122-125 */
static inline v3 mulv(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }          /* :127-130 */
static inline v3 scale(float t, v3 v) { return mk(t * v.x, t * v.y, t * v.z); }            /* :137-140, 147-150 */
static inline v3 divs(v3 v, float t) { return mk(v.x / t, v.y / t, v.z / t); }             /* :142-145 */
static inline v3 neg(v3 v) { return mk(-v.x, -v.y, -v.z); }                                 /* :57-60 */
static inline float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }          /* :152-155 */
static inline v3 cross(v3 a, v3 b) {                                                       /* :157-161 */
    return mk(a.y * b.z - a.z * b.y, -(a.x * b.z - a.z * b.x), a.x * b.y - a.y * b.x);
}
static inline float length(v3 v) { return sqrtf(v.x * v.x + v.y * v.y + v.z * v.z); }     /* :77-80 */
static inline v3 unit_vector(v3 v) { return divs(v, length(v)); }                          /* :220-223 */
static inline v3 normalize(v3 v) { float inv = 1 / sqrtf(dot(v, v)); return scale(inv, v); } /* :225-229 */
static inline float fclampf(float x, float a, float b) { return (x < a) ? a : ((x > b) ? b : x); } /* :307-310 */
static inline v3 reflect(v3 v, v3 n) { return sub(v, scale(2.0f * dot(v, n), n)); }       /* :287-290 */
static inline v3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }

/* Refract (Math.cuh:292-304) */
static inline int refract(v3 v, v3 n, float ni_over_nt, v3* refracted) {
    v3 uv = unit_vector(v);
    float dt = dot(uv, n);
    float discriminant = 1.0f - ni_over_nt * ni_over_nt * (1 - dt * dt);
    if (discriminant > 0) {
        *refracted = sub(scale(ni_over_nt, sub(uv, scale(dt, n))), scale(sqrtf(discriminant), n));
        return 1;
    }
    return 0;
}

/* ---------------------------------------------------------------------------------------------- */
/* cuRAND XORWOW restatement.  Published algorithm of curand_kernel.h (CUDA toolkit >= 12.0,        */
/* CMakeLists.txt:28): _curand_init_scratch seeding, curand() xorwow step, _curand_uniform.        */
/* Called with subsequence 0 and offset 0 (Kernel.cu:163,175), so no skip-ahead matrices apply.   */
/* ---------------------------------------------------------------------------------------------- */
/* The xorwow seeding scheme shared by cuRAND and rocRAND: the 64-bit seed's halves are scrambled by two
   xor constants and two multipliers into (d, v[5]) around Marsaglia's base state.  The two libraries differ
   only in those four constants (rocRAND: rocrand_xorwow.h:113-116), so checking this function with
   rocRAND's constants against rocRAND's own engine (tests/golden/rocrand_xorwow_kat.json) pins the base
   state, the Weyl step and the recurrence of orc_curand independently of the survey probe. */
void orc_xorwow_seed(unsigned long long seed, unsigned int xor0, unsigned int xor1, unsigned int mul0,
                     unsigned int mul1, rt_curand_state* s) {
    unsigned int s0 = ((unsigned int)seed) ^ xor0;
    unsigned int s1 = ((unsigned int)(seed >> 32)) ^ xor1;
    unsigned int t0 = mul0 * s0;
    unsigned int t1 = mul1 * s1;
    s->d = 6615241u + t1 + t0;
    s->v[0] = 123456789u + t0;
    s->v[1] = 362436069u ^ t0;
    s->v[2] = 521288629u + t1;
    s->v[3] = 88675123u ^ t1;
    s->v[4] = 5783321u + t0;
    s->boxmuller_flag = 0;
    s->boxmuller_flag_double = 0;
    s->boxmuller_extra = 0.0f;
    s->pad_ = 0;
    s->boxmuller_extra_double = 0.0;
}

void orc_curand_init(unsigned long long seed, rt_curand_state* s) {
    orc_xorwow_seed(seed, 0xaad26b49u, 0xf7dcefddu, 1099087573u, 2591861531u, s);
}

unsigned int orc_curand(rt_curand_state* s) {
    unsigned int t = s->v[0] ^ (s->v[0] >> 2);
    s->v[0] = s->v[1];
    s->v[1] = s->v[2];
    s->v[2] = s->v[3];
    s->v[3] = s->v[4];
    s->v[4] = (s->v[4] ^ (s->v[4] << 4)) ^ (t ^ (t << 1));
    s->d += 362437u;
    return s->v[4] + s->d;
}

/* uniform in (0, 1]: x·2^-32 + 2^-33 (CURAND_2POW32_INV = 2.3283064e-10f). */
float orc_curand_uniform(rt_curand_state* s) {
    unsigned int x = orc_curand(s);
    return (float)x * 2.3283064e-10f + (2.3283064e-10f / 2.0f);
}

/* ---------------------------------------------------------------------------------------------- */
/* Philox4x32-10: the perf-mode RNG BASELINE.json's north_star names ("hiprand (Philox) per-pixel   */
/* state").  Restates rocRAND's philox4x32_10_engine (/opt/rocm/include/rocrand/                    */
/* rocrand_philox4x32_10.h:270-303, the Random123 round) and rocrand_uniform (rocrand_uniform.h:    */
/* 65-68, 281-284).            A pixel's stream is rocrand_init(seed, subsequence = global pixel      */
/* index, offset = frame << 34), read as blocks philox10(ctr = {b, frame, pixel, 0}, key = {seed   */
/* lo, seed hi}) (rocrand_uniform4) in draw groups that start on a block boundary: the camera       */
/* jitter (Kernel.cu:139-140) and the dielectric's choice (Material.cuh:131) one group each, a      */
/* whole RandomInUnitSphere call (Math.cuh:252-260, 3 draws per attempt) one group (the kernel's   */
/* RngPhilox, render.hip).  Sample s of a pixel starts at block s << 16 (its own window of 2^16     */
/* blocks: offset (frame << 34) + (s << 18)), and the pixel's samples are summed in 2^-12 fixed      */
/* point (orc_quant), so neither depends on the order the samples run in.  Pinned by                */
/* tests/golden/philox_kat.json (rocRAND's own engine).                                              */
/* ---------------------------------------------------------------------------------------------- */
void orc_philox4x32_10(const unsigned int ctr_in[4], const unsigned int key_in[2], unsigned int out[4]) {
    unsigned int c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    unsigned int k0 = key_in[0], k1 = key_in[1];
    for (int round = 0; round < 10; round++) {
        unsigned long long m0 = 0xD2511F53ull * (unsigned long long)c0;
        unsigned long long m1 = 0xCD9E8D57ull * (unsigned long long)c2;
        unsigned int hi0 = (unsigned int)(m0 >> 32), lo0 = (unsigned int)m0;
        unsigned int hi1 = (unsigned int)(m1 >> 32), lo1 = (unsigned int)m1;
        c0 = hi1 ^ c1 ^ k0;
        c1 = lo1;
        c2 = hi0 ^ c3 ^ k1;
        c3 = lo0;
        k0 += 0x9E3779B9u; /* bumpkey */
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* uniform in (0, 1]: 2^-32 + x·2^-32 (rocrand_uniform.h:65-68).  x·2^-32 is exact, so a fused and an
 * unfused evaluation agree. */
static inline float philox_to_uniform(unsigned int x) { return 2.3283064e-10f + (float)x * 2.3283064e-10f; }

/* Philox mode's per-sample contribution in 2^-12 fixed point: NaN, negative and zero give 0, values from 2^20 - 1
 * on saturate; x · 4096 is exact, so the one rounding is the + 0.5's; the sum saturates at 2^32 - 1. */
static inline unsigned orc_quant(float x) {
    if (!(x > 0.0f)) return 0u;
    if (!(x < 1048575.0f)) return 0xffffffffu;
    return (unsigned)(x * 4096.0f + 0.5f);
}
static inline unsigned orc_sat_add(unsigned a, unsigned b) {
    unsigned s = a + b;
    return s < b ? 0xffffffffu : s;
}

float orc_philox_uniform_at(unsigned long long seed, unsigned int pixel, unsigned int frame, unsigned int n) {
    unsigned int ctr[4] = {n >> 2, frame, pixel, 0u};
    unsigned int key[2] = {(unsigned int)seed, (unsigned int)(seed >> 32)};
    unsigned int r[4];
    orc_philox4x32_10(ctr, key, r);
    return philox_to_uniform(r[n & 3u]);
}

/* The RNG of one pixel: the reference's cuRAND XORWOW state (parity mode) or a Philox stream. */
typedef struct {
    int philox;
    rt_curand_state* xs;
    unsigned int key[2], frame, pixel, n, r[4];
} orc_rng;

/* Start of a draw group: a Philox stream moves to the next block's first word (the rest of the current
 * block is skipped); the XORWOW stream is sequential. */
static inline void orc_group(orc_rng* g) {
    if (g->philox) g->n = (g->n + 3u) & ~3u;
}

static float orc_uniform(orc_rng* g) {
    if (!g->philox) return orc_curand_uniform(g->xs);
    if ((g->n & 3u) == 0u) {
        unsigned int ctr[4] = {g->n >> 2, g->frame, g->pixel, 0u};
        orc_philox4x32_10(ctr, g->key, g->r);
    }
    return philox_to_uniform(g->r[g->n++ & 3u]);
}

/* Random() (Math.cuh:231-234) + RandomInUnitSphere (Math.cuh:252-260). */
static inline v3 random_in_unit_sphere(orc_rng* st, int order, int* draws) {
    v3 p;
    orc_group(st); /* Philox: the call's attempts draw consecutive words from a block boundary on */
    do {
        float a = orc_uniform(st), b = orc_uniform(st), c = orc_uniform(st);
        v3 r = order == 0 ? mk(a, b, c) : mk(c, b, a);
        *draws += 3;
        p = sub(scale(2.0f, r), mk(1.0f, 1.0f, 1.0f));
    } while (p.x * p.x + p.y * p.y + p.z * p.z >= 1.0f); /* LengthSquared, Math.cuh:247-250 */
    return p;
}

/* ---------------------------------------------------------------------------------------------- */
/* Scene: primitives, materials, textures                                                          */
/* ---------------------------------------------------------------------------------------------- */
typedef struct {
    v3 p, normal;
    int mat;
    float t, u, v;
    int front_face;
} hitrec; /* HitRecord, Hittable.cuh:14-28 */

typedef struct {
    float bmin[3], bmax[3];
} aabb;

/* child reference: kind 0 = null, 1 = BVH node, 2 = primitive (Hittable* left/right, Hittable.cuh:300-301) */
typedef struct { int kind, idx; } childref;

typedef struct {
    aabb box;
    childref left, right;
} onode; /* BVHNode, Hittable.cuh:296-301 */

struct orc_scene {
    rt_hittable_desc* prims; /* all hittables in list order */
    int nprims;
    rt_material_desc* mats;
    int nmats;
    rt_image_desc* images;
    int nimages;
    onode* nodes;
    int nnodes, capnodes;
    int depth;
    int exact_closest_hit; /* 1: test every active primitive, no box culling (orc_scene_set_exact) */
};

/* SetFaceNormal (Hittable.cuh:23-27) */
static inline void set_face_normal(hitrec* rec, v3 d, v3 outward) {
    rec->front_face = dot(d, outward) < 0;
    rec->normal = rec->front_face ? outward : neg(outward);
}

/* acos / atan2 of GetSphereUV as a fixed sequence of binary32 +, -, *, / and sqrtf (Cephes asinf/atanf
   polynomials), operation for operation the same as render.hip's rt_acosf / rt_atan2f.  The reference calls
   CUDA's acos/atan2 under -use_fast_math (CudaRayTracer/CMakeLists.txt:36), which no CPU or ROCm library
   reproduces; libm's and the device library's own acosf/atan2f differ in the last bit now and then, which
   moves an 8192-wide texture lookup by one texel.  Documented deviation: the acos argument is clamped to
   [-1, 1] (a rounded normal can exceed 1 by an ulp; the reference's NaN would index the texture with
   int(NaN), undefined). */
static inline float orc_asin_poly(float x) { /* |x| <= 0.5 */
    float z = x * x;
    float p = (((4.2163199048e-2f * z + 2.4181311049e-2f) * z + 4.5470025998e-2f) * z + 7.4953002686e-2f) * z +
              1.6666752422e-1f;
    return p * z * x + x;
}
static inline float orc_acosf(float x) {
    x = x < -1.0f ? -1.0f : (x > 1.0f ? 1.0f : x);
    if (x < -0.5f) return 0x1.921fb6p+1f - 2.0f * orc_asin_poly(sqrtf(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * orc_asin_poly(sqrtf(0.5f * (1.0f - x)));
    return 0x1.921fb6p+0f - orc_asin_poly(x);
}
static inline float orc_atan_poly(float x) { /* |x| <= tan(pi/8) */
    float z = x * x;
    return (((8.05374449538e-2f * z - 1.38776856032e-1f) * z + 1.99777106478e-1f) * z - 3.33329491539e-1f) * z * x + x;
}
static inline float orc_atan01(float t) { /* t in [0, 1] */
    if (t > 0.41421356f) return 0x1.921fb6p-1f + orc_atan_poly((t - 1.0f) / (t + 1.0f));
    return orc_atan_poly(t);
}
static inline float orc_atan2f(float y, float x) {
    float ax = fabsf(x), ay = fabsf(y), r;
    if (ax == 0.0f && ay == 0.0f) r = 0.0f;
    else if (ay <= ax) r = orc_atan01(ay / ax);
    else r = 0x1.921fb6p+0f - orc_atan01(ax / ay);
    if (signbit(x)) r = 0x1.921fb6p+1f - r; /* IEEE atan2: x < 0 or -0 */
    return signbit(y) ? -r : r;
}
float orc_acos(float x) { return orc_acosf(x); }
float orc_atan2(float y, float x) { return orc_atan2f(y, x); }

/* GetSphereUV (Hittable.cuh:119-125) */
static inline void sphere_uv(v3 p, float* u, float* v) {
    float theta = orc_acosf(-p.y);
    float phi = orc_atan2f(-p.z, p.x) + ORC_PI;
    *u = phi / (2 * ORC_PI);
    *v = theta / ORC_PI;
}

/* Sphere::Hit (Hittable.cuh:80-110) */
static int sphere_hit(const rt_hittable_desc* s, v3 o, v3 d, float tmin, float tmax, hitrec* rec) {
    v3 c = ld3(s->center);
    v3 oc = sub(o, c);
    float a = dot(d, d);
    float b = dot(oc, d);
    float cc = dot(oc, oc) - s->radius * s->radius;
    float disc = b * b - a * cc;
    if (disc > 0) {
        float temp = (-b - sqrtf(disc)) / a;
        if (temp < tmax && temp > tmin) {
            rec->t = temp;
            rec->p = add(o, scale(temp, d));
            rec->normal = divs(sub(rec->p, c), s->radius);
            sphere_uv(rec->normal, &rec->u, &rec->v);
            rec->mat = s->material;
            return 1;
        }
        temp = (-b + sqrtf(disc)) / a;
        if (temp < tmax && temp > tmin) {
            rec->t = temp;
            rec->p = add(o, scale(temp, d));
            rec->normal = divs(sub(rec->p, c), s->radius);
            sphere_uv(rec->normal, &rec->u, &rec->v);
            rec->mat = s->material;
            return 1;
        }
    }
    return 0;
}

/* XYRect/XZRect/YZRect::Hit (Hittable.cuh:140-169, 196-225, 252-281).  axis k = plane normal axis,
 * (ia, ib) = in-plane axes giving (u, v). */
static int rect_hit(const rt_hittable_desc* r, v3 o, v3 d, float tmin, float tmax, hitrec* rec) {
    const float* c = r->center;
    float a0, a1, b0, b1, k, oa, ob, ok, da, db, dk;
    v3 nrm;
    float of[3] = {o.x, o.y, o.z}, df[3] = {d.x, d.y, d.z};
    int ia, ib, ik;
    if (r->type == RT_XYRECT) {
        a0 = c[0] - (r->width / 2); a1 = c[0] + (r->width / 2);
        b0 = c[1] - (r->height / 2); b1 = c[1] + (r->height / 2);
        k = c[2]; ia = 0; ib = 1; ik = 2; nrm = mk(0.0f, 0.0f, 1.0f);
    } else if (r->type == RT_XZRECT) {
        a0 = c[0] - (r->width / 2); a1 = c[0] + (r->width / 2);
        b0 = c[2] - (r->height / 2); b1 = c[2] + (r->height / 2);
        k = c[1]; ia = 0; ib = 2; ik = 1; nrm = mk(0.0f, 1.0f, 0.0f);
    } else { /* YZ: y from height, z from width (Hittable.cuh:255-258) */
        a0 = c[1] - (r->height / 2); a1 = c[1] + (r->height / 2);
        b0 = c[2] - (r->width / 2); b1 = c[2] + (r->width / 2);
        k = c[0]; ia = 1; ib = 2; ik = 0; nrm = mk(1.0f, 0.0f, 0.0f);
    }
    oa = of[ia]; ob = of[ib]; ok = of[ik];
    da = df[ia]; db = df[ib]; dk = df[ik];
    float inv = 1.0f / dk;
    float t = (k - ok) * inv;
    if (t < tmin || t > tmax) return 0;
    float x = oa + t * da;
    float y = ob + t * db;
    if (x < a0 || x > a1 || y < b0 || y > b1) return 0;
    rec->u = (x - a0) / (a1 - a0);
    rec->v = (y - b0) / (b1 - b0);
    rec->t = t;
    set_face_normal(rec, d, nrm);
    rec->mat = r->material;
    rec->p = add(o, scale(t, d));
    return 1;
}

static inline int prim_hit(const rt_hittable_desc* h, v3 o, v3 d, float tmin, float tmax, hitrec* rec) {
    switch (h->type) { /* PerformHit, Hittable.cuh:470-485 */
    case RT_SPHERE: return sphere_hit(h, o, d, tmin, tmax, rec);
    case RT_XYRECT:
    case RT_XZRECT:
    case RT_YZRECT: return rect_hit(h, o, d, tmin, tmax, rec);
    default: return 0;
    }
}

/* BoundingBox (Hittable.cuh:112-116, 171-181, 227-237, 283-293) */
static aabb prim_box(const rt_hittable_desc* h) {
    aabb b;
    const float* c = h->center;
    if (h->type == RT_SPHERE) {
        float r = h->radius;
        for (int i = 0; i < 3; i++) { b.bmin[i] = c[i] - r; b.bmax[i] = c[i] + r; }
    } else if (h->type == RT_XYRECT) {
        b.bmin[0] = c[0] - (h->width / 2); b.bmax[0] = c[0] + (h->width / 2);
        b.bmin[1] = c[1] - (h->height / 2); b.bmax[1] = c[1] + (h->height / 2);
        b.bmin[2] = c[2] - 0.0001f; b.bmax[2] = c[2] + 0.0001f;
    } else if (h->type == RT_XZRECT) {
        b.bmin[0] = c[0] - (h->width / 2); b.bmax[0] = c[0] + (h->width / 2);
        b.bmin[1] = c[1] - 0.0001f; b.bmax[1] = c[1] + 0.0001f;
        b.bmin[2] = c[2] - (h->height / 2); b.bmax[2] = c[2] + (h->height / 2);
    } else {
        b.bmin[0] = c[0] - 0.0001f; b.bmax[0] = c[0] + 0.0001f;
        b.bmin[1] = c[1] - (h->height / 2); b.bmax[1] = c[1] + (h->height / 2);
        b.bmin[2] = c[2] - (h->width / 2); b.bmax[2] = c[2] + (h->width / 2);
    }
    return b;
}

/* SurroundingBox (AABB.cuh:53-62) */
static aabb surrounding(aabb a, aabb b) {
    aabb r;
    for (int i = 0; i < 3; i++) {
        r.bmin[i] = fminf(a.bmin[i], b.bmin[i]);
        r.bmax[i] = fmaxf(a.bmax[i], b.bmax[i]);
    }
    return r;
}

/* AABB::Hit (AABB.cuh:30-50) */
static inline int aabb_hit(const aabb* b, v3 o, v3 d, float tmin, float tmax) {
    float of[3] = {o.x, o.y, o.z}, df[3] = {d.x, d.y, d.z};
    for (int a = 0; a < 3; a++) {
        float invD = 1.0f / df[a];
        float t0 = (b->bmin[a] - of[a]) * invD;
        float t1 = (b->bmax[a] - of[a]) * invD;
        if (invD < 0.0f) { float tmp = t0; t0 = t1; t1 = tmp; }
        tmin = t0 > tmin ? t0 : tmin;
        tmax = t1 < tmax ? t1 : tmax;
        if (tmax <= tmin) return 0;
    }
    return 1;
}

/* ---------------------------------------------------------------------------------------------- */
/* Reference BVH build (BVHNode ctor, Hittable.cuh:303-385)                                         */
/* ---------------------------------------------------------------------------------------------- */
static int new_node(orc_scene* s) {
    if (s->nnodes == s->capnodes) {
        s->capnodes = s->capnodes ? 2 * s->capnodes : 64;
        s->nodes = (onode*)realloc(s->nodes, (size_t)s->capnodes * sizeof(onode));
    }
    memset(&s->nodes[s->nnodes], 0, sizeof(onode));
    return s->nnodes++;
}

static aabb child_box(const orc_scene* s, childref c) {
    return c.kind == 1 ? s->nodes[c.idx].box : prim_box(&s->prims[c.idx]);
}

/* objs: hittable indices in the current order; [start, end) the range this node covers. */
static int build_node(orc_scene* s, int* objs, int start, int end, int depth) {
    int id = new_node(s);
    if (depth > s->depth) s->depth = depth;
    /* thrust::remove_if of inactive objects (stable) */
    int w = start;
    for (int i = start; i < end; i++)
        if (s->prims[objs[i]].is_active) objs[w++] = objs[i];
    int span = w - start;
    if (span == 0) { /* left = right = nullptr, box stays AABB() = zeros */
        s->nodes[id].left.kind = s->nodes[id].right.kind = 0;
        return id;
    }
    /* thrust::sort by HittableType: stable insertion sort keeps list order inside a type */
    for (int i = start + 1; i < w; i++) {
        int v = objs[i], j = i - 1;
        while (j >= start && s->prims[objs[j]].type > s->prims[v].type) { objs[j + 1] = objs[j]; j--; }
        objs[j + 1] = v;
    }
    childref L, R;
    if (span == 1) {
        L.kind = R.kind = 2; L.idx = R.idx = objs[start];
    } else if (span == 2) {
        L.kind = R.kind = 2; L.idx = objs[start]; R.idx = objs[start + 1];
    } else {
        /* thrust::partition by (type == first type): input is sorted by type, so the partition point is
         * the end of the first type group and the order is unchanged. */
        int t0 = s->prims[objs[start]].type;
        int mid = start;
        while (mid < w && s->prims[objs[mid]].type == t0) mid++;
        if (mid == start || mid == w) mid = start + span / 2;
        L.kind = R.kind = 1;
        L.idx = build_node(s, objs, start, mid, depth + 1);
        R.idx = build_node(s, objs, mid, w, depth + 1);
    }
    s->nodes[id].left = L;
    s->nodes[id].right = R;
    s->nodes[id].box = surrounding(child_box(s, L), child_box(s, R));
    return id;
}

orc_scene* orc_scene_build(const rt_scene_desc* desc) {
    orc_scene* s = (orc_scene*)calloc(1, sizeof(orc_scene));
    s->nprims = (int)desc->num_hittables;
    s->prims = (rt_hittable_desc*)malloc(sizeof(rt_hittable_desc) * (size_t)(s->nprims ? s->nprims : 1));
    if (s->nprims) memcpy(s->prims, desc->hittables, sizeof(rt_hittable_desc) * (size_t)s->nprims);
    s->nmats = (int)desc->num_materials;
    s->mats = (rt_material_desc*)malloc(sizeof(rt_material_desc) * (size_t)(s->nmats ? s->nmats : 1));
    if (s->nmats) memcpy(s->mats, desc->materials, sizeof(rt_material_desc) * (size_t)s->nmats);
    s->nimages = (int)desc->num_images;
    s->images = (rt_image_desc*)malloc(sizeof(rt_image_desc) * (size_t)(s->nimages ? s->nimages : 1));
    if (s->nimages) memcpy(s->images, desc->images, sizeof(rt_image_desc) * (size_t)s->nimages);
    int* objs = (int*)malloc(sizeof(int) * (size_t)(s->nprims ? s->nprims : 1));
    for (int i = 0; i < s->nprims; i++) objs[i] = i;
    build_node(s, objs, 0, s->nprims, 1);
    free(objs);
    return s;
}

void orc_scene_free(orc_scene* s) {
    if (!s) return;
    free(s->prims); free(s->mats); free(s->images); free(s->nodes); free(s);
}
int orc_scene_num_nodes(const orc_scene* s) { return s->nnodes; }
void orc_scene_set_exact(orc_scene* s, int exact) { s->exact_closest_hit = exact; }
int orc_scene_depth(const orc_scene* s) { return s->depth; }

/* BVHNode::Hit (Hittable.cuh:387-439): iterative DFS, stack of {node, t_min, t_max}.  The reference
 * stack holds 16 entries; depth here is bounded by the tree depth + 1 and asserted by the caller via
 * orc_scene_depth(). */
typedef struct { int node; float tmin, tmax; } stacknode;

#ifdef ORC_HIT_DIAG
/* Diagnostic build only (tools/bvh_hit_class.py compiles it with -DORC_HIT_DIAG into /tmp; the library the tests load
 * never has it): every reference-BVH closest-hit query is repeated as the exact linear scan and a disagreement is
 * classed as [1] tie (same t, another primitive's material/normal) or [2] culled (the BVH answer is farther or a miss:
 * a box rejected the ray at the precision edge of its slab test) or [3] other; [0] counts all disagreements. */
static unsigned long long orc_diag_counts[4];
unsigned long long orc_hit_diag(int k) { return k >= 0 && k < 4 ? orc_diag_counts[k] : 0; }
static int world_hit_bvh(const orc_scene* s, v3 o, v3 d, float tmin, float tmax, hitrec* rec,
                         unsigned long long* box_tests, unsigned long long* prim_tests, unsigned long long* rect_tests);
static int world_hit(const orc_scene* s, v3 o, v3 d, float tmin, float tmax, hitrec* rec,
                     unsigned long long* box_tests, unsigned long long* prim_tests, unsigned long long* rect_tests) {
    int r = world_hit_bvh(s, o, d, tmin, tmax, rec, box_tests, prim_tests, rect_tests);
    if (s->exact_closest_hit) return r;
    hitrec e;
    int he = 0;
    for (int i = 0; i < s->nprims; i++)
        if (s->prims[i].is_active) he |= prim_hit(&s->prims[i], o, d, tmin, he ? e.t : tmax, &e);
    if (he == r && (!he || (e.t == rec->t && e.mat == rec->mat && e.normal.x == rec->normal.x &&
                            e.normal.y == rec->normal.y && e.normal.z == rec->normal.z)))
        return r;
    int k = (he && r && e.t == rec->t) ? 1 : (he && (!r || rec->t > e.t)) ? 2 : 3;
#pragma omp atomic
    orc_diag_counts[0]++;
#pragma omp atomic
    orc_diag_counts[k]++;
    return r;
}
static int world_hit_bvh(const orc_scene* s, v3 o, v3 d, float tmin, float tmax, hitrec* rec,
                         unsigned long long* box_tests, unsigned long long* prim_tests, unsigned long long* rect_tests) {
#else
static int world_hit(const orc_scene* s, v3 o, v3 d, float tmin, float tmax, hitrec* rec,
                     unsigned long long* box_tests, unsigned long long* prim_tests, unsigned long long* rect_tests) {
#endif
    if (s->exact_closest_hit) {
        /* Geometric closest hit over the active primitives in list order, without box culling. */
        int hit_something = 0;
        for (int i = 0; i < s->nprims; i++) {
            if (!s->prims[i].is_active) continue;
            ++*prim_tests;
            *rect_tests += s->prims[i].type != RT_SPHERE;
            hit_something |= prim_hit(&s->prims[i], o, d, tmin, hit_something ? rec->t : tmax, rec);
        }
        return hit_something;
    }
    const onode* root = &s->nodes[0];
    ++*box_tests;
    if (!aabb_hit(&root->box, o, d, tmin, tmax)) return 0;
    stacknode stack[64];
    int top = -1;
    stack[++top] = (stacknode){0, tmin, tmax};
    int hit_something = 0;
    while (top >= 0) {
        stacknode cur = stack[top--];
        const onode* n = &s->nodes[cur.node];
        ++*box_tests;
        if (!aabb_hit(&n->box, o, d, cur.tmin, cur.tmax)) continue;
        childref ch[2] = {n->left, n->right};
        for (int k = 0; k < 2; k++) {
            if (ch[k].kind == 1) {
                stack[++top] = (stacknode){ch[k].idx, cur.tmin, hit_something ? rec->t : cur.tmax};
            } else if (ch[k].kind == 2) {
                ++*prim_tests;
                *rect_tests += s->prims[ch[k].idx].type != RT_SPHERE;
                hit_something |= prim_hit(&s->prims[ch[k].idx], o, d, cur.tmin, hit_something ? rec->t : cur.tmax, rec);
            }
        }
    }
    return hit_something;
}

/* ---------------------------------------------------------------------------------------------- */
/* Textures (Texture.cuh:32-109) and materials (Material.cuh:34-176)                               */
/* ---------------------------------------------------------------------------------------------- */
static v3 texture_value(const orc_scene* s, const rt_texture_desc* t, float u, float v, v3 p) {
    switch (t->type) {
    case RT_CONSTANT: return ld3(t->color); /* Constant::value :42-45 */
    case RT_CHECKER: {                      /* Checker::value :58-67 */
        float sines = sinf(10 * p.x) * sinf(10 * p.y) * sinf(10 * p.z);
        return sines < 0 ? ld3(t->color) : ld3(t->color2);
    }
    case RT_IMAGE: { /* Image::value :83-105 */
        /* data == nullptr → cyan (:83-84).  Documented deviation: an image with data but no texels (w·h == 0)
           is also cyan; the reference would read data[-3] (i = width - 1 = -1, :88-91), undefined. */
        if (t->image < 0 || t->image >= s->nimages || !s->images[t->image].data || s->images[t->image].width <= 0 ||
            s->images[t->image].height <= 0)
            return mk(0.0f, 1.0f, 1.0f);
        const rt_image_desc* im = &s->images[t->image];
        u = fclampf(u, 0.0f, 1.0f);
        v = 1.0f - fclampf(v, 0.0f, 1.0f);
        int i = (int)(u * im->width);
        int j = (int)(v * im->height);
        if (i >= im->width) i = im->width - 1;
        if (j >= im->height) j = im->height - 1;
        const float color_scale = 1.0f / 255.0f;
        const unsigned char* px = im->data + (size_t)j * (size_t)(3 * im->width) + (size_t)i * 3;
        return mk(color_scale * px[0], color_scale * px[1], color_scale * px[2]);
    }
    default: return mk(0.0f, 0.0f, 0.0f);
    }
}

/* Scatter of Lambertian (:43-62), Metal (:75-94), Dielectric (:106-145).  Returns the flag. */
static int scatter(const orc_scene* s, const rt_material_desc* m, v3 ro, v3 rd, const hitrec* rec,
                   orc_rng* st, v3* so, v3* sd, v3* att, int* draws, int order) {
    (void)ro;
    switch (m->type) {
    case RT_LAMBERTIAN: {
        v3 target = add(add(rec->p, rec->normal), random_in_unit_sphere(st, order, draws));
        *so = rec->p;
        *sd = sub(target, rec->p);
        *att = texture_value(s, &m->albedo, rec->u, rec->v, rec->p);
        return 1;
    }
    case RT_METAL: {
        v3 reflected = reflect(unit_vector(rd), rec->normal);
        *so = rec->p;
        *sd = add(reflected, scale(m->fuzz, random_in_unit_sphere(st, order, draws)));
        *att = texture_value(s, &m->albedo, rec->u, rec->v, rec->p);
        return dot(*sd, rec->normal) > 0;
    }
    case RT_DIELECTRIC: {
        v3 outward_normal;
        v3 reflected = reflect(rd, rec->normal);
        float ni_over_nt;
        float ir = m->ir;
        *att = mk(1.0f, 1.0f, 1.0f);
        v3 refracted = mk(0.0f, 0.0f, 0.0f);
        float reflect_prob;
        float cosine;
        if (dot(rd, rec->normal) > 0.0f) {
            outward_normal = neg(rec->normal);
            ni_over_nt = ir;
            cosine = dot(rd, rec->normal) / length(rd);
            cosine = sqrtf(1.0f - ir * ir * (1 - cosine * cosine));
        } else {
            outward_normal = rec->normal;
            ni_over_nt = 1.0f / ir;
            cosine = -dot(rd, rec->normal) / length(rd);
        }
        if (refract(rd, outward_normal, ni_over_nt, &refracted)) {
            /* Reflectance (Material.cuh:139-145) */
            float r0 = (1.0f - ir) / (1.0f + ir);
            r0 = r0 * r0;
            float x = 1.0f - cosine;
            float x2 = x * x;
            float x5 = (x2 * x2) * x;
            reflect_prob = r0 + (1.0f - r0) * x5;
        } else {
            reflect_prob = 1.0f;
        }
        *draws += 1;
        *so = rec->p;
        orc_group(st);
        *sd = orc_uniform(st) < reflect_prob ? reflected : refracted;
        return 1;
    }
    default: return 0; /* DiffuseLight::Scatter (:158-162) */
    }
}

/* color() (Kernel.cu:30-80) */
static v3 color(const orc_scene* s, v3 o, v3 d, int max_depth, orc_rng* st, const rt_input_struct* in,
                int order, orc_counters* c) {
    v3 cur_att = mk(1.0f, 1.0f, 1.0f);
    v3 black = mk(0.0f, 0.0f, 0.0f);
    hitrec rec;
    memset(&rec, 0, sizeof(rec));
    for (int i = 0; i < max_depth; i++) {
        c->rays++;
        if (!world_hit(s, o, d, 0.001f, FLT_MAX, &rec, &c->box_tests, &c->prim_tests, &c->rect_tests)) {
            v3 unit_direction = unit_vector(d);
            float t = 0.5f * (unit_direction.y + 1.0f);
            v3 bg = add(scale(1.0f - t, ld3(in->background_start)), scale(t, ld3(in->background_end)));
            return mulv(cur_att, bg);
        }
        const rt_material_desc* m = &s->mats[rec.mat];
        v3 emitted = mk(0.0f, 0.0f, 0.0f);
        v3 so, sd, att;
        int draws = 0;
        switch (m->type) {
        case RT_LAMBERTIAN:
        case RT_METAL:
        case RT_DIELECTRIC:
            if (!scatter(s, m, o, d, &rec, st, &so, &sd, &att, &draws, order)) return mulv(emitted, cur_att);
            break;
        case RT_DIFFUSELIGHT: /* DiffuseLight::Emitted (Material.cuh:164-176) */
            emitted = m->albedo.type <= RT_IMAGE
                          ? scale((float)m->light_intensity, texture_value(s, &m->albedo, rec.u, rec.v, rec.p))
                          : mk(0.0f, 0.0f, 0.0f);
            return mulv(emitted, cur_att);
        default: return black;
        }
        cur_att = mulv(att, cur_att);
        o = so;
        d = sd;
    }
    return black;
}

/* RgbToInt (Kernel.cu:12-19) with Clamp (Math.cuh:307-310). */
static inline int f2i(float f) { return f != f ? 0 : (int)f; }
unsigned int orc_rgb_to_int(float r, float g, float b) {
    r = fclampf(r, 0.0f, 255.0f);
    g = fclampf(g, 0.0f, 255.0f);
    b = fclampf(b, 0.0f, 255.0f);
    float a = 255.0f;
    return ((unsigned)(int)a << 24) | ((unsigned)f2i(b) << 16) | ((unsigned)f2i(g) << 8) | (unsigned)f2i(r);
}

/* RenderInit (Kernel.cu:166-176) over the floor grid (CudaLayer.cpp:97-100) or every pixel. */
void orc_render_init(rt_curand_state* state, unsigned width, unsigned height, unsigned long long seed_base,
                     int full) {
    unsigned gw = full ? width : (width / 16) * 16, gh = full ? height : (height / 16) * 16;
    for (unsigned j = 0; j < gh; j++)
        for (unsigned i = 0; i < gw; i++) {
            unsigned pixel_index = j * width + i;
            orc_curand_init(seed_base + pixel_index, &state[pixel_index]);
        }
}

/* Kernel (Kernel.cu:102-158) */
void orc_render(const orc_scene* s, unsigned int* pos, float* radiance, float* accum, unsigned width, unsigned height,
                unsigned spp, unsigned max_depth, rt_curand_state* state, const rt_input_struct* in,
                int faithful_grid, unsigned row_begin, unsigned row_end, unsigned row_step, int threads,
                int order, int philox, unsigned long long seed, unsigned frame, orc_counters* counters) {
    unsigned gw = faithful_grid ? (width / 16) * 16 : width;
    unsigned gh = faithful_grid ? (height / 16) * 16 : height;
    if (row_end > gh) row_end = gh;
    if (row_step == 0) row_step = 1;
    long nrows = row_end > row_begin ? (long)((row_end - row_begin + row_step - 1) / row_step) : 0;
    v3 origin = ld3(in->origin), fwd = ld3(in->orientation), up = ld3(in->up);
    v3 right = normalize(cross(up, fwd));
    v3 center = mk(width / 2.0f, height / 2.0f, 0.0f);
    unsigned long long rays = 0, boxes = 0, prims = 0, primary = 0, rects = 0;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : rays, boxes, prims, primary, rects)
#endif
    for (long ri = 0; ri < nrows; ri++) {
        int y = (int)(row_begin + (unsigned)ri * row_step);
        orc_counters c = {0, 0, 0, 0, 0};
        for (int x = 0; x < (int)gw; x++) {
            unsigned pixel_index = (unsigned)y * width + (unsigned)x;
            rt_curand_state st;
            orc_rng g;
            memset(&g, 0, sizeof(g));
            if (philox) { /* no per-pixel state in HBM: the stream is a function of (seed, pixel, frame) */
                g.philox = 1;
                g.key[0] = (unsigned)seed;
                g.key[1] = (unsigned)(seed >> 32);
                g.frame = frame;
                g.pixel = pixel_index;
            } else {
                st = state[pixel_index];
                g.xs = &st;
            }
            v3 col = mk(0.0f, 0.0f, 0.0f);
            unsigned q[3] = {0u, 0u, 0u}; /* Philox: the fixed-point sum */
            for (unsigned smp = 0; smp < spp; smp++) {
                if (philox) g.n = smp << 18; /* the sample's own window: block smp << 16 */
                orc_group(&g);
                float u = ((float)((float)x - center.x) + orc_uniform(&g)) / (float)width;
                float v = ((float)(center.y - (float)y) + orc_uniform(&g)) / (float)width;
                v3 dist = add(scale(u, right), scale(v, up));
                v3 start = add(add(scale(in->near_plane, dist), origin), scale(in->fov, fwd));
                v3 second = add(add(scale(in->far_plane, dist), scale(1.0f / in->fov * 10.0f, fwd)), origin);
                v3 dir = normalize(sub(second, start));
                c.primary++;
                v3 cs = color(s, start, dir, (int)max_depth, &g, in, order, &c);
                if (philox) {
                    q[0] = orc_sat_add(q[0], orc_quant(cs.x));
                    q[1] = orc_sat_add(q[1], orc_quant(cs.y));
                    q[2] = orc_sat_add(q[2], orc_quant(cs.z));
                } else {
                    col = add(col, cs);
                }
            }
            if (philox) col = mk((float)q[0] * (1.0f / 4096.0f), (float)q[1] * (1.0f / 4096.0f), (float)q[2] * (1.0f / 4096.0f));
            if (!philox) state[pixel_index] = st;
            if (accum) { /* progressive accumulation (not in the reference): running sum of
                            samples and sample count per pixel, the image shows their quotient */
                float* ap = accum + 4 * (size_t)pixel_index;
                ap[0] = ap[0] + col.x; ap[1] = ap[1] + col.y; ap[2] = ap[2] + col.z; ap[3] = ap[3] + (float)spp;
                col = divs(mk(ap[0], ap[1], ap[2]), ap[3]);
            } else {
                col = divs(col, (float)spp);
            }
            if (radiance) {
                float* rp = radiance + 4 * (size_t)pixel_index;
                rp[0] = col.x; rp[1] = col.y; rp[2] = col.z; rp[3] = 1.0f;
            }
            col.x = 255.0f * sqrtf(col.x);
            col.y = 255.0f * sqrtf(col.y);
            col.z = 255.0f * sqrtf(col.z);
            pos[pixel_index] = orc_rgb_to_int(col.x, col.y, col.z);
        }
        rays += c.rays; boxes += c.box_tests; prims += c.prim_tests; primary += c.primary; rects += c.rect_tests;
    }
    if (counters) {
        counters->rays = rays; counters->box_tests = boxes; counters->prim_tests = prims; counters->primary = primary;
        counters->rect_tests = rects;
    }
}

/* ---------------------------------------------------------------------------------------------- */
/* Known-answer helpers                                                                             */
/* ---------------------------------------------------------------------------------------------- */
int orc_hittable_hit(const rt_hittable_desc* h, const float o[3], const float d[3], float tmin, float tmax,
                     orc_hit* out) {
    hitrec rec;
    memset(&rec, 0, sizeof(rec));
    int hit = prim_hit(h, ld3(o), ld3(d), tmin, tmax, &rec);
    memset(out, 0, sizeof(*out));
    out->hit = hit;
    if (hit) {
        out->t = rec.t;
        out->p[0] = rec.p.x; out->p[1] = rec.p.y; out->p[2] = rec.p.z;
        out->normal[0] = rec.normal.x; out->normal[1] = rec.normal.y; out->normal[2] = rec.normal.z;
        out->u = rec.u; out->v = rec.v;
        out->front_face = rec.front_face;
    }
    return hit;
}

int orc_scatter(const rt_material_desc* m, const float o[3], const float d[3], const orc_hit* h,
                rt_curand_state* st, float so[3], float sd[3], float att[3], int* draws, int order) {
    orc_scene s;
    memset(&s, 0, sizeof(s));
    hitrec rec;
    rec.p = ld3(h->p); rec.normal = ld3(h->normal); rec.t = h->t; rec.u = h->u; rec.v = h->v;
    rec.front_face = h->front_face; rec.mat = 0;
    v3 o3, d3, a3 = mk(0.0f, 0.0f, 0.0f);
    o3 = d3 = a3;
    *draws = 0;
    orc_rng g;
    memset(&g, 0, sizeof(g));
    g.xs = st;
    int r = scatter(&s, m, ld3(o), ld3(d), &rec, &g, &o3, &d3, &a3, draws, order);
    so[0] = o3.x; so[1] = o3.y; so[2] = o3.z;
    sd[0] = d3.x; sd[1] = d3.y; sd[2] = d3.z;
    att[0] = a3.x; att[1] = a3.y; att[2] = a3.z;
    return r;
}
