// render.hip — the MI355X (gfx950) per-pixel path-trace kernel and its launchers.
//
// Replaces __global__ Kernel / RenderInit / RandInit and the extern "C" launchers of
// CudaRayTracer/src/Cuda/Kernel.cu:102-204.  Design:
//   * one lane per pixel; a 256-thread workgroup renders a 16×16 pixel tile, each wave64 an 8×8 sub-tile
//     so the primary rays of a wave are coherent;
//   * the sample loop (Kernel.cu:137) and the bounce loop of color() (Kernel.cu:39) are flattened into
//     ONE per-lane ray loop: a lane whose path ends starts its next sample at once instead of idling until
//     the slowest lane of the wave finishes its path.  The per-lane order of RNG draws, and so the result,
//     is unchanged;
//   * closest hit through a binary BVH whose child boxes sit in the parent node (one 64-B node fetch
//     tests two boxes), near-child-first traversal with a short per-lane stack; the scene tables are
//     read through the L1/L2 or staged in LDS (template choice);
//   * the cuRAND XORWOW state (Kernel.cu:123, 149) lives in VGPRs for the whole frame: 24 B loaded and
//     24 B stored per pixel;
//   * no MFMA: there is no dense contraction on this path.
//
// Arithmetic contract (bit-for-bit with oracle/rt_oracle.c): this file is compiled with
// -ffp-contract=off; every +,-,*,/ and sqrtf of the reference expressions is one correctly rounded
// binary32 operation, in the reference's association order.  Only the slab test of the BVH boxes uses
// explicit FMAs: boxes are padded outward on the host, so box culling never rejects a primitive the
// exact test accepts and the closest hit is decided by the exact primitive tests alone.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <map>
#include <numeric>
#include <memory>
#include <mutex>
#include <tuple>
#include <type_traits>
#include <vector>

#include "rt_internal.h"
#include "rt_scene_device.h"

namespace rt {
namespace dev {

// ---------------------------------------------------------------------------------------------------
// Vec3 algebra (Utils/Math.cuh:16-229), one IEEE op per component, reference association order.
// ---------------------------------------------------------------------------------------------------
struct f3 {
    float x, y, z;
};

// BVH node layouts read by the v3/v4 traversal (template argument NODES): 48 B of child boxes + a
// separate table of packed 16-bit child references, or the 64-B node with both (rt_internal.h)
enum NodeLayout { NODES_48 = 0, NODES_64 = 2 };
__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 mulv(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ f3 scale(float t, f3 v) { return mk(t * v.x, t * v.y, t * v.z); }
__device__ __forceinline__ f3 divs(f3 v, float t) { return mk(v.x / t, v.y / t, v.z / t); }
__device__ __forceinline__ f3 neg(f3 v) { return mk(-v.x, -v.y, -v.z); }
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// sqrtf(x) for x >= 2^-96 (finite or +inf): the instruction sequence LLVM emits for the correctly rounded
// square root — v_sqrt_f32 and a residual check of its two neighbours — without the small-input scaling
// and the 0/inf class test, neither of which changes the result in that range (saves ~24 of ~54 cycles).
__device__ __forceinline__ float sqrt_rn(const float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sdn = __uint_as_float(__float_as_uint(s) - 1u), sup = __uint_as_float(__float_as_uint(s) + 1u);
    float r = __builtin_fmaf(-sdn, s, x) <= 0.0f ? sdn : s;
    r = __builtin_fmaf(-sup, s, x) > 0.0f ? sup : r;
    return r;
}
// sqrtf(x) bit for bit: sqrt_rn in its range, LLVM's full sequence (a branch no lane usually takes) below it
__device__ __forceinline__ float sqrt_fast(const float x) { return x >= 0x1p-96f ? sqrt_rn(x) : sqrtf(x); }
// RN(1/a) for |a| in [2^-40, 2^40]: v_rcp_f32 and one FMA Newton step — equal to the IEEE division for every
// binary32 in that range, both signs (tools/check_rcp.hip, exhaustive on MI355X) — 12 issue cycles instead of
// the ~36-cycle division sequence.  rcp_ieee keeps the IEEE division outside the range (a branch no lane
// usually takes).
__device__ __forceinline__ bool in_rcp_range(const float a) {
    const float m = fabsf(a);
    return m >= 0x1p-40f && m <= 0x1p40f;
}
__device__ __forceinline__ float rcp_rn(const float a) {
    const float y = __builtin_amdgcn_rcpf(a);
    return __builtin_fmaf(__builtin_fmaf(-a, y, 1.0f), y, y);
}
__device__ __forceinline__ float rcp_ieee(const float a) {
    float r;
    if (in_rcp_range(a)) r = rcp_rn(a);
    else r = 1.0f / a;
    return r;
}
__device__ __forceinline__ float length(f3 v) { return sqrt_fast(v.x * v.x + v.y * v.y + v.z * v.z); }
__device__ __forceinline__ f3 unit_vector(f3 v) { return divs(v, length(v)); }
__device__ __forceinline__ f3 normalize(f3 v) {
    float inv = rcp_ieee(sqrt_fast(dot(v, v)));
    return scale(inv, v);
}
// x / a correctly rounded from y = RN(1/a) (a one-off IEEE division) in five 2-cycle ops instead of the
// ~36-cycle div_scale/rcp/div_fmas/div_fixup sequence: two residual corrections, the last of which is
// exact by Markstein's theorem once its input is within an ulp.  Valid for |a| in [2^-40, 2^40] and
// |x| >= 2^-100 or x == +0 (tools/check_fastdiv.c checks 1e10 random and near-tie cases bit for bit).
__device__ __forceinline__ float div_rn(const float x, const float a, const float y) {
    const float q0 = x * y;
    const float q1 = __builtin_fmaf(__builtin_fmaf(-a, q0, x), y, q0);
    return __builtin_fmaf(__builtin_fmaf(-a, q1, x), y, q1);
}
// divs(v, s) bit for bit, from y = RN(1/s) with |s| in [2^-40, 2^40] (y = 0 selects the IEEE division):
// the fast path needs every |v_i / s| >= 2^-50 (so |v_i| >= 2^-90), anything else divides the IEEE way.
__device__ __forceinline__ f3 divs_rn(const f3 v, const float s, const float y) {
    const f3 q0 = mk(v.x * y, v.y * y, v.z * y);
    if (fminf(fminf(fabsf(q0.x), fabsf(q0.y)), fabsf(q0.z)) >= 0x1p-50f) {
        const float qx = __builtin_fmaf(__builtin_fmaf(-s, q0.x, v.x), y, q0.x);
        const float qy = __builtin_fmaf(__builtin_fmaf(-s, q0.y, v.y), y, q0.y);
        const float qz = __builtin_fmaf(__builtin_fmaf(-s, q0.z, v.z), y, q0.z);
        return mk(__builtin_fmaf(__builtin_fmaf(-s, qx, v.x), y, qx), __builtin_fmaf(__builtin_fmaf(-s, qy, v.y), y, qy),
                  __builtin_fmaf(__builtin_fmaf(-s, qz, v.z), y, qz));
    }
    return divs(v, s);
}
// x / a bit for bit: div_rn from RN(1/a) inside its proven range (|a| in [2^-40, 2^40], |x| in [2^-100, 2^100] or
// x == +0), the IEEE division (a branch no lane usually takes) elsewhere.
__device__ __forceinline__ float fdiv(const float x, const float a) {
    const float m = fabsf(x);
    float r;
    if (in_rcp_range(a) && ((m >= 0x1p-100f && m <= 0x1p100f) || __float_as_uint(x) == 0u)) r = div_rn(x, a, rcp_rn(a));
    else r = x / a;
    return r;
}
__device__ __forceinline__ float recip_in_range(const float s) {
    return in_rcp_range(s) ? rcp_rn(s) : 0.0f;
}
__device__ __forceinline__ f3 reflect(f3 v, f3 n) { return sub(v, scale(2.0f * dot(v, n), n)); }
__device__ __forceinline__ float clampf(float x, float a, float b) { return (x < a) ? a : ((x > b) ? b : x); }
__device__ __forceinline__ f3 xyz(float4 v) { return mk(v.x, v.y, v.z); }

// ---------------------------------------------------------------------------------------------------
// cuRAND XORWOW (curand_kernel.h: curand(), _curand_uniform) in registers.
// ---------------------------------------------------------------------------------------------------
struct Rng {
    uint32_t d, v0, v1, v2, v3, v4;
};
__device__ __forceinline__ float uniform(Rng& s) {
    uint32_t t = s.v0 ^ (s.v0 >> 2);
    s.v0 = s.v1;
    s.v1 = s.v2;
    s.v2 = s.v3;
    s.v3 = s.v4;
    uint32_t t2;  // t << 1 as a full-rate add (v_lshlrev_b32 issues at half rate on gfx950)
    asm("v_add_u32 %0, %1, %1" : "=v"(t2) : "v"(t));
    s.v4 = (s.v4 ^ (s.v4 << 4)) ^ (t ^ t2);
    s.d += 362437u;
    uint32_t x = s.v4 + s.d;
    // x·2^-32 + 2^-33 (_curand_uniform): the product is exact, so one fma rounds like the mul + add
    return __builtin_fmaf((float)x, 2.3283064e-10f, 2.3283064e-10f / 2.0f);
}

// RandomInUnitSphere (Math.cuh:252-260) with Random() (Math.cuh:231-234).  rtl: the components of
// Vec3(ξa, ξb, ξc) are filled right to left (z = first draw), as the survey's g++ build evaluated it.
// Groups of consecutive draws (same values, same order as that many uniform() calls).  For the XORWOW
// state these are plain sequences; the Philox engine overloads them so a group generates at most one new
// block of four words (one generation site per group instead of one per draw).
template <class R> __device__ __forceinline__ void draw2(R& s, float& a, float& b) {
    a = uniform(s);
    b = uniform(s);
}
template <class R> __device__ __forceinline__ void draw3(R& s, float& a, float& b, float& c) {
    a = uniform(s);
    b = uniform(s);
    c = uniform(s);
}

// 2·ξ − 1 of each component with one fma: 2·ξ is exact, so it rounds like the reference's mul + sub.  The
// fill order is two selects per attempt (a launch-uniform branch around the loop measured the same).
template <class R>
__device__ __forceinline__ f3 random_in_unit_sphere(R& s, bool rtl) {
    f3 p;
    do {
        float a, b, c;
        draw3(s, a, b, c);
        const f3 r = rtl ? mk(c, b, a) : mk(a, b, c);
        p = mk(__builtin_fmaf(2.0f, r.x, -1.0f), __builtin_fmaf(2.0f, r.y, -1.0f), __builtin_fmaf(2.0f, r.z, -1.0f));
    } while (p.x * p.x + p.y * p.y + p.z * p.z >= 1.0f);
    return p;
}

// The same call resumable (flat kernels, RT_TUNE_RIUS_TRIPS): at most `cap` attempts now; false when every one of them was
// rejected, and the lane resumes the call at the wave's next shading pass (its RNG state advanced by exactly the
// attempts made, so the draws, and the accepted point, are those of the uninterrupted loop).  A wave otherwise runs
// the loop as long as its unluckiest lane: ~4.5 trips for ~1.9 attempts per lane (acceptance π/6).
__device__ __forceinline__ bool random_in_unit_sphere_capped(Rng& s, bool rtl, uint32_t cap, f3& p) {
    uint32_t n = 0u;
    bool inside;
    do {
        float a, b, c;
        draw3(s, a, b, c);
        const f3 r = rtl ? mk(c, b, a) : mk(a, b, c);
        p = mk(__builtin_fmaf(2.0f, r.x, -1.0f), __builtin_fmaf(2.0f, r.y, -1.0f), __builtin_fmaf(2.0f, r.z, -1.0f));
        inside = p.x * p.x + p.y * p.y + p.z * p.z < 1.0f;
    } while (!inside && ++n < cap);
    return inside;
}

// ---------------------------------------------------------------------------------------------------
// Kernel parameters (by value; everything launch-uniform precomputed on the host with the same
// binary32 operations the reference performs per thread).
// ---------------------------------------------------------------------------------------------------
struct KParams {
    const float4* nodes;
    const float4* nodes48;   // v3: three box float4 per node
    const uint32_t* refs;    // v3: child references per node: two 16-bit in one word, or (wide) two words
    const float4* prims;
    const float4* mats;
    const int4* imgs;
    const uint8_t* texels;
    uint32_t* pos;
    float4* radiance;
    float4* accum;
    uint32_t* state;  // XORWOW states: 12-word rt_curand_state per pixel, or (RT_FLAG_STATE_SOA) six planes
    uint32_t state_stride;  // distance between a pixel's state words: 1 (rt_curand_state) or the plane size
    unsigned long long* counters;
    uint32_t num_nodes, num_prims;
    uint32_t num_mats, num_imgs;  // material / image table entries (the persistent flat kernel stages them in LDS)
    uint32_t width, height, spp, max_depth, flags;
    uint32_t band_rows, num_ranks, rank, local_rows;
    uint32_t tiles_x;
    uint32_t grid_w, grid_h;  // pixels rendered: x < grid_w, global row < grid_h
    uint32_t rius_rtl;
    float width_f, cx, cy;
    float inv_width;  // RN(1.0f / width_f) for div_rn
    float near_plane, far_plane;
    float origin[3], up[3], right[3];
    float fov_fwd[3];  // inputs.fov * forwardV           (Kernel.cu:142)
    float k10_fwd[3];  // (1.0f / inputs.fov * 10.0f) * forwardV (Kernel.cu:143)
    float bg0[3], bg1[3];
    uint32_t regen_threshold;  // v2: lanes still tracing below which finished lanes are regenerated
    uint32_t* work_counter;    // v4: the frame's kQueueCounters queue heads, queue_stride words apart (zeroed before
                               // the launch), then the exhausted-heads word
    uint32_t queue_stride;     // v4: words between queue heads (RT_TUNE_QUEUE_STRIDE; 32 = 128 B)
    uint32_t work_chunk;       // v4: work indices a wave takes per atomic while its head has plenty left
                               // (RT_TUNE_QUEUE_CHUNK; a multiple of 64); 64 near the head's end
    uint32_t work_total;       // v4: work indices in the frame (64 per 8×8 tile)
    uint32_t work_per_counter; // v4: indices per queue head (a multiple of 64): head k owns [k·n, (k+1)·n)
    uint32_t queue_prefetch;   // persistent kernels: fetch the next chunk once at most this many indices are left (0: off)
    uint32_t queue_guide, queue_min;  // persistent kernels: guided chunk sizes (PixelQueue::chunk_want; 0: off)
    uint32_t lds_wave_words;   // v3/v4: LDS words per wave (parked state + stack)
    uint32_t rng_key_lo, rng_key_hi, rng_frame;  // RT_FLAG_RNG_PHILOX: Philox key (seed) and frame counter
    unsigned long long* wave_trace;  // diagnostic: v3 / flat per tile {start, end} of s_memrealtime (100 MHz); the
                                     // persistent kernels per wave kWaveTraceWords words (trace_persistent_wave)
    unsigned long long wave_trace_words;  // its size; a stamp that would not fit is not written
    const uint32_t* tile_order;      // v3: launch order of the 8×8 tiles (NULL = row-major); persistent kernels: the
                                     // tile of work tile slot i (the queue hands out slots in order)
    uint8_t* pixel_cost;             // persistent flat: per work index, the passes its pixel took (cost-ordered queue)
    float4* ray_dump;                // diagnostic (v3, COUNT_TESTS builds): rays that start at bounce ray_dump_depth,
    uint32_t* ray_dump_count;        // appended as (origin, 0), (direction, 0) pairs; the count of rays offered
    uint32_t ray_dump_cap, ray_dump_depth;  // (rt_set_ray_dump; tools/coherence.py)
    uint32_t* tile_cost;             // v3: per tile, the wave's lifetime (s_memtime cycles / 256) of this launch
    uint32_t num_tiles;              // v3: tiles of the (local) image; slots beyond it carry no tile
    uint32_t regen_live_frac;        // v3: threshold cap as a fraction of the wave's live pixels (x/64; 0 = off)
    uint32_t leaf_break;             // v3: leave the node loop once at most this many lanes still lack a leaf
    uint32_t rius_cap;               // flat: RandomInUnitSphere attempts per shading pass (0xffffffff = unbounded)
    const float4* ref_nodes;         // flat kernel: the reference BVH over the flat table (ref_trace_wave's root box)
    const float4* flat_ref_pairs;    // flat kernel: the same tree as child-pair records (ref_trace_wave)
    const float4* flat_boxes;        // flat kernel: per flat record its reference box (flat_trace's exactness check)
    uint32_t flat_runs[2];           // flat kernel: [begin, end) of each primitive type's run in the flat table
    const float4* bvh_ref_nodes;     // BVH kernels: the reference BVH over `prims` (bvh_clear), NULL = no replay
    const float4* bvh_boxes;         // BVH kernels: per `prims` record its reference box (bvh_clear)
    const float4* bvh_ref_pairs;     // BVH kernels: per reference node its children's boxes and refs (ref_trace_wave)
    uint32_t bvh_has_rects;          // BVH kernels: the scene holds a rectangle (bvh_clear's check of misses)
    uint32_t prefetch_stop;          // persistent flat: next pixels are taken ahead while the head holds > 1/this (0: never)
    uint32_t group_tiles;            // persistent flat, GROUP: tiles [0, group_tiles) are the workgroups' static shares
    uint32_t queue_base;             // persistent kernels: the queue's first work index (GROUP: group_tiles * 64; v4: 0)
    uint32_t group_perm_a;           // GROUP: 0 = interleaved shares; else the shares' golden-ratio step (GroupShare)
    uint32_t group_perm_b, group_perm_k;  // ... (group_perm_k · group_perm_a) mod group_tiles, and tiles per share
    uint32_t queue_host_reset;       // persistent kernels: 1 = rt_render zeroed the queue slot (no queue_release)
    uint32_t linger_ticks;           // persistent flat, GROUP: a finished workgroup waits at most this long (100 MHz
                                     // ticks) for the grid's others before it exits (group_linger; 0: it does not)
    uint32_t group_chunk;            // ... positions per chunk (a multiple of 64)
};

constexpr int kStackMax = 64;
constexpr int kBlock = 256;
// v4 work queue: the frame's work indices are split into this many contiguous ranges, each with its own
// head 128 B from the next — one shared head serialises every wave's atomic in one L2 channel (≈ 16 ns
// each: 0.5 ms for the 32400 chunks of a 1080p frame, the whole C5 frame time)
constexpr uint32_t kQueueCounters = 16;
// A work-queue slot's words (each queue_stride apart): the heads, the exhausted-heads word, the finished count
// (queue_release) and the arrived workgroups (group_linger)
constexpr uint32_t kQueueSlotWords = kQueueCounters + 3;  // <= 32: one word marks the exhausted heads (1-1024 heads measured)
static_assert(kQueueCounters >= 1 && kQueueCounters <= 32, "queue heads");
constexpr uint32_t kQueueAllDone = kQueueCounters == 32 ? 0xffffffffu : (1u << kQueueCounters) - 1u;

// Traversal stack of each kernel family: per-lane scratch array (v1, any scene), 32-bit LDS entries
// (v2, 32-bit references), 16-bit LDS entries (v3/v4, scenes whose references fit 16 bits)
enum StackKind { STACK_SCRATCH = 0, STACK_LDS = 1, STACK_LDS16 = 3, STACK_NONE = 4 };

// Per-lane traversal stack of the v1 kernel (the fallback for scenes the LDS kernels cannot hold)
struct ScratchStack {
    int s[kStackMax];
    int n;
    __device__ __forceinline__ void init(uint32_t*) { n = 0; }
    __device__ __forceinline__ void push(int v) { s[n++] = v; }
    __device__ __forceinline__ int pop() { return s[--n]; }
    __device__ __forceinline__ bool empty() const { return n == 0; }
};

struct Counts {
    uint32_t rays, boxes, prims, primary;
    uint32_t wnode, wleaf, wshade;  // COUNT_TESTS: wave-level iterations (counted on the first active lane)
    uint32_t rects = 0;  // COUNT_TESTS: the part of `prims` that are rectangle tests (12 FLOP vs a sphere's 23)
    uint32_t replays = 0;  // COUNT_TESTS: rays whose closest hit the exactness check sent through the reference BVH
    uint32_t wnode_uniform = 0, wleaf_uniform = 0;  // COUNT_TESTS (v3): ... of them with one node / primitive
    uint64_t ctrav = 0, cshade = 0, ctotal = 0, cleaf = 0;  // COUNT_TESTS (v3): wave clock cycles per phase
    // COUNT_TESTS (v3): idle lanes summed over node iterations: pixel done / ray finished, waiting for the
    // regeneration threshold / holding a leaf while the wave still visits nodes
    uint64_t idle_nt = 0, idle_fin = 0, idle_wait = 0;
};

// 1 on the lowest active lane of the wave, 0 elsewhere (diagnostic wave-iteration counts).
__device__ __forceinline__ uint32_t wave_leader() {
    return __lane_id() == (uint32_t)(__ffsll((unsigned long long)__ballot(1)) - 1) ? 1u : 0u;
}

constexpr int kEmpty = (int)0x80000000;
constexpr float kTmin = 0.001f;  // color(): world->Hit(cur_ray, 0.001f, FLT_MAX, rec) (Kernel.cu:40)
// Conservative box culling.  A slab distance (plane - o)·(1/d) computed as fma(plane, rcp(d), -o·rcp(d)), with
// rcp within 1 ulp, differs from the exact one by at most ~3·2^-24 of itself plus ~2^-24·|plane·rcp(d)|.  The
// second term is covered by the host's outward box padding (1e-5 of the plane coordinate, scene_build.cpp);
// the first grows with the distance travelled, so the far side of every slab interval is widened by a
// relative 2^-20 (≥ 2·(3·2^-24)): a box the exact ray meets is never culled, whatever the camera distance.
// (Widening only adds box visits; the closest hit is decided by the exact primitive tests.)
constexpr float kSlabSlack = 1.0f + 0x1p-20f;
// A hit index with this bit set (bvh_clear): a primitive tied with the closest hit so far (indices are < 2^26)
constexpr int kTieBit = 0x40000000;
#ifndef RT_REPLAY_SAME_PASS
#define RT_REPLAY_SAME_PASS 0  // (A/B builds: 1 = v3 replays and shades flagged lanes in the pass that flagged them)
#endif
#ifndef RT_BVH_EXACT
#define RT_BVH_EXACT 1  // (A/B builds only: 0 = the BVH kernels without the reference replay, the round-5 kernels;
                        //  2 = the tie tracking and the check without the replay; 3 = the tie tracking alone)
#endif

// Closest hit (BVHNode::Hit, Hittable.cuh:387-439, and the primitive tests of PerformHit :470-485).
// Returns the primitive index (BVH order) or -1, and the hit distance in t_best.
template <bool COUNT>
__device__ __forceinline__ int trace(const float4* __restrict__ nodes, const float4* __restrict__ prims,
                                     uint32_t num_nodes, f3 o, f3 d, float a_dd, float& t_best, Counts& cnt) {
    t_best = FLT_MAX;
    int hit = -1;
    if (num_nodes == 0) return -1;
    // Slab test in fma form, t = lo·invd − o·invd, on boxes padded outward on the host.  A direction
    // component that is exactly 0 (e.g. a Lambertian bounce whose tiny offset vanished against a large
    // hit coordinate, (p + n + q) − p) would give inf − inf; clamping 1/d to ±1e20 keeps the test
    // conservative: the position error of the fma form (~ulp of the coordinates) stays far below the
    // 1e-5-relative box padding.
    const f3 invd = mk(fminf(fmaxf(1.0f / d.x, -1e20f), 1e20f), fminf(fmaxf(1.0f / d.y, -1e20f), 1e20f),
                       fminf(fmaxf(1.0f / d.z, -1e20f), 1e20f));
    const float oix = o.x * invd.x, oiy = o.y * invd.y, oiz = o.z * invd.z;
    ScratchStack stack;
    stack.init(nullptr);
    int node = 0;
    while (true) {
        while (node >= 0) {
            const float4 n0 = nodes[4 * node + 0];
            const float4 n1 = nodes[4 * node + 1];
            const float4 n2 = nodes[4 * node + 2];
            const float4 n3 = nodes[4 * node + 3];
            const float a0 = __builtin_fmaf(n0.x, invd.x, -oix), a1 = __builtin_fmaf(n0.y, invd.x, -oix);
            const float a2 = __builtin_fmaf(n0.z, invd.y, -oiy), a3 = __builtin_fmaf(n0.w, invd.y, -oiy);
            const float a4 = __builtin_fmaf(n2.x, invd.z, -oiz), a5 = __builtin_fmaf(n2.y, invd.z, -oiz);
            const float b0 = __builtin_fmaf(n1.x, invd.x, -oix), b1 = __builtin_fmaf(n1.y, invd.x, -oix);
            const float b2 = __builtin_fmaf(n1.z, invd.y, -oiy), b3 = __builtin_fmaf(n1.w, invd.y, -oiy);
            const float b4 = __builtin_fmaf(n2.z, invd.z, -oiz), b5 = __builtin_fmaf(n2.w, invd.z, -oiz);
            const float c0min = fmaxf(fmaxf(fminf(a0, a1), fminf(a2, a3)), fmaxf(fminf(a4, a5), kTmin));
            const float c0max = fminf(fminf(fmaxf(a0, a1), fmaxf(a2, a3)), fminf(fmaxf(a4, a5), t_best)) * kSlabSlack;
            const float c1min = fmaxf(fmaxf(fminf(b0, b1), fminf(b2, b3)), fmaxf(fminf(b4, b5), kTmin));
            const float c1max = fminf(fminf(fmaxf(b0, b1), fmaxf(b2, b3)), fminf(fmaxf(b4, b5), t_best)) * kSlabSlack;
            if (COUNT) {
                cnt.boxes += 2;
                cnt.wnode += wave_leader();
            }
            const bool h0 = c0min <= c0max;
            const bool h1 = c1min <= c1max;
            const int ch0 = __float_as_int(n3.x), ch1 = __float_as_int(n3.y);
            if (h0 && h1) {
                const bool swap = c1min < c0min;
                node = swap ? ch1 : ch0;
                stack.push(swap ? ch0 : ch1);
            } else if (h0 | h1) {
                node = h0 ? ch0 : ch1;
            } else {
                node = stack.empty() ? kEmpty : stack.pop();
            }
        }
        if (node == kEmpty) break;
        // leaf: primitives [first, first + count)
        const uint32_t leaf = ~(uint32_t)node;
        const uint32_t first = leaf >> 2, count = (leaf & 3u) + 1u;
        for (uint32_t i = first; i < first + count; i++) {
            const float4 p0 = prims[2 * i + 0];
            const float4 p1 = prims[2 * i + 1];
            const uint32_t type = __float_as_uint(p1.w) & 15u;
            if (COUNT) {
                cnt.prims++;
                cnt.rects += type != RT_SPHERE ? 1u : 0u;
                cnt.wleaf += wave_leader();
            }
            if (type == RT_SPHERE) {  // Sphere::Hit (Hittable.cuh:80-110)
                const f3 oc = sub(o, xyz(p0));
                const float b = dot(oc, d);
                const float c = dot(oc, oc) - p1.x;  // p1.x = radius · radius
                const float disc = b * b - a_dd * c;
                if (disc > 0) {
                    const float sq = sqrtf(disc);
                    float t = (-b - sq) / a_dd;
                    if (t < t_best && t > kTmin) {
                        t_best = t;
                        hit = (int)i;
                    } else {
                        const bool tied = t == t_best;  // (bvh_clear: a tie at the closest hit so far)
                        t = (-b + sq) / a_dd;
                        if (t < t_best && t > kTmin) {
                            t_best = t;
                            hit = (int)i;
                        } else if (tied || t == t_best) {
                            hit |= kTieBit;
                        }
                    }
                }
            } else {  // XY/XZ/YZRect::Hit (Hittable.cuh:140-169, 196-225, 252-281)
                const float ok = type == RT_XYRECT ? o.z : (type == RT_XZRECT ? o.y : o.x);
                const float dk = type == RT_XYRECT ? d.z : (type == RT_XZRECT ? d.y : d.x);
                const float t = (p0.x - ok) * rcp_ieee(dk);
                if (!(t < kTmin || t > t_best)) {
                    const float oa = type == RT_YZRECT ? o.y : o.x, da = type == RT_YZRECT ? d.y : d.x;
                    const float ob = type == RT_XYRECT ? o.y : o.z, db = type == RT_XYRECT ? d.y : d.z;
                    const float x = oa + t * da;
                    const float y = ob + t * db;
                    if (!(x < p0.y || x > p0.z || y < p0.w || y > p1.x)) {
                        hit = t == t_best ? (int)i | kTieBit : (int)i;  // (a rectangle re-accepts an equal t)
                        t_best = t;
                    }
                }
            }
        }
        if (stack.empty()) break;
        node = stack.pop();
    }
    return hit;
}

// The reference's own closest-hit query, replayed exactly: BVHNode::Hit (Hittable.cuh:387-439) over the tree the
// BVHNode constructor builds (ref_nodes, scene_build.cpp), with AABB::Hit (AABB.cuh:30-50) on the reference's boxes and
// its t_max bookkeeping (a node's box is tested against the closest hit as of its push).  Per lane, with a private
// stack: the v1/v2 kernels call it for the rare rays whose answer box culling could change (bvh_replay); since round 6
// the v3/v4 and flat kernels replay wave-serially instead (ref_trace_wave), without a call or private memory.
constexpr int kRefStackBvh = 32;  // > kRefTreeMaxDepthBvh: the BVH kernels' (bvh_clear)
__device__ __forceinline__ bool ref_box(const float4 lo, const float4 hi, const f3 o, const f3 inv, float t_max) {
    float t_min = kTmin;
    const float los[3] = {lo.x, lo.y, lo.z}, his[3] = {hi.x, hi.y, hi.z};
    const float os[3] = {o.x, o.y, o.z}, invs[3] = {inv.x, inv.y, inv.z};
#pragma unroll
    for (int a = 0; a < 3; a++) {
        float t0 = (los[a] - os[a]) * invs[a];
        float t1 = (his[a] - os[a]) * invs[a];
        if (invs[a] < 0.0f) {
            const float tmp = t0;
            t0 = t1;
            t1 = tmp;
        }
        t_min = t0 > t_min ? t0 : t_min;
        t_max = t1 < t_max ? t1 : t_max;
        if (t_max <= t_min) return false;
    }
    return true;
}
struct HitOut {
    int hit;
    uint32_t tag;
    float t;
};
// (not inlined: the kernels' registers are sized for their common path; the result comes back in registers)
template <int STK>
__device__ __noinline__ HitOut ref_trace(const float4* __restrict__ rnodes, const float4* __restrict__ prims, const f3 o,
                                         const f3 d) {
    int hit = -1;
    uint32_t tag = 0u;
    float t_best = FLT_MAX;  // = rec.t once something is hit (the reference's "hit_something ? rec.t : t_max")
    const f3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const float a_dd = dot(d, d);
    int stk[STK];
    float stm[STK];
    if (!ref_box(rnodes[0], rnodes[1], o, inv, FLT_MAX)) return HitOut{hit, tag, t_best};  // its own box first (:389)
    int top = 0;
    stk[0] = 0;
    stm[0] = FLT_MAX;
    while (top >= 0) {
        const int n = stk[top];
        const float tm = stm[top];
        top--;
        const float4 lo = rnodes[2 * n], hi = rnodes[2 * n + 1];
        if (!ref_box(lo, hi, o, inv, tm)) continue;
        const int ch[2] = {__float_as_int(lo.w), __float_as_int(hi.w)};
        for (int k = 0; k < 2; k++) {
            if (ch[k] >= 0) {
                top++;
                stk[top] = ch[k];
                stm[top] = t_best;
                continue;
            }
            const int i = ~ch[k];  // PerformHit (Hittable.cuh:470-485) with t_max = the closest hit so far
            const float4 q0 = prims[2 * i], q1 = prims[2 * i + 1];
            const uint32_t type = __float_as_uint(q1.w) & 15u;
            if (type == RT_SPHERE) {  // Sphere::Hit (Hittable.cuh:80-110)
                const f3 oc = sub(o, xyz(q0));
                const float b = dot(oc, d);
                const float c = dot(oc, oc) - q1.x;
                const float disc = b * b - a_dd * c;
                if (disc > 0) {
                    float t = (-b - sqrtf(disc)) / a_dd;
                    if (!(t < t_best && t > kTmin)) t = (-b + sqrtf(disc)) / a_dd;
                    if (t < t_best && t > kTmin) {
                        t_best = t;
                        hit = i;
                        tag = __float_as_uint(q1.w);
                    }
                }
            } else {  // XY/XZ/YZRect::Hit
                const float ok = type == RT_XYRECT ? o.z : (type == RT_XZRECT ? o.y : o.x);
                const float ik = type == RT_XYRECT ? inv.z : (type == RT_XZRECT ? inv.y : inv.x);
                const float t = (q0.x - ok) * ik;
                if (!(t < kTmin || t > t_best)) {
                    const float oa = type == RT_YZRECT ? o.y : o.x, da = type == RT_YZRECT ? d.y : d.x;
                    const float ob = type == RT_XYRECT ? o.y : o.z, db = type == RT_XYRECT ? d.y : d.z;
                    const float xx = oa + t * da;
                    const float yy = ob + t * db;
                    if (!(xx < q0.y || xx > q0.z || yy < q0.w || yy > q1.x)) {
                        t_best = t;
                        hit = i;
                        tag = __float_as_uint(q1.w);
                    }
                }
            }
        }
    }
    return HitOut{hit, tag, t_best};
}

// Reference exactness of the BVH kernels (v1-v4).  Their SAH tree, on padded boxes with conservative culling, returns
// the geometric closest hit p* at t*: every primitive whose test accepts the ray is tested.  The reference's
// BVHNode::Hit (Hittable.cuh:387-439) returns the same unless (a) a box on p*'s path rejects the ray, (b) another
// primitive ties at t* (which one it keeps depends on its culling and order), or (c) a NaN took part.
//   (a) The boxes on p*'s path contain p*'s own reference box as floats (SurroundingBox is fmin / fmax), each is tested
//   against the closest hit as of its push, which is >= t*, and AABB::Hit's arithmetic — (bound - o) · (1/d), then
//   max / min — is monotone in the bound and in t_max (round-to-nearest is).  So if AABB::Hit(p*'s own box, 0.001, t*)
//   accepts the ray with the reference's own arithmetic, every box on the path accepts it too; only rays it rejects —
//   a ray grazing an edge or corner of that box, a hit within rounding of the box face it enters by — can differ.
//   (b) is tracked by the leaf tests: a candidate equal to the closest hit so far sets kTieBit in the hit index, a
//   strictly closer hit clears it.  (c): a slab distance or a rectangle's t is NaN only as 0 · inf, so only on a ray
//   with a direction component outside [2^-40, 2^40] in magnitude (zero included) or a non-finite origin; such a ray
//   replays whatever it hit (the reference may test a rectangle whose own box the SAH tree culls).
// Checked by shade() (EXACT) on the hit record it loads anyway, in two stages.  Stage 1, per ray: the hit point
// p = o + t*·d (the hit record's own expression) lies inside p*'s own box by a margin of 2^-20 · S, S = Σ_a (|o_a| +
// |t*·d_a|), on every axis — AABB::Hit's computed slab distances are within ~3 ulps of the true ones and p within ~2 ulps
// of o + t*·d, so the margin leaves a factor > 4 and AABB::Hit accepts.  A sphere's test reads |p - c| < r - 2^-19 (S +
// r) per axis from the hit record's own p - c (its box is c -/+ r; the extra terms cover the rounding of p - c and of
// c -/+ r); a rectangle's in-plane axes compare p with its extents; in its plane axis, where p lies on k inside the
// box's k -/+ 0.0001, the slab distances are computed exactly as AABB::Hit does, (k -/+ 0.0001 - o) · RN(1/d), and
// compared with t* = (k - o) · RN(1/d), the rectangle test's own expression.  Stage 2, for the rays stage 1 does not
// clear (a hit near a face of its box, or coordinates too large for the margin): AABB::Hit itself on the box
// (bvh_boxes).  A ray neither clears — a rejected own box, a tie, (c) — makes shade() return SHADE_REPLAY with its
// path state untouched; the kernel replays the reference BVH for it (ref_trace over bvh_ref_nodes, whose leaves index
// the BVH-order records, at a point of its loop where few registers are live: bvh_replay) and shades the answer, marked
// kVerifiedBit (a verified miss: kVerifiedMiss), without a second check.
constexpr int kVerifiedBit = 0x20000000;  // in a hit index: the reference traversal's own answer (bvh_replay)
constexpr int kVerifiedMiss = 0x3fffffff;  // (flags 001 with an index no scene has: primitive indices are < 2^26)
__device__ __forceinline__ bool bvh_odd_ray(const f3 ro, const f3 rd) {
    // (c): a direction component outside [2^-40, 2^40] in magnitude (zero, NaN and inf included: NaN fails every
    // comparison and propagates through the sum) or a non-finite origin
    const float ax = fabsf(rd.x), ay = fabsf(rd.y), az = fabsf(rd.z);
    const float lo = fminf(fminf(ax, ay), az), hi = fmaxf(fmaxf(ax, ay), az);
    const float so = fabsf(ro.x) + fabsf(ro.y) + fabsf(ro.z);
    return !(lo >= 0x1p-40f && hi <= 0x1p40f && ax + ay + az == ax + ay + az && so <= FLT_MAX);
}
// Whether (hit, t) is the reference's answer for the ray (see above); strips kTieBit / kVerifiedBit from `hit`.
// q = p - c of a sphere hit (its normal's numerator).  (c) is tested only where it can matter: stage 1 of a sphere hit
// needs no finite 1/d (a zero or tiny component leaves its axis unconstrained in AABB::Hit: an infinite slab; NaNs fail
// its comparisons), a rectangle hit needs its plane axis' RN(1/d) to be rcp_rn's, stage 2 needs every axis'; and a
// miss can be a NaN hit of the reference's only in a scene with rectangles.
template <class PP>
__device__ __forceinline__ bool bvh_clear(PP P, int& hit, const uint32_t tag, const float t, const f3 ro, const f3 rd,
                                          const float4 p0, const float4 p1, const f3 td, const f3 p, const f3 q) {
    // flags in bits 29-31 of the hit index: 000 a hit, 010 a tie, 001 verified, 111 a miss (-1); kVerifiedMiss
    const uint32_t flags = (uint32_t)hit >> 29;
    const bool miss = hit < 0 || hit == kVerifiedMiss, tie = flags == 2u, verified = flags == 1u;
    hit = miss ? -1 : (hit & (kVerifiedBit - 1));
    if (RT_BVH_EXACT == 0 || RT_BVH_EXACT == 3 || verified) return true;  // (bvh_ref_nodes: every scene, rt_render)
    bool clear;
    if (miss) {
        clear = !(P->bvh_has_rects && bvh_odd_ray(ro, rd));
    } else {
        clear = !tie && t > kTmin;  // (a rectangle accepts t* = 0.001, which AABB::Hit's t_min rejects)
        const float S = (fabsf(ro.x) + fabsf(td.x)) + (fabsf(ro.y) + fabsf(td.y)) + (fabsf(ro.z) + fabsf(td.z));
        const uint32_t type = tag & 15u;
        if (type == RT_SPHERE) {  // own box: centre -/+ radius (Hittable.cuh:112-116)
            const float r = p0.w;
            const float R = __builtin_fmaf(S, -0x1p-19f, r * (1.0f - 0x1p-19f));
            float qm;  // max |q_a| in one v_max3 (abs source modifiers; a NaN fails the comparison below)
            asm("v_max3_f32 %0, |%1|, |%2|, |%3|" : "=v"(qm) : "v"(q.x), "v"(q.y), "v"(q.z));
            clear = clear && qm < R;
        } else {  // own box: the extents, and k -/+ 0.0001 in the plane axis (Hittable.cuh:171-181, 227-237, 283-293)
            const float m = __builtin_fmaf(S, 0x1p-20f, 0x1p-100f);
            const bool yz = type == RT_YZRECT, xy = type == RT_XYRECT, xz = type == RT_XZRECT;
            const float pa = yz ? p.y : p.x, pb = xy ? p.y : p.z;
            const float dk = xy ? rd.z : (xz ? rd.y : rd.x);
            const float ok = xy ? ro.z : (xz ? ro.y : ro.x), ik = rcp_rn(dk);
            const float s0 = (p0.x - 0.0001f - ok) * ik, s1 = (p0.x + 0.0001f - ok) * ik;
            const bool neg = ik < 0.0f;
            clear = clear && in_rcp_range(dk) && (pa - p0.y) > m && (p0.z - pa) > m && (pb - p0.w) > m &&
                    (p1.x - pb) > m && (neg ? s1 : s0) < t && (neg ? s0 : s1) > t;
        }
        if (__builtin_expect(!clear && !tie && t > kTmin && !bvh_odd_ray(ro, rd), 0)) {
            // stage 2 (rare): AABB::Hit(own box, 0.001, t*) with the reference's arithmetic
            const float4* boxes = P->bvh_boxes;
            clear = ref_box(boxes[2 * hit], boxes[2 * hit + 1], ro, mk(rcp_rn(rd.x), rcp_rn(rd.y), rcp_rn(rd.z)), t);
        }
    }
    if (RT_BVH_EXACT == 2) {  // (A/B builds: the check without the replay)
        asm volatile("" ::"v"((uint32_t)clear));
        return true;
    }
    return clear;
}
// The reference traversal's answer for a ray shade() returned SHADE_REPLAY for, marked verified.
template <class PP>
__device__ __noinline__ void bvh_replay(PP P, const float4* __restrict__ prims, int& hit, uint32_t& tag, float& t,
                                        const f3 ro, const f3 rd) {
    if (RT_BVH_EXACT == 4) {  // (A/B builds: the replay's call without the reference traversal — wrong images)
        hit = hit >= 0 ? (hit | kVerifiedBit) : kVerifiedMiss;
        return;
    }
    const HitOut r = ref_trace<kRefStackBvh>(P->bvh_ref_nodes, prims, ro, rd);
    hit = r.hit >= 0 ? (r.hit | kVerifiedBit) : kVerifiedMiss;
    tag = r.tag;
    t = r.t;
}

// The reference traversal (ref_trace's algorithm and arithmetic) for one wave-uniform ray, without a call or private
// memory: every value is uniform — node and primitive records are scalar loads, the tests' arithmetic runs on uniform
// operands — and the stack lives across the lanes of one VGPR (entry j in lane j, v_writelane / v_readlane at the
// uniform top; at most kRefTreeMaxDepthBvh + 1 < 64 entries).  Every lane of the wave must be active (v3 and v4 keep
// all 64 lanes in their loops), so no copy of the stack registers can drop a lane.
typedef const __attribute__((address_space(4))) float ConstF32R;
__device__ __forceinline__ uint32_t lane_write(uint32_t vec, const uint32_t val, const uint32_t lane) {
    // (gfx9 reads one SGPR per VALU instruction: the lane select goes through M0)
    const uint32_t v = __builtin_amdgcn_readfirstlane(val), l = __builtin_amdgcn_readfirstlane(lane);
    asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(vec) : "s"(v), "{m0}"(l));
    return vec;
}
// The node records are the child-pair table (bvh_ref_pairs: per node both children's boxes and references, 64 B):
// a child's box is tested when its parent is processed, with the closest hit as of then — the t_max the reference
// pushes it with and tests it against when it pops it — so only accepted nodes are pushed and visited, each with one
// record load (round 6: the replay's share of C2 +1.0 % with the 32-B node records, a load per pushed node).
// lstk (the flat kernels): the stack in this wave's LDS words instead of VGPR lanes — a partial tile's flat kernel
// wave has inactive lanes, which a lane stack cannot use.
__device__ __forceinline__ HitOut ref_trace_wave(const float4* __restrict__ rnodes, const float4* __restrict__ rpairs,
                                                 const float4* __restrict__ prims, const f3 o, const f3 d,
                                                 uint32_t* lstk = nullptr) {
    int hit = -1;
    uint32_t tag = 0u;
    float t_best = FLT_MAX;
    const f3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const float a_dd = dot(d, d);
    const auto rec = [](const float4* base, const uint32_t i, float4& a, float4& b) {  // 32-B record i, scalar loads
        const ConstF32R* q = (const ConstF32R*)base + 8u * i;
        a = make_float4(q[0], q[1], q[2], q[3]);
        b = make_float4(q[4], q[5], q[6], q[7]);
    };
    float4 lo, hi;
    rec(rnodes, 0u, lo, hi);
    if (!ref_box(lo, hi, o, inv, FLT_MAX)) return HitOut{hit, tag, t_best};  // its own box first (Hittable.cuh:389)
    uint32_t stk_n = 0u;  // lane 0: the root (accepted)
    if (lstk) lstk[0] = 0u;
    int top = 0;
    while (top >= 0) {
        const uint32_t n = lstk ? (uint32_t)__builtin_amdgcn_readfirstlane((int)lstk[top])
                                : (uint32_t)__builtin_amdgcn_readlane((int)stk_n, top);
        top--;
        float4 cl[2], ch[2];
        rec(rpairs, 2u * n, cl[0], ch[0]);
        rec(rpairs, 2u * n + 1u, cl[1], ch[1]);
        for (int k = 0; k < 2; k++) {
            const int ref = __float_as_int(cl[k].w);
            if (ref >= 0) {  // an inner node: pushed if its box accepts with t_max = the closest hit so far
                if (ref_box(cl[k], ch[k], o, inv, t_best)) {
                    top++;
                    if (lstk) lstk[top] = (uint32_t)ref;
                    else stk_n = lane_write(stk_n, (uint32_t)ref, (uint32_t)top);
                }
                continue;
            }
            const uint32_t i = (uint32_t)~ref;  // PerformHit (Hittable.cuh:470-485) with t_max = the closest hit so far
            float4 q0, q1;
            rec(prims, i, q0, q1);
            const uint32_t type = __float_as_uint(q1.w) & 15u;
            if (type == RT_SPHERE) {  // Sphere::Hit (Hittable.cuh:80-110)
                const f3 oc = sub(o, xyz(q0));
                const float b = dot(oc, d);
                const float c = dot(oc, oc) - q1.x;
                const float disc = b * b - a_dd * c;
                if (disc > 0) {
                    float t = (-b - sqrtf(disc)) / a_dd;
                    if (!(t < t_best && t > kTmin)) t = (-b + sqrtf(disc)) / a_dd;
                    if (t < t_best && t > kTmin) {
                        t_best = t;
                        hit = (int)i;
                        tag = __float_as_uint(q1.w);
                    }
                }
            } else {  // XY/XZ/YZRect::Hit
                const float ok = type == RT_XYRECT ? o.z : (type == RT_XZRECT ? o.y : o.x);
                const float ik = type == RT_XYRECT ? inv.z : (type == RT_XZRECT ? inv.y : inv.x);
                const float t = (q0.x - ok) * ik;
                if (!(t < kTmin || t > t_best)) {
                    const float oa = type == RT_YZRECT ? o.y : o.x, da = type == RT_YZRECT ? d.y : d.x;
                    const float ob = type == RT_XYRECT ? o.y : o.z, db = type == RT_XYRECT ? d.y : d.z;
                    const float xx = oa + t * da;
                    const float yy = ob + t * db;
                    if (!(xx < q0.y || xx > q0.z || yy < q0.w || yy > q1.x)) {
                        t_best = t;
                        hit = (int)i;
                        tag = __float_as_uint(q1.w);
                    }
                }
            }
        }
    }
    return HitOut{hit, tag, t_best};
}
// acos / atan2 of GetSphereUV (Hittable.cuh:119-125) as fixed sequences of binary32 +, -, *, / and sqrt
// (Cephes asinf/atanf polynomials, ~2 ulp), identical operation for operation in oracle/rt_oracle.c.  The
// reference's CUDA acos/atan2 under -use_fast_math cannot be reproduced, and the device library's and
// libm's acosf/atan2f disagree in the last bit now and then, which moves a lookup into an 8192-wide texture
// by one texel.  The acos argument is clamped to [-1, 1] (a rounded normal can exceed 1 by an ulp).
__device__ __forceinline__ float rt_asin_poly(const float x) {  // |x| <= 0.5
    const float z = x * x;
    const float p = (((4.2163199048e-2f * z + 2.4181311049e-2f) * z + 4.5470025998e-2f) * z + 7.4953002686e-2f) * z +
                    1.6666752422e-1f;
    return p * z * x + x;
}
__device__ __forceinline__ float rt_acosf(float x) {
    x = x < -1.0f ? -1.0f : (x > 1.0f ? 1.0f : x);
    if (x < -0.5f) return 0x1.921fb6p+1f - 2.0f * rt_asin_poly(sqrt_fast(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * rt_asin_poly(sqrt_fast(0.5f * (1.0f - x)));
    return 0x1.921fb6p+0f - rt_asin_poly(x);
}
__device__ __forceinline__ float rt_atan_poly(const float x) {  // |x| <= tan(pi/8)
    const float z = x * x;
    return (((8.05374449538e-2f * z - 1.38776856032e-1f) * z + 1.99777106478e-1f) * z - 3.33329491539e-1f) * z * x + x;
}
__device__ __forceinline__ float rt_atan01(const float t) {  // t in [0, 1]
    if (t > 0.41421356f) return 0x1.921fb6p-1f + rt_atan_poly(fdiv(t - 1.0f, t + 1.0f));
    return rt_atan_poly(t);
}
__device__ __forceinline__ float rt_atan2f(const float y, const float x) {
    const float ax = fabsf(x), ay = fabsf(y);
    float r;
    if (ax == 0.0f && ay == 0.0f) r = 0.0f;
    else if (ay <= ax) r = rt_atan01(fdiv(ay, ax));
    else r = 0x1.921fb6p+0f - rt_atan01(fdiv(ax, ay));
    if (__builtin_signbit(x)) r = 0x1.921fb6p+1f - r;  // IEEE atan2: x < 0 or -0
    return __builtin_signbit(y) ? -r : r;
}

// Texture::value (Texture.cuh:42-45, 58-67, 83-105) in two steps: texture_fetch returns the colour, or for an image the
// address of the texel, texture_gather loads it as one dword and texture_resolve turns it into the colour.  shade()
// issues the gather for every lane of its Lambertian / Metal path (a lane without a texel reads a dummy word) and
// resolves it after RandomInUnitSphere: no branch between the load and its use, so the compiler waits for it only
// there and the round trip overlaps the rejection loop.  Each image is followed by >= 4 spare bytes (scene_build.cpp):
// the RGB8 layout's dword reads one byte past its texel, which the colour ignores.
struct TexFetch {
    f3 color;              // the colour, unless pending
    const uint8_t* texel;  // pending: the texel's first byte
    bool pending;
};
__device__ __forceinline__ TexFetch texture_fetch(const float4& m0, const float4& m1, const float4& m2, uint32_t tex_type,
                                                  float u, float v, f3 p, const int4* __restrict__ imgs,
                                                  const uint8_t* __restrict__ texels) {
    TexFetch f{mk(0.0f, 0.0f, 0.0f), nullptr, false};
    if (tex_type == RT_CONSTANT) {
        f.color = xyz(m1);
    } else if (tex_type == RT_CHECKER) {
        const float sines = sinf(10 * p.x) * sinf(10 * p.y) * sinf(10 * p.z);
        f.color = sines < 0 ? xyz(m1) : xyz(m2);
    } else if (tex_type == RT_IMAGE) {
        const int img = __float_as_int(m0.w);
        const int4 im = img < 0 ? make_int4(-1, 0, 0, 0) : imgs[img];  // (byte offset of the texels, width, height,
                                                                      //  bytes per texel)
        if (im.x < 0) {  // no image / data == nullptr (Texture.cuh:83-84) → cyan
            f.color = mk(0.0f, 1.0f, 1.0f);
        } else {
            u = clampf(u, 0.0f, 1.0f);
            v = 1.0f - clampf(v, 0.0f, 1.0f);
            int i = (int)(u * (float)im.y);
            int j = (int)(v * (float)im.z);
            if (i >= im.y) i = im.y - 1;
            if (j >= im.z) j = im.z - 1;
            // RGBA8-padded layout: 4 bytes per texel; the reference's RGB8 layout (Texture.cuh:76, 96-104): 3
            f.texel = texels + im.x + ((size_t)j * (size_t)im.y + (size_t)i) * (size_t)im.w;
            f.pending = true;
        }
    }
    return f;
}
// An RGB8 texel's dword is not 4-byte aligned: loaded through an alignment-1 type (one global_load_dword on gfx950,
// whose vector memory accesses need no alignment)
typedef uint32_t UnalignedU32 __attribute__((aligned(1)));
__device__ __forceinline__ uint32_t texture_gather(const TexFetch& f, const void* dummy) {
    return *reinterpret_cast<const UnalignedU32*>(f.pending ? f.texel : reinterpret_cast<const uint8_t*>(dummy));
}
__device__ __forceinline__ f3 texture_resolve(const TexFetch& f, uint32_t w) {
    if (!f.pending) return f.color;
    const float color_scale = 1.0f / 255.0f;
    return mk(color_scale * (float)(w & 0xffu), color_scale * (float)((w >> 8) & 0xffu),
              color_scale * (float)((w >> 16) & 0xffu));
}
__device__ __forceinline__ f3 texture_value(const float4& m0, const float4& m1, const float4& m2, uint32_t tex_type,
                                            float u, float v, f3 p, const int4* __restrict__ imgs,
                                            const uint8_t* __restrict__ texels) {
    const TexFetch f = texture_fetch(m0, m1, m2, tex_type, u, v, p, imgs, texels);
    return f.pending ? texture_resolve(f, *reinterpret_cast<const UnalignedU32*>(f.texel)) : f.color;
}

__device__ __forceinline__ uint32_t f2u8(float f) { return f != f ? 0u : (uint32_t)(int)f; }

// RgbToInt (Kernel.cu:12-19)
__device__ __forceinline__ uint32_t rgb_to_int(float r, float g, float b) {
    r = clampf(r, 0.0f, 255.0f);
    g = clampf(g, 0.0f, 255.0f);
    b = clampf(b, 0.0f, 255.0f);
    return (255u << 24) | (f2u8(b) << 16) | (f2u8(g) << 8) | f2u8(r);
}

__device__ __forceinline__ uint32_t global_row(const KParams& P, uint32_t local_row) {
    const uint32_t band = local_row / P.band_rows, within = local_row - band * P.band_rows;
    return (band * P.num_ranks + P.rank) * P.band_rows + within;
}

// Launch-uniform camera / background terms (kernel arguments, SGPR-resident).
struct Camera {
    f3 origin, up, right, fov_fwd, k10_fwd;
    float xf, yf;  // (x - center.x()), (center.y() - y) of this lane's pixel (Kernel.cu:139-140)
};

// Camera ray of one sample (Kernel.cu:139-146): two uniforms, then the reference's plane construction.
template <class PP, class R>
__device__ __forceinline__ void camera_ray(PP P, const Camera& cam, R& rng, f3& ro, f3& rd, uint32_t sample) {
    begin_sample(rng, sample);  // (Philox mode: the sample's own window of the pixel's stream)
    float xi1, xi2;
    draw2(rng, xi1, xi2);
    // (x - cx + ξ) / width: the dividend is +0 or at least 2^-33 in magnitude (ξ in (0, 1]), inside div_rn's range
    const float u = div_rn(cam.xf + xi1, P->width_f, P->inv_width);
    const float v = div_rn(cam.yf + xi2, P->width_f, P->inv_width);
    const f3 dist = add(scale(u, cam.right), scale(v, cam.up));
    const f3 start = add(add(scale(P->near_plane, dist), cam.origin), cam.fov_fwd);
    const f3 second = add(add(scale(P->far_plane, dist), cam.k10_fwd), cam.origin);
    ro = start;
    rd = normalize(sub(second, start));
}

// One iteration of color()'s bounce loop after the closest-hit query (Kernel.cu:40-76): sky on a miss,
// emission, or Scatter of the hit material.  Returns SHADE_ENDED when the path ended (contribution in
// `contrib`, `emitted * cur_attenuation` or `cur_attenuation * sky`), SHADE_CONTINUE when it continues with
// (ro, rd, att).
// DEFER (flat kernels): RandomInUnitSphere makes at most P->rius_cap attempts; SHADE_DEFERRED when all were rejected — ro, rd
// and att are untouched, and the lane shades the same hit again at the next pass, continuing the same call.
enum ShadeResult { SHADE_CONTINUE = 0, SHADE_ENDED = 1, SHADE_DEFERRED = 2 };
// EXACT (the BVH kernels): `hit` may carry kTieBit / kVerifiedBit; SHADE_REPLAY when the closest hit may not be the
// reference's (bvh_clear) — nothing is changed, and the kernel replays the reference traversal (bvh_replay).
enum { SHADE_REPLAY = 3 };
template <bool TEX = true, bool DEFER = false, bool EXACT = false, class PP, class R>
__device__ __forceinline__ int shade(PP P, const float4* __restrict__ prims, const float4* __restrict__ mats,
                                     const int4* __restrict__ imgs, int hit, uint32_t hit_tag, float t,
                                     f3& ro, f3& rd, f3& att, R& rng, bool rtl, f3& contrib) {
    float4 p0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), p1 = p0;
    // unit_vector(rd) is needed by the sky (y only), Metal and Dielectric: computed once for all lanes of
    // the wave that need it instead of once per material branch (same binary32 operations, Math.cuh:210-213)
    // hit_tag: the primitive's type | material << 4 word, which the traversal already read with the winning
    // primitive — the material load need not wait for the primitive's (nor for the exactness check)
    uint32_t mtype = 0xffu;  // 0xff: miss
    if constexpr (EXACT) {
        // the hit record's and the material's loads first, both in flight during the check (a replayed hit is shaded
        // by a later call); the record of primitive 0 for a miss: read, never used
        const int h = (hit >= 0 && hit != kVerifiedMiss) ? (hit & (kVerifiedBit - 1)) : 0;
        p0 = prims[2 * h + 0];
        p1 = prims[2 * h + 1];
        uint32_t mword = 0xffu;
        if (hit >= 0 && hit != kVerifiedMiss) mword = __float_as_uint(mats[3 * (hit_tag >> 4)].x);
        const f3 td = scale(t, rd);  // (the hit point and p - c: shared with the hit record below)
        const f3 ph = add(ro, td);
        if (__builtin_expect(!bvh_clear(P, hit, hit_tag, t, ro, rd, p0, p1, td, ph, sub(ph, xyz(p0))), 0)) return SHADE_REPLAY;
        mtype = hit >= 0 ? (mword & 15u) : 0xffu;
    } else {
        if (hit >= 0) mtype = __float_as_uint(mats[3 * (hit_tag >> 4)].x) & 15u;
    }
    const bool specular = mtype == RT_METAL || mtype == RT_DIELECTRIC;
    if (hit < 0) {  // sky (Kernel.cu:41-44)
        // rd.y / |rd|: below |rd.y| = 2^-100 the quotient's exact bits vanish in the + 1 (|q| < 2^-60)
        const float len = length(rd);
        float q;
        if (in_rcp_range(len)) q = div_rn(rd.y, len, rcp_rn(len));
        else q = rd.y / len;
        const float tt = 0.5f * (q + 1.0f);
        const f3 c = add(scale(1.0f - tt, mk(P->bg0[0], P->bg0[1], P->bg0[2])), scale(tt, mk(P->bg1[0], P->bg1[1], P->bg1[2])));
        contrib = mulv(att, c);
        return SHADE_ENDED;
    }
    if constexpr (!EXACT) {
        p0 = prims[2 * hit + 0];
        p1 = prims[2 * hit + 1];
    }
    const uint32_t type = hit_tag & 15u, mat = hit_tag >> 4;
    const float4 m0 = mats[3 * mat + 0];
    const uint32_t ttype = (__float_as_uint(m0.x) >> 4) & 15u;
    f3 p, normal;
    float hu = 0.0f, hv = 0.0f;
    if (type == RT_SPHERE) {  // hit record of Sphere::Hit (Hittable.cuh:91-95)
        p = add(ro, scale(t, rd));
        normal = divs_rn(sub(p, xyz(p0)), p0.w, p1.y);  // p1.y = RN(1/radius) or 0 (scene_build.cpp)
        if (TEX && ttype == RT_IMAGE && mtype != RT_DIELECTRIC) {  // GetSphereUV (Hittable.cuh:119-125)
            const float theta = rt_acosf(-normal.y);
            const float phi = rt_atan2f(-normal.z, normal.x) + 3.141592654f;
            hu = fdiv(phi, 2 * 3.141592654f);
            hv = fdiv(theta, 3.141592654f);
        }
    } else {  // hit record of *Rect::Hit (Hittable.cuh:155-166)
        const float oa = type == RT_YZRECT ? ro.y : ro.x, da = type == RT_YZRECT ? rd.y : rd.x;
        const float ob = type == RT_XYRECT ? ro.y : ro.z, db = type == RT_XYRECT ? rd.y : rd.z;
        const float xx = oa + t * da;
        const float yy = ob + t * db;
        hu = fdiv(xx - p0.y, p0.z - p0.y);
        hv = fdiv(yy - p0.w, p1.x - p0.w);
        const f3 outward = type == RT_XYRECT ? mk(0.0f, 0.0f, 1.0f)
                           : type == RT_XZRECT ? mk(0.0f, 1.0f, 0.0f)
                                               : mk(1.0f, 0.0f, 0.0f);
        const bool front = dot(rd, outward) < 0;  // SetFaceNormal (Hittable.cuh:23-27)
        normal = front ? outward : neg(outward);
        p = add(ro, scale(t, rd));
    }
    if (mtype == RT_DIFFUSELIGHT) {  // DiffuseLight::Emitted (Material.cuh:164-176)
        const float4 m1 = mats[3 * mat + 1];
        f3 tex = xyz(m1);
        if (TEX && ttype != RT_CONSTANT) {
            const float4 m2 = mats[3 * mat + 2];
            tex = texture_value(m0, m1, m2, ttype, hu, hv, p, imgs, P->texels);
        }
        const f3 e = scale(m0.z, tex);
        contrib = mulv(e, att);
        return SHADE_ENDED;
    }
    float len = 1.0f, y_len = 0.0f;
    f3 ud = mk(0.0f, 0.0f, 0.0f);
    if (specular) {
        len = length(rd);
        y_len = recip_in_range(len);
        ud = divs_rn(rd, len, y_len);
    }
    if (mtype == RT_DIELECTRIC) {  // Dielectric::Scatter (Material.cuh:106-136); attenuation (1,1,1)
        // Evaluated in an order that keeps few values live: every quantity is the same binary32 value the
        // reference computes (pure functions of rd, normal, ir), and only the chosen direction is formed.
        // m1 = (1.0f / ir, r0²) precomputed on the host with the same operations (rt_internal.h).
        const float ir = m0.y;
        const float4 m1 = mats[3 * mat + 1];
        const float dn = dot(rd, normal);
        const bool exiting = dn > 0.0f;
        const float cn = exiting ? dn : -dn;
        float cosine;
        if (y_len != 0.0f && fabsf(cn) >= 0x1p-100f) cosine = div_rn(cn, len, y_len);
        else cosine = cn / len;
        if (exiting) cosine = sqrt_fast(1.0f - ir * ir * (1 - cosine * cosine));  // (= sqrtf bit for bit)
        const float ni_over_nt = exiting ? ir : m1.x;
        const f3 outward_normal = exiting ? neg(normal) : normal;
        // Refract (Math.cuh:292-304): uv = UnitVector(v)
        const float dt = dot(ud, outward_normal);
        const float discriminant = 1.0f - ni_over_nt * ni_over_nt * (1 - dt * dt);
        float reflect_prob = 1.0f;
        if (discriminant > 0) {  // Reflectance (Material.cuh:139-145)
            const float r0 = m1.y;
            const float xs = 1.0f - cosine;
            const float x2 = xs * xs;
            reflect_prob = r0 + (1.0f - r0) * ((x2 * x2) * xs);
        }
        const bool refl = uniform(rng) < reflect_prob;
        if (refl) {
            rd = reflect(rd, normal);
        } else if (discriminant > 0) {
            rd = sub(scale(ni_over_nt, sub(ud, scale(dt, outward_normal))), scale(sqrt_fast(discriminant), outward_normal));
        } else {
            rd = mk(0.0f, 0.0f, 0.0f);  // uninitialised `refracted` in the reference (ξ = 1.0, TIR)
        }
        ro = p;
        return SHADE_CONTINUE;
    }
    // The attenuation (texture lookup) before the rejection loop, which it does not depend on: an image texel's gather
    // is in flight while RandomInUnitSphere runs instead of after it (no RNG draw moves)
    const float4 m1 = mats[3 * mat + 1];
    TexFetch tex{xyz(m1), nullptr, false};
    if (TEX && ttype != RT_CONSTANT) {
        const float4 m2 = mats[3 * mat + 2];
        tex = texture_fetch(m0, m1, m2, ttype, hu, hv, p, imgs, P->texels);
    }
    const uint32_t texel_word = TEX ? texture_gather(tex, P->prims) : 0u;  // (a dummy word of the primitive table)
    f3 q;
    if constexpr (DEFER) {
        if (!random_in_unit_sphere_capped(rng, rtl, P->rius_cap, q)) return SHADE_DEFERRED;
    } else {
        q = random_in_unit_sphere(rng, rtl);
    }
    const f3 attenuation = texture_resolve(tex, texel_word);
    bool ok = true;
    if (mtype == RT_LAMBERTIAN) {  // Lambertian::Scatter (Material.cuh:43-62)
        const f3 target = add(add(p, normal), q);
        rd = sub(target, p);
    } else {  // Metal::Scatter (Material.cuh:75-94)
        const f3 reflected = reflect(ud, normal);
        rd = add(reflected, scale(m0.y, q));
        ok = dot(rd, normal) > 0;
    }
    ro = p;
    if (ok) {
        att = mulv(attenuation, att);
        return SHADE_CONTINUE;
    }
    contrib = mulv(mk(0.0f, 0.0f, 0.0f), att);  // emitted * cur_attenuation
    return SHADE_ENDED;
}

// Pixel epilogue (Kernel.cu:149-157): RNG state store, average, gamma 2, RGBA8 pack; optional outputs.
__device__ __forceinline__ void store_rng(const KParams& P, uint32_t* st, const Rng& rng) {
    if (!(P.flags & RT_FLAG_NO_STATE_WRITEBACK)) {
        const uint32_t k = P.state_stride;
        if (k == 1u) {  // the reference's 48-B curandState: d, v[5] are its first 24 bytes
            *reinterpret_cast<uint4*>(st) = make_uint4(rng.d, rng.v0, rng.v1, rng.v2);
            *reinterpret_cast<uint2*>(st + 4) = make_uint2(rng.v3, rng.v4);
        } else {  // six planes: each word a coalesced 4-B access of the wave
            st[0] = rng.d;
            st[k] = rng.v0;
            st[2 * k] = rng.v1;
            st[3 * k] = rng.v2;
            st[4 * k] = rng.v3;
            st[5 * k] = rng.v4;
        }
    }
}

template <class R>
__device__ __forceinline__ void write_pixel(const KParams& P, size_t pix, uint32_t* st, const R& rng, f3 col,
                                            const float4* acc_pre = nullptr) {
    store_rng(P, st, rng);
    col = pixel_sum(rng, col);
    f3 c;
    if (P.flags & RT_FLAG_ACCUMULATE) {
        // (acc_pre: the value loaded when the pixel started; RT_FLAG_ACCUMULATE_RESET: a restart, nothing is read and
        // the sums below are 0 + x, as after a zero fill)
        float4 a = (P.flags & RT_FLAG_ACCUMULATE_RESET) ? make_float4(0.0f, 0.0f, 0.0f, 0.0f)
                                                        : (acc_pre ? *acc_pre : P.accum[pix]);
        a.x = a.x + col.x;
        a.y = a.y + col.y;
        a.z = a.z + col.z;
        a.w = a.w + (float)P.spp;
        P.accum[pix] = a;
        c = divs_rn(mk(a.x, a.y, a.z), a.w, recip_in_range(a.w));  // = divs(sum, a.w) bit for bit
    } else {
        const float n = (float)P.spp;
        c = divs_rn(col, n, recip_in_range(n));  // = divs(col, spp) bit for bit (IEEE division outside its range)
    }
    if (P.radiance) P.radiance[pix] = make_float4(c.x, c.y, c.z, 1.0f);
    if (P.pos) P.pos[pix] = rgb_to_int(255.0f * sqrt_fast(c.x), 255.0f * sqrt_fast(c.y), 255.0f * sqrt_fast(c.z));
}

template <bool COUNT_TESTS>
__device__ __forceinline__ void flush_counts(const KParams& P, const Counts& cnt) {
    if (P.counters) {
        atomicAdd(&P.counters[0], (unsigned long long)cnt.rays);
        if (COUNT_TESTS) {
            atomicAdd(&P.counters[1], (unsigned long long)cnt.boxes);
            atomicAdd(&P.counters[2], (unsigned long long)cnt.prims);
            atomicAdd(&P.counters[4], (unsigned long long)cnt.wnode);
            atomicAdd(&P.counters[5], (unsigned long long)cnt.wleaf);
            atomicAdd(&P.counters[6], (unsigned long long)cnt.wshade);
            atomicAdd(&P.counters[11], (unsigned long long)cnt.wnode_uniform);
            atomicAdd(&P.counters[12], (unsigned long long)cnt.wleaf_uniform);
            atomicAdd(&P.counters[13], (unsigned long long)cnt.idle_nt);
            atomicAdd(&P.counters[14], (unsigned long long)cnt.idle_fin);
            atomicAdd(&P.counters[15], (unsigned long long)cnt.idle_wait);
            atomicAdd(&P.counters[16], (unsigned long long)cnt.rects);
            atomicAdd(&P.counters[17], (unsigned long long)cnt.replays);
            if (cnt.ctotal && wave_leader()) {  // one lane per wave: the stamps are wave-uniform
                atomicAdd(&P.counters[7], (unsigned long long)cnt.ctrav);
                atomicAdd(&P.counters[8], (unsigned long long)cnt.cshade);
                atomicAdd(&P.counters[9], (unsigned long long)cnt.ctotal);
                atomicAdd(&P.counters[10], (unsigned long long)cnt.cleaf);
            }
        }
        atomicAdd(&P.counters[3], (unsigned long long)cnt.primary);
    }
}

template <bool COUNT_TESTS, class R>
__device__ __forceinline__ void finish_pixel(const KParams& P, size_t pix, uint32_t* st, const R& rng, f3 col,
                                             const Counts& cnt) {
    write_pixel(P, pix, st, rng, col);
    flush_counts<COUNT_TESTS>(P, cnt);
}

// Lane → pixel.  BLOCK = 256: a workgroup covers a 16×16 tile, each wave an 8×8 sub-tile (P.tiles_x =
// ceil(W/16)); BLOCK = 64: one wave per workgroup covering an 8×8 tile (P.tiles_x = ceil(W/8)).  Returns
// false for lanes outside the (local) image or outside the faithful floor-division grid (Kernel.cu:184).
template <int BLOCK = kBlock>
__device__ __forceinline__ bool lane_pixel(const KParams& P, uint32_t& x, uint32_t& g, size_t& pix,
                                           uint32_t tile = blockIdx.x) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t bx = tile % P.tiles_x, by = tile / P.tiles_x;
    uint32_t ly;
    if constexpr (BLOCK == 64) {
        x = bx * 8 + (lane & 7u);
        ly = by * 8 + (lane >> 3);
    } else {
        x = bx * 16 + (wave & 1u) * 8 + (lane & 7u);
        ly = by * 16 + (wave >> 1) * 8 + (lane >> 3);
    }
    if (x >= P.width || ly >= P.local_rows) return false;
    g = global_row(P, ly);
    if (x >= P.grid_w || g >= P.grid_h) return false;
    pix = (size_t)ly * P.width + x;
    return true;
}

template <class PP>
__device__ __forceinline__ Camera lane_camera(PP P, uint32_t x, uint32_t g) {
    Camera c;
    c.origin = mk(P->origin[0], P->origin[1], P->origin[2]);
    c.up = mk(P->up[0], P->up[1], P->up[2]);
    c.right = mk(P->right[0], P->right[1], P->right[2]);
    c.fov_fwd = mk(P->fov_fwd[0], P->fov_fwd[1], P->fov_fwd[2]);
    c.k10_fwd = mk(P->k10_fwd[0], P->k10_fwd[1], P->k10_fwd[2]);
    c.xf = (float)(int)x - P->cx;
    c.yf = P->cy - (float)(int)g;
    return c;
}

// The kernel-argument block as a constant-address-space pointer the compiler cannot see through: fields
// read through it are re-loaded with s_load where they are used, instead of being held in registers
// across the traversal loop (launch-uniform camera/shading constants otherwise overflow the SGPR budget
// and get parked in VGPRs, costing occupancy).
typedef __attribute__((address_space(4))) const KParams KParamsC;
__device__ __forceinline__ KParamsC* kparams_reload() {
    KParamsC* p = (KParamsC*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return p;
}

// The pixel's first state word; its words are P.state_stride apart (1: rt_curand_state; the plane size with
// RT_FLAG_STATE_SOA, whose planes hold the pixels 8×8 tile by tile — tile t, row r, column c at t·64 + 8r + c
// — so the wave that renders a tile reads and writes 256 contiguous bytes per plane).
__device__ __forceinline__ uint32_t soa_index(uint32_t x, uint32_t ly, uint32_t width) {
    return ((((ly >> 3) * ((width + 7u) >> 3)) + (x >> 3)) << 6) + ((ly & 7u) << 3) + (x & 7u);
}
__device__ __forceinline__ uint32_t* state_at(const KParams& P, size_t pix) {
    if (P.state_stride == 1u) return P.state + pix * 12;
    const uint32_t ly = (uint32_t)(pix / P.width), x = (uint32_t)(pix - (size_t)ly * P.width);  // once per pixel
    return P.state + soa_index(x, ly, P.width);
}
__device__ __forceinline__ Rng load_rng(const uint32_t* st, uint32_t k) {
    if (k == 1u) {
        const uint4 s03 = *reinterpret_cast<const uint4*>(st);
        const uint2 s45 = *reinterpret_cast<const uint2*>(st + 4);
        return Rng{s03.x, s03.y, s03.z, s03.w, s45.x, s45.y};
    }
    return Rng{st[0], st[k], st[2 * k], st[3 * k], st[4 * k], st[5 * k]};
}

// ---------------------------------------------------------------------------------------------------
// Perf-mode RNG (RT_FLAG_RNG_PHILOX): hipRAND/rocRAND Philox4x32-10 (rocrand_philox4x32_10.h:270-303,
// rocrand_uniform.h:65-68, 281-284).  The pixel's stream is rocrand_init(seed, subsequence = global
// pixel index, offset = frame << 34), consumed in draw groups that start on a block boundary (rocrand_uniform4
// per block, philox10(ctr = {b, frame, pixel, 0}, key = seed) for the frame's block b): the camera jitter (2
// draws) and the dielectric's choice (1) take the first words of one block each; a RandomInUnitSphere call takes
// consecutive words of as many blocks as its attempts need (3 per attempt).  No word is selected at a lane-varying
// offset; nothing per pixel lives in HBM and only the next block index is carried (plus the pixel index); key and
// frame are launch-uniform kernel arguments.
// ---------------------------------------------------------------------------------------------------
struct RngPhilox {
    uint32_t n, r0, r1, r2, r3, pix;  // n: the next group's block; r0..r3: the current block (not carried)
    uint32_t k0, k1, frame;  // launch-uniform key and frame, read once when the stream is (un)parked
};

// Per-sample RNG window and pixel sum.  XORWOW (the reference's mode): one sequential stream per pixel, samples
// summed in float in order (Kernel.cu:147).  Philox mode: sample s starts at block s << 16 of the pixel's stream
// (rocrand_init(seed, pixel, (frame << 34) + (s << 18))), and the samples are summed in 2^-12 fixed point,
// saturating (the float registers carry the uint32 sums) — so neither the draws nor the sum depend on the order the
// samples run in (oracle/rt_oracle.c orc_quant, the same operations).
__device__ __forceinline__ void begin_sample(Rng&, uint32_t) {}
__device__ __forceinline__ void begin_sample(RngPhilox& s, uint32_t sample) { s.n = sample << 16; }
__device__ __forceinline__ uint32_t quant12(const float x) {  // NaN, <= 0: 0; >= 2^20 - 1: saturated
    if (!(x > 0.0f)) return 0u;
    if (!(x < 1048575.0f)) return 0xffffffffu;
    return (uint32_t)(x * 4096.0f + 0.5f);  // (x · 4096 exact: one rounding, the + 0.5's)
}
__device__ __forceinline__ uint32_t sat_add(const uint32_t a, const uint32_t b) {
    const uint32_t t = a + b;
    return t < b ? 0xffffffffu : t;
}
__device__ __forceinline__ f3 add_sample(const Rng&, const f3 col, const f3 c) { return add(col, c); }
__device__ __forceinline__ f3 add_sample(const RngPhilox&, const f3 col, const f3 c) {
    return mk(__uint_as_float(sat_add(__float_as_uint(col.x), quant12(c.x))),
              __uint_as_float(sat_add(__float_as_uint(col.y), quant12(c.y))),
              __uint_as_float(sat_add(__float_as_uint(col.z), quant12(c.z))));
}
__device__ __forceinline__ f3 pixel_sum(const Rng&, const f3 col) { return col; }
__device__ __forceinline__ f3 pixel_sum(const RngPhilox&, const f3 col) {
    return mk((float)__float_as_uint(col.x) * (1.0f / 4096.0f), (float)__float_as_uint(col.y) * (1.0f / 4096.0f),
              (float)__float_as_uint(col.z) * (1.0f / 4096.0f));
}


// Block `blk` of the lane's stream: philox10(ctr = {blk, frame, pixel, 0}, key = seed) into s.r0..r3.
// The key and frame are re-read from the kernel arguments here (scalar loads) rather than carried: held across
// the kernel, the unrolled key schedule cost 12 SGPR spills (into VGPR lanes).
__device__ __forceinline__ void philox_block(RngPhilox& s, uint32_t blk) {
    KParamsC* q = kparams_reload();
    uint32_t c0 = blk, c1 = q->rng_frame, c2 = s.pix, c3 = 0u;
    uint32_t k0 = q->rng_key_lo, k1 = q->rng_key_hi;
#pragma unroll
    for (int i = 0; i < 10; i++) {  // single_round + bumpkey (rocrand_philox4x32_10.h:286-303)
        const uint64_t m0 = (uint64_t)0xD2511F53u * c0;  // one v_mad_u64_u32 for lo and hi
        const uint64_t m1 = (uint64_t)0xCD9E8D57u * c2;
        c0 = (uint32_t)(m1 >> 32) ^ c1 ^ k0;
        c1 = (uint32_t)m1;
        c2 = (uint32_t)(m0 >> 32) ^ c3 ^ k1;
        c3 = (uint32_t)m0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    s.r0 = c0;
    s.r1 = c1;
    s.r2 = c2;
    s.r3 = c3;
}

__device__ __forceinline__ float philox_to_uniform(uint32_t x) {
    return __builtin_fmaf((float)x, 2.3283064e-10f, 2.3283064e-10f);  // 2^-32 + x·2^-32 (exact product)
}

// A one-draw group (the dielectric's ξ, Material.cuh:131): word 0 of the next block.
__device__ __forceinline__ float uniform(RngPhilox& s) {
    philox_block(s, s.n++);
    return philox_to_uniform(s.r0);
}
__device__ __forceinline__ void draw2(RngPhilox& s, float& a, float& b) {  // camera jitter (Kernel.cu:139-140)
    philox_block(s, s.n++);
    a = philox_to_uniform(s.r0);
    b = philox_to_uniform(s.r1);
}
__device__ __forceinline__ void draw3(RngPhilox& s, float& a, float& b, float& c) {  // Random() (Math.cuh:233)
    philox_block(s, s.n++);
    a = philox_to_uniform(s.r0);
    b = philox_to_uniform(s.r1);
    c = philox_to_uniform(s.r2);
}

// RandomInUnitSphere (Math.cuh:252-260) in Philox mode: the whole call is one draw group, its attempts taking
// consecutive words of consecutive blocks (attempt a: words 3a .. 3a + 2 of the call's blocks; four attempts use
// three blocks, the fourth needs none).  Every lane still looping is at the same attempt, so which words an
// attempt takes is a wave-uniform branch, not a per-lane select.
__device__ __forceinline__ f3 random_in_unit_sphere(RngPhilox& s, bool rtl) {
    f3 p;
    uint32_t a = 0u;                      // attempt index (the same for every lane in the loop)
    uint32_t k1 = 0u, k2 = 0u, k3 = 0u;   // words 1-3 of the latest block not drawn yet
    do {
        uint32_t x, y, z;
        const uint32_t phase = a & 3u;
        if (phase == 0u) {
            philox_block(s, s.n++);
            x = s.r0, y = s.r1, z = s.r2, k3 = s.r3;
        } else if (phase == 1u) {
            x = k3;
            philox_block(s, s.n++);
            y = s.r0, z = s.r1, k2 = s.r2, k3 = s.r3;
        } else if (phase == 2u) {
            x = k2, y = k3;
            philox_block(s, s.n++);
            z = s.r0, k1 = s.r1, k2 = s.r2, k3 = s.r3;
        } else {
            x = k1, y = k2, z = k3;
        }
        a++;
        const float fa = philox_to_uniform(x), fb = philox_to_uniform(y), fc = philox_to_uniform(z);
        const f3 r = rtl ? mk(fc, fb, fa) : mk(fa, fb, fc);
        p = mk(__builtin_fmaf(2.0f, r.x, -1.0f), __builtin_fmaf(2.0f, r.y, -1.0f), __builtin_fmaf(2.0f, r.z, -1.0f));
    } while (p.x * p.x + p.y * p.y + p.z * p.z >= 1.0f);
    return p;
}

// Resumable form (RT_TUNE_RIUS_TRIPS): the cap is rounded up to whole four-attempt rounds, so a deferred call
// stops on a block boundary and resumes at attempt phase 0 with nothing but the block index carried.
__device__ __forceinline__ bool random_in_unit_sphere_capped(RngPhilox& s, bool rtl, uint32_t cap, f3& p) {
    cap = cap > 0xfffffff0u ? cap : (cap + 3u) & ~3u;
    uint32_t a = 0u;
    uint32_t k1 = 0u, k2 = 0u, k3 = 0u;
    bool inside;
    do {
        uint32_t x, y, z;
        const uint32_t phase = a & 3u;
        if (phase == 0u) {
            philox_block(s, s.n++);
            x = s.r0, y = s.r1, z = s.r2, k3 = s.r3;
        } else if (phase == 1u) {
            x = k3;
            philox_block(s, s.n++);
            y = s.r0, z = s.r1, k2 = s.r2, k3 = s.r3;
        } else if (phase == 2u) {
            x = k2, y = k3;
            philox_block(s, s.n++);
            z = s.r0, k1 = s.r1, k2 = s.r2, k3 = s.r3;
        } else {
            x = k1, y = k2, z = k3;
        }
        a++;
        const float fa = philox_to_uniform(x), fb = philox_to_uniform(y), fc = philox_to_uniform(z);
        const f3 r = rtl ? mk(fc, fb, fa) : mk(fa, fb, fc);
        p = mk(__builtin_fmaf(2.0f, r.x, -1.0f), __builtin_fmaf(2.0f, r.y, -1.0f), __builtin_fmaf(2.0f, r.z, -1.0f));
        inside = p.x * p.x + p.y * p.y + p.z * p.z < 1.0f;
    } while (!inside && a < cap);
    return inside;
}

__device__ __forceinline__ void store_rng(const KParams&, uint32_t*, const RngPhilox&) {}  // stateless in HBM

// Start of a pixel's frame: its XORWOW state from HBM, or its Philox stream at draw 0.
template <class R> __device__ __forceinline__ R begin_rng(const uint32_t* st, uint32_t stride, uint32_t pixel);
template <> __device__ __forceinline__ Rng begin_rng<Rng>(const uint32_t* st, uint32_t stride, uint32_t) {
    return load_rng(st, stride);
}
template <> __device__ __forceinline__ RngPhilox begin_rng<RngPhilox>(const uint32_t*, uint32_t, uint32_t pixel) {
    KParamsC* q = kparams_reload();
    return RngPhilox{0u, 0u, 0u, 0u, 0u, pixel, q->rng_key_lo, q->rng_key_hi, q->rng_frame};
}

// v1: Kernel (Kernel.cu:102-158) + color() (Kernel.cu:30-80), flattened into one per-lane ray loop: every
// iteration traces one ray per lane to completion (trace(), scratch stack, 32-bit references), then
// shades it.  The fallback for scenes whose BVH is too large or deep for the LDS-stack kernels.
template <bool COUNT_TESTS>
__global__ __launch_bounds__(kBlock) void render_kernel(const KParams P) {
    const float4* nodes = P.nodes;
    const float4* prims = P.prims;
    uint32_t x, g;
    size_t pix;
    if (!lane_pixel(P, x, g, pix)) return;
    uint32_t* st = state_at(P, pix);
    Rng rng = load_rng(st, P.state_stride);
    const Camera cam = lane_camera(&P, x, g);
    const bool rtl = P.rius_rtl != 0;

    Counts cnt{0, 0, 0, 0, 0, 0, 0};
    f3 col = mk(0.0f, 0.0f, 0.0f);
    f3 att = mk(1.0f, 1.0f, 1.0f);
    f3 ro = mk(0.0f, 0.0f, 0.0f), rd = ro;
    uint32_t sample = 0, depth = 0;
    bool need_camera = true;

    if (P.spp > 0) {
        while (true) {
            if (need_camera) {
                camera_ray(&P, cam, rng, ro, rd, sample);
                att = mk(1.0f, 1.0f, 1.0f);
                depth = 0;
                need_camera = false;
                cnt.primary++;
            }
            f3 contrib;
            bool done = true;
            if (depth >= P.max_depth) {
                contrib = mk(0.0f, 0.0f, 0.0f);  // exceeded recursion (Kernel.cu:79)
            } else {
                cnt.rays++;
                const float a_dd = dot(rd, rd);
                float t;
                int hit = trace<COUNT_TESTS>(nodes, prims, P.num_nodes, ro, rd, a_dd, t, cnt);
                if (COUNT_TESTS) cnt.wshade += wave_leader();
                uint32_t tag = hit >= 0 ? __float_as_uint(prims[2 * (hit & (kTieBit - 1)) + 1].w) : 0u;
                int res = shade<true, false, true>(&P, prims, P.mats, P.imgs, hit, tag, t, ro, rd, att, rng, rtl, contrib);
                if (res == SHADE_REPLAY) {  // (bvh_clear)
                    if (COUNT_TESTS) cnt.replays++;
                    bvh_replay(&P, prims, hit, tag, t, ro, rd);
                    res = shade<true, false, true>(&P, prims, P.mats, P.imgs, hit, tag, t, ro, rd, att, rng, rtl, contrib);
                }
                done = res == SHADE_ENDED;
                if (!done) depth++;
            }
            if (done) {
                col = add_sample(rng, col, contrib);
                if (++sample == P.spp) break;
                need_camera = true;
            }
        }
    }
    finish_pixel<COUNT_TESTS>(P, pix, st, rng, col, cnt);
}

// ---------------------------------------------------------------------------------------------------
// v2: resumable traversal.  Each lane carries its traversal state (node, postponed leaf, LDS stack,
// closest hit) across iterations of one loop, in the structure of Aila & Laine's persistent
// "while-while" kernel with speculative traversal:
//   * internal nodes are visited until every lane of the wave has found a leaf; a lane's first leaf is
//     postponed and it keeps traversing, so leaf tests run with most lanes active;
//   * when fewer than `regen_threshold` lanes are still tracing, the wave leaves the traversal loop and
//     the lanes whose query finished shade their hit and start their next ray (bounce or next sample),
//     instead of idling until the slowest ray of the wave is done (path regeneration).
// Per lane the sequence of rays, RNG draws and arithmetic is exactly that of render_kernel.
// ---------------------------------------------------------------------------------------------------
constexpr int kSentinel = 0x7fffffff;  // traversal finished (internal node ids are < it, leaves < 0)
enum LaneMode { MODE_TRAV = 0, MODE_SHADE = 1, MODE_DONE = 2 };
constexpr int MODE_NEED = 3;  // v4 / persistent flat: the lane waits for a pixel; v3 sample items: for a sample
constexpr int MODE_REPLAY = 4;  // v3 / v4: the closest hit replays the reference traversal before shading (bvh_replay)

template <bool COUNT_TESTS, int BLOCK = 64>
__global__ __launch_bounds__(BLOCK) void render_kernel_v2(const KParams P) {
    extern __shared__ float4 lds[];
    uint32_t* const stk = (uint32_t*)lds + threadIdx.x;  // [depth][BLOCK] per-lane stacks
    const float4* __restrict__ nodes = P.nodes;
    const float4* __restrict__ prims = P.prims;
    uint32_t x, g;
    size_t pix;
    if (!lane_pixel<BLOCK>(P, x, g, pix)) return;
    uint32_t* st = state_at(P, pix);
    Rng rng = load_rng(st, P.state_stride);
    const Camera cam = lane_camera(&P, x, g);
    const bool rtl = P.rius_rtl != 0;

    Counts cnt{0, 0, 0, 0, 0, 0, 0};
    f3 col = mk(0.0f, 0.0f, 0.0f);
    f3 att = mk(1.0f, 1.0f, 1.0f);
    f3 ro = mk(0.0f, 0.0f, 0.0f), rd = ro;
    uint32_t sample = 0, depth = 0;
    // traversal state of the current ray
    int node = kSentinel, leaf = 0, hit = -1;
    uint32_t sp = 0;
    float t_best = FLT_MAX, a_dd = 0.0f;
    f3 invd = ro, oi = ro;
    int mode = MODE_DONE;

    // Start the closest-hit query of (ro, rd) (BVHNode::Hit with t in (0.001, FLT_MAX), Kernel.cu:40).
    auto start_trace = [&]() {
        cnt.rays++;
        a_dd = dot(rd, rd);
        invd = mk(fminf(fmaxf(__builtin_amdgcn_rcpf(rd.x), -1e20f), 1e20f),
                  fminf(fmaxf(__builtin_amdgcn_rcpf(rd.y), -1e20f), 1e20f),
                  fminf(fmaxf(__builtin_amdgcn_rcpf(rd.z), -1e20f), 1e20f));
        oi = mk(ro.x * invd.x, ro.y * invd.y, ro.z * invd.z);
        t_best = FLT_MAX;
        hit = -1;
        node = P.num_nodes ? 0 : kSentinel;
        leaf = 0;
        sp = 0;
        mode = MODE_TRAV;
    };
    // A path ended with `contrib`: accumulate (Kernel.cu:147) and begin the next sample, or finish.
    auto next_sample = [&](f3 contrib) {
        col = add_sample(rng, col, contrib);
        while (++sample < P.spp) {
            camera_ray(&P, cam, rng, ro, rd, sample);
            att = mk(1.0f, 1.0f, 1.0f);
            depth = 0;
            cnt.primary++;
            if (P.max_depth > 0) {
                start_trace();
                return;
            }
            col = add_sample(rng, col, mk(0.0f, 0.0f, 0.0f));  // exceeded recursion (Kernel.cu:79)
        }
        mode = MODE_DONE;
    };

    if (P.spp > 0) {
        sample = (uint32_t)-1;
        next_sample(mk(0.0f, 0.0f, 0.0f));  // col += 0 leaves col = +0 bit-exactly
    }
    const uint32_t threshold = P.regen_threshold;

    while (true) {
        if (mode == MODE_TRAV) {
            while (node != kSentinel || leaf < 0) {
                // internal nodes until every lane here has a postponed leaf.  Branch-free visit: the two
                // stack entries a visit may pop are read before the node data arrives, the far child is
                // written unconditionally above the stack top (kept only when both children are hit).
                while ((uint32_t)node < (uint32_t)kSentinel) {
                    const int top1 = (int)stk[((sp > 0u ? sp : 1u) - 1u) * BLOCK];
                    const int top2 = (int)stk[((sp > 1u ? sp : 2u) - 2u) * BLOCK];
                    const float4 n0 = nodes[4 * node + 0];
                    const float4 n1 = nodes[4 * node + 1];
                    const float4 n2 = nodes[4 * node + 2];
                    const float4 n3 = nodes[4 * node + 3];
                    const float a0 = __builtin_fmaf(n0.x, invd.x, -oi.x), a1 = __builtin_fmaf(n0.y, invd.x, -oi.x);
                    const float a2 = __builtin_fmaf(n0.z, invd.y, -oi.y), a3 = __builtin_fmaf(n0.w, invd.y, -oi.y);
                    const float a4 = __builtin_fmaf(n2.x, invd.z, -oi.z), a5 = __builtin_fmaf(n2.y, invd.z, -oi.z);
                    const float b0 = __builtin_fmaf(n1.x, invd.x, -oi.x), b1 = __builtin_fmaf(n1.y, invd.x, -oi.x);
                    const float b2 = __builtin_fmaf(n1.z, invd.y, -oi.y), b3 = __builtin_fmaf(n1.w, invd.y, -oi.y);
                    const float b4 = __builtin_fmaf(n2.z, invd.z, -oi.z), b5 = __builtin_fmaf(n2.w, invd.z, -oi.z);
                    const float c0min = fmaxf(fmaxf(fminf(a0, a1), fminf(a2, a3)), fmaxf(fminf(a4, a5), kTmin));
                    const float c0max = fminf(fminf(fmaxf(a0, a1), fmaxf(a2, a3)), fminf(fmaxf(a4, a5), t_best)) * kSlabSlack;
                    const float c1min = fmaxf(fmaxf(fminf(b0, b1), fminf(b2, b3)), fmaxf(fminf(b4, b5), kTmin));
                    const float c1max = fminf(fminf(fmaxf(b0, b1), fmaxf(b2, b3)), fminf(fmaxf(b4, b5), t_best)) * kSlabSlack;
                    if (COUNT_TESTS) {
                        cnt.boxes += 2;
                        cnt.wnode += wave_leader();
                    }
                    const bool h0 = c0min <= c0max;
                    const bool h1 = c1min <= c1max;
                    const bool both = h0 && h1, none = !(h0 || h1);
                    const bool swap = c1min < c0min;
                    const int ch0 = __float_as_int(n3.x), ch1 = __float_as_int(n3.y);
                    const int nearc = both ? (swap ? ch1 : ch0) : (h0 ? ch0 : ch1);
                    const int farc = swap ? ch0 : ch1;
                    stk[sp * BLOCK] = (uint32_t)farc;
                    int nxt = none ? (sp > 0u ? top1 : kSentinel) : nearc;
                    uint32_t nsp = both ? sp + 1u : ((none && sp > 0u) ? sp - 1u : sp);
                    // first leaf: postpone it and pop the next entry (the stack top after this visit)
                    const bool postpone = nxt < 0 && leaf == 0;
                    const int after_top = both ? farc : (none ? (sp > 1u ? top2 : kSentinel) : (sp > 0u ? top1 : kSentinel));
                    leaf = postpone ? nxt : leaf;
                    nxt = postpone ? after_top : nxt;
                    nsp = (postpone && nsp > 0u) ? nsp - 1u : nsp;
                    node = nxt;
                    sp = nsp;
                    if (__ballot(leaf == 0) == 0) break;
                }
                // postponed leaves
                while (leaf < 0) {
                    const uint32_t l = ~(uint32_t)leaf;
                    const uint32_t first = l >> 2, count = (l & 3u) + 1u;
                    for (uint32_t i = first; i < first + count; i++) {
                        const float4 p0 = prims[2 * i + 0];
                        const float4 p1 = prims[2 * i + 1];
                        const uint32_t type = __float_as_uint(p1.w) & 15u;
                        if (COUNT_TESTS) {
                            cnt.prims++;
                            cnt.rects += type != RT_SPHERE ? 1u : 0u;
                            cnt.wleaf += wave_leader();
                        }
                        if (type == RT_SPHERE) {  // Sphere::Hit (Hittable.cuh:80-110)
                            const f3 oc = sub(ro, xyz(p0));
                            const float b = dot(oc, rd);
                            const float c = dot(oc, oc) - p1.x;
                            const float disc = b * b - a_dd * c;
                            if (disc > 0) {
                                const float sq = sqrtf(disc);
                                float t = (-b - sq) / a_dd;
                                if (t < t_best && t > kTmin) {
                                    t_best = t;
                                    hit = (int)i;
                                } else {
                                    const bool tied = t == t_best;  // (bvh_clear)
                                    t = (-b + sq) / a_dd;
                                    if (t < t_best && t > kTmin) {
                                        t_best = t;
                                        hit = (int)i;
                                    } else if (tied || t == t_best) {
                                        hit |= kTieBit;
                                    }
                                }
                            }
                        } else {  // *Rect::Hit
                            const float ok = type == RT_XYRECT ? ro.z : (type == RT_XZRECT ? ro.y : ro.x);
                            const float dk = type == RT_XYRECT ? rd.z : (type == RT_XZRECT ? rd.y : rd.x);
                            const float t = (p0.x - ok) * rcp_ieee(dk);
                            if (!(t < kTmin || t > t_best)) {
                                const float oa = type == RT_YZRECT ? ro.y : ro.x, da = type == RT_YZRECT ? rd.y : rd.x;
                                const float ob = type == RT_XYRECT ? ro.y : ro.z, db = type == RT_XYRECT ? rd.y : rd.z;
                                const float xx = oa + t * da;
                                const float yy = ob + t * db;
                                if (!(xx < p0.y || xx > p0.z || yy < p0.w || yy > p1.x)) {
                                    hit = t == t_best ? (int)i | kTieBit : (int)i;
                                    t_best = t;
                                }
                            }
                        }
                    }
                    leaf = 0;
                    if (node < 0) {  // another leaf was postponed in `node`: process it as well
                        leaf = node;
                        node = sp ? (int)stk[(--sp) * BLOCK] : kSentinel;
                    }
                }
                if ((uint32_t)__popcll(__ballot(1)) < threshold) break;  // regenerate finished lanes
            }
            if (node == kSentinel && leaf == 0) mode = MODE_SHADE;
        }
        if (mode == MODE_SHADE) {
            f3 contrib;
            if (COUNT_TESTS) cnt.wshade += wave_leader();
            uint32_t tag = hit >= 0 ? __float_as_uint(prims[2 * (hit & (kTieBit - 1)) + 1].w) : 0u;
            int res = shade<true, false, true>(&P, prims, P.mats, P.imgs, hit, tag, t_best, ro, rd, att, rng, rtl, contrib);
            if (res == SHADE_REPLAY) {  // (bvh_clear)
                if (COUNT_TESTS) cnt.replays++;
                bvh_replay(&P, prims, hit, tag, t_best, ro, rd);
                res = shade<true, false, true>(&P, prims, P.mats, P.imgs, hit, tag, t_best, ro, rd, att, rng, rtl, contrib);
            }
            if (res == SHADE_ENDED) {
                next_sample(contrib);
            } else if (++depth >= P.max_depth) {
                next_sample(mk(0.0f, 0.0f, 0.0f));  // exceeded recursion (Kernel.cu:79)
            } else {
                start_trace();
            }
        }
        if (__ballot(mode != MODE_DONE) == 0) break;
    }
    finish_pixel<COUNT_TESTS>(P, pix, st, rng, col, cnt);
}

// ---------------------------------------------------------------------------------------------------
// v3: v2's resumable traversal with the register footprint cut for occupancy.
//   * one wave per workgroup (no intra-workgroup coupling of wave lifetimes);
//   * per-lane path state that only shading needs (cuRAND state, colour sum, attenuation, sample and
//     depth counters) is parked in LDS while the lane traverses, and the ray's reciprocal direction /
//     |d|² are recomputed on entry to the traversal phase: only the ray, the traversal cursor and the
//     closest hit stay in VGPRs across phases;
//   * 16-bit traversal stack entries in LDS when node and leaf references fit a signed 16 bits (the scene
//     has < 32767 nodes and < 8192 primitives), 32-bit ones otherwise (WIDE instantiations, RefW below);
//   * the lane's ray count is parked with the path state; primary samples = spp per pixel.
// LDS per wave: 15 × 256 B of parked state + (depth + 2) × 128 B of stack (2 sentinel pads).
// ---------------------------------------------------------------------------------------------------
constexpr uint32_t kStackBase = 2;  // v3 stack entries start above two sentinel pads
// Reference width of the v3/v4 kernels: 16-bit child and stack references (scenes with < 32767 nodes and < 8192
// primitives: every BASELINE config), or 32-bit ones (WIDE: any scene the reference viewer can grow, AddHittable
// CudaLayer.cpp:918-1370; 4-B LDS stack entries; the references' upper halves ride in the low bytes of the y
// planes, scene_build.cpp).  References are unsigned in the width: internal nodes < kSentinel, leaves >= kLeaf.
template <bool WIDE> struct RefW {
    static constexpr uint32_t kSentinel = WIDE ? 0x7fffffffu : 0x7fffu;  // traversal finished
    static constexpr uint32_t kLeaf = WIDE ? 0x80000000u : 0x8000u;      // references >= kLeaf are leaves
    static constexpr uint32_t kMask = WIDE ? 0xffffffffu : 0xffffu;      // leaf ^ kMask = the leaf's ~ref
    static constexpr uint32_t kLevelShift = WIDE ? 8u : 7u;              // log2(LDS bytes per stack level)
    using Entry = typename std::conditional<WIDE, uint32_t, uint16_t>::type;
};
enum ParkSlot { PK_RNG = 0, PK_COL = 6, PK_ATT = 9, PK_SAMPLE = 12, PK_DEPTH = 13, PK_RAYS = 14, PK_WORDS = 15 };
// Compact parking (v3, COMPACT): sample (13 bits), depth (6 bits) and the lane's ray count (13 bits) share
// word PK_SD, so a wave parks 13 words instead of 15 — less LDS per wave, more resident waves (the v3
// kernels are LDS-limited).  Valid when spp < 8192, max_depth < 64 and spp · max_depth < 8192.
enum ParkSlotCompact { PK_SD = 12, PK_WORDS_COMPACT = 13 };
__host__ __device__ constexpr int park_words(bool compact) { return compact ? PK_WORDS_COMPACT : PK_WORDS; }

// Traversal cursor of one lane (v3).
struct Cursor {
    int node, leaf, hit;
    uint32_t tag;  // type | material << 4 of the closest primitive so far
    uint32_t sp;
    float t_best;
    int mode;
};

// v3 / v4: the lanes in MODE_REPLAY (shade() returned SHADE_REPLAY), one after another, through ref_trace_wave; each
// gets the reference traversal's answer, marked verified, and goes to MODE_SHADE.  Called where every lane is active.
template <class PP>
__device__ __forceinline__ void bvh_replay_wave(PP P, const float4* __restrict__ prims, Cursor& c, const f3 ro, const f3 rd,
                                                Counts& cnt, const bool count) {
    uint64_t need = __ballot(c.mode == MODE_REPLAY);
    while (need != 0u) {
        const int L = (int)__builtin_ctzll(need);
        need &= need - 1u;
        const auto bl = [L](const float v) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), L)); };
        const HitOut r = RT_BVH_EXACT == 4 ? HitOut{-1, 0u, 0.0f}
                                           : ref_trace_wave(P->bvh_ref_nodes, P->bvh_ref_pairs, prims, mk(bl(ro.x), bl(ro.y), bl(ro.z)),
                                                            mk(bl(rd.x), bl(rd.y), bl(rd.z)));
        if (__lane_id() == (uint32_t)L) {
            c.hit = RT_BVH_EXACT == 4 ? (c.hit >= 0 ? (c.hit | kVerifiedBit) : kVerifiedMiss)  // (A/B: no replay)
                                      : (r.hit >= 0 ? (r.hit | kVerifiedBit) : kVerifiedMiss);
            if (RT_BVH_EXACT != 4) {
                c.tag = r.tag;
                c.t_best = r.t;
            }
            c.mode = MODE_SHADE;
            if (count) cnt.replays++;
        }
    }
}

template <bool WIDE>
__device__ __forceinline__ void v3_start_trace(uint32_t num_nodes, Cursor& c, uint32_t& rays) {
    rays++;
    c.t_best = FLT_MAX;
    c.hit = -1;
    c.node = num_nodes ? 0 : (int)RefW<WIDE>::kSentinel;
    c.leaf = 0;
    c.sp = kStackBase;
    c.mode = MODE_TRAV;
}

// A path ended with `contrib`: accumulate (Kernel.cu:147), then the next sample's camera ray, or finish.
template <bool WIDE, class R>
__device__ __forceinline__ void v3_next_sample(const KParams& P, uint32_t x, uint32_t g, f3 contrib, R& rng,
                                               f3& col, f3& att, uint32_t& sample, uint32_t& depth, f3& ro,
                                               f3& rd, Cursor& c, uint32_t& rays) {
    col = add_sample(rng, col, contrib);
    KParamsC* q = kparams_reload();  // (launch-uniform operands re-read here, not held in SGPRs through the loop)
    const Camera cam = lane_camera(q, x, g);
    while (++sample < q->spp) {
        camera_ray(q, cam, rng, ro, rd, sample);
        att = mk(1.0f, 1.0f, 1.0f);
        depth = 0;
        if (q->max_depth > 0) {
            v3_start_trace<WIDE>(q->num_nodes, c, rays);
            return;
        }
        col = add_sample(rng, col, mk(0.0f, 0.0f, 0.0f));  // exceeded recursion (Kernel.cu:79)
    }
    c.mode = MODE_DONE;
}

// The six RNG words of a lane: XORWOW d, v[5]; Philox draw index, block of four words, pixel index.
__device__ __forceinline__ void park_rng(uint32_t* park, const Rng& r) {
    park[(PK_RNG + 0) * 64] = r.d;
    park[(PK_RNG + 1) * 64] = r.v0;
    park[(PK_RNG + 2) * 64] = r.v1;
    park[(PK_RNG + 3) * 64] = r.v2;
    park[(PK_RNG + 4) * 64] = r.v3;
    park[(PK_RNG + 5) * 64] = r.v4;
}
__device__ __forceinline__ void park_rng(uint32_t* park, const RngPhilox& r) {  // the block is not carried
    park[(PK_RNG + 0) * 64] = r.n;
    park[(PK_RNG + 5) * 64] = r.pix;
}
__device__ __forceinline__ void unpark_rng(const uint32_t* park, Rng& r) {
    r = Rng{park[(PK_RNG + 0) * 64], park[(PK_RNG + 1) * 64], park[(PK_RNG + 2) * 64],
            park[(PK_RNG + 3) * 64], park[(PK_RNG + 4) * 64], park[(PK_RNG + 5) * 64]};
}
__device__ __forceinline__ void unpark_rng(const uint32_t* park, RngPhilox& r) {
    KParamsC* q = kparams_reload();
    r = RngPhilox{park[(PK_RNG + 0) * 64], 0u, 0u, 0u, 0u, park[(PK_RNG + 5) * 64],
                  q->rng_key_lo, q->rng_key_hi, q->rng_frame};
}

template <bool COMPACT = false, bool COL = true, class R>
__device__ __forceinline__ void v3_park(uint32_t* park, const R& rng, f3 col, f3 att, uint32_t sample,
                                        uint32_t depth, uint32_t rays) {
    if constexpr (COMPACT) park[PK_SD * 64] = sample | (depth << 13) | (rays << 19);
    else park[PK_RAYS * 64] = rays;
    park_rng(park, rng);
    if constexpr (COL) {
        park[(PK_COL + 0) * 64] = __float_as_uint(col.x);
        park[(PK_COL + 1) * 64] = __float_as_uint(col.y);
        park[(PK_COL + 2) * 64] = __float_as_uint(col.z);
    }
    park[(PK_ATT + 0) * 64] = __float_as_uint(att.x);
    park[(PK_ATT + 1) * 64] = __float_as_uint(att.y);
    park[(PK_ATT + 2) * 64] = __float_as_uint(att.z);
    if constexpr (!COMPACT) {
        park[PK_SAMPLE * 64] = sample;
        park[PK_DEPTH * 64] = depth;
    }
}

template <bool COMPACT = false, bool COL = true, class R>
__device__ __forceinline__ void v3_unpark(const uint32_t* park, R& rng, f3& col, f3& att, uint32_t& sample,
                                          uint32_t& depth, uint32_t& rays) {
    if constexpr (COMPACT) {
        const uint32_t sd = park[PK_SD * 64];
        sample = sd & 0x1fffu;
        depth = (sd >> 13) & 0x3fu;
        rays = sd >> 19;
    } else {
        rays = park[PK_RAYS * 64];
    }
    unpark_rng(park, rng);
    if constexpr (COL)
        col = mk(__uint_as_float(park[(PK_COL + 0) * 64]), __uint_as_float(park[(PK_COL + 1) * 64]),
                 __uint_as_float(park[(PK_COL + 2) * 64]));
    else
        col = mk(0.0f, 0.0f, 0.0f);
    att = mk(__uint_as_float(park[(PK_ATT + 0) * 64]), __uint_as_float(park[(PK_ATT + 1) * 64]),
             __uint_as_float(park[(PK_ATT + 2) * 64]));
    if constexpr (!COMPACT) {
        sample = park[PK_SAMPLE * 64];
        depth = park[PK_DEPTH * 64];
    }
}


// Constant-address-space views of the read-only scene buffers: loads from them at wave-uniform indices become
// scalar loads (s_load_dword*) whose results feed VALU instructions as SGPR operands.
typedef const __attribute__((address_space(4))) float ConstF32;
typedef const __attribute__((address_space(4))) uint32_t ConstU32;
typedef const __attribute__((address_space(4))) uint8_t ConstU8;
template <class T> using Lds = __attribute__((address_space(3))) T;
// v_min/v_max(3)_f32 as plain instructions: the operands are finite FMA results or canonical values
__device__ __forceinline__ float vmax(float a, float b) { float r; asm("v_max_f32 %0, %1, %2" : "=v"(r) : "s"(a), "v"(b)); return r; }
__device__ __forceinline__ float vmin(float a, float b) { float r; asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
__device__ __forceinline__ float vmax3(float a, float b, float c) { float r; asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c)); return r; }
__device__ __forceinline__ float vmin3(float a, float b, float c) { float r; asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c)); return r; }
constexpr uint32_t kPrimStep = 32u;  // leaf cursor unit: bytes of one 32-B primitive record

// Traversal phase of one lane (v3/v4): resumes the cursor and runs the speculative while-while loop
// until this lane's closest hit is found (mode -> MODE_SHADE) or fewer than `threshold` lanes are
// still tracing (the wave then shades the finished lanes and regenerates them).
template <bool COUNT_TESTS, int NODES, uint32_t STK_OFF, bool WIDE, bool EXACT = RT_BVH_EXACT != 0>
__device__ __forceinline__ void v3_traverse(const __amdgpu_buffer_rsrc_t nrsrc,
                                            const float4* __restrict__ nodes_tab, const uint32_t* __restrict__ refs,
                                            const float4* __restrict__ prims, typename RefW<WIDE>::Entry* const stk,
                                            const uint32_t threshold, const f3 ro, const f3 rd, Cursor& c,
                                            Counts& cnt, const uint32_t ntrav = 64, const uint32_t leaf_break = 0) {
    // node / leaf references as unsigned values of the reference width (RefW): internal nodes < kSentinel, leaf
    // references (negative in the layout) >= kLeaf; leaf == 0: no postponed leaf
    using RW = RefW<WIDE>;
    using Entry = typename RW::Entry;
    uint32_t node = (uint32_t)c.node, leaf = (uint32_t)c.leaf;
    int hit = c.hit;
    uint32_t tag = c.tag;
    uint32_t sp = c.sp;
    float t_best = c.t_best;
    const float a_dd = dot(rd, rd);
    // RN(1/a) for the sphere roots (div_rn); outside [2^-40, 2^40] the test divides the IEEE way
    const bool fast_div = a_dd >= 0x1p-40f && a_dd <= 0x1p40f;
    const float inv_a = rcp_rn(a_dd);  // used only when fast_div
    const f3 invd = mk(fminf(fmaxf(__builtin_amdgcn_rcpf(rd.x), -1e20f), 1e20f),
                       fminf(fmaxf(__builtin_amdgcn_rcpf(rd.y), -1e20f), 1e20f),
                       fminf(fmaxf(__builtin_amdgcn_rcpf(rd.z), -1e20f), 1e20f));
    const f3 oi = mk(ro.x * invd.x, ro.y * invd.y, ro.z * invd.z);
    // (invd, 0) or (0, invd) by sign with one max / min each (invd is never NaN; a -0 that became +0
    // changes only the sign of a zero plane distance, which no comparison sees)
    const f3 pa = mk(fmaxf(invd.x, 0.0f), fmaxf(invd.y, 0.0f), fmaxf(invd.z, 0.0f));
    const f3 pc = mk(fminf(invd.x, 0.0f), fminf(invd.y, 0.0f), fminf(invd.z, 0.0f));
    const Entry* ustk = stk;
    // LDS address of this lane's stack entry 0 split into the lane part (VGPR) and the stack region's offset
    // STK_OFF (an immediate of the ds instructions)
    const uint32_t stk_lane = (uint32_t)(uintptr_t)(Lds<Entry>*)stk - STK_OFF;  // LDS base + the lane's column
    // structured (stride 48 B) view of the node boxes for the vector path's idxen loads
    const __amdgpu_buffer_rsrc_t rsrc_nodes_idx =
        __builtin_amdgcn_make_buffer_rsrc((void*)nodes_tab, (short)48, 0x7fffffff, 0x00020000);
    constexpr uint32_t stk_off = STK_OFF / sizeof(Entry);  // in entries
    const float tmin_s = kTmin;  // an SGPR operand of the slab test's v_max
    const __amdgpu_buffer_rsrc_t prsrc = __builtin_amdgcn_make_buffer_rsrc((void*)prims, (short)0, 0x7fffffff, 0x00020000);
    while (node != RW::kSentinel || leaf >= RW::kLeaf) {
        // t_best changes only in the leaf phase: canonicalised once here, not on every visit by fminf
        const float t_best_c = __builtin_canonicalizef(t_best);
        const uint32_t n_outer = COUNT_TESTS ? (uint32_t)__popcll(__ballot(1)) : 0u;  // lanes still tracing
        (void)n_outer;
        // lanes holding no leaf yet, carried through the visits as an SGPR mask
        uint64_t lzm = __ballot(leaf == 0);
        while (node < RW::kSentinel) {
            // the entry address as one v_lshl_add_u32 (LLVM emits a half-rate shift plus an add: C2 −0.2 %,
            // C3 −0.3 %, profiles/r02e_ab_stack_addr.txt)
            uint32_t sa;
            asm("v_lshl_add_u32 %0, %1, %3, %2" : "=v"(sa) : "v"(sp), "v"(stk_lane), "i"(RW::kLevelShift));
            Lds<Entry>* const sp_entry = (Lds<Entry>*)(uintptr_t)sa + stk_off;
            uint32_t top1 = sp_entry[-64];
            uint32_t top2 = sp_entry[-128];
            // materialise the zero-extended words here: used in another basic block, a loaded u16 would
            // otherwise be re-extended there with a v_and per word and visit
            asm("" : "+v"(top1));
            asm("" : "+v"(top2));
            float c0min, c0max, c1min, c1max;
            uint32_t ch0, ch1;
            // near/far plane distances without min/max (4-cycle ops on gfx950): with (pa, pc) = (1/d, 0) for a
            // positive direction component and (0, 1/d) for a negative one,
            //   near = fma(lo, pa, fma(hi, pc, -o/d)),  far = fma(hi, pa, fma(lo, pc, -o/d))
            // is fma(lo or hi, 1/d, -o/d) with one rounding — the value min/max of the two would pick — at four
            // 2-cycle FMAs per axis instead of two FMAs, a min and a max.
            const auto slab = [&](const float4 n0, const float4 n1, const float4 n2) {
                const float nx0 = __builtin_fmaf(n0.x, pa.x, __builtin_fmaf(n0.y, pc.x, -oi.x));
                const float fx0 = __builtin_fmaf(n0.y, pa.x, __builtin_fmaf(n0.x, pc.x, -oi.x));
                const float ny0 = __builtin_fmaf(n0.z, pa.y, __builtin_fmaf(n0.w, pc.y, -oi.y));
                const float fy0 = __builtin_fmaf(n0.w, pa.y, __builtin_fmaf(n0.z, pc.y, -oi.y));
                const float nz0 = __builtin_fmaf(n2.x, pa.z, __builtin_fmaf(n2.y, pc.z, -oi.z));
                const float fz0 = __builtin_fmaf(n2.y, pa.z, __builtin_fmaf(n2.x, pc.z, -oi.z));
                const float nx1 = __builtin_fmaf(n1.x, pa.x, __builtin_fmaf(n1.y, pc.x, -oi.x));
                const float fx1 = __builtin_fmaf(n1.y, pa.x, __builtin_fmaf(n1.x, pc.x, -oi.x));
                const float ny1 = __builtin_fmaf(n1.z, pa.y, __builtin_fmaf(n1.w, pc.y, -oi.y));
                const float fy1 = __builtin_fmaf(n1.w, pa.y, __builtin_fmaf(n1.z, pc.y, -oi.y));
                const float nz1 = __builtin_fmaf(n2.z, pa.z, __builtin_fmaf(n2.w, pc.z, -oi.z));
                const float fz1 = __builtin_fmaf(n2.w, pa.z, __builtin_fmaf(n2.z, pc.z, -oi.z));
                // the plane distances are FMA results and t_best_c is canonical, so min/max need no
                // canonicalising v_max (LLVM re-emits one per visit for a value carried into the loop:
                // C2 −1.8 %)
                c0min = vmax3(nx0, ny0, vmax(tmin_s, nz0));
                c0max = vmin3(fx0, fy0, vmin(fz0, t_best_c)) * kSlabSlack;
                c1min = vmax3(nx1, ny1, vmax(tmin_s, nz1));
                c1max = vmin3(fx1, fy1, vmin(fz1, t_best_c)) * kSlabSlack;
            };
            if constexpr (NODES == NODES_64) {  // 64-B node: f32 boxes + two int32 references
                const uint32_t noff = (uint32_t)node << 6;
                const uint2 r2 = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(nrsrc, noff + 48u, 0, 0));
                ch0 = r2.x & RW::kMask;
                ch1 = r2.y & RW::kMask;
                slab(__builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(nrsrc, noff, 0, 0)),
                     __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(nrsrc, noff + 16u, 0, 0)),
                     __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(nrsrc, noff + 32u, 0, 0)));
            } else {  // 48 B of f32 boxes + 4 B of references
                const uint32_t nu = __builtin_amdgcn_readfirstlane(node);
                if (__ballot(node != nu) == 0) {
                    // every active lane visits the same node: scalar loads through the constant cache, planes as
                    // SGPR operands of the FMAs — no vector-memory (TA/TD) traffic, the kernel's busiest unit
                    const ConstF32* cn = (const ConstF32*)((const ConstU8*)nodes_tab + nu * 48u);
                    if constexpr (WIDE) {
                        const ConstU32* r = (const ConstU32*)((const ConstU8*)refs + nu * 8u);
                        ch0 = r[0];
                        ch1 = r[1];
                    } else {
                        const uint32_t r = *(const ConstU32*)((const ConstU8*)refs + nu * 4u);
                        ch0 = r & 0xffffu;
                        ch1 = r >> 16;
                    }
                    slab(make_float4(cn[0], cn[1], cn[2], cn[3]), make_float4(cn[4], cn[5], cn[6], cn[7]),
                         make_float4(cn[8], cn[9], cn[10], cn[11]));
                } else {
                    // Three structured (idxen) buffer loads: the descriptor's 48-B stride scales the node index in
                    // the addresser (no VALU offset arithmetic: C2 −0.5 %), and the child references ride in the low
                    // bytes of the x planes (scene_build.cpp), so no fourth load (C2 −1.6 %: the texture addresser
                    // limits this loop as much as the VALU does — a fifth load costs +6.6 %;
                    // profiles/r02e_ab_idxen.txt, profiles/r02e_ab_node_loads.txt).  The builtins have no idxen form:
                    // the loads and their wait are one asm block.
                    float4 n0, n1, n2;
                    asm volatile(
                        "buffer_load_dwordx4 %0, %3, %4, 0 idxen\n\t"
                        "buffer_load_dwordx4 %1, %3, %4, 0 idxen offset:16\n\t"
                        "buffer_load_dwordx4 %2, %3, %4, 0 idxen offset:32\n\t"
                        "s_waitcnt vmcnt(0)"
                        : "=&v"(n0), "=&v"(n1), "=&v"(n2)
                        : "v"(node), "s"(rsrc_nodes_idx));
                    // byte 0 of lo_x | byte 0 of hi_x << 8 (v_perm: bytes 0-3 = src1, 4-7 = src0, 0x0c = zero)
                    // (a VOP3 takes no literal on gfx9: the selector is an SGPR operand)
                    asm("v_perm_b32 %0, %1, %2, %3" : "=v"(ch0) : "v"(n0.y), "v"(n0.x), "s"(0x0c0c0400u));
                    asm("v_perm_b32 %0, %1, %2, %3" : "=v"(ch1) : "v"(n1.y), "v"(n1.x), "s"(0x0c0c0400u));
                    if constexpr (WIDE) {  // bits 16-31: byte 0 of lo_y | byte 0 of hi_y << 8, then the two halves
                        uint32_t u0, u1;
                        asm("v_perm_b32 %0, %1, %2, %3" : "=v"(u0) : "v"(n0.w), "v"(n0.z), "s"(0x0c0c0400u));
                        asm("v_perm_b32 %0, %1, %2, %3" : "=v"(u1) : "v"(n1.w), "v"(n1.z), "s"(0x0c0c0400u));
                        asm("v_perm_b32 %0, %1, %2, %3" : "=v"(ch0) : "v"(u0), "v"(ch0), "s"(0x05040100u));
                        asm("v_perm_b32 %0, %1, %2, %3" : "=v"(ch1) : "v"(u1), "v"(ch1), "s"(0x05040100u));
                    }
                    slab(n0, n1, n2);
                }
            }
            if (COUNT_TESTS) {
                cnt.boxes += 2;
                cnt.wnode += wave_leader();
                if (__ballot(node != (uint32_t)__builtin_amdgcn_readfirstlane(node)) == 0) cnt.wnode_uniform += wave_leader();
                const uint32_t act = (uint32_t)__popcll(__ballot(1));
                if (wave_leader()) {
                    cnt.idle_nt += 64u - ntrav;
                    cnt.idle_fin += ntrav - n_outer;
                    cnt.idle_wait += n_outer - act;
                }
            }
            // The visit decision as one block of lane-mask arithmetic (C2 −0.7 % against its C++ statement,
            // profiles/r02h_ab_asm_decide.txt): the hit / order / leaf masks stay in SGPR pairs (SALU combines
            // them), the "no leaf held yet" mask is carried in SGPRs through the visits, and the exit test needs
            // no VALU materialisation of a ballot.  In C++ terms, with h0/h1 = child hit, swap = c1min < c0min:
            //   both = h0 && h1, none = !(h0 || h1); near = both ? (swap ? ch1 : ch0) : (h0 ? ch0 : ch1);
            //   far = swap ? ch0 : ch1 is written at the stack top unconditionally (kept when both);
            //   next = none ? top1 : near; sp += both - none (the sentinel pads make an empty pop yield the
            //   sentinel); a first leaf (next >= 0x8000 with no leaf held) is postponed: leaf = next and
            //   next = the new stack top (both ? far : none ? top2 : top1), sp -= 1.
            {
                uint32_t farc, xr, nxt, at;
                uint64_t m0, m1, m2, m3, m4, m5;
                asm volatile(
                    "v_cmp_le_f32 %[m0], %[a0], %[b0]\n\t"            // h0
                    "v_cmp_le_f32 %[m1], %[a1], %[b1]\n\t"            // h1
                    "v_cmp_lt_f32 %[m2], %[a1], %[a0]\n\t"            // swap
                    "v_cndmask_b32 %[farc], %[ch1], %[ch0], %[m2]\n\t" // far child = swap ? ch0 : ch1
                    "s_orn2_b64 %[m2], %[m2], %[m0]\n\t"              // swap | !h0
                    "s_and_b64 %[m2], %[m2], %[m1]\n\t"               // take ch1 first
                    "v_cndmask_b32 %[xr], %[ch0], %[ch1], %[m2]\n\t"
                    "s_and_b64 %[m2], %[m0], %[m1]\n\t"               // both
                    "s_or_b64 %[m0], %[m0], %[m1]\n\t"                // any
                    "v_cndmask_b32 %[nxt], %[t1], %[xr], %[m0]\n\t"    // next = any ? first : pop
                    "v_cndmask_b32 %[at], %[t2], %[t1], %[m0]\n\t"     // the stack top after this visit
                    "v_cndmask_b32 %[at], %[at], %[farc], %[m2]\n\t"
                    "v_addc_co_u32 %[sp], %[m3], %[sp], 0, %[m2]\n\t"  // push
                    "s_not_b64 %[m0], %[m0]\n\t"                      // none
                    "v_subb_co_u32 %[sp], %[m3], %[sp], 0, %[m0]\n\t"  // pop
                    "v_cmp_lt_u32 %[m1], %[sent], %[nxt]\n\t"         // next is a leaf
                    "s_mov_b64 %[m4], %[lzm]\n\t"                     // no leaf held yet (carried mask)
                    "s_and_b64 %[m1], %[m1], %[m4]\n\t"               // postpone
                    "v_cndmask_b32 %[leaf], %[leaf], %[nxt], %[m1]\n\t"
                    "v_cndmask_b32 %[node], %[nxt], %[at], %[m1]\n\t"
                    "v_subb_co_u32 %[sp], %[m3], %[sp], 0, %[m1]\n\t"  // pop the entry under the postponed leaf
                    "s_andn2_b64 %[m5], %[m4], %[m1]\n\t"             // lanes still without a leaf
                    "s_mov_b64 %[lzm], %[m5]\n\t"
                    "s_and_b64 %[m5], %[m5], exec"
                    : [farc] "=&v"(farc), [xr] "=&v"(xr), [nxt] "=&v"(nxt), [at] "=&v"(at), [node] "=&v"(node),
                      [sp] "+v"(sp), [leaf] "+v"(leaf), [m0] "=&s"(m0), [m1] "=&s"(m1), [m2] "=&s"(m2),
                      [m3] "=&s"(m3), [m4] "=&s"(m4), [m5] "=&s"(m5), [lzm] "+s"(lzm)
                    : [a0] "v"(c0min), [b0] "v"(c0max), [a1] "v"(c1min), [b1] "v"(c1max), [ch0] "v"(ch0),
                      [ch1] "v"(ch1), [t1] "v"(top1), [t2] "v"(top2), [sent] "s"(RW::kSentinel));
                (void)m0; (void)m2; (void)m3;
                *sp_entry = (Entry)farc;
                if ((uint32_t)__popcll(m5) <= leaf_break) break;  // (RT_TUNE_LEAF_BREAK)
            }
        }
        const uint64_t t_leaf = COUNT_TESTS ? __builtin_amdgcn_s_memtime() : 0;
        // One primitive per lane per iteration: a lane walks its leaf's primitives and then the leaves
        // that follow on its stack with its own cursor, so lanes with short leaves do not wait for the
        // wave's longest leaf (same primitives in the same order per lane as a per-leaf loop).
        // cursor and end in units of kPrimStep (bytes of the 32-B primitive record with RT_PRIM_BUFFER)
        uint32_t cur = 0u, end = 0u;
        if (leaf >= RW::kLeaf) {
            const uint32_t l = leaf ^ RW::kMask;
            cur = (l >> 2) * kPrimStep;
            end = cur + ((l & 3u) + 1u) * kPrimStep;
        }
        while (cur < end) {
            {
                const uint32_t i = cur / kPrimStep;  // the primitive's index (a shift, needed only on a hit)
                // byte offsets through a buffer descriptor: no 64-bit address arithmetic per primitive, and
                // two 16-B loads (two texture-addresser requests) per test
                const float4 p0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(prsrc, cur, 0, 0));
                const float4 p1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(prsrc, cur + 16u, 0, 0));
                const uint32_t type = __float_as_uint(p1.w) & 15u;
                if (COUNT_TESTS) {
                    cnt.prims++;
                    cnt.rects += type != RT_SPHERE ? 1u : 0u;
                    cnt.wleaf += wave_leader();
                    if (__ballot(cur != (uint32_t)__builtin_amdgcn_readfirstlane(cur)) == 0) cnt.wleaf_uniform += wave_leader();
                }
                if (type == RT_SPHERE) {  // Sphere::Hit (Hittable.cuh:80-110)
                    const f3 oc = sub(ro, xyz(p0));
                    const float b = dot(oc, rd);
                    const float c = dot(oc, oc) - p1.x;
                    const float disc = b * b - a_dd * c;
                    if (disc > 0) {
                        const float sq = sqrt_fast(disc);
                        float t = fast_div ? div_rn(-b - sq, a_dd, inv_a) : (-b - sq) / a_dd;
                        if (t < t_best && t > kTmin) {
                            t_best = t;
                            hit = (int)i;
                            tag = __float_as_uint(p1.w);
                        } else {
                            const bool tied = EXACT && t == t_best;  // (bvh_clear: a tie at the closest hit so far)
                            t = fast_div ? div_rn(-b + sq, a_dd, inv_a) : (-b + sq) / a_dd;
                            if (t < t_best && t > kTmin) {
                                t_best = t;
                                hit = (int)i;
                                tag = __float_as_uint(p1.w);
                            } else if (EXACT && (tied || t == t_best)) {
                                hit |= kTieBit;
                            }
                        }
                    }
                } else {  // *Rect::Hit
                    const float ok = type == RT_XYRECT ? ro.z : (type == RT_XZRECT ? ro.y : ro.x);
                    const float dk = type == RT_XYRECT ? rd.z : (type == RT_XZRECT ? rd.y : rd.x);
                    const float t = (p0.x - ok) * rcp_ieee(dk);
                    if (!(t < kTmin || t > t_best)) {
                        const float oa = type == RT_YZRECT ? ro.y : ro.x, da = type == RT_YZRECT ? rd.y : rd.x;
                        const float ob = type == RT_XYRECT ? ro.y : ro.z, db = type == RT_XYRECT ? rd.y : rd.z;
                        const float xx = oa + t * da;
                        const float yy = ob + t * db;
                        if (!(xx < p0.y || xx > p0.z || yy < p0.w || yy > p1.x)) {
                            hit = EXACT && t == t_best ? (int)i | kTieBit : (int)i;  // (a rectangle re-accepts an equal t)
                            t_best = t;
                            tag = __float_as_uint(p1.w);
                        }
                    }
                }
            }
            cur += kPrimStep;
            if (cur == end) {
                leaf = 0;
                if (node >= RW::kLeaf) {
                    leaf = node;
                    const uint32_t l = leaf ^ RW::kMask;
                    cur = (l >> 2) * kPrimStep;
                    end = cur + ((l & 3u) + 1u) * kPrimStep;
                    node = ustk[(sp - 1u) * 64];
                    sp--;
                }
            }
        }
        if (COUNT_TESTS) cnt.cleaf += __builtin_amdgcn_s_memtime() - t_leaf;
        if ((uint32_t)__popcll(__ballot(1)) < threshold) break;
    }
    c.node = (int)node;
    c.leaf = (int)leaf;
    c.hit = hit;
    c.tag = tag;
    c.sp = sp;
    c.t_best = t_best;
    if (node == RW::kSentinel && leaf == 0u) c.mode = MODE_SHADE;
}

// Diagnostic ray dump (COUNT_TESTS builds of v3): the lanes with `want` append their ray (one atomic per wave).
__device__ __forceinline__ void dump_ray(const KParams& P, const bool want, const f3 ro, const f3 rd) {
    const uint64_t m = __ballot(want);
    if (m == 0) return;
    const uint32_t leader = (uint32_t)__ffsll((unsigned long long)m) - 1u;
    uint32_t base = 0u;
    if (__lane_id() == leader) base = atomicAdd(P.ray_dump_count, (uint32_t)__popcll(m));
    base = __builtin_amdgcn_readlane(base, leader);
    const uint32_t i = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (want && i < P.ray_dump_cap) {
        P.ray_dump[2 * (size_t)i] = make_float4(ro.x, ro.y, ro.z, 0.0f);
        P.ray_dump[2 * (size_t)i + 1] = make_float4(rd.x, rd.y, rd.z, 0.0f);
    }
}

// v3 kernel: one wave per workgroup, one 8×8 pixel tile per wave; LDS holds the wave's parked path state
// and its traversal stacks (P.lds_wave_words words).
template <bool COUNT_TESTS, int WAVES_PER_SIMD, bool TEX, bool PHILOX = false, bool COMPACT = false, bool WIDE = false>
__global__ __launch_bounds__(64, WAVES_PER_SIMD) void render_kernel_v3(const KParams P) {
    using R = typename std::conditional<PHILOX, RngPhilox, Rng>::type;
    using Entry = typename RefW<WIDE>::Entry;
    constexpr int NODES = NODES_48;
    extern __shared__ float4 lds[];
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t* const wl = (uint32_t*)lds;
    uint32_t* const park = wl + lane;                                                  // word k: park[k * 64]
    Entry* const stk = reinterpret_cast<Entry*>(wl + park_words(COMPACT) * 64) + lane;  // stk[j * 64]
    // node boxes through a buffer descriptor: 32-bit offsets, no 64-bit address arithmetic per visit
    const __amdgpu_buffer_rsrc_t nrsrc =
        NODES == NODES_64 ? __builtin_amdgcn_make_buffer_rsrc((void*)P.nodes, (short)0, (int)(P.num_nodes * 64u), 0x00020000)
                          : __builtin_amdgcn_make_buffer_rsrc((void*)P.nodes48, (short)0, (int)(P.num_nodes * 48u), 0x00020000);
    const float4* __restrict__ prims = P.prims;
    uint32_t x, g;
    size_t pix;
    const uint32_t slot = blockIdx.x;
    const uint32_t tile = (P.tile_order && slot < P.num_tiles) ? P.tile_order[slot] : slot;
    // a lane outside the image (a partial tile) stays in the loop as a finished lane: the wave's reference replay
    // (bvh_replay_wave) keeps its stack across all 64 lanes
    const bool live = lane_pixel<64>(P, x, g, pix, tile);
    if (!live) x = g = 0u, pix = 0u;  // (renders pixel 0's first camera ray, then leaves it: nothing is written)
    const bool rtl = P.rius_rtl != 0;
    stk[0] = (Entry)RefW<WIDE>::kSentinel;   // two sentinel pads below the stack: popping an empty stack
    stk[64] = (Entry)RefW<WIDE>::kSentinel;  // yields the sentinel without a bounds test

    Counts cnt{0, 0, 0, 0, 0, 0, 0};
    f3 ro = mk(0.0f, 0.0f, 0.0f), rd = ro;
    Cursor c{(int)RefW<WIDE>::kSentinel, 0, -1, 0u, 0u, FLT_MAX, MODE_DONE};

    // Sample items (Philox mode, compact parking: the default Philox kernel; full tiles).  Philox draws and sums do not
    // depend on the order a pixel's samples run in (begin_sample, add_sample), so the tile's 64 × spp samples are work
    // items that whichever lane's path has ended takes next — no lane idles because its own pixel is done while the
    // wave's slowest pixel still renders (7 of 64 lanes per node iteration on C2).  Item i is sample i / 64 of pixel
    // i % 64 (the tile's pixels in lane order, sample-major: a wave's lanes stay on one tile); a path's sample goes
    // into its pixel's 64-bit fixed-point sums in LDS — parking words 1-4 (R, G) and 6-7 (B), which the Philox stream
    // (words 0, 5) and this mode's parking (no colour words) leave free; word 8 counts the lane's finished paths' rays
    // (the packed 13-bit ray field holds one path's); the packed sample field holds the item's pixel.
    constexpr bool kItemsBuild = PHILOX && COMPACT;
    const bool items = kItemsBuild && P.spp > 0 && P.max_depth > 0 && __ballot(live) == ~0ull;  // (wave-uniform)
    uint32_t next_item = 64u;  // wave-uniform: items 0-63 (every pixel's sample 0) start below
    const uint32_t n_items = P.spp * 64u;
    const auto item_sum = [&](uint32_t p, int ch) -> unsigned long long* {
        return (unsigned long long*)(wl + (ch < 2 ? 64u + 2u * ((uint32_t)ch * 64u + p) : 384u + 2u * p));
    };
    {  // first camera ray of the pixel
        uint32_t* st = state_at(P, pix);
        R rng = begin_rng<R>(st, P.state_stride, g * P.width + x);  // global pixel index (Kernel.cu:119)
        f3 col = mk(0.0f, 0.0f, 0.0f), att = mk(1.0f, 1.0f, 1.0f);
        // (sample = -1: v3_next_sample starts sample 0; with spp = 0 it stays 0, so compact parking's packed
        // sample field cannot spill into the ray count)
        uint32_t sample = P.spp > 0 ? (uint32_t)-1 : 0u, depth = 0, rays = 0;
        if (P.spp > 0) v3_next_sample<WIDE>(P, x, g, mk(0.0f, 0.0f, 0.0f), rng, col, att, sample, depth, ro, rd, c, rays);
        v3_park<COMPACT>(park, rng, col, att, items ? lane : sample, depth, rays);  // (col + 0 = +0 above)
        if (kItemsBuild && items) {  // (after the park above, which wrote colour words)
            park[1 * 64] = park[2 * 64] = park[3 * 64] = park[4 * 64] = 0u;
            park[6 * 64] = park[7 * 64] = park[8 * 64] = 0u;
        }
    }
    if (!live) c.mode = MODE_DONE;
    const uint32_t threshold = P.regen_threshold;

    const uint64_t t_start = COUNT_TESTS ? __builtin_amdgcn_s_memtime() : 0;
    const uint64_t rt_start = __builtin_amdgcn_s_memrealtime();
    const uint64_t w_start = __builtin_amdgcn_s_memtime();
    while (true) {
        // (RT_REPLAY_SAME_PASS = 0: shade() returned SHADE_REPLAY for these lanes last pass; the path state is parked)
        if (!RT_REPLAY_SAME_PASS && __builtin_expect(__ballot(c.mode == MODE_REPLAY) != 0u, 0))
            bvh_replay_wave(kparams_reload(), prims, c, ro, rd, cnt, COUNT_TESTS);
        const uint64_t t_a = COUNT_TESTS ? __builtin_amdgcn_s_memtime() : 0;
        const uint32_t ntrav = COUNT_TESTS ? (uint32_t)__popcll(__ballot(c.mode == MODE_TRAV)) : 64u;
        if (c.mode == MODE_TRAV) {
            // (RT_TUNE_REGEN_LIVE_FRAC: once pixels finish, the threshold follows the live pixels down)
            uint32_t thr = threshold;
            if (P.regen_live_frac) thr = min(thr, ((uint32_t)__popcll(__ballot(c.mode != MODE_DONE)) * P.regen_live_frac) >> 6);
            v3_traverse<COUNT_TESTS, NODES, park_words(COMPACT) * 256u, WIDE>(nrsrc, NODES == NODES_64 ? P.nodes : P.nodes48, P.refs, prims, stk, thr, ro, rd, c, cnt, ntrav, P.leaf_break);
        }
        const uint64_t t_b = COUNT_TESTS ? __builtin_amdgcn_s_memtime() : 0;
        if (COUNT_TESTS) cnt.ctrav += t_b - t_a;
        for (;;) {  // the shading pass, and once more for lanes whose hit the reference traversal replayed
            if (c.mode == MODE_SHADE) {
                R rng;
                f3 col, att;
                uint32_t sample, depth, rays;
                v3_unpark<COMPACT, false>(park, rng, col, att, sample, depth, rays);
                f3 contrib;
                if (COUNT_TESTS) cnt.wshade += wave_leader();
                KParamsC* const q = kparams_reload();
                const int res = shade<TEX, false, true>(q, prims, q->mats, q->imgs, c.hit, c.tag, c.t_best, ro, rd, att, rng,
                                                        rtl, contrib);
                bool ended = res == SHADE_ENDED;
                if (res != SHADE_REPLAY && !ended && ++depth >= q->max_depth) {  // exceeded recursion (Kernel.cu:79)
                    ended = true;
                    contrib = mk(0.0f, 0.0f, 0.0f);
                }
                if (res == SHADE_REPLAY) {  // (nothing changed: re-parked as it was, replayed at the loop's top)
                    c.mode = MODE_REPLAY;
                } else if (kItemsBuild && items && ended) {  // this sample into its pixel's sums; the lane takes the next item below
                    const uint32_t q0 = quant12(contrib.x), q1 = quant12(contrib.y), q2 = quant12(contrib.z);
                    if (q0) atomicAdd(item_sum(sample, 0), (unsigned long long)q0);
                    if (q1) atomicAdd(item_sum(sample, 1), (unsigned long long)q1);
                    if (q2) atomicAdd(item_sum(sample, 2), (unsigned long long)q2);
                    park[8 * 64] += rays;
                    rays = 0u;
                    c.mode = MODE_NEED;
                } else if (ended) {  // the colour sum stays parked until a path ends (3 fewer VGPRs live through shade())
                    col = mk(__uint_as_float(park[(PK_COL + 0) * 64]), __uint_as_float(park[(PK_COL + 1) * 64]),
                             __uint_as_float(park[(PK_COL + 2) * 64]));
                    v3_next_sample<WIDE>(P, x, g, contrib, rng, col, att, sample, depth, ro, rd, c, rays);
                    park[(PK_COL + 0) * 64] = __float_as_uint(col.x);
                    park[(PK_COL + 1) * 64] = __float_as_uint(col.y);
                    park[(PK_COL + 2) * 64] = __float_as_uint(col.z);
                } else {
                    v3_start_trace<WIDE>(P.num_nodes, c, rays);
                    if (COUNT_TESTS && P.ray_dump) dump_ray(P, depth == P.ray_dump_depth, ro, rd);
                }
                v3_park<COMPACT, false>(park, rng, col, att, sample, depth, rays);
            }
            // (RT_REPLAY_SAME_PASS: the lanes shade() returned SHADE_REPLAY for replay now, every lane active, and shade)
            if (!RT_REPLAY_SAME_PASS || __ballot(c.mode == MODE_REPLAY) == 0u) break;
            bvh_replay_wave(kparams_reload(), prims, c, ro, rd, cnt, COUNT_TESTS);
        }
        if constexpr (kItemsBuild) {
            // lanes whose path ended take the next items (ballot + mbcnt rank on the wave-uniform counter)
            const uint64_t needm = __ballot(c.mode == MODE_NEED);
            if (items && needm != 0) {
                const uint32_t item = next_item +
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(needm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)needm, 0u));
                next_item += (uint32_t)__popcll(needm);
                if (c.mode == MODE_NEED) {
                    if (item < n_items) {
                        const uint32_t p = item & 63u;
                        const uint32_t bx = tile % P.tiles_x, by = tile / P.tiles_x;
                        const uint32_t px = bx * 8u + (p & 7u), pg = global_row(P, by * 8u + (p >> 3));
                        R rng = begin_rng<R>(nullptr, 0u, pg * P.width + px);
                        KParamsC* q = kparams_reload();
                        camera_ray(q, lane_camera(q, px, pg), rng, ro, rd, item >> 6);
                        uint32_t rays = 0u;
                        v3_start_trace<WIDE>(P.num_nodes, c, rays);
                        v3_park<COMPACT, false>(park, rng, mk(0.0f, 0.0f, 0.0f), mk(1.0f, 1.0f, 1.0f), p, 0u, rays);
                    } else {
                        c.mode = MODE_DONE;
                    }
                }
            }
        }
        if (COUNT_TESTS) cnt.cshade += __builtin_amdgcn_s_memtime() - t_b;
        if (__ballot(c.mode != MODE_DONE) == 0) break;
    }
    if (COUNT_TESTS) cnt.ctotal = __builtin_amdgcn_s_memtime() - t_start;
    if (P.wave_trace && wave_leader() && 2ull * tile + 2ull <= P.wave_trace_words) {
        P.wave_trace[2 * tile] = rt_start;
        P.wave_trace[2 * tile + 1] = __builtin_amdgcn_s_memrealtime();
    }
    if (P.tile_cost && wave_leader()) {  // this tile's cost for the next launch's longest-first order
        const uint64_t c = (__builtin_amdgcn_s_memtime() - w_start) >> 8;
        P.tile_cost[tile] = c > 0xffffffffull ? 0xffffffffu : (uint32_t)c;
    }
    if (!live) return;
    R rng;
    f3 col, att;
    uint32_t sample, depth, rays;
    v3_unpark<COMPACT>(park, rng, col, att, sample, depth, rays);
    if (kItemsBuild && items) {  // this lane's pixel's sums (every lane's adds are done: LDS keeps a wave's order)
        const auto sat = [](unsigned long long v) { return __uint_as_float(v > 0xffffffffull ? 0xffffffffu : (uint32_t)v); };
        col = mk(sat(*item_sum(lane, 0)), sat(*item_sum(lane, 1)), sat(*item_sum(lane, 2)));
        rays += park[8 * 64];
    }
    cnt.rays = rays;
    cnt.primary = P.spp;  // every sample starts with one camera ray (Kernel.cu:137-146)
    finish_pixel<COUNT_TESTS>(P, pix, state_at(P, pix), rng, col, cnt);
}

// Closest hit of a batch of rays (rt_trace_rays): v3's traversal (while-while, postponed leaves, the regeneration
// threshold and leaf-break rules) without the shading — a wave owns `per_wave` consecutive rays of the batch and a
// lane whose ray is done takes the wave's next one (ballot + mbcnt on a wave-uniform counter).  Rays are
// (origin, -), (direction, -) float4 pairs; out[i] = (primitive index in the scene's BVH order or -1, t bits).
// For measuring how ray order changes traversal cost (tools/coherence.py: a frame's bounce-2 rays in generation
// order and sorted), and as a closest-hit query for callers that shade on their own.
template <bool COUNT_TESTS>
__global__ __launch_bounds__(64, 8) void trace_rays_kernel(const KParams P, const float4* __restrict__ rays,
                                                          const uint32_t n_rays, const uint32_t per_wave,
                                                          int2* __restrict__ out) {
    using Entry = uint16_t;
    extern __shared__ float4 lds[];
    const uint32_t lane = threadIdx.x & 63u;
    Entry* const stk = reinterpret_cast<Entry*>(lds) + lane;
    const __amdgpu_buffer_rsrc_t nrsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)P.nodes48, (short)0, (int)(P.num_nodes * 48u), 0x00020000);
    stk[0] = (Entry)RefW<false>::kSentinel;
    stk[64] = (Entry)RefW<false>::kSentinel;
    const uint32_t base = blockIdx.x * per_wave;
    const uint32_t end = min(base + per_wave, n_rays);
    Counts cnt{0, 0, 0, 0, 0, 0, 0};
    Cursor c{(int)RefW<false>::kSentinel, 0, -1, 0u, 0u, FLT_MAX, MODE_DONE};
    uint32_t ray = base + lane, nrays = 0u;
    f3 ro = mk(0.0f, 0.0f, 0.0f), rd = ro;
    const auto start = [&](uint32_t i) {
        const float4 o = rays[2 * (size_t)i], d = rays[2 * (size_t)i + 1];
        ro = xyz(o);
        rd = xyz(d);
        v3_start_trace<false>(P.num_nodes, c, nrays);
    };
    if (ray < end) start(ray);
    uint32_t next = base + 64u;  // wave-uniform
    while (__ballot(c.mode != MODE_DONE) != 0) {
        if (c.mode == MODE_TRAV) {
            uint32_t thr = P.regen_threshold;
            if (P.regen_live_frac) thr = min(thr, ((uint32_t)__popcll(__ballot(c.mode != MODE_DONE)) * P.regen_live_frac) >> 6);
            v3_traverse<COUNT_TESTS, NODES_48, 0u, false, false>(nrsrc, P.nodes48, P.refs, P.prims, stk, thr, ro, rd, c, cnt, 64u,
                                                           P.leaf_break);
        }
        if (c.mode == MODE_SHADE) {
            out[ray] = make_int2(c.hit, __float_as_int(c.t_best));
            c.mode = MODE_NEED;
        }
        const uint64_t needm = __ballot(c.mode == MODE_NEED);
        if (needm != 0) {
            const uint32_t i = next + __builtin_amdgcn_mbcnt_hi((uint32_t)(needm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)needm, 0u));
            next += (uint32_t)__popcll(needm);
            if (c.mode == MODE_NEED) {
                if (i < end) {
                    ray = i;
                    start(i);
                } else {
                    c.mode = MODE_DONE;
                }
            }
        }
    }
    cnt.rays = nrays;
    flush_counts<COUNT_TESTS>(P, cnt);
}

// ---------------------------------------------------------------------------------------------------
// v4: v3 made persistent, with per-lane pixel regeneration.
//   v3 gives each lane one pixel for the wave's lifetime, so a lane whose 64 samples are done idles
//   until the wave's slowest pixel finishes, and every wave pays a workgroup dispatch.  v4 launches
//   only as many single-wave workgroups as fit on the device at once; the frame is a queue of work
//   indices (8×8 tiles in row-major tile order, 64 indices per tile), and a lane that finishes its pixel
//   takes the next index at once.  The wave pulls 64-index chunks from the frame's counter with one
//   atomic per chunk; needy lanes take consecutive indices of the wave's chunk (ballot + mbcnt rank).
//   Every pixel still runs the reference's per-pixel sample loop on its own cuRAND stream, so the
//   result does not depend on which lane or wave renders it.  Every wave exits once the queue is empty
//   and its lanes are done (no wave waits on another).
// Requires spp ≥ 1 and max_depth ≥ 1 (rt_render uses v3 otherwise).
// LDS per wave: 18 × 256 B of parked state + (depth + 2) × 128 B of stack.
// ---------------------------------------------------------------------------------------------------
enum ParkSlotV4 { PK_X = PK_WORDS, PK_G = PK_WORDS + 1, PK_PIX = PK_WORDS + 2, PK_WORDS4 = PK_WORDS + 3 };

// Work index → pixel of the local image (8×8 tiles, row-major tile order); false when the index lies
// outside the image or outside the rendered grid.
__device__ __forceinline__ bool work_pixel(const KParams& P, uint32_t idx, uint32_t& x, uint32_t& g, uint32_t& pix) {
    const uint32_t slot = idx >> 6, l = idx & 63u;
    const uint32_t tile = P.tile_order ? P.tile_order[slot] : slot;
    const uint32_t by = tile / P.tiles_x, bx = tile - by * P.tiles_x;
    x = bx * 8u + (l & 7u);
    const uint32_t ly = by * 8u + (l >> 3);
    if (x >= P.width || ly >= P.local_rows) return false;
    g = global_row(P, ly);
    if (x >= P.grid_w || g >= P.grid_h) return false;
    pix = ly * P.width + x;
    return true;
}

// The persistent kernels' pixel queue (v4, persistent flat), all fields wave-uniform.  The frame's work indices
// are split over kQueueCounters heads, each owning a contiguous range; a wave draws chunks from its head with one
// atomic each and moves on to the next live head when its own is exhausted.  Chunks are P.work_chunk indices while
// the head had plenty left at this wave's last grab, then 64 (other waves draining the same head make that count
// stale, so a chunk above 64 can still lengthen the frame's tail: RT_TUNE_QUEUE_CHUNK defaults to 128).
// TRACE: the wave-trace build (a persistent kernel's instance picked only while rt_set_wave_trace holds a buffer); the
// product instances carry none of the trace's stamps and counters, whose SGPRs spilled to VGPR lanes (C5 kernel: 105
// spilled SGPRs with them, 53 without; -2.5 % per frame, profiles/r05q_ab_c5_trace_build.txt).
template <bool TRACE>
struct PixelQueue {
    uint32_t qc;                           // the head the wave draws from
    uint32_t qtried = 0u;                  // heads found exhausted
    uint32_t wq_next = 0u, wq_end = 0u;    // the wave's current chunk
    uint32_t head_left = 0xffffffffu;      // the head's remaining indices as of this wave's last grab from it
    uint32_t wave_pixels = 0u;             // pixels this wave has taken
    bool drained = false;                  // the frame's queue is empty
    uint64_t rt_drained = 0u;              // (wave trace) when it found the queue empty
    uint64_t rt_last = 0u;                 // (wave trace) when it last handed a pixel to a lane
    uint64_t rt_atomic = 0u;               // (wave trace) realtime ticks spent waiting for queue atomics
    uint32_t n_grab = 0u, n_probe = 0u;    // (wave trace) chunk atomics that returned work / found a head exhausted
    // The next chunk's atomic, issued ahead (P.queue_prefetch): its result stays in the issuing lane's VGPR until the
    // current chunk runs out, so its round trip (1-5 us under load, profiles/r05b_c5_tail.txt) overlaps the wave's work
    bool pf_valid = false;                 // wave-uniform: an atomic on head qc is in flight for the next chunk
    uint32_t pf_base = 0u, pf_leader = 0u, pf_want = 0u;
    __device__ explicit PixelQueue(uint32_t head) : qc(head) {}
    // Indices to take per atomic.  Guided (P.queue_guide > 0, RT_TUNE_QUEUE_GUIDE): the head's remaining indices over
    // (waves per head × k), in multiples of 16 between P.queue_min and P.work_chunk — the private reserve of every
    // wave shrinks as its head drains, so when the queue runs dry no wave still holds a full chunk that its lanes
    // take out over a whole pixel lifetime before rendering it (C5's tail, profiles/r05b_c5_tail.txt).  Otherwise
    // round 3's rule: P.work_chunk while the head had at least four chunks at this wave's last grab, then 64.
    __device__ __forceinline__ uint32_t chunk_want(const KParams& P) const {
        if (P.queue_guide) {
            const uint32_t g = (head_left / P.queue_guide) & ~15u;
            return min(P.work_chunk, max(g, P.queue_min));
        }
        return head_left > 4u * P.work_chunk ? P.work_chunk : 64u;
    }
    // Lanes with `need` take the next work indices of the wave's chunk (ballot + mbcnt rank); start(x, g, pix) runs on
    // every lane that gets a pixel, and its `need` clears.  A lane still needing one afterwards found the queue empty.
    template <class F>
    __device__ __forceinline__ void take(const KParams& P, bool& need, F&& start) {
        uint64_t needm = __ballot(need);
        while (needm != 0 && !drained) {
            if (wq_next >= wq_end) {
                uint32_t leader = (uint32_t)__ffsll((unsigned long long)__ballot(1)) - 1u;
                uint32_t base = 0u, want;
                const uint64_t ta = TRACE ? __builtin_amdgcn_s_memrealtime() : 0u;
                if (pf_valid) {  // the chunk fetched ahead (same head: qc changes only below, after consuming it)
                    leader = pf_leader;
                    want = pf_want;
                    base = __builtin_amdgcn_readlane(pf_base, leader);
                    pf_valid = false;
                } else {
                    want = chunk_want(P);
                    if (__lane_id() == leader) base = atomicAdd(P.work_counter + qc * P.queue_stride, want);
                    base = __builtin_amdgcn_readlane(base, leader);
                }
                const uint32_t idx = P.queue_base + qc * P.work_per_counter + base;
                if (TRACE) {  // (diagnostic: the atomic's round trip, stamped after its result is in)
                    __builtin_amdgcn_s_waitcnt(0);
                    rt_atomic += __builtin_amdgcn_s_memrealtime() - ta;
                }
                if (base >= P.work_per_counter || idx >= P.work_total) {  // this head is exhausted
                    // mark it in the exhausted-heads word and move to the next live head (so a wave probes a few
                    // heads at the frame's end, not every one of them)
                    const uint64_t tb = TRACE ? __builtin_amdgcn_s_memrealtime() : 0u;
                    uint32_t done = 0u;
                    if (__lane_id() == leader) done = atomicOr(P.work_counter + kQueueCounters * P.queue_stride, 1u << qc);
                    done = __builtin_amdgcn_readlane(done, leader) | (1u << qc);
                    if (TRACE) {
                        __builtin_amdgcn_s_waitcnt(0);
                        rt_atomic += __builtin_amdgcn_s_memrealtime() - tb;
                        n_probe++;
                    }
                    if (done == kQueueAllDone || ++qtried >= kQueueCounters) {
                        drained = true;
                        if (TRACE) rt_drained = __builtin_amdgcn_s_memrealtime();
                        break;
                    }
                    const uint32_t live = ~done & kQueueAllDone;        // (nonzero here)
                    const uint32_t above = live & ~((2u << qc) - 1u);   // live heads after qc
                    qc = (uint32_t)__builtin_ctz(above ? above : live);
                    head_left = 0u;  // (unknown: small chunks until the first grab there)
                    continue;
                }
                wq_next = idx;
                if (TRACE) n_grab++;
                // (a chunk ends at its head's range: a head's range is a multiple of 64, not of work_chunk)
                wq_end = idx + min(want, P.work_per_counter - base);
                head_left = P.work_per_counter - base - min(want, P.work_per_counter - base);
            }
            const uint32_t avail = wq_end - wq_next;
            const uint32_t rank =
                __builtin_amdgcn_mbcnt_hi((uint32_t)(needm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)needm, 0u));
            if (need && rank < avail) {
                uint32_t x, g, pix;
                if (work_pixel(P, wq_next + rank, x, g, pix)) {
                    need = false;
                    start(x, g, pix, wq_next + rank);
                }
            }
            const uint32_t taken = min((uint32_t)__popcll(needm), avail);
            wq_next += taken;
            if (TRACE && taken) rt_last = __builtin_amdgcn_s_memrealtime();
            const uint64_t still = __ballot(need);
            wave_pixels += (uint32_t)__popcll(needm & ~still);
            needm = still;
        }
        // fetch the next chunk ahead once the current one is nearly used up (never after the queue ran dry: a chunk
        // fetched ahead is always consumed by a later take before the wave can find the queue empty)
        if (P.queue_prefetch && !drained && !pf_valid && wq_end - wq_next <= P.queue_prefetch) {
            pf_leader = (uint32_t)__ffsll((unsigned long long)__ballot(1)) - 1u;
            pf_want = chunk_want(P);
            if (__lane_id() == pf_leader) pf_base = atomicAdd(P.work_counter + qc * P.queue_stride, pf_want);
            pf_valid = true;
        }
    }
};

// End of a persistent wave: the grid's last wave to finish zeroes the queue slot (its heads, the exhausted-heads word
// and the finished-waves count kQueueCounters + 1 strides in), so the slot is clean for the launch that reuses it and
// rt_render needs no memset per frame (5 us per C5 frame, profiles/r04p_kernel_stats_by_grid_c5.csv).  Every wave
// reaches this point after its last queue atomic has returned.
__device__ __forceinline__ uint32_t grid_waves() { return gridDim.x * (blockDim.x >> 6); }
__device__ __forceinline__ uint32_t grid_wave_id() {  // (wave-uniform: an SGPR, not a per-lane value)
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)));
}
// arrivals: how many callers the launch has (its waves, or — GROUP — its workgroups, whose last wave calls it)
__device__ __forceinline__ void queue_release(const KParams& P, const uint32_t arrivals) {
    if (P.queue_host_reset) return;
    const uint32_t leader = (uint32_t)__ffsll((unsigned long long)__ballot(1)) - 1u;
    uint32_t fin = 0u;
    if (__lane_id() == leader) fin = atomicAdd(P.work_counter + (kQueueCounters + 1u) * P.queue_stride, 1u);
    fin = __builtin_amdgcn_readlane(fin, leader);
    if (fin == arrivals - 1u && __lane_id() < kQueueSlotWords)
        __hip_atomic_store(P.work_counter + __lane_id() * P.queue_stride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The end of a GROUP workgroup (wave 0, after a barrier the group's 16 waves all reached).  With P.linger_ticks
// (RT_TUNE_GROUP_LINGER_US, off by default) the group stays resident — asleep, polling the count of arrived workgroups
// — until every workgroup of the grid has finished its pixels, or the deadline passes, then leaves (queue_release
// counts the leavers; the last zeroes the slot).  Measured (profiles/r06h_c5_linger.txt): waves that exit while others
// still render stall those (a depth-1 frame's stragglers spent 24-84 us in their last pass), and with the finished
// groups resident the stragglers run at full speed and every group leaves within ~1-4 us of the last pixel — but the
// kernel then ends ~100 us after the groups leave together, where exits spread over the tail cost ~10 us: C5 0.23 ->
// 0.31 ms.  The deadline bounds the wait when a workgroup of the grid is not resident, so every wave always exits.
__device__ __forceinline__ void group_linger(const KParams& P) {
    if (P.linger_ticks && !P.queue_host_reset && __lane_id() == 0) {
        uint32_t* const arrived = P.work_counter + (kQueueCounters + 2u) * P.queue_stride;
        atomicAdd(arrived, 1u);
        const uint64_t deadline = __builtin_amdgcn_s_memrealtime() + P.linger_ticks;
        while (__hip_atomic_load(arrived, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gridDim.x &&
               __builtin_amdgcn_s_memrealtime() < deadline)
            __builtin_amdgcn_s_sleep(8);
    }
    queue_release(P, gridDim.x);
}

// Wave trace of the persistent kernels (rt_set_wave_trace; tools/v4_timeline.py), kWaveTraceWords words per wave:
// [0] start, [1] queue found empty, [2] end, [3] pixels taken | grid waves << 32, [4] HW_REG_HW_ID | HW_REG_XCC_ID << 32 (the wave's
// SIMD / CU / shader engine and XCD), [5] when it last handed out a pixel, [6] chunk grabs | exhausted-head probes
// << 32, [7] realtime ticks spent waiting for the queue's atomics.  Times: s_memrealtime (100 MHz).
constexpr uint32_t kWaveTraceWords = 8;
template <bool TRACE>
__device__ __forceinline__ void trace_persistent_wave(const KParams& P, const PixelQueue<TRACE>& queue, uint64_t rt_start,
                                                      uint32_t wave_pixels) {
    if (TRACE && P.wave_trace && wave_leader() && (uint64_t)kWaveTraceWords * (grid_wave_id() + 1ull) <= P.wave_trace_words) {
        unsigned long long* w = P.wave_trace + (size_t)kWaveTraceWords * grid_wave_id();
        w[0] = rt_start;
        w[1] = queue.rt_drained;
        w[2] = __builtin_amdgcn_s_memrealtime();
        w[3] = wave_pixels | ((unsigned long long)grid_waves() << 32);
        w[4] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
               ((unsigned long long)__builtin_amdgcn_s_getreg((15 << 11) | 20) << 32);
        w[5] = queue.rt_last;
        w[6] = (unsigned long long)queue.n_grab | ((unsigned long long)queue.n_probe << 32);
        w[7] = queue.rt_atomic;
    }
}

// v4 persistent kernel.  It must not exit early: every wave runs to queue_release, whose last caller re-zeroes the
// frame's queue slot for the launch that reuses it (render_kernel_flat_persistent has the same rule).
template <bool COUNT_TESTS, bool TEX, int NODES = NODES_64, bool PHILOX = false, bool WIDE = false, int WAVES_PER_SIMD = 1,
          bool TRACE = false>
__global__ __launch_bounds__(64, WAVES_PER_SIMD) void render_kernel_v4(const KParams P) {
    using R = typename std::conditional<PHILOX, RngPhilox, Rng>::type;
    using Entry = typename RefW<WIDE>::Entry;
    extern __shared__ float4 lds[];
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t* const wl = (uint32_t*)lds;
    uint32_t* const park = wl + lane;
    Entry* const stk = reinterpret_cast<Entry*>(wl + PK_WORDS4 * 64) + lane;
    const __amdgpu_buffer_rsrc_t nrsrc =
        NODES == NODES_64 ? __builtin_amdgcn_make_buffer_rsrc((void*)P.nodes, (short)0, (int)(P.num_nodes * 64u), 0x00020000)
                          : __builtin_amdgcn_make_buffer_rsrc((void*)P.nodes48, (short)0, (int)(P.num_nodes * 48u), 0x00020000);
    const float4* __restrict__ prims = P.prims;
    const bool rtl = P.rius_rtl != 0;
    stk[0] = (Entry)RefW<WIDE>::kSentinel;
    stk[64] = (Entry)RefW<WIDE>::kSentinel;
    park[PK_RAYS * 64] = 0u;

    Counts cnt{0, 0, 0, 0, 0, 0, 0};
    f3 ro = mk(0.0f, 0.0f, 0.0f), rd = ro;
    Cursor c{(int)RefW<WIDE>::kSentinel, 0, -1, 0u, 0u, FLT_MAX, MODE_NEED};
    PixelQueue<TRACE> queue(blockIdx.x % kQueueCounters);
    const uint32_t threshold = P.regen_threshold;
    const uint64_t rt_start = TRACE ? __builtin_amdgcn_s_memrealtime() : 0u;

    while (true) {
        // shade() returned SHADE_REPLAY for these lanes: the path state is parked, few registers are live
        if (__builtin_expect(__ballot(c.mode == MODE_REPLAY) != 0u, 0))
            bvh_replay_wave(kparams_reload(), prims, c, ro, rd, cnt, COUNT_TESTS);
        if (c.mode == MODE_TRAV) v3_traverse<COUNT_TESTS, NODES, PK_WORDS4 * 256u, WIDE>(nrsrc, NODES == NODES_64 ? P.nodes : P.nodes48, P.refs, prims, stk, threshold, ro, rd, c, cnt);
        R rng;
        f3 col, att;
        uint32_t sample, depth, rays;
        bool cam = false, fin = false;
        const bool shading = c.mode == MODE_SHADE;
        if (shading) {
            v3_unpark(park, rng, col, att, sample, depth, rays);
            f3 contrib;
            if (COUNT_TESTS) cnt.wshade += wave_leader();
            KParamsC* const q = kparams_reload();
            const int res = shade<TEX, false, true>(q, prims, q->mats, q->imgs, c.hit, c.tag, c.t_best, ro, rd, att, rng,
                                                    rtl, contrib);
            bool ended = res == SHADE_ENDED;
            if (res != SHADE_REPLAY && !ended && ++depth >= q->max_depth) {  // exceeded recursion (Kernel.cu:79)
                ended = true;
                contrib = mk(0.0f, 0.0f, 0.0f);
            }
            if (res == SHADE_REPLAY) {  // (nothing changed: re-parked as it was, replayed at the loop's top)
                c.mode = MODE_REPLAY;
            } else if (ended) {
                col = add_sample(rng, col, contrib);  // Kernel.cu:147
                if (++sample < P.spp) {
                    cam = true;
                } else {  // the pixel is done (Kernel.cu:149-157)
                    const uint32_t pix = park[PK_PIX * 64];
                    write_pixel(P, pix, state_at(P, pix), rng, col);
                    fin = true;
                }
            } else {
                v3_start_trace<WIDE>(P.num_nodes, c, rays);
            }
        }
        // pixel regeneration: lanes without a pixel take the next work indices
        bool need = fin || c.mode == MODE_NEED;
        if (__ballot(need) != 0) {
            if (!shading && need) rays = park[PK_RAYS * 64];
            queue.take(P, need, [&](uint32_t x, uint32_t g, uint32_t pix, uint32_t) {
                park[PK_X * 64] = x;
                park[PK_G * 64] = g;
                park[PK_PIX * 64] = pix;
                rng = begin_rng<R>(state_at(P, pix), P.state_stride, g * P.width + x);
                col = mk(0.0f, 0.0f, 0.0f);
                sample = 0u;
                cam = true;
            });
            if (need) c.mode = MODE_DONE;
        }
        if (cam) {  // next sample's camera ray (Kernel.cu:139-146)
            KParamsC* q = kparams_reload();
            const Camera cam_l = lane_camera(q, park[PK_X * 64], park[PK_G * 64]);
            camera_ray(q, cam_l, rng, ro, rd, sample);
            att = mk(1.0f, 1.0f, 1.0f);
            depth = 0u;
            v3_start_trace<WIDE>(P.num_nodes, c, rays);
        }
        if (shading || cam) v3_park(park, rng, col, att, sample, depth, rays);
        if (__ballot(c.mode != MODE_DONE) == 0) break;
    }
    cnt.rays = park[PK_RAYS * 64];
    // every sample starts with one camera ray (Kernel.cu:137-146): spp primary rays per pixel taken
    cnt.primary = __lane_id() == 0 ? queue.wave_pixels * P.spp : 0u;
    trace_persistent_wave(P, queue, rt_start, queue.wave_pixels);
    queue_release(P, grid_waves());
    flush_counts<COUNT_TESTS>(P, cnt);
}

// ---------------------------------------------------------------------------------------------------
// Flat kernel (variant 5): scenes of at most RT_TUNE_FLAT_MAX primitives — BASELINE configs 1, 3 and 5 have 3, 8
// and 5.  Over a handful of primitives a BVH saves few tests and makes the lanes of a wave diverge: different
// node paths, leaves of different lengths, a stack per lane.  Here every ray tests every primitive, in the order
// the reference's own BVH tests them (prims_flat, scene_build.cpp), so all lanes of a wave step through the same
// primitive at the same time: its record is a scalar load whose values are SGPR operands, its type a wave-uniform
// branch, and there is no traversal state.  A pass traces one ray for every lane that needs one and then shades
// every lane; the path state stays in registers (nothing to park: no traversal competes for them).
// RandomInUnitSphere is capped per pass (P.rius_cap): a lane still rejecting resumes the call at the next pass and
// skips that pass's trace, instead of every lane of the wave waiting for the wave's slowest sampler.  Per lane the
// rays, RNG draws and arithmetic are those of the other kernels (tests/test_gpu_parity.py runs it on every case).
// ---------------------------------------------------------------------------------------------------
// Closest hit over all n primitives of the flat table (PerformHit, Hittable.cuh:470-485, for each in turn), then
// whether the reference's box culling could have answered differently.  Without culling the query returns the
// geometric closest hit p* at t*; the reference returns it too unless (a) a box on p*'s path rejects the ray — its
// boxes contain p*'s own (SurroundingBox), so only if p*'s hit point lies on or within rounding of a face of p*'s own
// box: within 2^-18 relative of a face in the axes where t* and the box test compute differently, or a slab distance
// of the rect's own plane axis equal to t* (both are (plane - o) · (1/d), monotone in the plane), — or (b) another
// primitive ties with t* (which one the reference keeps depends on its culling and order), or (c) a NaN took part:
// a rectangle's t is NaN only as 0 · inf, so only on rays with a zero or infinite 1/d component or a non-finite
// origin (geometry is finite, scene_build.cpp); a wave holding such a ray re-runs the rectangles' t for it after the
// scan.  Those rays (about 1e-5 of them) replay the reference exactly (ref_trace); the rest are exact as they stand.
// m's lane bit ? a : b, with the lane mask m read from SGPRs by the select itself (v_cndmask_b32 with an SGPR-pair
// condition)
__device__ __forceinline__ float select_m(const uint64_t m, const float a, const float b) {
    float r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(m));
    return r;
}
__device__ __forceinline__ uint32_t select_m(const uint64_t m, const uint32_t a, const uint32_t b) {
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(m));
    return r;
}

template <bool COUNT_TESTS>
__device__ __forceinline__ void flat_trace(const float4* __restrict__ prims, const float4* __restrict__ rnodes,
                                           const float4* __restrict__ boxes, const uint32_t n, const uint32_t runs0,
                                           const uint32_t runs1, const f3 ro, const f3 rd, int& hit, uint32_t& tag,
                                           float& t_best, Counts& cnt, bool& replay) {
    hit = -1;
    tag = 0u;
    t_best = FLT_MAX;
    // lanes where a candidate equals the closest hit so far, as a wave-uniform lane mask (scalar mask arithmetic, no
    // per-lane VALU bookkeeping)
    uint64_t tie_m = 0u;
    const float a_dd = dot(rd, rd);
    const bool fast_div = a_dd >= 0x1p-40f && a_dd <= 0x1p40f;  // RN(1/a) for the sphere roots (div_rn)
    const float inv_a = rcp_rn(a_dd);
    // 1.0f / d of each axis (the rect tests' inv_d*, Hittable.cuh:149), once per ray instead of once per rect
    const float ix = rcp_ieee(rd.x), iy = rcp_ieee(rd.y), iz = rcp_ieee(rd.z);
    // (c): a rectangle's t can be NaN only if a 1/d component is infinite or zero or the origin is not finite
    // (x · 0 is NaN exactly when x is infinite or NaN)
    const float z = __builtin_fmaf(ix, 0.0f, __builtin_fmaf(iy, 0.0f, __builtin_fmaf(iz, 0.0f, __builtin_fmaf(
                        ro.x, 0.0f, __builtin_fmaf(ro.y, 0.0f, ro.z * 0.0f)))));
    const bool odd = !(z == 0.0f) || ix == 0.0f || iy == 0.0f || iz == 0.0f;
    // Both tests branch-free: every lane evaluates the whole test and the closest hit moves by selects (the tests'
    // results are those of the reference's branches: x and y are pure functions of t, computed whatever t is).
    // XY/XZ/YZRect::Hit (Hittable.cuh:140-169, 196-225, 252-281) with the plane axis k and in-plane axes a, b
    const auto rect = [&](const float4 q0, const float4 q1, const uint32_t i, const float ok, const float ik,
                          const float oa, const float da, const float ob, const float db) {
        const float t = (q0.x - ok) * ik;
        const float xx = oa + t * da;
        const float yy = ob + t * db;
        // the acceptance as an SGPR lane mask: each comparison's ballot is one v_cmp into SGPRs, combined by SALU; the
        // selects read the mask directly (a bool would be materialised as 0/1 and compared again, 8 issue cycles)
        const uint64_t acc_m = __ballot(!(t < kTmin)) & __ballot(!(t > t_best)) & __ballot(!(xx < q0.y)) &
                               __ballot(!(xx > q0.z)) & __ballot(!(yy < q0.w)) & __ballot(!(yy > q1.x));
        tie_m = (tie_m & ~acc_m) | (acc_m & __ballot(t == t_best));
        t_best = select_m(acc_m, t, t_best);
        hit = (int)select_m(acc_m, i, (uint32_t)hit);
        tag = select_m(acc_m, __float_as_uint(q1.w), tag);
    };
    // wave-uniform record: scalar loads through the constant cache
    const auto record = [&](const uint32_t i, float4& q0, float4& q1) {
        const ConstF32* q = (const ConstF32*)((const ConstU8*)prims + i * 32u);
        q0 = make_float4(q[0], q[1], q[2], q[3]);
        q1 = make_float4(q[4], q[5], q[6], q[7]);
        if (COUNT_TESTS) cnt.prims++;
    };
    // One primitive type at a time: prims_flat keeps each type as one contiguous run (scene_build.cpp, `runs`: [begin,
    // end) of type t in bytes 2t, 2t + 1), so no test sits behind a per-primitive type branch (whose merges cost ~8
    // register copies per rectangle).  The scan order does not change the answer: without a tie the closest hit is the
    // unique minimum, and a tie at the minimum is flagged in whichever order its primitives come (the second one seen
    // either ties t_best or, for a rectangle, re-accepts it), then replayed below.
    const auto run = [&](const int t, uint32_t& b, uint32_t& e) {
        const uint32_t v = (t < 2 ? runs0 : runs1) >> (16 * (t & 1));
        b = v & 0xffu;
        e = (v >> 8) & 0xffu;
    };
    uint32_t rb, re;
    run(RT_SPHERE, rb, re);
    for (uint32_t i = rb; i < re; i++) {
        float4 q0, q1;
        record(i, q0, q1);
        {  // Sphere::Hit (Hittable.cuh:80-110)
            const f3 oc = sub(ro, xyz(q0));
            const float b = dot(oc, rd);
            const float c = dot(oc, oc) - q1.x;
            const float disc = b * b - a_dd * c;
            const bool real = disc > 0;
            const float sq = sqrt_fast(real ? disc : 1.0f);  // (a dummy argument keeps sqrt_fast's fast path)
            const float tn = fast_div ? div_rn(-b - sq, a_dd, inv_a) : (-b - sq) / a_dd;
            const float tf = fast_div ? div_rn(-b + sq, a_dd, inv_a) : (-b + sq) / a_dd;
            // (lane masks in SGPRs, as the rectangles' acceptance below)
            const uint64_t real_m = __ballot(real);
            const uint64_t near_m = __ballot(tn < t_best) & __ballot(tn > kTmin);
            const float t = select_m(near_m, tn, tf);  // the far root is tried only when the near one is out of range
            const uint64_t acc_m = real_m & __ballot(t < t_best) & __ballot(t > kTmin);
            tie_m = (tie_m | (real_m & (__ballot(tn == t_best) | (~near_m & __ballot(tf == t_best))))) & ~acc_m;
            t_best = select_m(acc_m, t, t_best);
            hit = (int)select_m(acc_m, i, (uint32_t)hit);
            tag = select_m(acc_m, __float_as_uint(q1.w), tag);
        }
    }
    run(RT_XYRECT, rb, re);
    for (uint32_t i = rb; i < re; i++) {
        float4 q0, q1;
        record(i, q0, q1);
        if (COUNT_TESTS) cnt.rects++;
        rect(q0, q1, i, ro.z, iz, ro.x, rd.x, ro.y, rd.y);
    }
    run(RT_XZRECT, rb, re);
    for (uint32_t i = rb; i < re; i++) {
        float4 q0, q1;
        record(i, q0, q1);
        if (COUNT_TESTS) cnt.rects++;
        rect(q0, q1, i, ro.y, iy, ro.x, rd.x, ro.z, rd.z);
    }
    run(RT_YZRECT, rb, re);
    for (uint32_t i = rb; i < re; i++) {  // YZRect: y from the height, z from the width (Hittable.cuh:255-258)
        float4 q0, q1;
        record(i, q0, q1);
        if (COUNT_TESTS) cnt.rects++;
        rect(q0, q1, i, ro.x, ix, ro.y, rd.y, ro.z, rd.z);
    }
    // (a): p*'s hit point against the faces of p*'s own reference box (boxes: scene_build.cpp pack_flat_box)
    bool edge = false;
    if (hit >= 0) {
        const float4 lo = boxes[2 * hit], hi = boxes[2 * hit + 1];
        // a rect's plane axis: its box's slab distances (k -/+ 0.0001 - o) · (1/d) against t* = (k - o) · (1/d)
        // (lo.w, hi.w: NaN for a sphere)
        const uint32_t type = tag & 15u;
        const bool kz = type == RT_XYRECT, ky = type == RT_XZRECT;
        const float ok = kz ? ro.z : (ky ? ro.y : ro.x), ik = kz ? iz : (ky ? iy : ix);
        edge = ((lo.w - ok) * ik) == t_best || ((hi.w - ok) * ik) == t_best;
        // the other faces, within 2^-18 relative (a rect's plane axis holds 1e30 there: never within)
        const auto near_face = [&](const float o, const float d, const float l, const float h) {
            const float td = t_best * d;
            const float p = o + td;
            const float slack = 0x1p-18f * (fabsf(o) + fabsf(td) + fabsf(l) + fabsf(h)) + 0x1p-120f;
            return fabsf(p - l) <= slack || fabsf(p - h) <= slack;
        };
        edge = edge || near_face(ro.x, rd.x, lo.x, hi.x) || near_face(ro.y, rd.y, lo.y, hi.y) ||
               near_face(ro.z, rd.z, lo.z, hi.z);
    }
    // (c) for the rare waves holding such a ray: the rectangles' t once more (the scan's expression), NaN or not
    bool nan = false;
    if (__ballot(odd) != 0) {
        for (uint32_t i = 0; i < n; i++) {
            const ConstF32* q = (const ConstF32*)((const ConstU8*)prims + i * 32u);
            const uint32_t type = __float_as_uint(q[7]) & 15u;
            if (type == RT_SPHERE) continue;
            const float ok = type == RT_XYRECT ? ro.z : (type == RT_XZRECT ? ro.y : ro.x);
            const float ik = type == RT_XYRECT ? iz : (type == RT_XZRECT ? iy : ix);
            const float t = (q[0] - ok) * ik;
            nan = nan || (odd && t != t);
        }
    }
    const bool tie = (tie_m >> __lane_id()) & 1u;
    // such a ray replays the reference traversal at the top of the next pass, where every lane of the wave is active
    // (flat_replay_wave: wave-serial, no call, no private stack; round 5's called ref_trace with its 16-entry private
    // stack cost C3 10.6 % and C5 3.8 % through the call's register convention in the hot loop, not its ~1e-5 replays)
    replay = tie || nan || edge || t_best != t_best;
    if (COUNT_TESTS && replay) cnt.replays++;
}

// The flat kernels' lanes in MODE_REPLAY (flat_trace flagged their closest hit), one after another through
// ref_trace_wave over the reference tree of the flat table; each gets the reference's answer and shades it (MODE_SHADE).
// Its stack is in LDS (lstk, 32 words per wave): a partial tile's wave has inactive lanes.
__device__ __forceinline__ void flat_replay_wave(KParamsC* q, uint32_t* lstk, int& mode, int& hit, uint32_t& tag,
                                                 float& t, const f3 ro, const f3 rd) {
    uint64_t need = __ballot(mode == MODE_REPLAY);
    while (need != 0u) {
        const int L = (int)__builtin_ctzll(need);
        need &= need - 1u;
        const auto bl = [L](const float v) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), L)); };
        const HitOut r = ref_trace_wave(q->ref_nodes, q->flat_ref_pairs, q->prims, mk(bl(ro.x), bl(ro.y), bl(ro.z)),
                                        mk(bl(rd.x), bl(rd.y), bl(rd.z)), lstk);
        if (__lane_id() == (uint32_t)L) {
            hit = r.hit;
            tag = r.tag;
            t = r.t;
            mode = MODE_SHADE;
        }
    }
}

template <bool COUNT_TESTS, bool TEX, bool PHILOX, int WAVES_PER_SIMD>
__global__ __launch_bounds__(64, WAVES_PER_SIMD) void render_kernel_flat(const KParams P) {
    using R = typename std::conditional<PHILOX, RngPhilox, Rng>::type;
    const float4* __restrict__ prims = P.prims;  // the flat table (rt_render)
    uint32_t x, g;
    size_t pix;
    const uint32_t slot = blockIdx.x;
    const uint32_t tile = (P.tile_order && slot < P.num_tiles) ? P.tile_order[slot] : slot;
    if (!lane_pixel<64>(P, x, g, pix, tile)) return;
    const bool rtl = P.rius_rtl != 0;
    __shared__ uint32_t replay_stk[32];  // flat_replay_wave's stack (one wave per workgroup)
    uint32_t* st = state_at(P, pix);
    R rng = begin_rng<R>(st, P.state_stride, g * P.width + x);  // global pixel index (Kernel.cu:119)

    Counts cnt{0, 0, 0, 0, 0, 0, 0};
    f3 col = mk(0.0f, 0.0f, 0.0f), att = mk(1.0f, 1.0f, 1.0f);
    f3 ro = col, rd = col;
    // (sample = -1: next_sample starts sample 0)
    uint32_t sample = P.spp > 0 ? (uint32_t)-1 : 0u, depth = 0u, rays = 0u;
    int mode = MODE_DONE;
    // A path ended with `contrib` (Kernel.cu:147): the next sample's camera ray (Kernel.cu:139-146), or done.  With
    // max_depth = 0 every sample is black but still draws its camera jitter (Kernel.cu:79).
    const auto next_sample = [&](const f3 contrib) {
        // (COUNT_TESTS: counted on the call's lowest active lane, summed over all lanes at the end)
        const uint64_t c0 = COUNT_TESTS ? __builtin_amdgcn_s_memtime() : 0;
        const uint32_t lead = COUNT_TESTS ? wave_leader() : 0u;
        if (COUNT_TESTS) cnt.idle_wait += lead * (uint32_t)__popcll(__ballot(1));
        col = add_sample(rng, col, contrib);
        KParamsC* q = kparams_reload();
        const Camera cam = lane_camera(q, x, g);
        while (++sample < P.spp) {
            camera_ray(q, cam, rng, ro, rd, sample);
            att = mk(1.0f, 1.0f, 1.0f);
            depth = 0u;
            if (P.max_depth > 0u) {
                mode = MODE_TRAV;
                return;
            }
            col = add_sample(rng, col, mk(0.0f, 0.0f, 0.0f));  // exceeded recursion (Kernel.cu:79)
        }
        mode = MODE_DONE;
        if (COUNT_TESTS) cnt.wleaf += lead * (uint32_t)(__builtin_amdgcn_s_memtime() - c0);
    };
    if (P.spp > 0) next_sample(mk(0.0f, 0.0f, 0.0f));  // (col + 0 = +0)
    // Sample items (Philox mode, full tiles; as render_kernel_v3): a path that ends puts its sample into its pixel's
    // 64-bit fixed-point sums in LDS, and the lane takes the tile's next sample item (i: sample i / 64 of pixel i % 64)
    constexpr bool kItemsBuild = PHILOX;
    __shared__ unsigned long long item_sums[kItemsBuild ? 192 : 1];  // R, G, B x 64 pixels
    const bool items = kItemsBuild && P.spp > 0 && P.max_depth > 0 && __ballot(1) == ~0ull;  // (wave-uniform)
    uint32_t next_item = 64u, item_p = threadIdx.x & 63u;
    if (kItemsBuild && items) item_sums[item_p] = item_sums[64u + item_p] = item_sums[128u + item_p] = 0ull;
    const auto end_path = [&](const f3 contrib) {
        if (kItemsBuild && items) {
            const uint32_t q0 = quant12(contrib.x), q1 = quant12(contrib.y), q2 = quant12(contrib.z);
            if (q0) atomicAdd(&item_sums[item_p], (unsigned long long)q0);
            if (q1) atomicAdd(&item_sums[64u + item_p], (unsigned long long)q1);
            if (q2) atomicAdd(&item_sums[128u + item_p], (unsigned long long)q2);
            mode = MODE_NEED;
        } else {
            next_sample(contrib);
        }
    };

    const uint64_t w_start = __builtin_amdgcn_s_memtime();
    const uint64_t rt_start = __builtin_amdgcn_s_memrealtime();
    int hit = -1;
    uint32_t tag = 0u;
    float t = FLT_MAX;
    // COUNT_TESTS (tools/flat_phases.py): wave cycles in the trace (ctrav) / shading, camera rays included (cshade) /
    // camera-ray code (wleaf), passes (wnode), and per pass the lanes tracing (idle_nt), shading (idle_fin) and
    // starting a sample (idle_wait)
    while (__ballot(mode != MODE_DONE) != 0) {
        const uint64_t c0 = COUNT_TESTS ? __builtin_amdgcn_s_memtime() : 0;
        if (COUNT_TESTS) {
            const uint32_t lead = wave_leader();
            cnt.wnode += lead;
            cnt.idle_nt += lead * (uint32_t)__popcll(__ballot(mode == MODE_TRAV));
            cnt.idle_fin += lead * (uint32_t)__popcll(__ballot(mode == MODE_TRAV || mode == MODE_SHADE));
        }
        // flat_trace flagged these lanes' closest hits last pass: the reference traversal, then they shade below
        if (__builtin_expect(__ballot(mode == MODE_REPLAY) != 0u, 0))
            flat_replay_wave(kparams_reload(), replay_stk, mode, hit, tag, t, ro, rd);
        if (mode == MODE_TRAV) {  // (a lane resuming its RandomInUnitSphere call keeps its hit)
            rays++;
            // the scan's launch-uniform operands re-read per pass (as the persistent flat kernel's)
            KParamsC* const q = kparams_reload();
            bool replay;
            flat_trace<COUNT_TESTS>(q->prims, q->ref_nodes, q->flat_boxes, q->num_prims, q->flat_runs[0], q->flat_runs[1], ro,
                                    rd, hit, tag, t, cnt, replay);
            mode = replay ? MODE_REPLAY : MODE_SHADE;
        }
        const uint64_t c1 = COUNT_TESTS ? __builtin_amdgcn_s_memtime() : 0;
        if (COUNT_TESTS) cnt.ctrav += c1 - c0;
        if (mode == MODE_SHADE) {
            if (COUNT_TESTS) cnt.wshade += wave_leader();
            f3 contrib;
            KParamsC* const q = kparams_reload();
            const int res = shade<TEX, true>(q, prims, q->mats, q->imgs, hit, tag, t, ro, rd, att, rng, rtl, contrib);
            if (res == SHADE_ENDED) {
                end_path(contrib);
            } else if (res == SHADE_CONTINUE) {
                if (++depth >= P.max_depth) end_path(mk(0.0f, 0.0f, 0.0f));  // Kernel.cu:79
                else mode = MODE_TRAV;
            }
        }
        if constexpr (kItemsBuild) {  // lanes whose path ended take the next items (as render_kernel_v3)
            const uint64_t needm = __ballot(mode == MODE_NEED);
            if (items && needm != 0) {
                const uint32_t item = next_item +
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(needm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)needm, 0u));
                next_item += (uint32_t)__popcll(needm);
                if (mode == MODE_NEED) {
                    if (item < P.spp * 64u) {
                        item_p = item & 63u;
                        const uint32_t bx = tile % P.tiles_x, by = tile / P.tiles_x;
                        const uint32_t px = bx * 8u + (item_p & 7u), pg = global_row(P, by * 8u + (item_p >> 3));
                        rng = begin_rng<R>(nullptr, 0u, pg * P.width + px);
                        KParamsC* q = kparams_reload();
                        camera_ray(q, lane_camera(q, px, pg), rng, ro, rd, item >> 6);
                        att = mk(1.0f, 1.0f, 1.0f);
                        depth = 0u;
                        mode = MODE_TRAV;
                    } else {
                        mode = MODE_DONE;
                    }
                }
            }
        }
        if (COUNT_TESTS) cnt.cshade += __builtin_amdgcn_s_memtime() - c1;
    }
    if (kItemsBuild && items) {  // this lane's pixel's sums (every lane's adds are done: LDS keeps a wave's order)
        const auto sat = [](unsigned long long v) { return __uint_as_float(v > 0xffffffffull ? 0xffffffffu : (uint32_t)v); };
        const uint32_t l = threadIdx.x & 63u;
        col = mk(sat(item_sums[l]), sat(item_sums[64u + l]), sat(item_sums[128u + l]));
    }
    if (COUNT_TESTS) cnt.ctotal = __builtin_amdgcn_s_memtime() - w_start;
    if (P.wave_trace && wave_leader() && 2ull * tile + 2ull <= P.wave_trace_words) {
        P.wave_trace[2 * tile] = rt_start;
        P.wave_trace[2 * tile + 1] = __builtin_amdgcn_s_memrealtime();
    }
    if (P.tile_cost && wave_leader()) {  // this tile's cost for the next launch's longest-first order
        const uint64_t c = (__builtin_amdgcn_s_memtime() - w_start) >> 8;
        P.tile_cost[tile] = c > 0xffffffffull ? 0xffffffffu : (uint32_t)c;
    }
    cnt.rays = rays;
    cnt.primary = P.spp;
    finish_pixel<COUNT_TESTS>(P, pix, st, rng, col, cnt);
}

// The persistent flat kernel's workgroup share (GROUP builds, round 6).  One 16-wave workgroup per CU owns a static
// interleaved share of the frame's 8×8 tiles — tile k for k ≡ group (mod groups), k < P.group_tiles — and hands its
// positions (64 per tile, in order) to whichever of its 1 024 lanes needs a pixel through one LDS counter: a
// ds_add_rtn per take, no device-scope atomic, and no private reserve.  Today's per-wave queue keeps a reserve per wave
// (its chunk of up to 128 indices, the chunk fetched ahead, and every lane's next pixel) that it hands out long after
// the queue ran dry while other waves idle: C5's tail was 149 of 262 us (profiles/r05ad_c5_tail_final.txt).  The
// tiles past group_tiles stay in the per-wave queue (PixelQueue over [queue_base, work_total)), which the waves turn
// to once their group's share is handed out, so CUs that run slow or hold costly tiles are evened out at the end.
struct GroupShare {
    uint32_t* next;        // LDS: positions of the share handed out (may run past total)
    uint32_t total;        // positions in the share
    uint32_t left;         // positions left as of this wave's last take
    bool done = false;     // wave-uniform: the share is handed out
    __device__ GroupShare(const KParams& P, uint32_t* lds_next) : next(lds_next) {
        const uint32_t lo = blockIdx.x * P.group_perm_k;  // (permuted: the share is j in [lo, lo + K) ∩ [0, S))
        const uint32_t own = P.group_perm_a ? (lo < P.group_tiles ? min(P.group_perm_k, P.group_tiles - lo) : 0u)
                           : blockIdx.x < P.group_tiles ? (P.group_tiles - 1u - blockIdx.x) / gridDim.x + 1u : 0u;
        total = own * 64u;
        left = total;
        done = total == 0u;
    }
    // Lanes with `need` take the next positions (ballot + mbcnt rank); start(x, g, pix, idx) runs on every lane that
    // gets a pixel.  A lane still needing one afterwards found the share handed out (done).
    template <class F>
    __device__ __forceinline__ uint32_t take(const KParams& P, bool& need, F&& start) {
        uint64_t needm = __ballot(need);
        uint32_t taken_px = 0u;
        while (needm != 0 && !done) {
            const uint32_t k = (uint32_t)__popcll(needm);
            const uint32_t leader = (uint32_t)__ffsll((unsigned long long)needm) - 1u;
            uint32_t base = 0u;
            if (__lane_id() == leader) base = __hip_atomic_fetch_add(next, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            base = __builtin_amdgcn_readlane(base, leader);
            const uint32_t avail = base < total ? min(k, total - base) : 0u;
            left = base < total ? total - base - avail : 0u;
            if (avail < k) done = true;
            const uint32_t rank =
                __builtin_amdgcn_mbcnt_hi((uint32_t)(needm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)needm, 0u));
            if (need && rank < avail) {
                const uint32_t pos = base + rank;
                // interleaved: tile g + k·groups; permuted: tile (j · A) mod S for j = g·K + k, i.e. (g·B + k·A) mod S
                // (rt_render keeps both terms below 2^32 or leaves the shares interleaved)
                const uint32_t tile = P.group_perm_a
                                          ? (blockIdx.x * P.group_perm_b + (pos >> 6) * P.group_perm_a) % P.group_tiles
                                          : blockIdx.x + (pos >> 6) * gridDim.x;
                const uint32_t idx = tile * 64u + (pos & 63u);
                uint32_t x, g, pix;
                if (work_pixel(P, idx, x, g, pix)) {  // (a position outside the image: the lane takes another)
                    need = false;
                    start(x, g, pix, idx);
                }
            }
            const uint64_t still = __ballot(need);
            taken_px += (uint32_t)__popcll(needm & ~still);
            needm = still;
        }
        return taken_px;
    }
};

// The persistent flat kernel's workgroup chunk queue (GROUP 2: RT_TUNE_PERSISTENT_GROUP 2, the default since round
// 6).  Static shares leave the load balance to the shares' sizes, but the XCDs of one MI355X do not render at one
// speed (equal shares ended 196-253 us per XCD, profiles/r06b_ab_c5_group_shares.txt).  Here a workgroup draws chunks
// of tiles from the frame's queue heads (one device atomic per chunk and group, not per wave) and hands their positions
// to its lanes through its LDS counter.  Chunk c covers positions [c·C, c·C + C) (C = P.group_chunk); it is fetched
// by the wave whose claim holds the first position of chunk c - kGqAhead (chunks 0 .. kGqAhead - 1 by thread 0 at the
// start), in chunk order (a fetch waits for the previous chunk's slot), so a chunk that comes back empty means every
// later one is empty too, and every position of a non-empty chunk has been claimed by then.  A lane resolves the
// position it claimed from its chunk's slot in an LDS ring of kGqRing (waiting for the slot if its fetch is in
// flight); positions past a partial chunk's valid indices are claimed again.  Near the end of a head the chunks shrink
// (guided by the indices the head had left at the group's last fetch).
constexpr uint32_t kGqRing = 16;   // chunk slots in LDS (a slot is reused kGqRing chunks later)
constexpr uint32_t kGqAhead = 2;   // chunks fetched ahead of the one being handed out
constexpr uint32_t kGqWords = 8 + 4 * kGqRing;
// LDS words from w: [0] positions claimed, [1] head the group draws from, [2] indices that head had left at the
// group's last fetch; slot s at [8 + 4s]: tag (chunk id + 1; 0 = empty), first work index, valid indices
struct GroupQueue {
    uint32_t* w;
    bool done = false;  // wave-uniform: a chunk came back empty (the frame's queue is exhausted)
    __device__ explicit GroupQueue(uint32_t* lds) : w(lds) {}
    __device__ static uint32_t lds_load(const uint32_t* a) {
        return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __device__ static void lds_store(uint32_t* a, uint32_t v) {
        __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    // one lane: the next chunk's indices from the group's head — guided near the head's end — moving on to the next
    // live head when it is exhausted.  Returns (first index, count), count 0 once every head is exhausted.
    __device__ static uint2 fetch(const KParams& P, uint32_t* w) {
        uint32_t qc = lds_load(w + 1);
        const uint32_t left = lds_load(w + 2), per_head = max(1u, gridDim.x / kQueueCounters);
        const uint32_t want = min(P.group_chunk, max(64u, (left / (2u * per_head)) & ~63u));
        for (uint32_t tries = 0; tries <= kQueueCounters; tries++) {
            const uint32_t b = atomicAdd(P.work_counter + qc * P.queue_stride, want);
            const uint32_t idx = P.queue_base + qc * P.work_per_counter + b;
            if (b < P.work_per_counter && idx < P.work_total) {
                const uint32_t n = min(want, min(P.work_per_counter - b, P.work_total - idx));
                lds_store(w + 1, qc);
                lds_store(w + 2, P.work_per_counter - b - min(want, P.work_per_counter - b));
                return make_uint2(idx, n);
            }
            const uint32_t done = atomicOr(P.work_counter + kQueueCounters * P.queue_stride, 1u << qc) | (1u << qc);
            if (done == kQueueAllDone) break;
            const uint32_t live = ~done & kQueueAllDone, above = live & ~((2u << qc) - 1u);
            qc = (uint32_t)__builtin_ctz(above ? above : live);
            lds_store(w + 2, 0xffffffffu);  // (a new head: its remaining count is not known yet)
        }
        lds_store(w + 1, qc);
        return make_uint2(0u, 0u);
    }
    __device__ static void publish(uint32_t* w, uint32_t chunk, uint2 r) {
        uint32_t* slot = w + 8 + 4 * (chunk % kGqRing);
        lds_store(slot + 1, r.x);
        lds_store(slot + 2, r.y);
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the slot's words before its tag
        __hip_atomic_store(slot, chunk + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    // thread 0, before the kernel's first barrier
    __device__ static void init(const KParams& P, uint32_t* w) {
        w[0] = 0u;
        w[1] = blockIdx.x % kQueueCounters;
        w[2] = 0xffffffffu;
        for (uint32_t s = 0; s < kGqRing; s++) w[8 + 4 * s] = 0u;
        for (uint32_t c = 0; c < kGqAhead; c++) publish(w, c, fetch(P, w));
    }
    // Lanes with `need` claim positions (ballot + mbcnt rank) and start(x, g, pix, idx) runs on every lane that gets a
    // pixel.  A lane still needing one afterwards found the frame's queue exhausted (done).
    template <class F>
    __device__ __forceinline__ uint32_t take(const KParams& P, bool& need, F&& start) {
        uint64_t needm = __ballot(need);
        uint32_t taken_px = 0u;
        const uint32_t C = P.group_chunk;
        while (needm != 0 && !done) {
            const uint32_t k = (uint32_t)__popcll(needm);
            const uint32_t leader = (uint32_t)__ffsll((unsigned long long)needm) - 1u;
            uint32_t p = 0u;
            if (__lane_id() == leader) p = __hip_atomic_fetch_add(w, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            p = __builtin_amdgcn_readlane(p, leader);
            const uint32_t cs = (p + C - 1u) / C;  // the first chunk starting at or after p
            if (cs * C < p + k && __lane_id() == leader) {  // this claim holds chunk cs's first position
                const uint32_t j = cs + kGqAhead;
                while (lds_load(w + 8 + 4 * ((j - 1u) % kGqRing)) < j) __builtin_amdgcn_s_sleep(1);  // chunk j - 1 first
                publish(w, j, fetch(P, w));
            }
            const uint32_t rank =
                __builtin_amdgcn_mbcnt_hi((uint32_t)(needm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)needm, 0u));
            bool dry = false;
            if (need && rank < k) {
                const uint32_t pos = p + rank, c = pos / C, off = pos - c * C;
                const uint32_t* slot = w + 8 + 4 * (c % kGqRing);
                // (its fetch is in flight; the slot is reused only kGqRing chunks later, far beyond any claim)
                while (__hip_atomic_load(slot, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < c + 1u)
                    __builtin_amdgcn_s_sleep(1);
                const uint32_t first = lds_load(slot + 1), cnt = lds_load(slot + 2);
                if (cnt == 0u) {
                    dry = true;
                } else if (off < cnt) {
                    uint32_t x, g, pix;
                    if (work_pixel(P, first + off, x, g, pix)) {
                        need = false;
                        start(x, g, pix, first + off);
                    }
                }
            }
            if (__ballot(dry) != 0) done = true;
            const uint64_t still = __ballot(need);
            taken_px += (uint32_t)__popcll(needm & ~still);
            needm = still;
        }
        return taken_px;
    }
    // indices the group's head had left at its last fetch (0xffffffff: unknown)
    __device__ uint32_t head_left() const { return lds_load(w + 2); }
};

// Persistent flat kernel (variant 6): the flat kernel's closest-hit query in v4's persistent grid — a device-filling
// grid whose lanes take the next pixel from the frame's work queue as soon as theirs is done (PixelQueue), for frames
// with few samples per pixel (BASELINE config 5: 1 spp), where a tile wave would idle on its slowest pixels.  The path
// state stays in registers (no traversal, nothing to park).  Requires spp >= 1 and max_depth >= 1 (rt_render).
// Such a frame is bound by each pixel's chain of dependent memory round trips (RNG state, texel gathers, the
// accumulator), so PREFETCH hides two of them: bit 0 — a lane that starts a pixel also takes its NEXT pixel from the
// queue and issues that pixel's XORWOW state loads, consumed only when it starts it; bit 1 — the float4 accumulator
// of the current pixel is loaded when it starts, not when it is written.  The next pixel is taken early only while
// the wave's queue head holds more than 1/kPrefetchStop of its range: near the end a pixel parked in a busy lane's
// prefetch slot waits out that lane's current pixel while other lanes idle (always-on prefetch lengthened the tail
// 168 -> 211 us; profiles/r04e_ab_c5_prefetch.txt).  Like v4 it must not exit early: every wave reaches
// queue_release, which leaves the queue slot zeroed for its next user.
constexpr int kFlatPrefetch = 1;
constexpr uint32_t kPrefetchStop = 8;
// GROUP (RT_TUNE_PERSISTENT_GROUP, round 6): 2 (the default) — 1024-thread workgroups, one per CU, drawing chunks of
// tiles from the queue heads for their lanes (GroupQueue); 1 — the same workgroups handing out a static share of the
// tiles (GroupShare), then the per-wave queue over the tiles past the shares; 0 — one-wave workgroups on the per-wave
// queue alone (round 5).  Each build carries only its own scheduling code.
template <bool COUNT_TESTS, bool TEX, bool PHILOX, int WAVES_PER_SIMD, bool TRACE = false, int GROUP = 2>
__global__ __launch_bounds__(GROUP ? 1024 : 64, WAVES_PER_SIMD) void render_kernel_flat_persistent(const KParams P) {
    using R = typename std::conditional<PHILOX, RngPhilox, Rng>::type;
    constexpr bool kNext = (kFlatPrefetch & 1) && !PHILOX;  // (Philox has no per-pixel state to load)
    constexpr bool kAcc = (kFlatPrefetch & 2) != 0;
    constexpr uint32_t kNone = 0xffffffffu;
    const float4* __restrict__ prims = P.prims;  // the flat table (rt_render)
    const bool rtl = P.rius_rtl != 0;
    const bool accumulate = (P.flags & RT_FLAG_ACCUMULATE) != 0;
    // The scene's per-lane-indexed tables — the hit primitive's record and reference box, the materials, the image
    // descriptors: under 8 KB for a flat scene (rt_render checks flat_lds_bytes) — staged in LDS once per persistent
    // wave: a pass's dependent loads (box check, material, image descriptor before the texel gather) become LDS reads
    // instead of L2 round trips.  The scan itself keeps its wave-uniform scalar loads of `prims`.
    extern __shared__ float4 lds_tabs[];
    float4* const tprims = lds_tabs;
    float4* const tboxes = tprims + 2u * P.num_prims;
    float4* const tmats = tboxes + 2u * P.num_prims;
    int4* const timgs = reinterpret_cast<int4*>(tmats + 3u * P.num_mats);
    __shared__ uint32_t replay_stk[(GROUP ? 16 : 1) * 32];  // flat_replay_wave's stacks, 32 words per wave
    // GROUP: the share's LDS counter after the tables (rt_render sizes the LDS for it)
    uint32_t* const share_next = reinterpret_cast<uint32_t*>(timgs + P.num_imgs);
    {
        const uint32_t tid = threadIdx.x, nt = blockDim.x;
        for (uint32_t i = tid; i < 2u * P.num_prims; i += nt) {
            tprims[i] = prims[i];
            tboxes[i] = P.flat_boxes[i];
        }
        for (uint32_t i = tid; i < 3u * P.num_mats; i += nt) tmats[i] = P.mats[i];
        for (uint32_t i = tid; i < P.num_imgs; i += nt) timgs[i] = P.imgs[i];
        if (GROUP && tid < 2u) share_next[tid] = 0u;  // (the share's counter, the group's finished waves)
        if (GROUP == 2 && tid == 0u) GroupQueue::init(P, share_next + 2);
        __syncthreads();
    }
    Counts cnt{0, 0, 0, 0, 0, 0, 0};
    R rng{};
    Rng nrng{};               // kNext: the prefetched pixel's state (loads in flight until it starts)
    uint32_t npix = kNone, nx = 0u, ng = 0u, nwidx = 0u;
    uint32_t widx = 0u, life = 0u;  // the pixel's work index and the passes it has taken (P.pixel_cost)
    float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);  // kAcc: the current pixel's accumulator
    f3 col = mk(0.0f, 0.0f, 0.0f), att = col, ro = col, rd = col;
    uint32_t x = 0u, g = 0u, pix = 0u, sample = 0u, depth = 0u, rays = 0u;
    int mode = MODE_NEED;
    int hit = -1;
    uint32_t tag = 0u;
    float t = FLT_MAX;
    const uint32_t wave_id = grid_wave_id(), n_waves = grid_waves();
    PixelQueue<TRACE> queue(wave_id % kQueueCounters);
    GroupShare share(P, share_next);
    if (GROUP != 1) share.done = true;
    // (GROUP 1 with no tail: every tile is in the shares; GROUP 2: the workgroups draw the queue themselves)
    if (GROUP == 2 || P.work_per_counter == 0u) queue.drained = true;
    GroupQueue gq(share_next + 2);
    if (GROUP != 2) gq.done = true;
    uint32_t wave_pixels = 0u;  // pixels this wave took from its group's share
    const uint64_t rt_start = TRACE ? __builtin_amdgcn_s_memrealtime() : 0u;
    // pass trace (diagnostic, tools/c5_tail.py): every 64th wave stamps each of its first kPassTrace / 4 passes with 4
    // words: s_memrealtime at the pass start (bits 0-39) with the lanes about to trace (40-46), shade (47-53) and with a
    // pixel at all (54-60); then s_memrealtime after the trace, after the shading and after the queue
    constexpr uint32_t kPassTrace = 1024;
    // (one wave of every 64 consecutive wave ids, at a different offset in each block: in 16-wave groups every wave
    // index of a group is sampled, not only each group's first wave)
    const bool pass_traced = TRACE && P.wave_trace && (wave_id & 63u) == ((wave_id >> 6) * 17u & 63u) &&
                             (uint64_t)P.wave_trace_words >= (uint64_t)kWaveTraceWords * n_waves +
                                 (uint64_t)kPassTrace * (wave_id / 64u + 1u);
    unsigned long long* const pass_rec =
        pass_traced ? P.wave_trace + (size_t)kWaveTraceWords * n_waves + (size_t)kPassTrace * (wave_id / 64u) : nullptr;
    uint32_t pass_no = 0u;
    while (true) {
        life++;
        if (pass_traced) {
            const uint64_t tr = __builtin_amdgcn_s_memrealtime() & 0xffffffffffull;
            const uint64_t n_t = (uint64_t)__popcll(__ballot(mode == MODE_TRAV));
            const uint64_t n_s = (uint64_t)__popcll(__ballot(mode == MODE_SHADE));
            const uint64_t n_a = (uint64_t)__popcll(__ballot(mode == MODE_TRAV || mode == MODE_SHADE));
            if (4u * pass_no < kPassTrace && wave_leader()) pass_rec[4u * pass_no] = tr | (n_t << 40) | (n_s << 47) | (n_a << 54);
        }
        const auto pass_stamp = [&](uint32_t k) {
            if (pass_traced && 4u * pass_no < kPassTrace && wave_leader()) pass_rec[4u * pass_no + k] = __builtin_amdgcn_s_memrealtime();
        };
        // flat_trace flagged these lanes' closest hits last pass: the reference traversal, then they shade below
        if (__builtin_expect(__ballot(mode == MODE_REPLAY) != 0u, 0))
            flat_replay_wave(kparams_reload(), replay_stk + 32u * (threadIdx.x >> 6), mode, hit, tag, t, ro, rd);
        if (mode == MODE_TRAV) {  // (a lane resuming its RandomInUnitSphere call keeps its hit)
            rays++;
            // the scan's launch-uniform operands re-read per pass (s_load): hoisted out of the loop, the per-run
            // pointers, counts and masks derived from them overflowed the SGPR budget into VGPR-lane spills
            KParamsC* const q = kparams_reload();
            bool replay;
            flat_trace<COUNT_TESTS>(q->prims, q->ref_nodes, tboxes, q->num_prims, q->flat_runs[0], q->flat_runs[1], ro, rd,
                                    hit, tag, t, cnt, replay);
            mode = replay ? MODE_REPLAY : MODE_SHADE;
        }
        pass_stamp(1);
        bool cam = false;
        if (mode == MODE_SHADE) {
            if (COUNT_TESTS) cnt.wshade += wave_leader();
            f3 contrib;
            const int res = shade<TEX, true>(kparams_reload(), tprims, tmats, timgs, hit, tag, t, ro, rd, att, rng, rtl, contrib);
            bool ended = res == SHADE_ENDED;
            if (res == SHADE_CONTINUE && ++depth >= P.max_depth) {  // exceeded recursion (Kernel.cu:79)
                ended = true;
                contrib = mk(0.0f, 0.0f, 0.0f);
            }
            if (ended) {
                col = add_sample(rng, col, contrib);  // Kernel.cu:147
                if (++sample < P.spp) {
                    cam = true;
                } else {  // the pixel is done (Kernel.cu:149-157)
                    write_pixel(P, pix, state_at(P, pix), rng, col, kAcc && accumulate ? &acc : nullptr);
                    if (P.pixel_cost) P.pixel_cost[widx] = (uint8_t)min(life, 255u);
                    mode = MODE_NEED;
                }
            } else if (res == SHADE_CONTINUE) {
                mode = MODE_TRAV;
            }
        }
        pass_stamp(2);
        // pixel regeneration: a lane without a pixel starts its prefetched one, or takes the next work index
        bool need = mode == MODE_NEED;
        if (__ballot(need) != 0) {
            bool started = false;
            const auto start = [&](uint32_t sx, uint32_t sg, uint32_t spix, uint32_t swidx, const R& srng) {
                x = sx;
                g = sg;
                pix = spix;
                widx = swidx;
                life = 0u;
                rng = srng;
                if (kAcc && accumulate && !(P.flags & RT_FLAG_ACCUMULATE_RESET)) acc = P.accum[spix];
                col = mk(0.0f, 0.0f, 0.0f);
                sample = 0u;
                cam = true;
                started = true;
            };
            if constexpr (kNext) {
                if (need && npix != kNone) {
                    need = false;
                    start(nx, ng, npix, nwidx, nrng);
                    npix = kNone;
                }
            }
            const auto start_new = [&](uint32_t qx, uint32_t qg, uint32_t qpix, uint32_t qidx) {  // Kernel.cu:119-123
                start(qx, qg, qpix, qidx, begin_rng<R>(state_at(P, qpix), P.state_stride, qg * P.width + qx));
            };
            if (GROUP == 1 && !share.done) {
                const uint32_t n = share.take(P, need, start_new);
                wave_pixels += n;
                if (TRACE && n) queue.rt_last = __builtin_amdgcn_s_memrealtime();  // (last pixel handed out)
            }
            if (GROUP == 2 && !gq.done) {
                const uint32_t n = gq.take(P, need, start_new);
                wave_pixels += n;
                if (TRACE && n) queue.rt_last = __builtin_amdgcn_s_memrealtime();
                if (TRACE && gq.done && !queue.rt_drained) queue.rt_drained = __builtin_amdgcn_s_memrealtime();
            }
            if (GROUP != 2 && __ballot(need) != 0) queue.take(P, need, start_new);
            if (need) mode = MODE_DONE;
            if constexpr (kNext) {  // the next pixel of every lane that just started one: its state loads go out now
                const auto take_next = [&](uint32_t qx, uint32_t qg, uint32_t qpix, uint32_t qidx) {
                    nx = qx;
                    ng = qg;
                    npix = qpix;
                    nwidx = qidx;
                    nrng = load_rng(state_at(P, qpix), P.state_stride);
                };
                // (from the group's share while it holds more than 1/prefetch_stop of itself; then from the queue by
                // the same rule on the wave's head)
                bool want = started && npix == kNone && P.prefetch_stop != 0u;
                if (GROUP == 1 && !share.done) {
                    want = want && share.left > share.total / P.prefetch_stop;
                    if (__ballot(want) != 0) wave_pixels += share.take(P, want, take_next);
                } else if (GROUP == 2) {
                    want = want && !gq.done && gq.head_left() > P.work_per_counter / P.prefetch_stop;
                    if (__ballot(want) != 0) wave_pixels += gq.take(P, want, take_next);
                } else {
                    want = want && queue.head_left > P.work_per_counter / P.prefetch_stop;
                    if (__ballot(want) != 0) queue.take(P, want, take_next);
                }
            }
        }
        pass_stamp(3);
        pass_no++;
        if (cam) {  // next sample's camera ray (Kernel.cu:139-146)
            KParamsC* q = kparams_reload();
            camera_ray(q, lane_camera(q, x, g), rng, ro, rd, sample);
            att = mk(1.0f, 1.0f, 1.0f);
            depth = 0u;
            mode = MODE_TRAV;
        }
        if (__ballot(mode != MODE_DONE) == 0) break;
    }
    cnt.rays = rays;
    wave_pixels += queue.wave_pixels;
#ifdef RT_LINGER_US
    {  // (diagnostic A/B builds only: the wave stays resident, asleep, this long after its last pixel)
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + 100u * (uint64_t)(RT_LINGER_US);
        while (__builtin_amdgcn_s_memrealtime() < t_end) __builtin_amdgcn_s_sleep(127);
    }
#endif
    cnt.primary = __lane_id() == 0 ? wave_pixels * P.spp : 0u;  // spp camera rays per pixel taken
    trace_persistent_wave(P, queue, rt_start, wave_pixels);
    if constexpr (GROUP) {
        // one device-scope arrival per workgroup (4 096 waves ending within tens of microseconds serialised on the one
        // finished-waves word, ~12 ns each, MI355X_MICROARCH.md fan-in); with RT_TUNE_GROUP_LINGER_US the group's waves
        // wait for each other at a barrier (asleep), then for the grid (group_linger), and leave together
        if (P.linger_ticks) {  // (launch-uniform: every wave of the group takes the same branch)
            __syncthreads();
            if (threadIdx.x < 64u) group_linger(P);
            __syncthreads();
            // (wave trace: word 7, the queue-atomic wait of the per-wave queue, holds when the group left instead)
            if (TRACE && P.wave_trace && wave_leader() && (uint64_t)kWaveTraceWords * (wave_id + 1ull) <= P.wave_trace_words)
                P.wave_trace[(size_t)kWaveTraceWords * wave_id + 7] = __builtin_amdgcn_s_memrealtime();
        } else {  // each wave exits when its lanes are done; the group's last wave (an LDS count) releases the slot
            const uint32_t leader = (uint32_t)__ffsll((unsigned long long)__ballot(1)) - 1u;
            uint32_t fin = 0u;
            if (__lane_id() == leader)
                fin = __hip_atomic_fetch_add(share_next + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            fin = __builtin_amdgcn_readlane(fin, leader);
            if (fin == (blockDim.x >> 6) - 1u) queue_release(P, gridDim.x);
        }
    } else {
        queue_release(P, grid_waves());
    }
    flush_counts<COUNT_TESTS>(P, cnt);
}

// RenderInit (Kernel.cu:166-176): curand_init(seed_base + global_pixel_index, 0, 0).
__device__ __forceinline__ void curand_init_state(unsigned long long seed, uint32_t* st, uint32_t k = 1u) {
    const uint32_t s0 = ((uint32_t)seed) ^ 0xaad26b49u;
    const uint32_t s1 = ((uint32_t)(seed >> 32)) ^ 0xf7dcefddu;
    const uint32_t t0 = 1099087573u * s0;
    const uint32_t t1 = 2591861531u * s1;
    if (k != 1u) {  // RT_FLAG_STATE_SOA: d, v[5] only, one plane each
        st[0] = 6615241u + t1 + t0;
        st[k] = 123456789u + t0;
        st[2 * k] = 362436069u ^ t0;
        st[3 * k] = 521288629u + t1;
        st[4 * k] = 88675123u ^ t1;
        st[5 * k] = 5783321u + t0;
        return;
    }
    *reinterpret_cast<uint4*>(st) = make_uint4(6615241u + t1 + t0, 123456789u + t0, 362436069u ^ t0, 521288629u + t1);
    *reinterpret_cast<uint4*>(st + 4) = make_uint4(88675123u ^ t1, 5783321u + t0, 0u, 0u);
    *reinterpret_cast<uint4*>(st + 8) = make_uint4(0u, 0u, 0u, 0u);  // boxmuller_extra, pad, extra_double
}

__global__ __launch_bounds__(kBlock) void render_init_kernel(uint32_t* state, uint32_t width, uint32_t local_rows,
                                                              uint32_t band_rows, uint32_t num_ranks, uint32_t rank,
                                                              unsigned long long seed_base, uint32_t soa) {  // soa: plane size
    const size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t n = (size_t)width * local_rows;
    if (i >= n) return;
    const uint32_t ly = (uint32_t)(i / width), x = (uint32_t)(i - (size_t)ly * width);
    const uint32_t band = ly / band_rows, within = ly - band * band_rows;
    const uint32_t g = (band * num_ranks + rank) * band_rows + within;
    const uint32_t pixel_index = g * width + x;  // unsigned, as Kernel.cu:174
    if (soa) curand_init_state(seed_base + pixel_index, state + soa_index(x, ly, width), soa);
    else curand_init_state(seed_base + pixel_index, state + i * 12);
}

// LaunchRenderInit's kernel honours the caller's grid/block exactly (Kernel.cu:166-176).
__global__ void render_init_grid_kernel(uint32_t* state, uint32_t width, uint32_t height) {
    const uint32_t i = threadIdx.x + blockIdx.x * blockDim.x;
    const uint32_t j = threadIdx.y + blockIdx.y * blockDim.y;
    if (i >= width || j >= height) return;
    const uint32_t pixel_index = j * width + i;
    curand_init_state(1984ull + pixel_index, state + (size_t)pixel_index * 12);
}

// Longest-first launch order.  Wave lifetimes differ several-fold between tiles (glass and metal paths
// run to depth 8, sky pixels end at once), and a frame's last waves otherwise run on a nearly empty GPU:
// in a row-major launch the final quarter of a config-2 frame holds < 50 % of the steady-state waves.
// After each launch this one-workgroup kernel buckets the tiles by the lifetime their wave just measured
// (4 buckets per octave, most expensive first) into the order the next launch with the same tile grid
// dispatches them in.  The order changes when waves start, never what they compute.
__device__ __forceinline__ uint32_t cost_bucket(uint32_t c) {  // 0 = most expensive
    if (c == 0u) return 127u;
    const uint32_t msb = 31u - (uint32_t)__clz(c);
    const uint32_t frac = msb >= 2u ? (c >> (msb - 2u)) & 3u : (c << (2u - msb)) & 3u;
    return 127u - (msb * 4u + frac);
}

__global__ __launch_bounds__(1024) void plan_order_kernel(const uint32_t* __restrict__ cost,
                                                          uint32_t* __restrict__ order, uint32_t n) {
    __shared__ uint32_t start[128];
    if (threadIdx.x < 128) start[threadIdx.x] = 0u;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += 1024u) atomicAdd(&start[cost_bucket(cost[i])], 1u);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0u;
        for (int b = 0; b < 128; b++) {
            const uint32_t c = start[b];
            start[b] = acc;
            acc += c;
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += 1024u) order[atomicAdd(&start[cost_bucket(cost[i])], 1u)] = i;
}

__global__ void rand_init_kernel(uint32_t* state) {  // RandInit (Kernel.cu:160-164)
    if (threadIdx.x == 0 && blockIdx.x == 0) curand_init_state(1984ull, state);
}

}  // namespace dev

// ---------------------------------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------------------------------
namespace {

thread_local bool g_timing = false;
thread_local float g_last_ms = -1.0f;
thread_local float g_last_host_ms = -1.0f;  // LaunchKernel: host time of the scene-cache step
thread_local int g_variant = -1;
thread_local int g_last_variant = -1;  // the variant the last rt_render on this thread launched

int hip_check(hipError_t e, const char* what, int code = RT_ERR_DEVICE) {
    if (e == hipSuccess) return RT_OK;
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return code;
}

using KernelFn = void (*)(const dev::KParams);

// The kernels librt_hip.so ships (rt_set_variant(i) selects kVariants[i]).  Round 1 measured 37 variants;
// the ones that lost their A/B (LDS-staged scene tables, binary16 and 4-wide nodes, several waves per
// workgroup, register-bound occupancy targets) were dropped (DESIGN.md §4 keeps their numbers).
//   0  v1: scratch stack, 32-bit references       — fallback for scenes beyond 16-bit references and deep BVHs
//   1  v2: 64-thread resumable, 32-bit LDS stacks — fallback for scenes beyond 16-bit references
//   2  v3: 15-word parking                        — spp/depth too large for compact parking
//   3  v3: 13-word compact parking                — automatic choice from 64 spp; below, timed against 4
//   4  v4: persistent work queue, 64-B nodes      — timed against 3 below 64 spp (a compact-parking, 48-B-node,
//         longest-first-ordered v4 measured slower on C2, C3 and C5: profiles/r02_ab_v3_v4compact_c2.txt,
//         profiles/r02_configs_v345.txt)
//   5  flat: no BVH, every primitive per ray        — automatic choice (in 3's place) for scenes of at most
//         RT_TUNE_FLAT_MAX primitives
//   6  persistent flat: 5 in v4's persistent grid — in 4's place for those scenes
struct Variant {
    int stack;        // StackKind
    int lds_depth;    // v2: LDS stack entries per lane
    int block;        // threads per workgroup
    int kernel;       // 1, 2, 3, 4: v1..v4
    bool compact;     // v3: 13-word parking (needs spp < 8192, max_depth < 64, spp · max_depth < 8192)
};
constexpr Variant kVariants[] = {
    {dev::STACK_SCRATCH, 0, 256, 1, false}, {dev::STACK_LDS, 24, 64, 2, false}, {dev::STACK_LDS16, 0, 64, 3, false},
    {dev::STACK_LDS16, 0, 64, 3, true},     {dev::STACK_LDS16, 0, 64, 4, false}, {dev::STACK_NONE, 0, 64, 5, false},
    {dev::STACK_NONE, 0, 64, 6, false},
};
constexpr int kNumVariants = (int)(sizeof(kVariants) / sizeof(kVariants[0]));
constexpr int kVarV1 = 0, kVarV2 = 1, kVarV3 = 2, kVarV3Compact = 3, kVarV4 = 4, kVarFlat = 5, kVarFlatPersistent = 6;

template <int W, bool PH = false, bool C = false, bool WD = false>
KernelFn v3_pick(bool count, bool tex) {
    if (tex) return count ? dev::render_kernel_v3<true, W, true, PH, C, WD> : dev::render_kernel_v3<false, W, true, PH, C, WD>;
    return count ? dev::render_kernel_v3<true, W, false, PH, C, WD> : dev::render_kernel_v3<false, W, false, PH, C, WD>;
}

// __launch_bounds__ waves per SIMD of the textured v4 build (config 5): the compiler's 98 VGPRs (4 waves/SIMD).  The
// config-5 frame is not occupancy-bound: held to 5 / 6 / 8 waves it runs 0.30 / 0.33 / 0.51 ms against 0.293
// (profiles/r03g_ab_v4_tex_waves.txt; 6 and 8 spill to scratch)
constexpr int kV4TexWaves = 1;
// trace: the wave-trace build of a persistent kernel (rt_set_wave_trace holds a buffer; counting builds carry no trace)
template <bool PH = false, bool WD = false>
KernelFn v4_pick(bool count, bool tex, bool trace) {
    if (tex)
        return count   ? dev::render_kernel_v4<true, true, dev::NODES_64, PH, WD>
               : trace ? dev::render_kernel_v4<false, true, dev::NODES_64, PH, WD, kV4TexWaves, true>
                       : dev::render_kernel_v4<false, true, dev::NODES_64, PH, WD, kV4TexWaves>;
    return count   ? dev::render_kernel_v4<true, false, dev::NODES_64, PH, WD>
           : trace ? dev::render_kernel_v4<false, false, dev::NODES_64, PH, WD, 1, true>
                   : dev::render_kernel_v4<false, false, dev::NODES_64, PH, WD>;
}

constexpr int kXorwowCompactWaves = 8;  // __launch_bounds__ waves per SIMD of the XORWOW build of variant 3
constexpr int kPhiloxCompactWaves = 8;  // ... of the non-texture Philox build of variant 3

constexpr int kFlatWaves = 8;  // __launch_bounds__ waves per SIMD of the untextured flat kernel
constexpr int kFlatPersistentWaves = 4;  // resident waves per SIMD of the persistent flat kernel's grid
// RT_TUNE_PERSISTENT_GROUP: the persistent flat kernel's 16-wave workgroups drawing chunks from the queue heads (2,
// default: GroupQueue), with static tile shares (1: GroupShare), or the round-5 one-wave workgroups on the per-wave
// queue alone (0); profiles/r06b_ab_c5_group_shares.txt
thread_local int g_persistent_group = 2;
// RT_TUNE_GROUP_TAIL: permille of the frame's tiles left to the per-wave queue behind the groups' static shares
thread_local int g_group_tail = 0;
// RT_TUNE_GROUP_ORDER: the shares' tiles interleaved (0: tile g + k·groups) or in golden-ratio order (1)
thread_local int g_group_order = 0;
// RT_TUNE_GROUP_CHUNK: positions per chunk of the workgroup chunk queue (RT_TUNE_PERSISTENT_GROUP 2)
thread_local int g_group_chunk = 1024;
// RT_TUNE_GROUP_WAVES: waves per workgroup of the GROUP builds (4, 8, 12 or 16)
thread_local int g_group_waves = 16;
// RT_TUNE_GROUP_LINGER_US: a finished workgroup waits up to this long for the grid's others before it exits (0: off)
thread_local int g_group_linger_us = 0;
// RT_TUNE_QUEUE_RESET: 1 = rt_render zeroes the persistent kernels' queue slot per launch (and they skip queue_release)
thread_local int g_queue_host_reset = 0;
template <bool PH, int G>
KernelFn flat_persistent_pick(bool count, bool tex, bool trace) {
    if (tex)
        return count   ? dev::render_kernel_flat_persistent<true, true, PH, 1, false, G>
               : trace ? dev::render_kernel_flat_persistent<false, true, PH, 1, true, G>
                       : dev::render_kernel_flat_persistent<false, true, PH, 1, false, G>;
    return count   ? dev::render_kernel_flat_persistent<true, false, PH, 1, false, G>
           : trace ? dev::render_kernel_flat_persistent<false, false, PH, 1, true, G>
                   : dev::render_kernel_flat_persistent<false, false, PH, 1, false, G>;
}
template <bool PH>
KernelFn flat_pick(bool count, bool tex, bool persistent, bool trace) {
    if (persistent)
        return g_persistent_group == 2 ? flat_persistent_pick<PH, 2>(count, tex, trace)
               : g_persistent_group == 1 ? flat_persistent_pick<PH, 1>(count, tex, trace)
                                         : flat_persistent_pick<PH, 0>(count, tex, trace);
    if (tex) return count ? dev::render_kernel_flat<true, true, PH, 1> : dev::render_kernel_flat<false, true, PH, 1>;
    return count ? dev::render_kernel_flat<true, false, PH, 1> : dev::render_kernel_flat<false, false, PH, kFlatWaves>;
}

KernelFn pick(int variant, bool count, bool tex, bool philox, bool wide, bool trace) {
    if (variant == kVarFlat || variant == kVarFlatPersistent)
        return philox ? flat_pick<true>(count, tex, variant == kVarFlatPersistent, trace)
                      : flat_pick<false>(count, tex, variant == kVarFlatPersistent, trace);
    if (wide) {  // 32-bit references: builds of the compact v3 and of v4 only (rt_render maps wide scenes there)
        if (variant == kVarV3Compact)
            return philox ? v3_pick<1, true, true, true>(count, tex) : v3_pick<1, false, true, true>(count, tex);
        return philox ? v4_pick<true, true>(count, tex, trace) : v4_pick<false, true>(count, tex, trace);
    }
    switch (variant) {
    case kVarV1: return count ? dev::render_kernel<true> : dev::render_kernel<false>;
    case kVarV2: return count ? dev::render_kernel_v2<true> : dev::render_kernel_v2<false>;
    case kVarV3: return philox ? v3_pick<1, true>(count, tex) : v3_pick<1>(count, tex);
    case kVarV3Compact:
        // Waves per SIMD by registers (profiles/r02_ab_builds_c2.txt, profiles/r03_ab_philox.txt): XORWOW held to 64
        // VGPRs (8 waves, 8 B of cold spills) 16.98 vs 17.25 ms at the compiler's 68; Philox, once its key is read
        // per block and the colour sum stays parked during shading, to 64 as well (20 B of cold spills): 20.24 vs
        // 20.6 ms at 7 waves
        if (philox)
            return tex ? v3_pick<1, true, true>(count, true) : v3_pick<kPhiloxCompactWaves, true, true>(count, false);
        return tex ? v3_pick<1, false, true>(count, true) : v3_pick<kXorwowCompactWaves, false, true>(count, false);
    default: return philox ? v4_pick<true>(count, tex, trace) : v4_pick<false>(count, tex, trace);
    }
}

// RT_TUNE_REGEN_THRESHOLD: 56 together with the live-pixel cap below (the pair's plateau, 56-64 x 52-60/64, is
// flat within 0.3 %; 40 without the cap was round 2's optimum: profiles/r03o_sweep_regen_live_frac.txt)
thread_local int g_regen_threshold = 56;
thread_local int g_lds_pad = 0;  // diagnostic: extra LDS bytes per wave (occupancy experiments)
thread_local unsigned long long* g_wave_trace = nullptr;  // diagnostic: rt_set_wave_trace
thread_local unsigned long long g_wave_trace_words = 0;
thread_local uint8_t* g_pixel_cost = nullptr;  // diagnostic: rt_set_pixel_cost
thread_local float4* g_ray_dump = nullptr;     // diagnostic: rt_set_ray_dump
thread_local uint32_t* g_ray_dump_count = nullptr;
thread_local uint32_t g_ray_dump_cap = 0, g_ray_dump_depth = 1;
thread_local uint64_t g_pixel_cost_bytes = 0;
thread_local const uint32_t* g_tile_order = nullptr;       // experiment: rt_set_tile_order
thread_local int g_adaptive_order = 1;                      // RT_TUNE_ADAPTIVE_ORDER
// RT_TUNE_REGEN_LIVE_FRAC: v3's regeneration threshold is capped at 48/64 of the wave's live pixels, so a wave whose
// pixels are finishing keeps tracing until most of its remaining lanes are done instead of shading a few lanes per
// leaf pass; with it a higher base threshold pays (C2 −2.1 % for the pair against 40 without the cap, C4 −2.4 %,
// C3 ±0.2 %: profiles/r03o_sweep_regen_live_frac.txt; 48 rather than 56 once the leaf-break rule is on, −0.6 %:
// profiles/r03s_ab_node_min_cap.txt)
thread_local int g_regen_live_frac = 48;
// RT_TUNE_LEAF_BREAK: leave the node loop for the leaf tests once at most 3 traversing lanes still lack a leaf
// (with the threshold pair above: C2 −2.4 %, C4 −3.5 %, C3 ±0; round 2 measured −1.2 / +1 % at 2 with threshold 40
// and no cap: profiles/r03r_ab_leaf_break.txt)
thread_local int g_leaf_break = 3;
// RT_TUNE_FLAT_MAX: scenes of at most this many primitives run the flat kernels (variants 5, 6) where the automatic
// choice would run v3 / v4.  RT_TUNE_RIUS_TRIPS: the tile flat kernel's RandomInUnitSphere attempts per pass before a
// rejecting lane defers the rest of the call to the next pass (0 = unbounded; 4: C3's optimum, a wave otherwise runs
// the loop as long as its unluckiest lane).  RT_TUNE_RIUS_TRIPS_PERSISTENT: the same for the persistent flat kernel,
// unbounded by default — a C5 frame is bound by its last pixels' chains of passes, and a deferred call adds a pass to
// one (C5 0.262 -> 0.253 ms per step unbounded, K = 4 / 6 / 8: 0.262 / 0.260 / 0.255; profiles/r05u_c5_rius_trips.txt)
thread_local int g_flat_max = 16;
thread_local int g_rius_trips = 4;
thread_local int g_rius_trips_persistent = 0;
// RT_TUNE_PREFETCH_STOP: the persistent flat kernel's lanes take their next pixel ahead (kFlatPrefetch) only while their
// wave's queue head holds more than 1/value of its range (0 = never); kPrefetchStop (8) by default
thread_local int g_prefetch_stop = (int)dev::kPrefetchStop;

// Per (device, stream, tile grid): the tile costs the v3 kernel records and the order planned from them.
// Plans are held by shared_ptr: a caller keeps its plan alive across the launch even if another thread
// evicts the cache meanwhile (the buffers are freed when the last holder drops it; hipFree waits for the
// device, so a launch still reading them completes first).
struct TilePlan {
    uint32_t* cost = nullptr;
    uint32_t* order = nullptr;
    std::atomic<bool> valid{false};  // an order has been planned (by an earlier launch on the same stream)
    ~TilePlan() {
        if (cost) (void)hipFree(cost);
        if (order) (void)hipFree(order);
    }
};
struct PlanKey {
    int device;
    void* stream;
    uint32_t tiles_x, tiles;
    int kind;  // kernel family
    bool operator<(const PlanKey& o) const {
        if (kind != o.kind) return kind < o.kind;
        if (device != o.device) return device < o.device;
        if (stream != o.stream) return stream < o.stream;
        if (tiles_x != o.tiles_x) return tiles_x < o.tiles_x;
        return tiles < o.tiles;
    }
};
// Automatic kernel choice below 64 spp, by measurement.  Which of v3 (tile waves, longest-first order) and v4
// (persistent, per-lane pixel queue) is faster there depends on the scene as much as on spp (config 2's scene
// at 4 spp: v3 1.54 vs v4 1.77 ms; config 5's at 4 spp: 0.89 vs 0.65; config 3's at 8 spp: 14.1 vs 12.8,
// profiles/r02_ab_v3_v4_low_spp.txt).  Both render the same bits, so the library times one frame of each
// for a (device, stream, scene, frame shape, spp, depth, RNG mode) and keeps the faster: the first frame
// runs v3 untimed (it builds the tile order), the second v3 timed, the third v4 timed, and the choice is
// made once both timings have completed (until then: v4 below 32 spp, v3 from 32).
struct AutoKey {
    int device;
    void* stream;
    const void* scene;
    uint32_t width, rows, spp, depth, philox;
    uint32_t flat;  // the trial's pair is the flat kernels (RT_TUNE_FLAT_MAX may change between frames)
    bool operator<(const AutoKey& o) const {
        return std::tie(device, stream, scene, width, rows, spp, depth, philox, flat) <
               std::tie(o.device, o.stream, o.scene, o.width, o.rows, o.spp, o.depth, o.philox, o.flat);
    }
};
struct AutoChoice {
    int stage = 0;      // frames of the trial already launched
    int chosen = -1;    // the decided variant
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};  // v3 start/end, v4 start/end
    ~AutoChoice() {
        for (hipEvent_t& e : ev)
            if (e) (void)hipEventDestroy(e);
    }
};
constexpr uint32_t kAutoSpp = 64;  // from here on v3 always (configs 2-4: 64-256 spp)
std::mutex g_auto_mu;
// never destroyed (holds HIP events, see g_plans)
// entries held by shared_ptr: a frame being timed keeps its AutoChoice (and events) alive even if another
// thread clears the map meanwhile
std::map<AutoKey, std::shared_ptr<AutoChoice>>& g_auto = *new std::map<AutoKey, std::shared_ptr<AutoChoice>>();

// never destroyed: plans free device memory, which must not run after the HIP runtime has shut down
std::map<PlanKey, std::shared_ptr<TilePlan>>& g_plans = *new std::map<PlanKey, std::shared_ptr<TilePlan>>();
std::mutex g_plans_mu;
constexpr size_t kMaxPlans = 32;

int acquire_plan(const PlanKey& key, hipStream_t s, std::shared_ptr<TilePlan>* out) {
    std::lock_guard<std::mutex> lock(g_plans_mu);
    auto it = g_plans.find(key);
    if (it == g_plans.end()) {
        if (g_plans.size() >= kMaxPlans) g_plans.clear();  // holders keep their plans alive
        auto p = std::make_shared<TilePlan>();
        void* c = nullptr;
        void* o = nullptr;
        int rc = hip_check(hipMalloc(&c, (size_t)key.tiles * 4), "rt_render: tile cost allocation");
        p->cost = (uint32_t*)c;
        if (rc == RT_OK) rc = hip_check(hipMalloc(&o, (size_t)key.tiles * 4), "rt_render: tile order allocation");
        p->order = (uint32_t*)o;
        if (rc == RT_OK) rc = hip_check(hipMemsetAsync(c, 0, (size_t)key.tiles * 4, s), "rt_render: tile cost reset");
        if (rc != RT_OK) return rc;
        it = g_plans.emplace(key, std::move(p)).first;
    }
    *out = it->second;
    return RT_OK;
}
thread_local int g_persistent_waves = 0;  // 0: occupancy query

constexpr size_t kLdsLimit = 160 * 1024;
constexpr size_t kFlatTabLdsMax = 16 * 1024;  // LDS per persistent flat wave for the scene tables (64 primitives: 4 KB)

// Work-queue heads of the persistent kernel: a ring of counters per device, one slot per launch, zeroed
// on the launch's stream right before it.  A slot holds the kQueueCounters heads RT_TUNE_QUEUE_STRIDE apart
// plus the exhausted-heads word) and is reused after kQueueSlots further persistent launches on that device:
// a caller may keep at most kQueueSlots persistent launches in flight per device (rt_hip.h, rt_render).
constexpr uint32_t kQueueSlots = 256;
constexpr uint32_t kQueueMaxStride = 4096;  // bytes between heads (RT_TUNE_QUEUE_STRIDE)
thread_local int g_queue_stride = 128;  // RT_TUNE_QUEUE_STRIDE: bytes between the v4 kernel's queue heads
// RT_TUNE_QUEUE_CHUNK: work indices per queue atomic while the head has plenty left.  128 since the texel gather
// overlaps RandomInUnitSphere: C5 -3.6 % against 64 (0.2525 vs 0.2620 ms, 6 alternations; 192 / 256 lose,
// profiles/r05ag_c5_queue_chunk.txt); round 3 had measured 64..256 within 3 %
thread_local int g_queue_chunk = 128;
thread_local int g_queue_prefetch = 32; // RT_TUNE_QUEUE_PREFETCH: fetch the next chunk ahead at this many indices left
thread_local int g_queue_guide = 0;     // RT_TUNE_QUEUE_GUIDE: guided chunks, head_left / (waves per head × this)
thread_local int g_queue_min = 16;      // RT_TUNE_QUEUE_MIN_CHUNK: the guided chunks' floor
constexpr int kMaxDevices = 64;
struct QueueRing {
    uint32_t* buf = nullptr;
    size_t slot_bytes = 0;  // kQueueCounters heads + the exhausted and finished words at the largest stride used
    std::atomic<uint32_t> next{0};
    int cus = 0;
    std::vector<void*> retired;  // rings outgrown by a larger stride: never freed (see acquire_queue)
};
QueueRing g_queues[kMaxDevices];
std::mutex g_queue_mu;

// The next queue slot of `device` for heads `stride` bytes apart.  The ring is sized for the stride in use (2 KB
// slots at the default 128 B); a larger stride allocates a larger ring.  The outgrown ring is retired, not freed:
// another thread may hold a head pointer into it, taken under the lock, whose memset and launch it has not yet
// enqueued (rt_render), so freeing it could hand the kernel freed memory.  Strides are powers of two in
// [128, kQueueMaxStride], so a device retires at most five rings (≤ 8.9 MB together).
int acquire_queue(int device, uint32_t stride, uint32_t** head, int* cus) {
    if (device < 0 || device >= kMaxDevices) {
        set_error("rt_render: device ordinal out of range");
        return RT_ERR_DEVICE;
    }
    QueueRing& q = g_queues[device];
    const size_t need = (size_t)dev::kQueueSlotWords * stride;
    std::lock_guard<std::mutex> lock(g_queue_mu);
    if (!q.buf || q.slot_bytes < need) {
        if (q.buf) {
            q.retired.push_back(q.buf);
            q.buf = nullptr;
        }
        void* p = nullptr;
        int rc = hip_check(hipMalloc(&p, (size_t)kQueueSlots * need), "rt_render: work queue allocation");
        if (rc != RT_OK) return rc;
        // zeroed once, before any launch can take a slot (every launch leaves its slot zeroed: queue_release)
        rc = hip_check(hipMemset(p, 0, (size_t)kQueueSlots * need), "rt_render: work queue reset");
        if (rc == RT_OK) rc = hip_check(hipDeviceSynchronize(), "rt_render: work queue reset");
        if (rc != RT_OK) {
            (void)hipFree(p);
            return rc;
        }
        q.buf = (uint32_t*)p;
        q.slot_bytes = need;
        if (q.cus == 0) {
            int n = 0;
            rc = hip_check(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device),
                           "rt_render: compute unit count");
            if (rc != RT_OK) return rc;
            q.cus = n;
        }
    }
    *head = q.buf + (size_t)(q.next.fetch_add(1u) % kQueueSlots) * (q.slot_bytes / 4u);
    *cus = q.cus;
    return RT_OK;
}

}  // namespace

}  // namespace rt

using namespace rt;

namespace {
// Process-wide flags LaunchKernel adds to its own (rt_set_launch_flags); the environment's RT_LAUNCH_RANDOM_FILL=ltr sets
// RT_FLAG_RIUS_LEFT_TO_RIGHT before the first call, so a viewer switches Random()'s fill order without a code change.
std::atomic<uint32_t> g_launch_flags{0u};
std::once_flag g_launch_env_once;
constexpr uint32_t kLaunchFlagsAllowed = RT_FLAG_RIUS_LEFT_TO_RIGHT;

}  // namespace

extern "C" {

int rt_set_wave_trace(void* buffer, uint64_t words) {
    g_wave_trace = (unsigned long long*)buffer;
    g_wave_trace_words = buffer ? words : 0;
    return RT_OK;
}

int rt_set_ray_dump(void* rays, uint32_t capacity, uint32_t* count, uint32_t depth) {
    if (rays && (!count || capacity == 0)) {
        set_error("rt_set_ray_dump: a ray buffer needs a count word and a capacity");
        return RT_ERR_INVALID_ARGUMENT;
    }
    g_ray_dump = (float4*)rays;
    g_ray_dump_count = rays ? count : nullptr;
    g_ray_dump_cap = rays ? capacity : 0u;
    g_ray_dump_depth = depth;
    return RT_OK;
}

int rt_trace_rays(const rt_scene* scene, const float* rays, uint32_t n, int32_t* hits, uint64_t* counters,
                  int count_tests, rt_stream stream) {
    if (!scene || (n && (!rays || !hits))) { set_error("rt_trace_rays: NULL argument"); return RT_ERR_INVALID_ARGUMENT; }
    if (n == 0) return RT_OK;
    const DeviceScene& S = scene->dev;
    if (S.wide_refs) { set_error("rt_trace_rays: scenes with 32-bit references are not supported"); return RT_ERR_UNSUPPORTED; }
    const size_t lds = (size_t)(S.depth + 2) * 64 * 2;
    if (S.depth > (uint32_t)dev::kStackMax || lds > kLdsLimit) { set_error("rt_trace_rays: BVH too deep"); return RT_ERR_UNSUPPORTED; }
    dev::KParams P;
    std::memset(&P, 0, sizeof(P));
    P.nodes48 = (const float4*)S.nodes48;
    P.refs = (const uint32_t*)S.refs;
    P.prims = (const float4*)S.prims;
    P.num_nodes = S.num_nodes;
    P.num_prims = S.num_prims;
    P.counters = (unsigned long long*)counters;
    P.regen_threshold = (uint32_t)g_regen_threshold;
    P.regen_live_frac = (uint32_t)g_regen_live_frac;
    P.leaf_break = (uint32_t)g_leaf_break;
    // rays per wave: enough waves to fill the device (8 per SIMD), at most 16 rays per lane
    const uint32_t per_lane = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(16, (uint64_t)n / (64ull * 8192ull)));
    const uint32_t per_wave = 64u * per_lane;
    const uint32_t grid = (uint32_t)(((uint64_t)n + per_wave - 1) / per_wave);
    hipStream_t s = (hipStream_t)stream;
    (void)hipGetLastError();
    if (count_tests && counters)
        hipLaunchKernelGGL(dev::trace_rays_kernel<true>, dim3(grid), dim3(64), lds, s, P, (const float4*)rays, n, per_wave,
                           (int2*)hits);
    else
        hipLaunchKernelGGL(dev::trace_rays_kernel<false>, dim3(grid), dim3(64), lds, s, P, (const float4*)rays, n, per_wave,
                           (int2*)hits);
    return hip_check(hipGetLastError(), "rt_trace_rays: kernel launch", RT_ERR_LAUNCH);
}

int rt_set_pixel_cost(void* buffer, uint64_t bytes) {
    g_pixel_cost = (bytes && buffer) ? (uint8_t*)buffer : nullptr;
    g_pixel_cost_bytes = g_pixel_cost ? bytes : 0;
    return RT_OK;
}

int rt_set_tile_order(const void* order) {
    g_tile_order = (const uint32_t*)order;
    return RT_OK;
}

int rt_set_timing(int enabled) {
    g_timing = enabled != 0;
    return RT_OK;
}

float rt_last_kernel_ms(void) { return g_last_ms; }

float rt_last_launch_host_ms(void) { return g_last_host_ms; }

// Benchmark/tuning knob: -1 = automatic, else an index into kVariants.  Returns the previous value.
int rt_set_variant(int variant) {
    int prev = g_variant;
    g_variant = variant;
    return prev;
}

int rt_last_variant(void) { return g_last_variant; }

int rt_set_tuning(int key, int value) {
    if (key == RT_TUNE_REGEN_THRESHOLD) {
        if (value < 1 || value > 64) {
            set_error("rt_set_tuning: regen threshold must be in [1, 64]");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int prev = g_regen_threshold;
        g_regen_threshold = value;
        return prev;
    }
    if (key == RT_TUNE_LEAF_MAX) {
        if (value < 1 || value > kLeafMax) {
            set_error("rt_set_tuning: leaf max must be in [1, 4]");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int prev = g_leaf_max;
        g_leaf_max = value;
        return prev;
    }
    if (key == RT_TUNE_SAH_TRAVERSAL) {
        if (value < 1 || value > 1000) {
            set_error("rt_set_tuning: SAH traversal cost (x10) must be in [1, 1000]");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int prev = g_sah_traversal_x10;
        g_sah_traversal_x10 = value;
        return prev;
    }
    if (key == RT_TUNE_ADAPTIVE_ORDER) {
        if (value < 0 || value > 1) {
            set_error("rt_set_tuning: adaptive order must be 0 or 1");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int prev = g_adaptive_order;
        g_adaptive_order = value;
        return prev;
    }
    if (key == RT_TUNE_TEXEL_LAYOUT) {
        if (value != 3 && value != 4) {
            set_error("rt_set_tuning: texel layout must be 3 (RGB8) or 4 (RGBA8)");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int prev = g_texel_bytes;
        g_texel_bytes = value;
        return prev;
    }
    if (key == RT_TUNE_LDS_PAD) {
        if (value < 0 || value > 65536 || value % 4) {
            set_error("rt_set_tuning: LDS pad must be a multiple of 4 in [0, 65536]");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int prev = g_lds_pad;
        g_lds_pad = value;
        return prev;
    }
    if (key == RT_TUNE_QUEUE_CHUNK) {
        if (value < 64 || value > 4096 || value % 64) {
            set_error("rt_set_tuning: queue chunk must be a multiple of 64 in [64, 4096]");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int prev = g_queue_chunk;
        g_queue_chunk = value;
        return prev;
    }
    if (key == RT_TUNE_QUEUE_STRIDE) {
        if (value < 128 || value > (int)kQueueMaxStride || (value & (value - 1))) {
            set_error("rt_set_tuning: queue head stride must be a power of two in [128, 4096] bytes");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int prev = g_queue_stride;
        g_queue_stride = value;
        return prev;
    }
    if (key == RT_TUNE_REGEN_LIVE_FRAC) {
        if (value < 0 || value > 64) {
            set_error("rt_set_tuning: live fraction must be in [0, 64]");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int prev = g_regen_live_frac;
        g_regen_live_frac = value;
        return prev;
    }
    if (key == RT_TUNE_LEAF_BREAK) {
        if (value < 0 || value > 64) {
            set_error("rt_set_tuning: leaf break must be in [0, 64]");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int prev = g_leaf_break;
        g_leaf_break = value;
        return prev;
    }
    if (key == RT_TUNE_RIUS_TRIPS || key == RT_TUNE_RIUS_TRIPS_PERSISTENT) {
        if (value < 0 || value > 64) {
            set_error("rt_set_tuning: RandomInUnitSphere trips must be in [0, 64]");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int& knob = key == RT_TUNE_RIUS_TRIPS ? g_rius_trips : g_rius_trips_persistent;
        int prev = knob;
        knob = value;
        return prev;
    }
    if (key == RT_TUNE_PREFETCH_STOP) {
        if (value < 0 || value > 1024) {
            set_error("rt_set_tuning: prefetch stop must be in [0, 1024]");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int prev = g_prefetch_stop;
        g_prefetch_stop = value;
        return prev;
    }
    if (key == RT_TUNE_GROUP_WAVES) {
        if (value < 4 || value > 16 || value % 4) {
            set_error("rt_set_tuning: group waves must be 4, 8, 12 or 16");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int prev = g_group_waves;
        g_group_waves = value;
        return prev;
    }
    if (key == RT_TUNE_GROUP_LINGER_US) {
        if (value < 0 || value > 100000) {
            set_error("rt_set_tuning: group linger must be in [0, 100000] us");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int prev = g_group_linger_us;
        g_group_linger_us = value;
        return prev;
    }
    if (key == RT_TUNE_GROUP_CHUNK) {
        if (value < 64 || value > 4096 || value % 64) {
            set_error("rt_set_tuning: group chunk must be a multiple of 64 in [64, 4096]");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int prev = g_group_chunk;
        g_group_chunk = value;
        return prev;
    }
    if (key == RT_TUNE_PERSISTENT_GROUP) {
        if (value < 0 || value > 2) {
            set_error("rt_set_tuning: persistent group must be 0, 1 or 2");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int prev = g_persistent_group;
        g_persistent_group = value;
        return prev;
    }
    if (key == RT_TUNE_QUEUE_RESET) {
        if (value < 0 || value > 1) {
            set_error("rt_set_tuning: queue reset must be 0 or 1");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int prev = g_queue_host_reset;
        g_queue_host_reset = value;
        return prev;
    }
    if (key == RT_TUNE_GROUP_ORDER) {
        if (value < 0 || value > 1) {
            set_error("rt_set_tuning: group order must be 0 or 1");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int prev = g_group_order;
        g_group_order = value;
        return prev;
    }
    if (key == RT_TUNE_GROUP_TAIL) {
        if (value < 0 || value > 1000) {
            set_error("rt_set_tuning: group tail must be in [0, 1000] permille");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int prev = g_group_tail;
        g_group_tail = value;
        return prev;
    }
    if (key == RT_TUNE_FLAT_MAX) {
        if (value < 0 || value > (int)kFlatMaxPrims) {
            set_error("rt_set_tuning: flat kernel primitive limit must be in [0, 64]");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int prev = g_flat_max;
        g_flat_max = value;
        return prev;
    }
    if (key == RT_TUNE_QUEUE_GUIDE) {
        if (value < 0 || value > 64) {
            set_error("rt_set_tuning: queue guide factor must be in [0, 64]");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int prev = g_queue_guide;
        g_queue_guide = value;
        return prev;
    }
    if (key == RT_TUNE_QUEUE_MIN_CHUNK) {
        if (value < 16 || value > 64 || value % 16) {
            set_error("rt_set_tuning: guided chunk floor must be 16, 32, 48 or 64");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int prev = g_queue_min;
        g_queue_min = value;
        return prev;
    }
    if (key == RT_TUNE_QUEUE_PREFETCH) {
        if (value < 0 || value > 64) {
            set_error("rt_set_tuning: queue prefetch must be in [0, 64]");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int prev = g_queue_prefetch;
        g_queue_prefetch = value;
        return prev;
    }
    if (key == RT_TUNE_PERSISTENT_WAVES) {
        if (value < 0 || value > 16) {
            set_error("rt_set_tuning: persistent waves per SIMD must be in [0, 16]");
            return RT_ERR_INVALID_ARGUMENT;
        }
        int prev = g_persistent_waves;
        g_persistent_waves = value;
        return prev;
    }
    set_error("rt_set_tuning: unknown key");
    return RT_ERR_INVALID_ARGUMENT;
}

int rt_render(const rt_scene* scene, const rt_render_args* a, rt_stream stream) {
    if (!scene || !a) { set_error("rt_render: NULL scene or args"); return RT_ERR_INVALID_ARGUMENT; }
    if (a->tiling.local_rows == 0 || a->width == 0 || a->height == 0) return RT_OK;  // nothing to render
    const bool philox = (a->flags & RT_FLAG_RNG_PHILOX) != 0;
    if (!a->state && !philox) { set_error("rt_render: state is NULL"); return RT_ERR_INVALID_ARGUMENT; }
    if (philox && a->samples_per_pixel > RT_PHILOX_MAX_SPP) {  // sample s reads the window at word s << 18
        set_error("rt_render: RT_FLAG_RNG_PHILOX supports at most RT_PHILOX_MAX_SPP (16384) samples per pixel");
        return RT_ERR_INVALID_ARGUMENT;
    }
    if (a->reserved != 0 || a->reserved2 != 0) { set_error("rt_render: reserved fields must be 0"); return RT_ERR_INVALID_ARGUMENT; }
    if (!a->pos && !a->radiance && !a->accum) { set_error("rt_render: no output buffer"); return RT_ERR_INVALID_ARGUMENT; }
    if ((a->flags & RT_FLAG_ACCUMULATE) && !a->accum) { set_error("rt_render: ACCUMULATE without accum"); return RT_ERR_INVALID_ARGUMENT; }
    if ((a->flags & RT_FLAG_ACCUMULATE_RESET) && !(a->flags & RT_FLAG_ACCUMULATE)) {
        set_error("rt_render: ACCUMULATE_RESET without ACCUMULATE");
        return RT_ERR_INVALID_ARGUMENT;
    }
    if (a->width == 0 || a->height == 0) return RT_OK;
    const rt_tiling& T = a->tiling;
    if (T.band_rows == 0 || T.num_ranks == 0 || T.rank >= T.num_ranks) {
        set_error("rt_render: invalid tiling");
        return RT_ERR_INVALID_ARGUMENT;
    }
    if (T.local_rows == 0) return RT_OK;
    {
        // the last local row must map into the image
        uint32_t l = T.local_rows - 1, band = l / T.band_rows, within = l % T.band_rows;
        uint64_t g = ((uint64_t)band * T.num_ranks + T.rank) * T.band_rows + within;
        if (g >= a->height) { set_error("rt_render: tiling maps local rows outside the image"); return RT_ERR_INVALID_ARGUMENT; }
    }
    const DeviceScene& S = scene->dev;
    if (S.depth > (uint32_t)dev::kStackMax) {
        set_error("rt_render: BVH deeper than the traversal stack");
        return RT_ERR_UNSUPPORTED;
    }
    dev::KParams P;
    std::memset(&P, 0, sizeof(P));
    P.nodes = (const float4*)S.nodes;
    P.nodes48 = (const float4*)S.nodes48;
    P.refs = (const uint32_t*)S.refs;
    P.prims = (const float4*)S.prims;
    P.mats = (const float4*)S.mats;
    P.imgs = (const int4*)S.imgs;
    P.texels = (const uint8_t*)S.texels;
    P.pos = a->pos;
    P.radiance = (float4*)a->radiance;
    P.accum = (float4*)a->accum;
    P.state = (uint32_t*)a->state;
    if (a->flags & RT_FLAG_STATE_SOA) {  // six planes of whole 8×8 tiles
        const uint64_t plane = rt_soa_plane_words(a->width, T.local_rows);
        if (plane > 0xffffffffull) {
            set_error("rt_render: RT_FLAG_STATE_SOA needs < 2^32 pixels per rank");
            return RT_ERR_INVALID_ARGUMENT;
        }
        P.state_stride = (uint32_t)plane;
    } else {
        P.state_stride = 1u;
    }
    P.counters = (unsigned long long*)a->counters;
    P.num_nodes = S.num_nodes;
    P.num_prims = S.num_prims;
    P.num_mats = S.num_mats;
    P.num_imgs = S.num_imgs;
    P.width = a->width;
    P.height = a->height;
    P.spp = a->samples_per_pixel;
    P.max_depth = a->max_depth;
    P.flags = a->flags;
    P.band_rows = T.band_rows;
    P.num_ranks = T.num_ranks;
    P.rank = T.rank;
    P.local_rows = T.local_rows;
    P.tiles_x = 0;  // set below for the chosen workgroup shape
    const bool faithful = (a->flags & RT_FLAG_FAITHFUL_GRID) != 0;
    P.grid_w = faithful ? (a->width / 16) * 16 : a->width;
    P.grid_h = faithful ? (a->height / 16) * 16 : a->height;
    P.rius_rtl = (a->flags & RT_FLAG_RIUS_LEFT_TO_RIGHT) ? 0u : 1u;
    P.regen_threshold = (uint32_t)g_regen_threshold;
    P.regen_live_frac = (uint32_t)g_regen_live_frac;
    P.leaf_break = (uint32_t)g_leaf_break;
    P.rng_key_lo = (uint32_t)a->rng_seed;
    P.rng_key_hi = (uint32_t)(a->rng_seed >> 32);
    P.rng_frame = a->rng_frame;
    P.wave_trace = g_wave_trace;
    P.wave_trace_words = g_wave_trace_words;
    P.tile_order = g_tile_order;
    P.ray_dump = g_ray_dump;
    P.ray_dump_count = g_ray_dump_count;
    P.ray_dump_cap = g_ray_dump_cap;
    P.ray_dump_depth = g_ray_dump_depth;
    // Launch-uniform camera terms, with the binary32 operations of Kernel.cu:130-143.
    const rt_input_struct& in = a->inputs;
    P.width_f = (float)a->width;
    P.inv_width = 1.0f / P.width_f;
    P.cx = (float)a->width / 2.0f;
    P.cy = (float)a->height / 2.0f;
    P.near_plane = in.near_plane;
    P.far_plane = in.far_plane;
    {
        volatile float up[3] = {in.up[0], in.up[1], in.up[2]};
        volatile float fw[3] = {in.orientation[0], in.orientation[1], in.orientation[2]};
        // rightV = Normalize(Cross(upV, forwardV)) (Kernel.cu:133, Math.cuh:157-161, 225-229)
        volatile float cx = up[1] * fw[2] - up[2] * fw[1];
        volatile float t = up[0] * fw[2] - up[2] * fw[0];
        volatile float cy = -t;
        volatile float cz = up[0] * fw[1] - up[1] * fw[0];
        volatile float d0 = cx * cx, d1 = cy * cy, d2 = cz * cz;
        volatile float dd = d0 + d1;
        dd = dd + d2;
        volatile float s = std::sqrt((float)dd);
        volatile float inv = 1.0f / s;
        P.right[0] = inv * cx;
        P.right[1] = inv * cy;
        P.right[2] = inv * cz;
        volatile float k10 = 1.0f / in.fov;
        k10 = k10 * 10.0f;
        for (int i = 0; i < 3; i++) {
            P.origin[i] = in.origin[i];
            P.up[i] = in.up[i];
            P.fov_fwd[i] = in.fov * fw[i];
            P.k10_fwd[i] = k10 * fw[i];
            P.bg0[i] = in.background_start[i];
            P.bg1[i] = in.background_end[i];
        }
    }

    const bool count_tests = a->counters && (a->flags & RT_FLAG_COUNT_TESTS);
    int variant = g_variant;
    // auto: the fastest measured kernel per workload shape (profiles/r01d_*, r01e_*): the persistent v4 when a
    // pixel has few paths (config 5: 1 spp, 0.51-0.54 vs 0.80 ms), otherwise v3 with the adaptive
    // longest-first tile order and compact parking: 13 words of parked state + a depth + 2 stack fit config
    // 2's wave in 5 KB of LDS, 8 waves per SIMD (config 2: 17.05 vs 17.8 ms with 15-word parking; config 3,
    // depth 16: 365 vs 408 ms for v4).  Compact parking falls back to 15 words where its packed counters
    // would overflow.
    std::shared_ptr<AutoChoice> trial;  // this frame is timed for the automatic choice: events ev[trial_slot..+1]
    int trial_slot = 0;
    const bool automatic = variant < 0 || variant >= kNumVariants;
    // small scenes: the flat kernel takes v3's place (in the trial below 64 spp as well).  (Until round 5 also scenes of
    // up to kFlatMaxPrims primitives whose rectangles touch others, where only the flat kernels were exact; the BVH
    // kernels now replay the reference traversal where it could differ, bvh_clear, and are faster beyond 16.)
    const bool flat_ok = S.prims_flat && S.num_prims <= (uint32_t)g_flat_max;
    const int tile_kernel = flat_ok ? kVarFlat : kVarV3Compact;
    const int persistent_kernel = flat_ok ? kVarFlatPersistent : kVarV4;
    if (automatic) {
        variant = a->samples_per_pixel < 32 ? persistent_kernel : tile_kernel;
        if (a->samples_per_pixel > 0 && a->samples_per_pixel < kAutoSpp && a->max_depth > 0) {
            int device = 0;
            (void)hipGetDevice(&device);
            const AutoKey key{device, stream, scene, a->width, T.local_rows, a->samples_per_pixel, a->max_depth,
                              philox ? 1u : 0u, flat_ok ? 1u : 0u};
            std::lock_guard<std::mutex> lock(g_auto_mu);
            auto it = g_auto.find(key);
            if (it == g_auto.end()) {
                if (g_auto.size() >= 64) g_auto.clear();
                it = g_auto.emplace(key, std::make_shared<AutoChoice>()).first;
            }
            const std::shared_ptr<AutoChoice> held = it->second;
            AutoChoice& ac = *held;
            if (ac.chosen >= 0) {
                variant = ac.chosen;
            } else if (ac.stage < 3) {
                variant = ac.stage < 2 ? tile_kernel : persistent_kernel;
                if (ac.stage >= 1) {
                    trial_slot = ac.stage == 1 ? 0 : 2;
                    if ((ac.ev[trial_slot] || hipEventCreate(&ac.ev[trial_slot]) == hipSuccess) &&
                        (ac.ev[trial_slot + 1] || hipEventCreate(&ac.ev[trial_slot + 1]) == hipSuccess))
                        trial = held;
                }
                ac.stage++;
            } else if (ac.ev[1] && ac.ev[3] && hipEventQuery(ac.ev[1]) == hipSuccess &&
                       hipEventQuery(ac.ev[3]) == hipSuccess) {
                float t3 = -1.0f, t4 = -1.0f;
                (void)hipEventElapsedTime(&t3, ac.ev[0], ac.ev[1]);
                (void)hipEventElapsedTime(&t4, ac.ev[2], ac.ev[3]);
                ac.chosen = (t3 >= 0.0f && t4 >= 0.0f && t4 < t3) ? persistent_kernel : tile_kernel;
                variant = ac.chosen;
            } else if (!ac.ev[1] || !ac.ev[3]) {
                ac.chosen = variant;  // no events: keep the static rule
            }
            (void)hipGetLastError();  // (hipEventQuery reports hipErrorNotReady while pending)
        }
    }
    const bool packable =
        a->samples_per_pixel < 8192u && a->max_depth < 64u && (uint64_t)a->samples_per_pixel * a->max_depth < 8192u;
    if (variant == kVarFlat && !S.prims_flat) variant = kVarV3Compact;  // (a scene beyond kFlatMaxPrims)
    // the persistent flat kernel stages the flat tables in LDS: a scene whose materials overflow kFlatTabLdsMax runs v4
    const size_t flat_tab_bytes = ((size_t)4 * S.num_prims + (size_t)3 * S.num_mats + S.num_imgs) * 16u;
    if (variant == kVarFlatPersistent && (!S.prims_flat || flat_tab_bytes > kFlatTabLdsMax)) variant = kVarV4;
    if (kVariants[variant].compact && !packable) variant = kVarV3;  // packed counters would overflow
    if ((kVariants[variant].kernel == 4 || kVariants[variant].kernel == 6) && (a->samples_per_pixel == 0 || a->max_depth == 0))
        variant = kVariants[variant].kernel == 6 ? kVarFlat  // the persistent kernels assume every pixel traces a ray
                                                 : (packable ? kVarV3Compact : kVarV3);
    if (philox && kVariants[variant].stack != dev::STACK_LDS16 && kVariants[variant].stack != dev::STACK_NONE)
        variant = packable ? kVarV3Compact : kVarV3;  // the v1/v2 kernels have no Philox build
    // Scenes whose references need 32 bits (S.wide_refs: >= 32767 nodes or >= 8192 primitives) run the WIDE builds
    // of the compact v3 and of v4; the 15-word v3 has none: v2 / v1 there (no Philox build either).
    bool wide = false;
    if (kVariants[variant].stack == dev::STACK_LDS16 && S.wide_refs) {
        if (variant == kVarV3) {
            if (philox) {
                set_error("rt_render: RT_FLAG_RNG_PHILOX on a scene with 32-bit references needs spp < 8192, "
                          "max_depth < 64 and spp * max_depth < 8192");
                return RT_ERR_UNSUPPORTED;
            }
            variant = S.depth <= 25u ? kVarV2 : kVarV1;  // 32-bit LDS stacks, or scratch if deep
        } else {
            wide = true;
        }
    }
    const Variant& V = kVariants[variant];
    const bool persistent = V.kernel == 4 || V.kernel == 6;
    // near-first traversal holds at most one deferred child per level below the root
    if (V.stack == dev::STACK_LDS && S.depth > (uint32_t)V.lds_depth + 1) {
        set_error("rt_render: BVH too deep for the LDS stack of kernel variant " + std::to_string(variant));
        return RT_ERR_UNSUPPORTED;
    }
    // v3/v4: per wave, the parked path state + a 16-bit stack of depth + 2 entries: two sentinel pads, and
    // a visit at level L (root = 1) holds at most L - 1 deferred children, so its unconditional write of
    // the far child lands at index 2 + (L - 1) <= depth + 1 (the 128-B saving keeps config 2's wave
    // inside 10 × 512 B of LDS)
    const int group_mode = V.kernel == 6 ? g_persistent_group : 0;
    const size_t wave_bytes = V.stack == dev::STACK_LDS16
                                  ? (size_t)(persistent ? dev::PK_WORDS4 : dev::park_words(V.compact)) * 64 * 4 +
                                        (size_t)(S.depth + 2) * 64 * (wide ? 4 : 2) + (size_t)g_lds_pad
                                  : 0;
    P.lds_wave_words = (uint32_t)(wave_bytes / 4);
    // the persistent flat kernel's GROUP build: 16-wave workgroups (one per CU) whose share counter follows the tables
    const bool group = V.kernel == 6 && g_persistent_group != 0;
    const uint32_t block = group ? (uint32_t)g_group_waves * 64u : (uint32_t)V.block;
    // GROUP: the workgroups per CU the grid is sized for (kFlatPersistentWaves waves per SIMD, e.g. 1 of 16 waves)
    const int group_per_cu = std::max(1, kFlatPersistentWaves * 4 / std::max(1, g_group_waves));
    size_t lds_bytes = (V.stack == dev::STACK_LDS ? (size_t)V.lds_depth * V.block * 4 : 0) + wave_bytes +
                       (V.kernel == 6 ? flat_tab_bytes + (group ? 4u * (2u + dev::kGqWords) : 0u) : 0);  // (GROUP)
    if (lds_bytes > kLdsLimit) {
        set_error("rt_render: BVH too deep for the LDS stack of kernel variant " + std::to_string(variant));
        return RT_ERR_UNSUPPORTED;
    }
    KernelFn fn = pick(variant, count_tests, S.has_textures, philox, wide, g_wave_trace != nullptr);
    P.bvh_ref_nodes = (const float4*)S.bvh_ref_nodes;  // (the BVH kernels' exactness, bvh_clear)
    P.bvh_boxes = (const float4*)S.bvh_boxes;
    P.bvh_ref_pairs = (const float4*)S.bvh_ref_pairs;
    P.bvh_has_rects = S.has_rects ? 1u : 0u;
    P.prefetch_stop = (uint32_t)g_prefetch_stop;
    if (V.kernel == 5 || V.kernel == 6) {  // the flat kernels' tables: primitives in the reference's test order, its BVH
        P.prims = (const float4*)S.prims_flat;
        P.ref_nodes = (const float4*)S.ref_nodes;
        P.flat_ref_pairs = (const float4*)S.flat_ref_pairs;
        P.flat_boxes = (const float4*)S.flat_boxes;
        P.flat_runs[0] = S.flat_runs[0];
        P.flat_runs[1] = S.flat_runs[1];
    }
    const int rius_trips = V.kernel == 6 ? g_rius_trips_persistent : g_rius_trips;  // (the flat kernels')
    P.rius_cap = rius_trips > 0 ? (uint32_t)rius_trips : 0xffffffffu;
    const uint32_t tile = V.block == 64 ? 8u : 16u;  // v2/v3/v4: one 8×8 tile per wave
    P.tiles_x = (a->width + tile - 1) / tile;
    const uint32_t tiles = P.tiles_x * ((T.local_rows + tile - 1) / tile);
    hipStream_t s = (hipStream_t)stream;
    uint32_t grid = tiles;
    if (persistent) {
        int device = 0, cus = 0, per_cu = 0;
        int rc = hip_check(hipGetDevice(&device), "rt_render: hipGetDevice");
        if (rc == RT_OK) rc = acquire_queue(device, (uint32_t)g_queue_stride, &P.work_counter, &cus);
        if (rc == RT_OK)
            rc = hip_check(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)fn, block, lds_bytes),
                           "rt_render: occupancy query");
        if (rc != RT_OK) return rc;
        if (group && per_cu > group_per_cu) {
            // more groups would fit a CU by registers than the grid is sized for: claim enough of the CU's LDS that
            // the grid cannot put more on one CU and leave another short
            lds_bytes = std::max(lds_bytes, kLdsLimit / (size_t)(group_per_cu + 1) + 1024u);
            rc = hip_check(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes),
                           "rt_render: LDS size attribute");
            if (rc != RT_OK) return rc;
        }
        P.work_total = tiles * 64u;
        P.pixel_cost = g_pixel_cost_bytes >= (uint64_t)P.work_total ? g_pixel_cost : nullptr;
        P.work_chunk = (uint32_t)g_queue_chunk;
        P.queue_prefetch = (uint32_t)g_queue_prefetch;
        P.queue_min = (uint32_t)g_queue_min;
        P.queue_stride = (uint32_t)g_queue_stride / 4u;
        // GROUP: the groups' static shares cover the first tiles, the per-wave queue the last g_group_tail permille
        const uint32_t tail_tiles =
            group && group_mode == 1 ? (uint32_t)(((uint64_t)tiles * (uint32_t)g_group_tail + 999u) / 1000u) : tiles;
        P.group_chunk = (uint32_t)g_group_chunk;
        P.linger_ticks = group ? (uint32_t)g_group_linger_us * 100u : 0u;
        P.group_tiles = tiles - tail_tiles;
        P.queue_base = P.group_tiles * 64u;
        P.work_per_counter = (tail_tiles + dev::kQueueCounters - 1u) / dev::kQueueCounters * 64u;
        // the persistent flat kernel runs 4 waves per SIMD even where its registers allow 5-6: C5 0.294 vs 0.307 ms
        // (XORWOW), 0.300 vs 0.314 (Philox), 3 rounds on one box (profiles/r04f_ab_pflat_waves.txt)
        if (V.kernel == 6) per_cu = std::min(per_cu, group ? group_per_cu : std::max(1, kFlatPersistentWaves * 4 * 64 / (int)block));
        if (g_persistent_waves > 0) per_cu = std::max(1, g_persistent_waves * 4 * 64 / (int)block);
        const uint64_t resident = (uint64_t)(per_cu > 0 ? per_cu : 1) * (uint64_t)(cus > 0 ? cus : 1);
        if (group) grid = (tiles + block / 64u - 1u) / (block / 64u);  // (no more waves than tiles, as one-wave grids)
        grid = (uint32_t)(resident < grid ? resident : grid);
        // GROUP shares in golden-ratio order (RT_TUNE_GROUP_ORDER 1): share g holds tiles (j · A) mod S for j in
        // [g·K, g·K + K), A ≈ 0.618 S coprime with S — every share (and every XCD's) a spread sample of the frame, and
        // the tiles the groups render at one moment scattered over it, not one band or one comb of tile columns
        P.group_perm_a = P.group_perm_b = P.group_perm_k = 0u;
        const uint64_t S = P.group_tiles;
        if (group && g_group_order == 1 && S > 1u) {
            const uint64_t K = (S + grid - 1u) / grid;
            uint64_t A = (uint64_t)((double)S * 0.6180339887498949) | 1u;
            while (std::gcd(A, S) != 1u) A++;
            if ((uint64_t)(grid - 1u) * (S - 1u) + (K - 1u) * (S - 1u) < (1ull << 32)) {
                P.group_perm_a = (uint32_t)A;
                P.group_perm_b = (uint32_t)(K * A % S);
                P.group_perm_k = (uint32_t)K;
            }
        }
        P.queue_guide = g_queue_guide > 0 ? std::max(1u, grid / dev::kQueueCounters) * (uint32_t)g_queue_guide : 0u;
        // (no reset here: the slot is zero, the previous launch that used it left it so, queue_release — unless
        // RT_TUNE_QUEUE_RESET asks for the round-4 host memset)
        P.queue_host_reset = g_queue_host_reset ? 1u : 0u;
        if (g_queue_host_reset) {
            int rc2 = hip_check(hipMemsetAsync(P.work_counter, 0, (size_t)dev::kQueueSlotWords * P.queue_stride * 4u, s),
                                "rt_render: queue reset");
            if (rc2 != RT_OK) return rc2;
        }
    }
    P.num_tiles = tiles;
    std::shared_ptr<TilePlan> plan;
    if ((V.kernel == 3 || V.kernel == 5) && g_adaptive_order && !g_tile_order) {
        int device = 0;
        int rc = hip_check(hipGetDevice(&device), "rt_render: hipGetDevice");
        if (rc == RT_OK) rc = acquire_plan(PlanKey{device, (void*)s, P.tiles_x, tiles, V.kernel}, s, &plan);
        if (rc != RT_OK) return rc;
        P.tile_cost = plan->cost;
        P.tile_order = plan->valid.load() ? plan->order : nullptr;
    }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (g_timing) {
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0, s);
    }
    g_last_variant = variant;
    if (trial) (void)hipEventRecord(trial->ev[trial_slot], s);
    (void)hipGetLastError();
    hipLaunchKernelGGL(fn, dim3(grid), dim3(block), lds_bytes, s, P);
    int rc = hip_check(hipGetLastError(), "rt_render: kernel launch", RT_ERR_LAUNCH);
    // A persistent launch that did not run leaves its queue slot as it found it, but the slot is re-zeroed anyway, so
    // that the launch reusing it kQueueSlots launches later never finds exhausted heads (the slot is
    // otherwise clean only because the grid's last wave zeroes it in queue_release)
    if (rc != RT_OK && persistent)
        (void)hipMemsetAsync(P.work_counter, 0, (size_t)dev::kQueueSlotWords * P.queue_stride * 4u, s);
    if (trial) (void)hipEventRecord(trial->ev[trial_slot + 1], s);  // the render kernel alone (v4 has no plan step)
    if (rc == RT_OK && plan) {  // the next launch on this stream dispatches this frame's costliest tiles first
        hipLaunchKernelGGL(dev::plan_order_kernel, dim3(1), dim3(1024), 0, s, (const uint32_t*)plan->cost, plan->order,
                           tiles);
        rc = hip_check(hipGetLastError(), "rt_render: plan kernel launch", RT_ERR_LAUNCH);
        if (rc == RT_OK) plan->valid.store(true);
    }
    if (g_timing) {
        (void)hipEventRecord(e1, s);
        if (rc == RT_OK && hipEventSynchronize(e1) == hipSuccess) {
            float ms = -1.0f;
            (void)hipEventElapsedTime(&ms, e0, e1);
            g_last_ms = ms;
        } else {
            g_last_ms = -1.0f;
        }
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    }
    return rc;
}

uint64_t rt_soa_plane_words(uint32_t width, uint32_t local_rows) {
    return (((uint64_t)width + 7u) / 8u) * (((uint64_t)local_rows + 7u) / 8u) * 64u;
}

namespace {
int render_init(void* d_state, uint32_t width, const rt_tiling* tiling, uint64_t seed_base, rt_stream stream,
                uint32_t soa, const char* who) {  // soa: 0 = rt_curand_state, else the plane layout
    if (!tiling) { set_error(std::string(who) + ": NULL tiling"); return RT_ERR_INVALID_ARGUMENT; }
    if ((size_t)width * tiling->local_rows == 0) return RT_OK;  // nothing to seed
    if (!d_state) { set_error(std::string(who) + ": NULL state"); return RT_ERR_INVALID_ARGUMENT; }
    if (tiling->band_rows == 0 || tiling->num_ranks == 0 || tiling->rank >= tiling->num_ranks) {
        set_error(std::string(who) + ": invalid tiling");
        return RT_ERR_INVALID_ARGUMENT;
    }
    const size_t n = (size_t)width * tiling->local_rows;
    if (soa) {
        const uint64_t plane = rt_soa_plane_words(width, tiling->local_rows);
        if (plane > 0xffffffffull) {
            set_error(std::string(who) + ": needs < 2^32 pixels per rank");
            return RT_ERR_INVALID_ARGUMENT;
        }
        soa = (uint32_t)plane;  // the kernel's plane stride
    }
    (void)hipGetLastError();
    hipLaunchKernelGGL(dev::render_init_kernel, dim3((unsigned)((n + dev::kBlock - 1) / dev::kBlock)), dim3(dev::kBlock), 0,
                       (hipStream_t)stream, (uint32_t*)d_state, width, tiling->local_rows, tiling->band_rows,
                       tiling->num_ranks, tiling->rank, (unsigned long long)seed_base, soa);
    return hip_check(hipGetLastError(), (std::string(who) + ": kernel launch").c_str(), RT_ERR_LAUNCH);
}
}  // namespace

int rt_render_init(rt_curand_state* d_state, uint32_t width, uint32_t height, const rt_tiling* tiling,
                   uint64_t seed_base, rt_stream stream) {
    (void)height;
    return render_init(d_state, width, tiling, seed_base, stream, 0u, "rt_render_init");
}

int rt_render_init_soa(uint32_t* d_planes, uint32_t width, uint32_t height, const rt_tiling* tiling,
                       uint64_t seed_base, rt_stream stream) {
    (void)height;
    return render_init(d_planes, width, tiling, seed_base, stream, 1u, "rt_render_init_soa");
}

// ----- reference-named drop-in launchers (synchronous, void) ----------------------------------------

void LaunchRenderInit(rt_dim3 grid, rt_dim3 block, unsigned int window_width, unsigned int window_height,
                      rt_curand_state* d_rand_state) {
    (void)hipGetLastError();
    hipLaunchKernelGGL(dev::render_init_grid_kernel, dim3(grid.x, grid.y, grid.z), dim3(block.x, block.y, block.z), 0, 0,
                       (uint32_t*)d_rand_state, window_width, window_height);
    if (hip_check(hipGetLastError(), "LaunchRenderInit: kernel launch", RT_ERR_LAUNCH) == RT_OK)
        hip_check(hipDeviceSynchronize(), "LaunchRenderInit: hipDeviceSynchronize");
}

void LaunchRandInit(rt_curand_state* d_rand_state2) {
    (void)hipGetLastError();
    hipLaunchKernelGGL(dev::rand_init_kernel, dim3(1), dim3(1), 0, 0, (uint32_t*)d_rand_state2);
    if (hip_check(hipGetLastError(), "LaunchRandInit: kernel launch", RT_ERR_LAUNCH) == RT_OK)
        hip_check(hipDeviceSynchronize(), "LaunchRandInit: hipDeviceSynchronize");
}

int rt_set_launch_flags(uint32_t flags) {
    if (flags & ~kLaunchFlagsAllowed) {
        set_error("rt_set_launch_flags: only RT_FLAG_RIUS_LEFT_TO_RIGHT may be set");
        return RT_ERR_INVALID_ARGUMENT;
    }
    std::call_once(g_launch_env_once, [] {});  // (an explicit setting wins over the environment)
    return (int)g_launch_flags.exchange(flags);
}

void LaunchKernel(unsigned int* pos, unsigned int image_width, unsigned int image_height,
                  const unsigned int samples_per_pixel, const unsigned int max_depth, const void* world,
                  rt_curand_state* d_rand_state, rt_input_struct inputs) {
    std::call_once(g_launch_env_once, [] {
        const char* e = std::getenv("RT_LAUNCH_RANDOM_FILL");
        if (e && std::strcmp(e, "ltr") == 0) g_launch_flags.store(RT_FLAG_RIUS_LEFT_TO_RIGHT);
    });
    // The viewer mutates the graph in place between frames: the cache re-flattens it on
    // every call and updates the device scene by what changed (reference_scene_for_launch, api.cpp).
    std::shared_ptr<rt_scene> cached;  // held until the frame is done (another thread may evict the entry)
    double host_ms = 0.0;
    const int rc = reference_scene_for_launch(world, &cached, &host_ms);
    g_last_host_ms = (float)host_ms;
    if (rc != RT_OK) return;
    rt_render_args a;
    std::memset(&a, 0, sizeof(a));
    a.pos = pos;
    a.state = d_rand_state;
    a.width = image_width;
    a.height = image_height;
    a.samples_per_pixel = samples_per_pixel;
    a.max_depth = max_depth;
    a.flags = RT_FLAG_FAITHFUL_GRID | g_launch_flags.load();
    a.tiling.band_rows = image_height ? image_height : 1;
    a.tiling.num_ranks = 1;
    a.tiling.rank = 0;
    a.tiling.local_rows = image_height;
    a.inputs = inputs;
    if (rt_render(cached.get(), &a, nullptr) != RT_OK) return;
    hip_check(hipDeviceSynchronize(), "LaunchKernel: hipDeviceSynchronize");  // Kernel.cu:190
}

}  // extern "C"
