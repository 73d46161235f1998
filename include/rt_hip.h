/*
 * rt_hip.h — C ABI of librt_hip.so, the MI355X (gfx950) per-pixel path-tracing kernel.
 *
 * This header is the drop-in boundary for the hot path of Trippasch/CudaRayTracer.  The reference binds
 * its render kernel through three extern "C" launchers compiled in CudaRayTracer/src/Cuda/Kernel.cu:178-204
 * and declared by the caller in CudaRayTracer/src/Cuda/CudaLayer.cpp:12-19.  Every entry point below names
 * the reference interface it replaces.  Only plain C types cross the boundary (no torch / HIP C++ types);
 * `rt_stream` is an opaque hipStream_t (NULL = the legacy default stream).
 *
 * Conventions:
 *   - rt_* functions return 0 on success or a negative rt_status; they never exit the process.
 *     The message of the last failure on the calling thread is available from rt_last_error().
 *   - The caller owns framebuffers and RNG-state buffers (device pointers).  The library owns the
 *     device-side scene tables behind an rt_scene handle.
 *   - rt_* launches are asynchronous on the given stream; the reference-named launchers are synchronous
 *     (they end in a device synchronize, as Kernel.cu:190/196/203 do).
 */
#ifndef RT_HIP_H
#define RT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------------------------------ */
/* Status codes                                                                                     */
/* ------------------------------------------------------------------------------------------------ */
typedef enum rt_status {
    RT_OK = 0,
    RT_ERR_INVALID_ARGUMENT = -1,
    RT_ERR_INVALID_SCENE = -2,
    RT_ERR_OUT_OF_MEMORY = -3,
    RT_ERR_DEVICE = -4,        /* a HIP runtime call failed (message holds hipGetErrorString) */
    RT_ERR_LAUNCH = -5,        /* hipGetLastError() after a kernel launch was not hipSuccess */
    RT_ERR_UNSUPPORTED = -6
} rt_status;

/* ------------------------------------------------------------------------------------------------ */
/* Scene data model (flat).  Mirrors the reference's pointer graph:                                 */
/*   Hittable{type,isActive,Object->{Sphere|XYRect|XZRect|YZRect}}   Hittables/Hittable.cuh:30-294   */
/*   Material{type,Object->{Lambertian|Metal|Dielectric|DiffuseLight}} Hittables/Material.cuh:6-177 */
/*   Texture{type,Object->{Constant|Checker|Image}}                    Hittables/Texture.cuh:6-109   */
/* ------------------------------------------------------------------------------------------------ */
typedef enum rt_hittable_type { /* HittableType, Hittable.cuh:30-38 (same numeric values) */
    RT_SPHERE = 0,
    RT_XYRECT = 1,
    RT_XZRECT = 2,
    RT_YZRECT = 3
} rt_hittable_type;

typedef enum rt_material_type { /* MaterialType, Material.cuh:6-12 */
    RT_LAMBERTIAN = 0,
    RT_METAL = 1,
    RT_DIELECTRIC = 2,
    RT_DIFFUSELIGHT = 3
} rt_material_type;

typedef enum rt_texture_type { /* TextureType, Texture.cuh:6-10 */
    RT_CONSTANT = 0,
    RT_CHECKER = 1,
    RT_IMAGE = 2
} rt_texture_type;

typedef struct rt_texture_desc {
    int32_t type;      /* rt_texture_type */
    int32_t image;     /* RT_IMAGE: index into rt_scene_desc.images, or -1 for "no data" (Texture.cuh:83-84) */
    float color[3];    /* RT_CONSTANT: Constant::color; RT_CHECKER: odd colour (Texture.cuh:58-67) */
    float color2[3];   /* RT_CHECKER: even colour */
} rt_texture_desc;     /* 32 B */

typedef struct rt_material_desc {
    int32_t type;            /* rt_material_type */
    float fuzz;              /* RT_METAL: Metal::fuzz as the kernel reads it (ctor clamp Material.cuh:71 is the caller's) */
    float ir;                /* RT_DIELECTRIC: Dielectric::ir */
    int32_t light_intensity; /* RT_DIFFUSELIGHT: DiffuseLight::light_intensity (an int, Material.cuh:152) */
    rt_texture_desc albedo;  /* Lambertian/Metal/DiffuseLight albedo texture */
} rt_material_desc;          /* 48 B */

typedef struct rt_hittable_desc {
    int32_t type;      /* rt_hittable_type */
    int32_t is_active; /* Hittable::isActive — inactive entries are dropped (Hittable.cuh:311-312) */
    float center[3];   /* Sphere::center / *Rect::center */
    float radius;      /* RT_SPHERE; >= 0 (the reference editor's range, CudaLayer.cpp:496), else RT_ERR_INVALID_SCENE */
    float width;       /* rects: XY width along x, XZ width along x, YZ width along z (Hittable.cuh:255-258) */
    float height;      /* rects: XY height along y, XZ height along z, YZ height along y */
    int32_t material;  /* index into rt_scene_desc.materials */
    int32_t reserved;
} rt_hittable_desc;    /* 40 B */

typedef struct rt_image_desc {
    const uint8_t* data; /* host pointer, RGB8, 3 bytes per texel, row-major (Texture.cuh:76, RawStbImage.h:13) */
    int32_t width;
    int32_t height;
} rt_image_desc;

typedef struct rt_scene_desc {
    const rt_hittable_desc* hittables; /* in list order (m_List, CudaLayer.cpp:131) */
    uint32_t num_hittables;
    const rt_material_desc* materials;
    uint32_t num_materials;
    const rt_image_desc* images;
    uint32_t num_images;
} rt_scene_desc;

/* InputStruct (Utils/SharedStructs.h:3-24): 18 floats, 72 B, same layout. */
typedef struct rt_input_struct {
    float origin[3];
    float orientation[3];
    float up[3];
    float far_plane;
    float near_plane;
    float fov; /* radians (CudaLayer.cpp:62) */
    float background_start[3];
    float background_end[3];
} rt_input_struct;

/* curandStateXORWOW layout (48 B).  The caller allocates W·H of these exactly as CudaLayer.cpp:72 does
 * (cudaMalloc(W·H·sizeof(curandState))); only d and v[5] are read or written by the kernel. */
typedef struct rt_curand_state {
    uint32_t d;
    uint32_t v[5];
    int32_t boxmuller_flag;
    int32_t boxmuller_flag_double;
    float boxmuller_extra;
    uint32_t pad_;
    double boxmuller_extra_double;
} rt_curand_state;

typedef struct rt_dim3 { /* binary-compatible with HIP/CUDA dim3 passed by value */
    uint32_t x, y, z;
} rt_dim3;

typedef struct rt_scene rt_scene; /* opaque: device-resident flat scene (BVH + primitive + material tables) */
typedef void* rt_stream;          /* hipStream_t */

/* ------------------------------------------------------------------------------------------------ */
/* Reference-named drop-in launchers (same names, argument meaning, synchronous, void return).      */
/* ------------------------------------------------------------------------------------------------ */

/* Replaces `extern "C" void LaunchKernel(unsigned int* pos, unsigned int image_width, unsigned int
 * image_height, const unsigned int samples_per_pixel, const unsigned int max_depth, Hittable* world,
 * curandState* d_rand_state, InputStruct inputs)` — Kernel.cu:178-191.
 * `world` is the reference's Hittable* scene graph (see rt_reference_graph.h); it is re-flattened on
 * every call because the viewer mutates it in place and the device scene cached per
 * (device, world) is updated by what changed: materials in place, geometry by a BVH rebuild, images only
 * when an image's data pointer, width or height changes (the reference re-allocates texture data to change
 * it, CudaLayer.cpp:889-903; texel bytes are never re-read per frame).  Floor-division grid as in
 * Kernel.cu:184: pixels outside the last whole 16×16 block are not written.  Errors: rt_last_error(). */
void LaunchKernel(unsigned int* pos, unsigned int image_width, unsigned int image_height,
                  const unsigned int samples_per_pixel, const unsigned int max_depth, const void* world,
                  rt_curand_state* d_rand_state, rt_input_struct inputs);

/* Flags LaunchKernel adds to its own (RT_FLAG_FAITHFUL_GRID), process-wide: RT_FLAG_RIUS_LEFT_TO_RIGHT selects the
 * left-to-right fill of Random()'s Vec3(ξ, ξ, ξ) (Utils/Math.cuh:231-234; default right to left)
 * for a viewer whose CUDA build filled it that way.  Any other bit is rejected (RT_ERR_INVALID_ARGUMENT).  Returns the
 * previous flags.  Without a call, the environment variable RT_LAUNCH_RANDOM_FILL=ltr sets the same flag when
 * LaunchKernel first runs. */
int rt_set_launch_flags(uint32_t flags);

/* Replaces `extern "C" void LaunchRandInit(curandState* d_rand_state2)` — Kernel.cu:193-197
 * (curand_init(1984, 0, 0) of one state). */
void LaunchRandInit(rt_curand_state* d_rand_state2);

/* Replaces `extern "C" void LaunchRenderInit(dim3 grid, dim3 block, unsigned int window_width,
 * unsigned int window_height, curandState* d_rand_state)` — Kernel.cu:199-204: curand_init(1984 +
 * pixel_index, 0, 0) for every thread (i, j) = threadIdx + blockIdx·blockDim of the given grid. */
void LaunchRenderInit(rt_dim3 grid, rt_dim3 block, unsigned int window_width, unsigned int window_height,
                      rt_curand_state* d_rand_state);

/* ------------------------------------------------------------------------------------------------ */
/* Native API                                                                                       */
/* ------------------------------------------------------------------------------------------------ */

/* Last error message of the calling thread ("" if none). */
const char* rt_last_error(void);

/* Library version string. */
const char* rt_version(void);

/* Version of this C ABI (structure layouts, counter words, entry points); a caller built against an older header
 * can refuse a newer library.  6: RT_COUNTERS_WORDS (24) counter words with RT_FLAG_COUNT_TESTS, rt_set_launch_flags. */
#define RT_ABI_VERSION 6
int rt_abi_version(void);

/* hipSetDevice on the calling thread. */
int rt_set_device(int device);

/* Upload a flat scene: validates, drops inactive hittables, builds a binned-SAH BVH on the host and
 * copies the tables to the current device.  Replaces the managed-memory pointer graph of
 * CudaLayer::GenerateWorld (CudaLayer.cpp:103-256) + BVHNode ctor (Hittable.cuh:303-385). */
int rt_scene_create(const rt_scene_desc* desc, rt_scene** out_scene);

/* Re-read the scene from the reference's Hittable* graph (host-visible memory) — see
 * rt_reference_graph.h — into a new rt_scene. */
int rt_scene_from_reference_graph(const void* world, rt_scene** out_scene);

/* Replace materials/textures in place (no BVH rebuild), like the viewer's material edits
 * (CudaLayer.cpp:719-872).  num_materials must equal the scene's material count. */
int rt_scene_update_materials(rt_scene* scene, const rt_material_desc* materials, uint32_t num_materials);

int rt_scene_destroy(rt_scene* scene);

typedef struct rt_scene_info {
    uint32_t num_primitives; /* active hittables */
    uint32_t num_nodes;      /* BVH nodes */
    uint32_t num_materials;
    uint32_t bvh_depth;
    uint64_t device_bytes;   /* bytes of device tables */
} rt_scene_info;
int rt_scene_get_info(const rt_scene* scene, rt_scene_info* info);

/* Row mapping of a (possibly tiled) render.  Local row l of the caller's buffers is global image row
 *   g = ((l / band_rows) * num_ranks + rank) * band_rows + (l % band_rows)
 * (block-cyclic row bands).  {band_rows = H, num_ranks = 1, rank = 0} is the whole
 * image.  Pixel index for RNG seeding and the camera is always the GLOBAL g·W + x (Kernel.cu:119,175). */
typedef struct rt_tiling {
    uint32_t band_rows;
    uint32_t num_ranks;
    uint32_t rank;
    uint32_t local_rows; /* rows held by the local buffers */
} rt_tiling;

/* curand_init(seed_base + global_pixel_index, 0, 0) for every local pixel (Kernel.cu:166-176). */
int rt_render_init(rt_curand_state* d_state, uint32_t width, uint32_t height, const rt_tiling* tiling,
                   uint64_t seed_base, rt_stream stream);
/* The same states in the native plane layout of RT_FLAG_STATE_SOA: six uint32 planes (d, v[0..4]) of
 * rt_soa_plane_words(width, local_rows) words each; a plane holds the pixels 8×8 tile by tile (tile
 * t = (row / 8) · ceil(width / 8) + column / 8 at word t·64 + 8·(row % 8) + column % 8), so the wave that
 * renders a tile moves 256 contiguous bytes per plane: 24 bytes per pixel, no partial cache lines. */
uint64_t rt_soa_plane_words(uint32_t width, uint32_t local_rows);
int rt_render_init_soa(uint32_t* d_planes, uint32_t width, uint32_t height, const rt_tiling* tiling,
                       uint64_t seed_base, rt_stream stream);

#define RT_COUNTERS_WORDS 24u /* rt_render_args.counters length with RT_FLAG_COUNT_TESTS (16 without) */
#define RT_PHILOX_MAX_SPP 16384u /* RT_FLAG_RNG_PHILOX: samples per pixel (2^14 windows of 2^18 words) */

enum rt_render_flags {
    RT_FLAG_FAITHFUL_GRID = 1u << 0, /* skip pixels outside whole 16×16 blocks (Kernel.cu:184) */
    RT_FLAG_NO_STATE_WRITEBACK = 1u << 1, /* do not store the advanced RNG state (benchmark repeatability) */
    RT_FLAG_ACCUMULATE = 1u << 2, /* accum[px].rgb += Σ samples, accum[px].w += spp; pos shows rgb / w */
    RT_FLAG_RIUS_LEFT_TO_RIGHT = 1u << 3, /* fill Random()'s Vec3(ξ,ξ,ξ) left to right (default: right to
                                             left, the order the survey's g++ build of Math.cuh:233 used — the
                                             only build of the reference available here; C++ leaves the order
                                             unspecified and nvcc's is not established).
                                             Both orders are tested against the oracle on every config. */
    RT_FLAG_COUNT_TESTS = 1u << 4, /* also count box, primitive and rectangle tests into counters[1], [2], [16]
                                      (counters must then hold RT_COUNTERS_WORDS words) */
    RT_FLAG_RNG_PHILOX = 1u << 5,  /* perf-mode RNG: sample s of a pixel draws from the hipRAND/rocRAND
                                      Philox4x32-10 stream rocrand_init(rng_seed, subsequence = global pixel
                                      index, offset = (rng_frame << 34) + (s << 18)), read as rocrand_uniform4
                                      blocks in draw groups that start on a block boundary (the camera jitter,
                                      the dielectric's choice, a whole RandomInUnitSphere call), instead of its
                                      cuRAND XORWOW state; the pixel's samples are summed in 2^-12 fixed point
                                      (each sample's channel rounded to the nearest multiple of 2^-12, the sum
                                      saturating at 2^20), so neither the draws nor the sum depend on the order
                                      the samples run in — the kernels hand a tile's samples to whichever lane
                                      is free.  `state` is neither read nor written (may be NULL): no per-pixel
                                      RNG bytes in HBM.  Not the reference's stream (its images match the parity
                                      mode statistically, not bit for bit).  Limits: spp <= RT_PHILOX_MAX_SPP
                                      (each sample's window is 2^18 words; larger spp is rejected); a sample's
                                      channel below 2^-13 (and any negative or NaN value) rounds to 0, so a
                                      very dim image loses up to 2^-13 per sample and channel against the
                                      parity mode's float sum (tests/test_oracle.py::test_philox_mode_dim_scene_bias_is_bounded). */
    RT_FLAG_ACCUMULATE_RESET = 1u << 7, /* with RT_FLAG_ACCUMULATE: the accumulation restarts with this frame
                                            (a camera move or scene edit): accum is written, never read — the
                                            same bits as zeroing it first (0 + x rounds as the kernel adds),
                                            without the fill kernel and the read of zeros */
    RT_FLAG_STATE_SOA = 1u << 6    /* `state` holds the XORWOW states as six uint32 planes (rt_render_init_soa)
                                      instead of rt_curand_state structs: the same streams and images, 24 B
                                      per pixel read and written with coalesced 4-B accesses (the 48-B
                                      struct moves whole cache lines for its 24 used bytes) */
};

typedef struct rt_render_args {
    uint32_t* pos;            /* device RGBA8 framebuffer, local_rows × width (may be NULL if accum given) */
    float* radiance;          /* optional device float[local_rows·width·4]: pre-gamma mean colour (col/spp) */
    float* accum;             /* RT_FLAG_ACCUMULATE: device float4 running sum of samples */
    rt_curand_state* state;   /* device RNG states, local_rows × width (RT_FLAG_STATE_SOA: the six planes) */
    uint64_t* counters;       /* optional device uint64[RT_COUNTERS_WORDS] with RT_FLAG_COUNT_TESTS (the
                                 kernels then write up to word 17; ABI versions < 6 wrote 16 words: see
                                 rt_abi_version), else uint64[16]: rays, box tests, primitive tests, primary samples;
                                 with RT_FLAG_COUNT_TESTS
                                 also [4..6] = wave-level iterations of node visits,
                                 primitive tests and shading (SIMD-efficiency diagnostics) and, for the v3
                                 kernels, [7..10] = wave clock cycles spent tracing, shading, in total and
                                 in leaves, [11..12] = node / primitive wave-iterations whose active lanes
                                 all test the same node / primitive, [13..15] = idle lanes per node iteration
                                 (pixel done, ray finished, holding a leaf), [16] = rectangle tests (the
                                 part of [2] that are XY/XZ/YZRect::Hit; the FLOP model prices them apart),
                                 [17] = rays whose closest hit the exactness check replayed through the
                                 reference BVH (render.hip bvh_clear / flat_trace) */
    uint32_t width;
    uint32_t height;          /* global image height */
    uint32_t samples_per_pixel;
    uint32_t max_depth;
    uint32_t flags;           /* rt_render_flags */
    uint32_t reserved;        /* must be 0 */
    rt_tiling tiling;
    rt_input_struct inputs;
    uint64_t rng_seed;        /* RT_FLAG_RNG_PHILOX: Philox key (e.g. 1984, the reference's seed base) */
    uint32_t rng_frame;       /* RT_FLAG_RNG_PHILOX: frame counter; each frame draws fresh numbers */
    uint32_t reserved2;       /* must be 0 */
} rt_render_args;

/* One frame of the per-pixel render kernel (Kernel.cu:102-158) on `stream`, asynchronous.  At most 256
 * frames may be in flight per device at once (the persistent kernel's work-queue slots are reused after
 * 256 launches); synchronise at least that often when queueing frames on several streams. */
int rt_render(const rt_scene* scene, const rt_render_args* args, rt_stream stream);

/* Kernel duration of the last rt_render on this thread measured with HIP events on its stream
 * (milliseconds); requires rt_set_timing(1) before the launch.  Returns <0 when unavailable. */
int rt_set_timing(int enabled);
float rt_last_kernel_ms(void);

/* Host milliseconds of the last LaunchKernel's scene step on this thread (graph flatten + change detection +
 * any device update); < 0 before the first call. */
float rt_last_launch_host_ms(void);

/* Diagnostic (per thread): device buffer of `words` uint64 that later launches fill with s_memrealtime stamps
 * (100 MHz): v3 and flat, 2 per 8×8 tile (its wave's start and end; tools/wave_timeline.py); v4 and persistent flat,
 * 8 per persistent wave (start, the moment its work queue ran dry, end, pixels taken, HW_REG_HW_ID | XCC id << 32,
 * when it last handed out a pixel, chunk grabs | exhausted-head probes << 32, ticks spent waiting for queue atomics;
 * tools/v4_timeline.py).  Stamps that would fall beyond `words` are not written.  NULL = off.  The persistent kernels
 * run a separate trace build while a buffer is set (the product build carries no stamps); RT_FLAG_COUNT_TESTS
 * launches of them run the counting build, which writes no per-wave records. */
int rt_set_wave_trace(void* buffer, uint64_t words);

/* Experiment (per thread): device uint32 permutation of the frame's 8×8 tiles giving the v3 kernels' launch
 * order, and the order the persistent kernels' work queue hands tiles out in (NULL = row-major).  Results do not
 * depend on it (every pixel is independent); the time does. */
int rt_set_tile_order(const void* order);

/* Diagnostic (per thread): device buffer of `bytes` uint8 that later persistent-flat launches fill, per work index
 * (tile slot · 64 + pixel of the 8×8 tile), with the loop passes the pixel took (clamped at 255) — the cost
 * measure a cost-ordered queue plans from.  Ignored when smaller than the frame's work indices.  NULL = off. */
int rt_set_pixel_cost(void* buffer, uint64_t bytes);

/* Diagnostic (per thread): later rt_render calls with RT_FLAG_COUNT_TESTS on the v3 kernels (variants 2, 3) append
 * every ray that starts at bounce `depth` (1 = the first scattered ray; 0 is not recorded) to `rays` as (origin, 0),
 * (direction, 0) float4 pairs, up to `capacity` rays; *count (device uint32, caller-zeroed) counts the rays offered,
 * so min(*count, capacity) were written.  rays = NULL: off.  (tools/coherence.py) */
int rt_set_ray_dump(void* rays, uint32_t capacity, uint32_t* count, uint32_t depth);

/* Closest hit of n rays (device (origin, -), (direction, -) float4 pairs) against the scene, with v3's traversal
 * (BVHNode::Hit semantics, Hittable.cuh:387-439; t in (0.001, FLT_MAX)): hits[2i] = the primitive's index in the
 * scene's BVH order or -1, hits[2i + 1] = the hit distance's bits.  counters: optional device uint64[RT_COUNTERS_WORDS]
 * ([0] rays; with count_tests also box and primitive tests and wave iterations, as rt_render).  Asynchronous on
 * `stream`.  Scenes with 32-bit references are not supported (RT_ERR_UNSUPPORTED). */
int rt_trace_rays(const rt_scene* scene, const float* rays, uint32_t n, int32_t* hits, uint64_t* counters,
                  int count_tests, rt_stream stream);

/* Tuning/benchmark knob (per thread): the kernel rt_render launches.  -1 = automatic: 3 from 64 spp; below,
 * the faster of 3 and 4 as timed on the first frames of each (device, stream, scene, frame shape, spp, depth,
 * RNG mode) — both render identical bits — with fallbacks where a kernel's limits are exceeded; 0 = v1
 * (scratch stack, any scene), 1 = v2 (resumable, 32-bit LDS stacks), 2 = v3 (resumable, path state parked in
 * LDS, 16-bit stacks, longest-first tile order), 3 = v3 with compact parking, 4 = v4 (v3 made persistent with
 * a pixel work queue), 5 = flat (no BVH; scenes of at most 64 primitives, else 3), 6 = flat in the persistent grid
 * of 4 (else 4).  Returns the previous value. */
int rt_set_variant(int variant);
/* The variant the last rt_render on this thread launched (-1 before any). */
int rt_last_variant(void);

/* Tuning knob (per thread); returns the previous value or a negative rt_status.
 *   RT_TUNE_REGEN_THRESHOLD: resumable kernels leave traversal to shade/regenerate finished lanes when
 *   fewer than this many of a wave's 64 lanes are still tracing (1..64, default 56). */
/*   RT_TUNE_LEAF_MAX: maximum primitives per BVH leaf used by later rt_scene_create calls (1..4, default 4). */
/*   RT_TUNE_PERSISTENT_WAVES: waves per SIMD of the persistent kernels' grid (0 = default: the occupancy query,
 *   capped at 4 for the persistent flat kernel; 1..16). */
/*   RT_TUNE_SAH_TRAVERSAL: cost of a node visit relative to a primitive test in the SAH leaf decision, ×10
  *   (1..1000, default 16), used by later rt_scene_create calls. */
/*   RT_TUNE_LDS_PAD: diagnostic, extra LDS bytes per wave of the v3/v4 kernels (occupancy experiments; 0).
 *   RT_TUNE_ADAPTIVE_ORDER: 1 (default) = the v3 kernels dispatch a frame's tiles longest-first, ordered by
 *   the per-tile wave lifetimes the previous launch on the same stream with the same tile grid measured;
 *   0 = row-major.  The image does not depend on it. */
/*   RT_TUNE_TEXEL_LAYOUT: device bytes per texel of the images of later rt_scene_create calls: 3 (default,
 *   the reference's RGB8 layout, Texture.cuh:76) or 4 (RGBA8-padded, 4/3 the memory); the kernels gather one dword
 *   per lookup in either.  The image does not depend on it. */
/*   RT_TUNE_QUEUE_CHUNK: work indices (pixels) a persistent (v4) wave takes from its queue head per atomic
 *   (a multiple of 64 in [64, 4096], default 128; 64 near a head's end).  RT_TUNE_QUEUE_STRIDE: bytes between the v4 kernel's 16
 *   queue heads (a power of two in [128, 4096], default 128).  Neither changes the image.
 *   RT_TUNE_REGEN_LIVE_FRAC: the v3 kernels cap the regeneration threshold at this fraction (x/64) of the wave's
 *   pixels still rendering (0 = off; 0..64; default 48).  The image does not depend on it.
 *   RT_TUNE_LEAF_BREAK: the v3 kernels leave the node-visit loop for the leaf tests once at most this many of
 *   the still-traversing lanes hold no leaf (0..64, default 3; 0 = once every lane holds one).  Nor does this.
 *   RT_TUNE_FLAT_MAX: scenes of at most this many active primitives (0..64, default 16) run the flat kernels
 *   (variants 5 and 6: no BVH, every ray tests every primitive in the reference BVH's test order, and rays whose
 *   answer the reference's box culling could change replay the reference BVH: the reference's pixels for any
 *   geometry) where the automatic choice would run variant 3 or 4.  The BVH kernels (0-4) return the reference's
 *   answer too: their closest hit is the geometric one, which can differ from the reference traversal's only on
 *   exact ties, rays its own box test of the hit primitive rejects and rays with a zero or non-finite component, and
 *   those rays replay the reference BVH (render.hip bvh_clear).  RT_TUNE_RIUS_TRIPS: the tile
 *   flat kernel (variant 5) makes at most this many RandomInUnitSphere attempts (Math.cuh:252-260) per shading pass; a
 *   lane whose attempts were all rejected continues the same call at the wave's next pass (0 = unbounded; 0..64;
 *   default 4; Philox mode rounds it up to whole blocks of four attempts).  RT_TUNE_RIUS_TRIPS_PERSISTENT: the same for
 *   the persistent flat kernel (variant 6; default 0 = unbounded: C5 -3.5 %).  Neither changes the image.
 *   RT_TUNE_QUEUE_PREFETCH: the persistent kernels (variants 4, 6) fetch their next chunk of work indices (the queue
 *   atomic) ahead, once at most this many indices of the current chunk are left, so the atomic's round trip overlaps
 *   the wave's work (0 = off: fetched when the chunk runs out; 0..64; default 32: C5 -7 %,
 *   profiles/r05g_ab_c5_queue_prefetch.txt).  RT_TUNE_QUEUE_GUIDE: guided chunk sizes for
 *   the persistent kernels — a wave takes (its head's remaining indices) / (waves per head × this factor), rounded
 *   down to a multiple of 16, at least RT_TUNE_QUEUE_MIN_CHUNK (16..64) and at most RT_TUNE_QUEUE_CHUNK (0 = off:
 *   RT_TUNE_QUEUE_CHUNK while plenty is left, then 64; 0..64).  RT_TUNE_PREFETCH_STOP: the persistent flat kernel's lanes
 *   take their next pixel (and its RNG state) ahead while their wave's queue head holds more than 1/value of its
 *   range (default 8; 0 = never ahead; 0..1024).  RT_TUNE_PERSISTENT_GROUP: the persistent flat kernel runs 16-wave
 *   workgroups, one per CU, each handing a static interleaved share of the frame's tiles to its lanes through an LDS
 *   counter before its waves turn to the per-wave queue (1; round 6), or one-wave workgroups on the queue alone (0,
 *   round 5), or 16-wave workgroups drawing chunks of RT_TUNE_GROUP_CHUNK positions (64..4096, default 1024) from the
 *   queue heads themselves, one device atomic per chunk and group (2, default).  RT_TUNE_GROUP_TAIL: permille of the frame's tiles left to the per-wave queue behind the
 *   shares (0..1000, default 0).  RT_TUNE_GROUP_ORDER: the shares' tiles interleaved (0, default: tile g + k·groups) or in
 *   golden-ratio order (1: share g holds tiles (j · A) mod S, j in [g·K, g·K + K)).  None of these changes
 *   the image.  RT_TUNE_QUEUE_RESET: 1 = rt_render zeroes the persistent kernels' work-queue slot with a memset per
 *   launch; 0 (default) = the launch's last wave (GROUP: last workgroup) leaves it zeroed.  RT_TUNE_GROUP_LINGER_US: a
 *   workgroup of the persistent flat kernel that has finished its pixels stays resident, asleep, until every workgroup
 *   has (waves exiting while others render stall them), at most this long (0..100000; default 0 = exit at once: the
 *   groups' simultaneous exit then costs the kernel's end ~100 us, more than the stall it avoids).
 *   RT_TUNE_GROUP_WAVES: waves per workgroup of those builds (4, 8, 12 or 16, default 16; the grid keeps 4 waves per
 *   SIMD where the group size divides 16, else the one group per CU that fits). */
enum rt_tuning_key { RT_TUNE_REGEN_THRESHOLD = 0, RT_TUNE_LEAF_MAX = 1, RT_TUNE_PERSISTENT_WAVES = 2,
                     RT_TUNE_SAH_TRAVERSAL = 3, RT_TUNE_LDS_PAD = 4, RT_TUNE_ADAPTIVE_ORDER = 5,
                     RT_TUNE_TEXEL_LAYOUT = 6, RT_TUNE_QUEUE_CHUNK = 7, RT_TUNE_QUEUE_STRIDE = 8,
                     RT_TUNE_REGEN_LIVE_FRAC = 9, RT_TUNE_LEAF_BREAK = 10, RT_TUNE_RIUS_TRIPS = 11,
                     RT_TUNE_FLAT_MAX = 12, RT_TUNE_QUEUE_PREFETCH = 13, RT_TUNE_QUEUE_GUIDE = 14,
                     RT_TUNE_QUEUE_MIN_CHUNK = 15, RT_TUNE_RIUS_TRIPS_PERSISTENT = 16, RT_TUNE_PREFETCH_STOP = 17,
                     RT_TUNE_PERSISTENT_GROUP = 18, RT_TUNE_GROUP_TAIL = 19, RT_TUNE_GROUP_ORDER = 20,
                     RT_TUNE_QUEUE_RESET = 21, RT_TUNE_GROUP_CHUNK = 22,
                     RT_TUNE_GROUP_LINGER_US = 23, RT_TUNE_GROUP_WAVES = 24 };
int rt_set_tuning(int key, int value);

/* ------------------------------------------------------------------------------------------------ */
/* Multi-device image tiling in one process (the reference is single-device,    */
/* LaunchKernel at Kernel.cu:178-191).  Band rank r renders the block-cyclic row bands b ≡ r (mod N) */
/* on devices[r] (entries may repeat a device: one stream per rank), then copies its bands into     */
/* their rows of the caller's W·H framebuffer with one strided peer copy over xGMI: gather and      */
/* unshuffle in one transfer per rank.  The frame is bit-identical to a one-rank render (the RNG    */
/* streams are keyed by the global pixel index).                                                     */
/* ------------------------------------------------------------------------------------------------ */
typedef struct rt_tiled rt_tiled; /* opaque: per-rank device scene, stream, framebuffer band store, RNG states */

typedef struct rt_tiled_desc {
    const int* devices;  /* device ordinal of each band rank (copied) */
    uint32_t num_ranks;
    uint32_t band_rows;  /* rows per band (0 = 16) */
    uint32_t width, height;
    uint32_t flags;      /* RT_FLAG_RNG_PHILOX: stateless Philox streams, no per-rank RNG state */
    uint32_t reserved;   /* must be 0 */
    uint64_t seed;       /* XORWOW: curand_init(seed + global pixel index, 0, 0) (Kernel.cu:175; 1984); Philox key */
} rt_tiled_desc;

typedef struct rt_tiled_frame {
    uint32_t* pos;       /* device W·H RGBA8 framebuffer (row 0 = bottom) on any device: the gather target */
    uint32_t samples_per_pixel;
    uint32_t max_depth;
    uint32_t flags;      /* RT_FLAG_FAITHFUL_GRID / NO_STATE_WRITEBACK / COUNT_TESTS / RIUS_LEFT_TO_RIGHT */
    uint32_t rng_frame;  /* Philox frame counter when rng_frame_set != 0, else the object's own counter */
    uint32_t rng_frame_set;
    uint32_t reserved;   /* must be 0 */
    rt_input_struct inputs;
} rt_tiled_frame;

typedef struct rt_tiled_timing {
    float render_ms;     /* slowest rank's kernel time (HIP events on its stream) */
    float gather_ms;     /* slowest rank's gather copy (HIP events on its stream) */
    float total_ms;      /* host wall time of the call */
    uint32_t reserved;
    uint64_t rays;       /* closest-hit queries over all ranks */
} rt_tiled_timing;

/* Uploads `scene` to every distinct device, allocates each rank's band store and seeds its RNG states. */
int rt_tiled_create(const rt_tiled_desc* desc, const rt_scene_desc* scene, rt_tiled** out);
/* One frame over all ranks + the gather into frame->pos; synchronous (as LaunchKernel, Kernel.cu:190).
 * timing may be NULL. */
int rt_tiled_render(rt_tiled* tiled, const rt_tiled_frame* frame, rt_tiled_timing* timing);
int rt_tiled_destroy(rt_tiled* tiled);

/* ------------------------------------------------------------------------------------------------ */
/* Display and headless output of the RGBA8 framebuffer.                        */
/* ------------------------------------------------------------------------------------------------ */
typedef struct rt_gl_target rt_gl_target; /* opaque: a registered OpenGL texture */

/* Replaces cudaGraphicsGLRegisterImage(&res, texture, GL_TEXTURE_2D, cudaGraphicsRegisterFlagsWriteDiscard)
 * (CudaLayer.cpp:89-90).  Needs the caller's current GL context; gl_target is e.g. GL_TEXTURE_2D (0x0DE1). */
int rt_gl_register_texture(uint32_t gl_texture, uint32_t gl_target, rt_gl_target** out);
/* Replaces the per-frame map → mapped array → cudaMemcpy2DToArray(W·4 B × H rows, device to device) → unmap
 * (CudaLayer.cpp:379-386), on `stream`. */
int rt_gl_copy_image(rt_gl_target* target, const uint32_t* device_pos, uint32_t width, uint32_t height,
                     rt_stream stream);
int rt_gl_unregister(rt_gl_target* target);

/* Host-staging fallback when there is no GL interop: the device framebuffer into host memory (synchronous on
 * `stream`); flip_rows != 0 puts the image's top row first (buffer row 0 is the bottom, CudaLayer.cpp:402). */
int rt_copy_image_to_host(uint32_t* host, const uint32_t* device_pos, uint32_t width, uint32_t height, int flip_rows,
                          rt_stream stream);

/* Headless output: binary PPM (P6) of a host RGBA8 buffer; flip_rows != 0 writes buffer row H-1 first, so the
 * file shows the image upright (the reference's display flip, CudaLayer.cpp:402). */
int rt_write_ppm(const char* path, const uint32_t* rgba, uint32_t width, uint32_t height, int flip_rows);

/* Host-side helpers (no device needed). */

/* Flatten the reference's Hittable* graph (rt_reference_graph.h) into flat arrays (size query with NULL
 * arrays; counts are in/out).  This is the host step of rt_scene_from_reference_graph / LaunchKernel. */
int rt_reference_graph_flatten(const void* world, rt_hittable_desc* hittables, uint32_t* num_hittables,
                               rt_material_desc* materials, uint32_t* num_materials, rt_image_desc* images,
                               uint32_t* num_images);

/* Build the device tables on the host only and copy them out (for inspection/tests): nodes 16 floats,
 * prims 8 floats, materials 12 floats each; prim_source[i] = hittable index of primitive i.  Size query
 * with NULL arrays. */
typedef struct rt_host_tables_info {
    uint32_t num_nodes, num_prims, num_materials, depth;
} rt_host_tables_info;
int rt_build_host_tables(const rt_scene_desc* desc, float* nodes, float* prims, float* materials,
                         int32_t* prim_source, rt_host_tables_info* info);

/* glibc random_r TYPE_3 restatement: rand() sequence after srand(seed) (RND macro, Math.cuh:12). */
typedef struct rt_glibc_rand { int32_t r[34]; uint32_t idx; } rt_glibc_rand;
void rt_glibc_srand(rt_glibc_rand* g, uint32_t seed);
int32_t rt_glibc_rand_next(rt_glibc_rand* g);

/* Built-in scenes, written into caller-provided arrays (query sizes with NULL arrays).
 *   0 = CudaLayer::GenerateWorld default world (CudaLayer.cpp:103-256): XZ checker ground + 16 spheres
 *   1 = 3-sphere Lambertian scene (BASELINE config 1)
 *   2 = RTIOW book-1 final random-spheres scene in the reference's types (BASELINE config 2/4)
 *   3 = Cornell-style emissive box of XY/XZ/YZ rects (BASELINE config 3)
 *   4 = textured spheres (BASELINE config 5); images 0, 1, 2 (earth, moon, sun) are the caller's
 * `seed` seeds rt_glibc_srand for the scenes that draw random numbers (glibc default is 1). */
int rt_builtin_scene(int which, uint32_t seed, rt_hittable_desc* hittables, uint32_t* num_hittables,
                     rt_material_desc* materials, uint32_t* num_materials);

/* Procedural RGB8 texture (3 bytes per texel, row-major, row 0 = top as stb loads it) standing in for the
 * reference's 8192×4096 planet maps (assets/textures/8k_*.jpg, loaded by RawStbImage.h:11-22): kind 0 = earth,
 * 1 = moon, 2 = sun.  Deterministic: every texel is a pure function of (kind, x, y, width, height). */
int rt_procedural_texture(int kind, int32_t width, int32_t height, uint8_t* rgb);

/* Camera → InputStruct exactly as CudaLayer.cpp:43-65: up = normalize(cross(o, normalize(cross(o, up0)))). */
void rt_camera_inputs(const float position[3], const float orientation[3], const float world_up[3],
                      float fov_degrees, float near_plane, float far_plane, const float bg_start[3],
                      const float bg_end[3], rt_input_struct* out);

#ifdef __cplusplus
}
#endif

#endif /* RT_HIP_H */
