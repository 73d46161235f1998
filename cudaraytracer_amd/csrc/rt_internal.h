// rt_internal.h — internal (non-ABI) definitions shared by the host scene builder and the gfx950 kernels.
//
// Device data layout (all tables are read-only during a launch and small: an RTIOW scene of 488 spheres
// is ~40 KB, so a workgroup can stage the node + primitive tables in LDS):
//
//   nodes   : BVH2 with the two child boxes stored in the parent (4 × float4 = 64 B per node):
//               n0 = (c0.lo.x, c0.hi.x, c0.lo.y, c0.hi.y)
//               n1 = (c1.lo.x, c1.hi.x, c1.lo.y, c1.hi.y)
//               n2 = (c0.lo.z, c0.hi.z, c1.lo.z, c1.hi.z)
//               n3 = (int c0, int c1, 0, 0)    child >= 0: internal node; child < 0: leaf ~(first<<2 | count-1)
//               (count 1..4; with < 32767 nodes and < 8192 primitives every reference fits a signed 16 bits)
//   prims   : 2 × float4 = 32 B per primitive, in BVH leaf order:
//               sphere: p0 = (cx, cy, cz, r),         p1 = (r·r, 0, 0, bits(type | mat << 4))
//               rect  : p0 = (k, a0, a1, b0),         p1 = (b1, 0, 0, bits(type | mat << 4))
//                       k = plane coordinate, [a0,a1]×[b0,b1] the in-plane extent, exactly the floats
//                       XYRect/XZRect/YZRect::Hit compute (Hittable.cuh:142-147, 198-203, 254-259)
//   mats    : 3 × float4 = 48 B per material:
//               m0 = (bits(type | textype << 4), fuzz|ir, float(light_intensity), bits(image))
//               m1 = (color.rgb, 0)   m2 = (color2.rgb, 0)
//               dielectric: m1 = (1.0f / ir, r0², 0, 0) — the ir-only terms of Scatter, same binary32 ops
//   images  : texels of every image back to back, RGB8 (3 B, the reference's layout, Texture.cuh:76) or
//             RGBA8 (4 B, alpha 0: one dword gather per lookup); imgs[i] = (byte offset, width, height,
//             bytes per texel) as int4, offset -1 = no data
//
// Box padding: child boxes are the reference's primitive boxes (Hittable.cuh:112-116, 171-181, ...)
// grown outward by 1e-5 of the plane coordinate + 1e-6.  That covers the slab test's error term that scales
// with the plane coordinate (~2^-24·|plane/d|); the term that scales with the distance along the ray is
// covered in the kernel by widening every slab interval's far side by a relative 2^-20 (kSlabSlack,
// render.hip), so culling stays conservative for any camera distance (tests/test_gpu_parity.py,
// far-camera brute-force check).  Boxes only cull: the closest hit is decided by the primitive tests,
// which follow the reference arithmetic exactly.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/rt_hip.h"

namespace rt {

constexpr int kLeafMax = 4;         // max primitives per leaf (2-bit count in the leaf reference)
// Deepest BVH the compact v3 kernel holds at 8 waves per SIMD: 13 parked words × 256 B + (depth + 2) × 128 B of
// 16-bit stack per wave must fit 160 KB / 32 waves = 5120 B (render.hip, rt_render's LDS sizing)
constexpr uint32_t kOccupancyDepth = 12;
extern thread_local int g_leaf_max;  // rt_set_tuning(RT_TUNE_LEAF_MAX): 1..kLeafMax, read by the BVH build
extern thread_local int g_sah_traversal_x10;  // rt_set_tuning(RT_TUNE_SAH_TRAVERSAL): SAH node cost × 10
extern thread_local int g_texel_bytes;  // rt_set_tuning(RT_TUNE_TEXEL_LAYOUT): device bytes per texel, 3 or 4
constexpr int kRegStackDepth = 24;  // depth limit of the register (shift) traversal stack
constexpr uint32_t kFlatMaxPrims = 64;  // scenes up to this many primitives also get the flat kernel's tables
constexpr uint32_t kRefTreeMaxDepth = 14;  // deepest reference BVH the flat kernel replays (render.hip kRefStack)
// ... and the BVH kernels (render.hip kRefStackBvh).  The reference tree splits at most 3 times by type and otherwise
// in the middle, so 2^26 primitives (the library's limit) give depth <= 3 + 26 + 1.
constexpr uint32_t kRefTreeMaxDepthBvh = 31;

struct HostScene {
    std::vector<float> nodes;   // 16 floats per node
    std::vector<float> nodes48; // 12 floats per node: the three box float4 of `nodes` (v3 kernels), each child
                                // reference also in the low bytes of its x planes (and, wide, of its y planes;
                                // moved outward; scene_build.cpp)
    std::vector<uint32_t> refs;    // per node: child 0 | child 1 << 16 as 16-bit references, or (wide_refs) the
                                   // two 32-bit references
    bool wide_refs = false;        // references need 32 bits: >= 32767 nodes or >= 8192 primitives
    std::vector<float> prims;   // 8 floats per primitive
    std::vector<float> mats;    // 12 floats per material
    std::vector<int32_t> imgs;  // 4 ints per image
    std::vector<uint8_t> texels;
    uint32_t num_nodes = 0;
    uint32_t num_prims = 0;
    uint32_t num_mats = 0;
    uint32_t depth = 0;          // max root-to-leaf node count
    bool has_image_textures = false;
    bool has_textures = false;  // any CHECKER or IMAGE albedo
    bool has_rects = false;     // any active rectangle (render.hip bvh_clear: only rectangles can turn a miss into a
                                // NaN hit of the reference's)
    std::vector<int32_t> prim_source;  // desc index of each primitive (BVH order)
    std::vector<float> prims_flat;     // scenes of <= kFlatMaxPrims primitives: the records in the reference BVH's
                                       // test order (the flat kernel's table), else empty
    std::vector<float> ref_nodes;      // ... and the reference BVH itself: 8 floats per node (scene_build.cpp)
    std::vector<float> flat_ref_pairs; // ... and the same tree as child-pair records (16 floats per node)
    std::vector<float> flat_boxes;     // ... and per flat record its reference box for the flat kernels' exactness
                                       // check: 8 floats (scene_build.cpp)
    uint32_t flat_runs[2] = {0u, 0u};  // prims_flat holds each primitive type as one contiguous run: [begin, end) of
                                        // type t in bytes 2t, 2t + 1 of the pair (t = RT_SPHERE .. RT_YZRECT)
    std::vector<float> bvh_ref_nodes;  // every scene: the reference BVH (ref_nodes' layout) with its primitive children
                                       // as ~(BVH-order index) — the BVH kernels' replay (render.hip bvh_clear)
    std::vector<float> bvh_boxes;      // ... and per BVH-order primitive its reference box: (lo.xyz, 0), (hi.xyz, 0)
    std::vector<float> bvh_ref_pairs;  // ... and per reference node its two children: (lo.xyz, ref), (hi.xyz, 0) each
                                       // (a primitive child's box is not used) — the wave-serial replay's records
};

// Validate + build (host only).  Returns RT_OK or an rt_status, with `err` set.  with_texels = false computes
// the image table but leaves `texels` empty (a rebuild that reuses an uploaded texel block).
int build_host_scene(const rt_scene_desc* desc, HostScene* out, std::string* err, bool with_texels = true);

// Material table packing only (used by rt_scene_update_materials).
int pack_materials(const rt_material_desc* mats, uint32_t n, uint32_t num_images, std::vector<float>* out,
                   std::string* err);

// Flatten the reference's pointer graph (rt_reference_graph.h) into a flat description.
struct FlatDesc {
    std::vector<rt_hittable_desc> hittables;
    std::vector<rt_material_desc> materials;
    std::vector<rt_image_desc> images;
    rt_scene_desc desc() const {
        rt_scene_desc d;
        d.hittables = hittables.data();
        d.num_hittables = (uint32_t)hittables.size();
        d.materials = materials.data();
        d.num_materials = (uint32_t)materials.size();
        d.images = images.data();
        d.num_images = (uint32_t)images.size();
        return d;
    }
};
int flatten_reference_graph(const void* world, FlatDesc* out, std::string* err);

void set_error(const std::string& msg);

inline float bits_to_float(uint32_t u) {
    float f;
    static_assert(sizeof(f) == sizeof(u), "");
    __builtin_memcpy(&f, &u, 4);
    return f;
}

}  // namespace rt
