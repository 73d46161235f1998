// rt_scene_device.h — the opaque rt_scene handle: host copy of the packed tables + device pointers.
#pragma once

#include <cstdint>
#include <memory>

#include "rt_internal.h"

namespace rt {

struct DeviceScene {
    const void* nodes = nullptr;   // float4 × 4 per node
    const void* nodes48 = nullptr; // float4 × 3 per node (boxes only)
    const void* refs = nullptr;    // per node: uint32 of two 16-bit child references, or (wide_refs) two uint32
    bool wide_refs = false;
    const void* prims = nullptr;   // float4 × 2 per primitive
    const void* prims_flat = nullptr;  // the same records in the reference BVH's test order (small scenes), or NULL
    const void* ref_nodes = nullptr;   // the reference BVH (boxes + shape) over prims_flat, or NULL
    const void* flat_ref_pairs = nullptr;  // ... as child-pair records (the flat kernels' wave-serial replay)
    const void* flat_boxes = nullptr;  // per prims_flat record its reference box (exactness check), or NULL
    const void* bvh_ref_nodes = nullptr;  // the reference BVH over `prims` (BVH order), or NULL (bvh_clear, render.hip)
    const void* bvh_boxes = nullptr;      // per `prims` record its reference box, or NULL
    const void* bvh_ref_pairs = nullptr;  // per reference node its children's boxes and references (ref_trace_wave)
    uint32_t flat_runs[2] = {0u, 0u};  // HostScene::flat_runs
    const void* mats = nullptr;    // float4 × 3 per material
    const void* imgs = nullptr;    // int4 per image
    const void* texels = nullptr;  // RGB8
    uint32_t num_nodes = 0, num_prims = 0, num_mats = 0, depth = 0;
    uint32_t num_imgs = 0;  // image descriptors (int4 each)
    bool has_image_textures = false;
    bool has_textures = false;  // any CHECKER or IMAGE albedo (selects the texture-capable kernel)
    bool has_rects = false;     // HostScene::has_rects
    uint64_t device_bytes = 0;
};

// Upload the tables of `h` to the current device.  shared_texels: an existing device texel block (same image
// table) to reference instead of uploading h.texels.  The host copy of the texels is not kept.
int create_device_scene(const HostScene& h, rt_scene** out, std::shared_ptr<void> shared_texels = nullptr);

// The device scene of the reference graph `world` for LaunchKernel (Kernel.cu:178-191), cached per
// (device, world): materials edited in place are re-uploaded, geometry edits rebuild the BVH and tables but
// keep the uploaded texels, a new image (data pointer, width or height, CudaLayer.cpp:889-903) re-uploads
// them.  *host_ms: host time spent (flatten + compare + any update).
int reference_scene_for_launch(const void* world, std::shared_ptr<rt_scene>* out, double* host_ms);

}  // namespace rt

struct rt_scene {
    rt::HostScene host;  // packed tables (texels dropped after the upload)
    rt::DeviceScene dev;
    std::shared_ptr<void> texel_block;  // device texels, shared by scenes rebuilt from the same images
};
