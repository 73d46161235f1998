// rt_scene_device.h — the opaque rt_scene handle: host copy of the packed tables + device pointers.
#pragma once

#include <cstdint>

#include "rt_internal.h"

namespace rt {

struct DeviceScene {
    const void* nodes = nullptr;   // float4 × 4 per node
    const void* nodes48 = nullptr; // float4 × 3 per node (boxes only)
    const void* refs16 = nullptr;  // uint32 per node: two signed 16-bit child references
    const void* prims = nullptr;   // float4 × 2 per primitive
    const void* mats = nullptr;    // float4 × 3 per material
    const void* imgs = nullptr;    // int4 per image
    const void* texels = nullptr;  // RGB8
    uint32_t num_nodes = 0, num_prims = 0, num_mats = 0, depth = 0;
    bool has_image_textures = false;
    bool has_textures = false;  // any CHECKER or IMAGE albedo (selects the texture-capable kernel)
    uint64_t device_bytes = 0;
};

int create_device_scene(const HostScene& h, rt_scene** out);

}  // namespace rt

struct rt_scene {
    rt::HostScene host;
    rt::DeviceScene dev;
};
