/*
 * rt_reference_graph.h — memory layout of the reference's scene graph, as the reference viewer builds it in
 * host-visible (CUDA managed / HIP managed) memory and hands it to LaunchKernel as `Hittable* world`.
 *
 * The structs below are plain-C descriptions of the reference classes' data members (x86-64 / 64-bit
 * device ABI: pointers 8 B, enums 4 B, bool 1 B).  librt_hip.so only READS such a graph, on the host, to
 * flatten it (rt_scene_from_reference_graph / LaunchKernel); it never writes it.
 *
 *   Hittable      Hittables/Hittable.cuh:47-67     16 B  {type, isActive, Object*}
 *   ObjectUnion   Hittables/Hittable.cuh:53-60      8 B  one pointer
 *   Sphere        Hittables/Hittable.cuh:69-74     24 B  {center, radius, mat_ptr}
 *   XY/XZ/YZRect  Hittables/Hittable.cuh:128-134   32 B  {center, width, height, mat_ptr}
 *   BVHNode       Hittables/Hittable.cuh:296-301   48 B  {box, left, right, memory}
 *   Material      Hittables/Material.cuh:19-32     16 B  {type, Object*}
 *   Lambertian    Hittables/Material.cuh:34-37      8 B  {albedo}
 *   Metal         Hittables/Material.cuh:65-69     16 B  {albedo, fuzz}
 *   Dielectric    Hittables/Material.cuh:97-100     4 B  {ir}
 *   DiffuseLight  Hittables/Material.cuh:148-152   16 B  {albedo, light_intensity}
 *   Texture       Hittables/Texture.cuh:16-28      16 B  {type, Object*}
 *   Constant      Hittables/Texture.cuh:30-34      16 B  {color, padding}
 *   Checker       Hittables/Texture.cuh:47-51      16 B  {odd, even}
 *   Image         Hittables/Texture.cuh:70-108     32 B  {data, path, width, height, bytes_per_scanline}
 */
#ifndef RT_REFERENCE_GRAPH_H
#define RT_REFERENCE_GRAPH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { RTREF_SPHERE = 0, RTREF_XYRECT = 1, RTREF_XZRECT = 2, RTREF_YZRECT = 3, RTREF_HITTABLELIST = 4,
       RTREF_BVHNODE = 5 };

typedef struct rtref_vec3 { float e[3]; } rtref_vec3;

typedef struct rtref_hittable {
    int32_t type;
    uint8_t is_active;
    uint8_t pad_[3];
    void** object; /* ObjectUnion*: *object points at the Sphere, XYRect, ..., or BVHNode */
} rtref_hittable;

typedef struct rtref_sphere { rtref_vec3 center; float radius; void* mat_ptr; } rtref_sphere;
typedef struct rtref_rect { rtref_vec3 center; float width; float height; void* mat_ptr; } rtref_rect;
typedef struct rtref_aabb { rtref_vec3 minimum, maximum; } rtref_aabb;
typedef struct rtref_bvh_node {
    rtref_aabb box;
    rtref_hittable* left;
    rtref_hittable* right;
    char* memory;
} rtref_bvh_node;

typedef struct rtref_material { int32_t type; void** object; } rtref_material;
typedef struct rtref_lambertian { void* albedo; } rtref_lambertian;
typedef struct rtref_metal { void* albedo; float fuzz; } rtref_metal;
typedef struct rtref_dielectric { float ir; } rtref_dielectric;
typedef struct rtref_diffuse_light { void* albedo; int32_t light_intensity; } rtref_diffuse_light;

typedef struct rtref_texture { int32_t type; void** object; } rtref_texture;
typedef struct rtref_constant { rtref_vec3 color; float padding; } rtref_constant;
typedef struct rtref_checker { rtref_constant* odd; rtref_constant* even; } rtref_checker;
typedef struct rtref_image {
    unsigned char* data;
    const char* path;
    int32_t width, height;
    int32_t bytes_per_scanline;
} rtref_image;

#ifdef __cplusplus
static_assert(sizeof(rtref_hittable) == 16, "Hittable layout");
static_assert(sizeof(rtref_sphere) == 24, "Sphere layout");
static_assert(sizeof(rtref_rect) == 32, "Rect layout");
static_assert(sizeof(rtref_bvh_node) == 48, "BVHNode layout");
static_assert(sizeof(rtref_material) == 16, "Material layout");
static_assert(sizeof(rtref_metal) == 16, "Metal layout");
static_assert(sizeof(rtref_diffuse_light) == 16, "DiffuseLight layout");
static_assert(sizeof(rtref_texture) == 16, "Texture layout");
static_assert(sizeof(rtref_constant) == 16, "Constant layout");
static_assert(sizeof(rtref_image) == 32, "Image layout");
}
#endif

#endif
