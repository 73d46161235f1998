// api.cpp — host half of the C ABI: error reporting, device scene tables, and the flattener for the
// reference's pointer-graph scene (the `Hittable* world` argument of LaunchKernel, Kernel.cu:178-180).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <new>
#include <stdexcept>
#include <cstring>
#include <mutex>
#include <unordered_set>

#include "../../include/rt_reference_graph.h"
#include "rt_internal.h"
#include "rt_scene_device.h"

namespace rt {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

// Host steps allocate (std::vector, std::string): a failed allocation must come back as a status code, not
// as an exception through the extern "C" boundary (which would terminate the caller's process).
template <class F>
static int guarded(const char* what, F&& f) {
    try {
        return f();
    } catch (const std::bad_alloc&) {
        set_error(std::string(what) + ": host allocation failed");
        return RT_ERR_OUT_OF_MEMORY;
    } catch (const std::exception& e) {
        set_error(std::string(what) + ": " + e.what());
        return RT_ERR_INVALID_SCENE;
    }
}

static int hip_fail(hipError_t e, const char* what) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? RT_ERR_OUT_OF_MEMORY : RT_ERR_DEVICE;
}

template <typename T>
static int upload(const std::vector<T>& host, void** dev, const char* what) {
    *dev = nullptr;
    if (host.empty()) return RT_OK;
    hipError_t e = hipMalloc(dev, host.size() * sizeof(T));
    if (e != hipSuccess) return hip_fail(e, what);
    e = hipMemcpy(*dev, host.data(), host.size() * sizeof(T), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(*dev);
        *dev = nullptr;
        return hip_fail(e, what);
    }
    return RT_OK;
}

static void free_device(DeviceScene* s) {
    if (s->nodes) (void)hipFree((void*)s->nodes);
    if (s->nodes48) (void)hipFree((void*)s->nodes48);
    if (s->refs) (void)hipFree((void*)s->refs);
    s->nodes48 = s->refs = nullptr;
    if (s->prims) (void)hipFree((void*)s->prims);
    if (s->prims_flat) (void)hipFree((void*)s->prims_flat);
    if (s->ref_nodes) (void)hipFree((void*)s->ref_nodes);
    if (s->flat_boxes) (void)hipFree((void*)s->flat_boxes);
    if (s->flat_ref_pairs) (void)hipFree((void*)s->flat_ref_pairs);
    s->prims_flat = s->ref_nodes = s->flat_boxes = s->flat_ref_pairs = nullptr;
    if (s->bvh_ref_nodes) (void)hipFree((void*)s->bvh_ref_nodes);
    if (s->bvh_boxes) (void)hipFree((void*)s->bvh_boxes);
    if (s->bvh_ref_pairs) (void)hipFree((void*)s->bvh_ref_pairs);
    s->bvh_ref_nodes = s->bvh_boxes = s->bvh_ref_pairs = nullptr;
    if (s->mats) (void)hipFree((void*)s->mats);
    if (s->imgs) (void)hipFree((void*)s->imgs);  // texels: owned by rt_scene::texel_block
    s->nodes = s->prims = s->mats = nullptr;
    s->imgs = nullptr;
    s->texels = nullptr;
}

int create_device_scene(const HostScene& h, rt_scene** out, std::shared_ptr<void> shared_texels) {
    rt_scene* s = new rt_scene();
    s->host = h;
    s->host.texels = std::vector<uint8_t>();  // uploaded below (or shared); no host copy is kept
    DeviceScene& d = s->dev;
    int rc;
    void* p;
    if ((rc = upload(h.nodes, &p, "hipMalloc/hipMemcpy(nodes)"))) goto fail;
    d.nodes = p;
    if ((rc = upload(h.nodes48, &p, "hipMalloc/hipMemcpy(nodes48)"))) goto fail;
    d.nodes48 = p;
    if ((rc = upload(h.refs, &p, "hipMalloc/hipMemcpy(refs)"))) goto fail;
    d.refs = p;
    d.wide_refs = h.wide_refs;
    if ((rc = upload(h.prims, &p, "hipMalloc/hipMemcpy(prims)"))) goto fail;
    d.prims = p;
    if ((rc = upload(h.prims_flat, &p, "hipMalloc/hipMemcpy(prims_flat)"))) goto fail;
    d.prims_flat = p;
    if ((rc = upload(h.ref_nodes, &p, "hipMalloc/hipMemcpy(ref_nodes)"))) goto fail;
    d.ref_nodes = p;
    if ((rc = upload(h.flat_ref_pairs, &p, "hipMalloc/hipMemcpy(flat_ref_pairs)"))) goto fail;
    d.flat_ref_pairs = p;
    if ((rc = upload(h.flat_boxes, &p, "hipMalloc/hipMemcpy(flat_boxes)"))) goto fail;
    d.flat_boxes = p;
    if ((rc = upload(h.bvh_ref_nodes, &p, "hipMalloc/hipMemcpy(bvh_ref_nodes)"))) goto fail;
    d.bvh_ref_nodes = p;
    if ((rc = upload(h.bvh_boxes, &p, "hipMalloc/hipMemcpy(bvh_boxes)"))) goto fail;
    d.bvh_boxes = p;
    if ((rc = upload(h.bvh_ref_pairs, &p, "hipMalloc/hipMemcpy(bvh_ref_pairs)"))) goto fail;
    d.bvh_ref_pairs = p;
    d.flat_runs[0] = h.flat_runs[0];
    d.flat_runs[1] = h.flat_runs[1];
    if ((rc = upload(h.mats, &p, "hipMalloc/hipMemcpy(materials)"))) goto fail;
    d.mats = p;
    if ((rc = upload(h.imgs, &p, "hipMalloc/hipMemcpy(images)"))) goto fail;
    d.imgs = p;
    if (shared_texels) {
        s->texel_block = std::move(shared_texels);
    } else {
        if ((rc = upload(h.texels, &p, "hipMalloc/hipMemcpy(texels)"))) goto fail;
        if (p) s->texel_block = std::shared_ptr<void>(p, [](void* q) { (void)hipFree(q); });
    }
    d.texels = s->texel_block.get();
    d.num_nodes = h.num_nodes;
    d.num_prims = h.num_prims;
    d.num_mats = h.num_mats;
    d.num_imgs = (uint32_t)(h.imgs.size() / 4);
    d.depth = h.depth;
    d.has_image_textures = h.has_image_textures;
    d.has_textures = h.has_textures;
    d.has_rects = h.has_rects;
    d.device_bytes = (h.nodes.size() + h.nodes48.size() + h.refs.size() + h.prims.size() + h.prims_flat.size() + h.ref_nodes.size() +
                      h.flat_boxes.size() + h.flat_ref_pairs.size() + h.bvh_ref_nodes.size() + h.bvh_boxes.size() + h.bvh_ref_pairs.size() + h.mats.size()) * 4 +
                     h.imgs.size() * 4 + h.texels.size();
    *out = s;
    return RT_OK;
fail:
    free_device(&d);
    delete s;
    return rc;
}

// ------------------------------------------------------------------------------------------------
// Reference pointer-graph flattener.  Walks BVHNode::left/right (Hittable.cuh:296-301) from `world`,
// collects each distinct leaf hittable once (span-1 leaves reference one object twice, Hittable.cuh:
// 326-327), and resolves Material → {Lambertian|Metal|Dielectric|DiffuseLight} → Texture →
// {Constant|Checker|Image} (Material.cuh:19-177, Texture.cuh:16-109).  The graph only contains active
// objects (the BVH is rebuilt without inactive ones), so every collected hittable is active.
// ------------------------------------------------------------------------------------------------
static int read_texture(const void* tex_ptr, rt_texture_desc* t, FlatDesc* out, std::string* err) {
    std::memset(t, 0, sizeof(*t));
    t->image = -1;
    if (!tex_ptr) { *err = "material without texture"; return RT_ERR_INVALID_SCENE; }
    const rtref_texture* tex = (const rtref_texture*)tex_ptr;
    t->type = tex->type;
    if (!tex->object || !*tex->object) { *err = "texture without object"; return RT_ERR_INVALID_SCENE; }
    const void* obj = *tex->object;
    switch (tex->type) {
    case RT_CONSTANT: {
        const rtref_constant* c = (const rtref_constant*)obj;
        std::memcpy(t->color, c->color.e, sizeof(t->color));
        break;
    }
    case RT_CHECKER: {
        const rtref_checker* c = (const rtref_checker*)obj;
        if (!c->odd || !c->even) { *err = "checker without constants"; return RT_ERR_INVALID_SCENE; }
        std::memcpy(t->color, c->odd->color.e, sizeof(t->color));
        std::memcpy(t->color2, c->even->color.e, sizeof(t->color2));
        break;
    }
    case RT_IMAGE: {
        const rtref_image* im = (const rtref_image*)obj;
        rt_image_desc d;
        d.data = im->data;
        d.width = im->data ? im->width : 0;
        d.height = im->data ? im->height : 0;
        t->image = (int32_t)out->images.size();
        out->images.push_back(d);
        break;
    }
    default: *err = "unknown texture type " + std::to_string(tex->type); return RT_ERR_INVALID_SCENE;
    }
    return RT_OK;
}

static int read_material(const void* mat_ptr, rt_material_desc* m, FlatDesc* out, std::string* err) {
    std::memset(m, 0, sizeof(*m));
    m->albedo.image = -1;
    if (!mat_ptr) { *err = "hittable without material"; return RT_ERR_INVALID_SCENE; }
    const rtref_material* mat = (const rtref_material*)mat_ptr;
    if (!mat->object || !*mat->object) { *err = "material without object"; return RT_ERR_INVALID_SCENE; }
    const void* obj = *mat->object;
    m->type = mat->type;
    switch (mat->type) {
    case RT_LAMBERTIAN: return read_texture(((const rtref_lambertian*)obj)->albedo, &m->albedo, out, err);
    case RT_METAL:
        m->fuzz = ((const rtref_metal*)obj)->fuzz;
        return read_texture(((const rtref_metal*)obj)->albedo, &m->albedo, out, err);
    case RT_DIELECTRIC: m->ir = ((const rtref_dielectric*)obj)->ir; return RT_OK;
    case RT_DIFFUSELIGHT:
        m->light_intensity = ((const rtref_diffuse_light*)obj)->light_intensity;
        return read_texture(((const rtref_diffuse_light*)obj)->albedo, &m->albedo, out, err);
    default: *err = "unknown material type " + std::to_string(mat->type); return RT_ERR_INVALID_SCENE;
    }
}

int flatten_reference_graph(const void* world, FlatDesc* out, std::string* err) {
    *out = FlatDesc();
    if (!world) { *err = "world is NULL"; return RT_ERR_INVALID_ARGUMENT; }
    const rtref_hittable* root = (const rtref_hittable*)world;
    if (root->type != RTREF_BVHNODE) { *err = "world is not a BVHNode hittable"; return RT_ERR_INVALID_SCENE; }
    std::vector<const rtref_hittable*> stack{root};
    std::unordered_set<const void*> seen_nodes, seen_prims;
    while (!stack.empty()) {
        const rtref_hittable* h = stack.back();
        stack.pop_back();
        if (!h->object || !*h->object) { *err = "hittable without object"; return RT_ERR_INVALID_SCENE; }
        const void* obj = *h->object;
        if (h->type == RTREF_BVHNODE) {
            if (!seen_nodes.insert(obj).second) continue;
            if (seen_nodes.size() > (1u << 24)) { *err = "BVH graph too large or cyclic"; return RT_ERR_INVALID_SCENE; }
            const rtref_bvh_node* n = (const rtref_bvh_node*)obj;
            // right first so that the left subtree is emitted first (list order of the build)
            if (n->right) stack.push_back(n->right);
            if (n->left) stack.push_back(n->left);
            continue;
        }
        if (!seen_prims.insert(obj).second) continue;
        rt_hittable_desc d;
        std::memset(&d, 0, sizeof(d));
        d.type = h->type;
        d.is_active = 1;
        const void* mat_ptr;
        if (h->type == RTREF_SPHERE) {
            const rtref_sphere* s = (const rtref_sphere*)obj;
            std::memcpy(d.center, s->center.e, sizeof(d.center));
            d.radius = s->radius;
            mat_ptr = s->mat_ptr;
        } else if (h->type == RTREF_XYRECT || h->type == RTREF_XZRECT || h->type == RTREF_YZRECT) {
            const rtref_rect* r = (const rtref_rect*)obj;
            std::memcpy(d.center, r->center.e, sizeof(d.center));
            d.width = r->width;
            d.height = r->height;
            mat_ptr = r->mat_ptr;
        } else {
            *err = "unsupported hittable type " + std::to_string(h->type) + " in BVH";
            return RT_ERR_INVALID_SCENE;
        }
        rt_material_desc m;
        int rc = read_material(mat_ptr, &m, out, err);
        if (rc) return rc;
        d.material = (int32_t)out->materials.size();
        out->materials.push_back(m);
        out->hittables.push_back(d);
    }
    return RT_OK;
}

// ------------------------------------------------------------------------------------------------
// LaunchKernel's scene cache.  The viewer mutates its managed-memory graph in place
// between frames without notifying anyone, so every launch re-flattens it (microseconds for ~500
// objects) and compares the flat description with the cached one:
//   * hittables (geometry, activity) differ → rebuild BVH + tables, keep the uploaded texels;
//   * only materials differ → re-upload the material table in place (no rebuild, CudaLayer.cpp:719-872);
//   * an image's (data pointer, width, height) differs → rebuild with a new texel upload.  The reference
//     replaces texture data by cudaFree + a new allocation (CudaLayer.cpp:889-903), so the pointer is the
//     change key: texel bytes are never read per frame.
// One entry per (device, world pointer), least recently used evicted beyond kLaunchCacheEntries.
// ------------------------------------------------------------------------------------------------
namespace {

struct ImageKey {
    const void* data;
    int32_t width, height;
    bool operator==(const ImageKey& o) const { return data == o.data && width == o.width && height == o.height; }
};

struct LaunchEntry {
    int device = 0;
    const void* world = nullptr;
    uint64_t last_use = 0;
    std::vector<rt_hittable_desc> hittables;
    std::vector<rt_material_desc> materials;
    std::vector<ImageKey> images;
    int texel_bytes = 0;  // device bytes per texel of the uploaded block (RT_TUNE_TEXEL_LAYOUT when it was made)
    // shared with the LaunchKernel calls rendering it: an entry evicted or rebuilt by another thread frees
    // its device scene only when the last of them has finished
    std::shared_ptr<rt_scene> scene;
};

std::shared_ptr<rt_scene> own_scene(rt_scene* s, int device) {
    return std::shared_ptr<rt_scene>(s, [device](rt_scene* p) {
        int cur = 0;
        const bool restore = hipGetDevice(&cur) == hipSuccess;
        (void)hipSetDevice(device);
        rt_scene_destroy(p);
        if (restore) (void)hipSetDevice(cur);
    });
}

constexpr size_t kLaunchCacheEntries = 8;
std::mutex g_launch_mu;
// never destroyed: the entries free device memory, which must not run after the HIP runtime has shut down
std::vector<LaunchEntry>& g_launch_cache = *new std::vector<LaunchEntry>();
uint64_t g_launch_clock = 0;

template <class T>
bool same_bytes(const std::vector<T>& a, const std::vector<T>& b) {
    return a.size() == b.size() && (a.empty() || std::memcmp(a.data(), b.data(), a.size() * sizeof(T)) == 0);
}

}  // namespace

int reference_scene_for_launch(const void* world, std::shared_ptr<rt_scene>* out, double* host_ms) {
    const auto t0 = std::chrono::steady_clock::now();
    int device = 0;
    hipError_t e = hipGetDevice(&device);
    if (e != hipSuccess) return hip_fail(e, "LaunchKernel: hipGetDevice");
    std::lock_guard<std::mutex> lock(g_launch_mu);
    int rc = guarded("LaunchKernel", [&]() -> int {
        FlatDesc f;
        std::string err;
        int r = flatten_reference_graph(world, &f, &err);
        if (r) { set_error("LaunchKernel: " + err); return r; }
        std::vector<ImageKey> images;
        for (const rt_image_desc& im : f.images) images.push_back(ImageKey{im.data, im.width, im.height});
        LaunchEntry* ent = nullptr;
        for (LaunchEntry& c : g_launch_cache)
            if (c.device == device && c.world == world) ent = &c;
        if (!ent) {
            if (g_launch_cache.size() >= kLaunchCacheEntries) {  // evict the least recently used entry
                auto lru = std::min_element(g_launch_cache.begin(), g_launch_cache.end(),
                                            [](const LaunchEntry& a, const LaunchEntry& b) { return a.last_use < b.last_use; });
                g_launch_cache.erase(lru);  // (its scene is freed once no call renders it)
            }
            g_launch_cache.emplace_back();
            ent = &g_launch_cache.back();
            ent->device = device;
            ent->world = world;
        }
        ent->last_use = ++g_launch_clock;
        const bool geometry = !ent->scene || !same_bytes(ent->hittables, f.hittables) ||
                              ent->materials.size() != f.materials.size();
        // the image table of a rebuilt scene takes this thread's texel layout: a block uploaded in the other
        // layout cannot be shared with it (its offsets and strides differ), so a layout change re-uploads
        const int texel_bytes = g_texel_bytes == 4 ? 4 : 3;
        const bool new_images = !ent->scene || !(ent->images == images) || ent->texel_bytes != texel_bytes;
        if (geometry || new_images) {
            rt_scene_desc d = f.desc();
            HostScene h;
            r = build_host_scene(&d, &h, &err, new_images);
            if (r) { set_error("LaunchKernel: " + err); return r; }
            rt_scene* fresh = nullptr;
            r = create_device_scene(h, &fresh, new_images ? nullptr : ent->scene->texel_block);
            if (r) return r;
            ent->scene = own_scene(fresh, device);
            ent->texel_bytes = texel_bytes;
        } else if (!same_bytes(ent->materials, f.materials)) {
            r = rt_scene_update_materials(ent->scene.get(), f.materials.data(), (uint32_t)f.materials.size());
            if (r) return r;
        }
        ent->hittables.swap(f.hittables);
        ent->materials.swap(f.materials);
        ent->images.swap(images);
        *out = ent->scene;
        return RT_OK;
    });
    if (host_ms) *host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

}  // namespace rt

using namespace rt;

extern "C" {

const char* rt_last_error(void) { return g_last_error.c_str(); }

const char* rt_version(void) { return "librt_hip 0.1 (gfx950)"; }
int rt_abi_version(void) { return RT_ABI_VERSION; }

int rt_set_device(int device) {
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    return RT_OK;
}

int rt_scene_create(const rt_scene_desc* desc, rt_scene** out_scene) {
    if (!out_scene) { set_error("rt_scene_create: out_scene is NULL"); return RT_ERR_INVALID_ARGUMENT; }
    *out_scene = nullptr;
    return guarded("rt_scene_create", [&]() -> int {
        HostScene h;
        std::string err;
        int rc = build_host_scene(desc, &h, &err);
        if (rc) { set_error("rt_scene_create: " + err); return rc; }
        return create_device_scene(h, out_scene);
    });
}

int rt_scene_from_reference_graph(const void* world, rt_scene** out_scene) {
    if (!out_scene) { set_error("rt_scene_from_reference_graph: out_scene is NULL"); return RT_ERR_INVALID_ARGUMENT; }
    *out_scene = nullptr;
    return guarded("rt_scene_from_reference_graph", [&]() -> int {
        FlatDesc f;
        std::string err;
        int rc = flatten_reference_graph(world, &f, &err);
        if (rc) { set_error("rt_scene_from_reference_graph: " + err); return rc; }
        rt_scene_desc d = f.desc();
        return rt_scene_create(&d, out_scene);
    });
}

int rt_scene_update_materials(rt_scene* scene, const rt_material_desc* materials, uint32_t num_materials) {
    if (!scene || (!materials && num_materials)) {
        set_error("rt_scene_update_materials: NULL argument");
        return RT_ERR_INVALID_ARGUMENT;
    }
    if (num_materials != scene->dev.num_mats) {
        set_error("rt_scene_update_materials: material count differs from the scene's");
        return RT_ERR_INVALID_ARGUMENT;
    }
    return guarded("rt_scene_update_materials", [&]() -> int {
        std::vector<float> packed;
        std::string err;
        int rc = pack_materials(materials, num_materials, (uint32_t)(scene->host.imgs.size() / 4), &packed, &err);
        if (rc) { set_error("rt_scene_update_materials: " + err); return rc; }
        bool img = false, tex = false;
        for (uint32_t i = 0; i < num_materials; i++) {
            if (materials[i].type == RT_DIELECTRIC) continue;
            img |= materials[i].albedo.type == RT_IMAGE;
            tex |= materials[i].albedo.type != RT_CONSTANT;
        }
        if (!packed.empty()) {
            // renders are asynchronous on the callers' streams: let every launch that may still read the
            // old table finish before it is overwritten (the viewer edits between frames, CudaLayer.cpp:719-872)
            hipError_t e = hipDeviceSynchronize();
            if (e != hipSuccess) return hip_fail(e, "rt_scene_update_materials: hipDeviceSynchronize");
            e = hipMemcpy((void*)scene->dev.mats, packed.data(), packed.size() * 4, hipMemcpyHostToDevice);
            if (e != hipSuccess) return hip_fail(e, "rt_scene_update_materials: hipMemcpy");
        }
        scene->dev.has_image_textures = img;
        scene->dev.has_textures = tex;
        scene->host.mats = packed;
        return RT_OK;
    });
}

int rt_reference_graph_flatten(const void* world, rt_hittable_desc* hittables, uint32_t* num_hittables,
                               rt_material_desc* materials, uint32_t* num_materials, rt_image_desc* images,
                               uint32_t* num_images) {
    if (!num_hittables || !num_materials || !num_images) {
        set_error("rt_reference_graph_flatten: count pointers must not be NULL");
        return RT_ERR_INVALID_ARGUMENT;
    }
    FlatDesc f;
    int rc = guarded("rt_reference_graph_flatten", [&]() -> int {
        std::string err;
        int r = flatten_reference_graph(world, &f, &err);
        if (r) set_error("rt_reference_graph_flatten: " + err);
        return r;
    });
    if (rc) return rc;
    bool fits = (!hittables || f.hittables.size() <= *num_hittables) &&
                (!materials || f.materials.size() <= *num_materials) && (!images || f.images.size() <= *num_images);
    if (fits) {
        if (hittables) std::copy(f.hittables.begin(), f.hittables.end(), hittables);
        if (materials) std::copy(f.materials.begin(), f.materials.end(), materials);
        if (images) std::copy(f.images.begin(), f.images.end(), images);
    }
    *num_hittables = (uint32_t)f.hittables.size();
    *num_materials = (uint32_t)f.materials.size();
    *num_images = (uint32_t)f.images.size();
    if (!fits) { set_error("rt_reference_graph_flatten: output arrays too small"); return RT_ERR_INVALID_ARGUMENT; }
    return RT_OK;
}

int rt_build_host_tables(const rt_scene_desc* desc, float* nodes, float* prims, float* materials,
                         int32_t* prim_source, rt_host_tables_info* info) {
    if (!info) { set_error("rt_build_host_tables: info is NULL"); return RT_ERR_INVALID_ARGUMENT; }
    HostScene h;
    int rc = guarded("rt_build_host_tables", [&]() -> int {
        std::string err;
        int r = build_host_scene(desc, &h, &err);
        if (r) set_error("rt_build_host_tables: " + err);
        return r;
    });
    if (rc) return rc;
    info->num_nodes = h.num_nodes;
    info->num_prims = h.num_prims;
    info->num_materials = h.num_mats;
    info->depth = h.depth;
    if (nodes) std::copy(h.nodes.begin(), h.nodes.end(), nodes);
    // (num_prims records: an empty scene's table carries one zero record for the device, not for the caller)
    if (prims) std::copy(h.prims.begin(), h.prims.begin() + (size_t)h.num_prims * 8, prims);
    if (materials) std::copy(h.mats.begin(), h.mats.end(), materials);
    if (prim_source) std::copy(h.prim_source.begin(), h.prim_source.end(), prim_source);
    return RT_OK;
}

int rt_scene_destroy(rt_scene* scene) {
    if (!scene) return RT_OK;
    free_device(&scene->dev);
    delete scene;
    return RT_OK;
}

int rt_scene_get_info(const rt_scene* scene, rt_scene_info* info) {
    if (!scene || !info) { set_error("rt_scene_get_info: NULL argument"); return RT_ERR_INVALID_ARGUMENT; }
    info->num_primitives = scene->dev.num_prims;
    info->num_nodes = scene->dev.num_nodes;
    info->num_materials = scene->dev.num_mats;
    info->bvh_depth = scene->dev.depth;
    info->device_bytes = scene->dev.device_bytes;
    return RT_OK;
}

}  // extern "C"
