// scene_build.cpp — host side of the scene boundary: validation, flat-table packing and the BVH build.
//
// Replaces the reference's host-side scene construction: the managed-memory pointer graph of
// CudaLayer::GenerateWorld (CudaLayer.cpp:103-256) and the recursive BVHNode constructor
// (Hittable.cuh:303-385).  The reference splits by hittable type, then in list order (no spatial
// criterion), which costs ~50 box tests per ray on the RTIOW scene.  Here a full-sweep
// SAH build over padded reference boxes produces a BVH with the same closest-hit semantics: the
// primitive tests alone decide the hit, boxes only cull (see rt_internal.h).
#include <algorithm>
#include <limits>
#include <functional>
#include <array>
#include <cmath>
#include <cstring>
#include <numeric>

#include "rt_internal.h"

namespace rt {
namespace {

struct Box {
    float lo[3], hi[3];
    void empty() {
        for (int i = 0; i < 3; i++) { lo[i] = INFINITY; hi[i] = -INFINITY; }
    }
    void grow(const Box& b) {
        for (int i = 0; i < 3; i++) { lo[i] = std::min(lo[i], b.lo[i]); hi[i] = std::max(hi[i], b.hi[i]); }
    }
    float area() const {
        float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        if (!(dx >= 0) || !(dy >= 0) || !(dz >= 0)) return 0.0f;
        return 2.0f * (dx * dy + dy * dz + dz * dx);
    }
};

// Rect plane/extent exactly as XYRect/XZRect/YZRect::Hit compute them (Hittable.cuh:142-147, 198-203,
// 254-259): a0 = c.a - (w / 2) etc.  Evaluated in binary32 so the device sees identical floats.
struct RectGeom { float k, a0, a1, b0, b1; int ia, ib, ik; };
RectGeom rect_geom(const rt_hittable_desc& h) {
    RectGeom g;
    const float* c = h.center;
    volatile float w2 = h.width / 2, h2 = h.height / 2;  // keep binary32 rounding of each step
    if (h.type == RT_XYRECT) {
        g.a0 = c[0] - w2; g.a1 = c[0] + w2; g.b0 = c[1] - h2; g.b1 = c[1] + h2; g.k = c[2];
        g.ia = 0; g.ib = 1; g.ik = 2;
    } else if (h.type == RT_XZRECT) {
        g.a0 = c[0] - w2; g.a1 = c[0] + w2; g.b0 = c[2] - h2; g.b1 = c[2] + h2; g.k = c[1];
        g.ia = 0; g.ib = 2; g.ik = 1;
    } else {  // YZ: y from height, z from width
        g.a0 = c[1] - h2; g.a1 = c[1] + h2; g.b0 = c[2] - w2; g.b1 = c[2] + w2; g.k = c[0];
        g.ia = 1; g.ib = 2; g.ik = 0;
    }
    return g;
}

// Reference primitive box (Hittable.cuh:112-116, 171-181, 227-237, 283-293), grown outward.
Box prim_box(const rt_hittable_desc& h) {
    Box b;
    if (h.type == RT_SPHERE) {
        for (int i = 0; i < 3; i++) { b.lo[i] = h.center[i] - h.radius; b.hi[i] = h.center[i] + h.radius; }
    } else {
        RectGeom g = rect_geom(h);
        b.lo[g.ia] = g.a0; b.hi[g.ia] = g.a1;
        b.lo[g.ib] = g.b0; b.hi[g.ib] = g.b1;
        b.lo[g.ik] = g.k - 0.0001f; b.hi[g.ik] = g.k + 0.0001f;
    }
    for (int i = 0; i < 3; i++) {
        float m = std::max(std::fabs(b.lo[i]), std::fabs(b.hi[i]));
        float pad = 1e-5f * m + 1e-6f;
        b.lo[i] -= pad;
        b.hi[i] += pad;
    }
    return b;
}

// v with the low byte of its binary32 representation replaced by `payload`, moved outward: the result is <= v
// (up = false) or >= v (up = true).  Works on the magnitude, whose bit pattern orders like the value; a zero
// or tiny magnitude crosses to the other sign's side (a denormal of the right sign).
float with_low_byte(float v, uint32_t payload, bool up) {
    uint32_t b;
    std::memcpy(&b, &v, 4);
    const uint32_t sign = b & 0x80000000u, mag = b & 0x7fffffffu;
    const bool grow = (sign == 0) == up;  // the magnitude must not shrink (else: must not grow)
    uint32_t out;
    // (a plane at the float range's end keeps its magnitude just under FLT_MAX: no finite ray reaches past it)
    if (grow) {
        out = sign | (((mag >> 8) + 1u) << 8) | payload;  // > mag
    } else if ((mag >> 8) > 0u) {
        out = sign | (((mag >> 8) - 1u) << 8) | payload;  // < mag
    } else {
        out = (sign ^ 0x80000000u) | 0x100u | payload;  // |v| < 256 ulps of 2^-149: a denormal past zero
    }
    if ((out & 0x7fffffffu) >= 0x7f7fff00u) out = (out & 0x80000000u) | 0x7f7fff00u | payload;  // stay finite
    float r;
    std::memcpy(&r, &out, 4);
    return r;
}

struct BuildPrim {
    Box box;
    float centroid[3];
    int src;  // index into desc.hittables
};

struct Builder {
    int leaf_max = kLeafMax;
    float traversal = 1.6f;  // SAH: node visit cost / primitive test cost
    std::vector<BuildPrim> prims;
    std::vector<int> order;  // final primitive order
    struct Node {
        Box box[2];
        int child[2];
    };
    std::vector<Node> nodes;
    uint32_t max_depth = 0;
    // > 0: every leaf at a depth <= depth_limit (root = 1).  Each split then keeps both sides within what a
    // subtree of the remaining depth can hold (leaf_max << levels left), choosing the best SAH split among those.
    uint32_t depth_limit = 0;

    Box range_box(int b, int e) const {
        Box r;
        r.empty();
        for (int i = b; i < e; i++) r.grow(prims[order[i]].box);
        return r;
    }

    // leaf reference: ~(first << 2 | (count - 1)), count in 1..4 (rt_internal.h)
    int make_leaf(int b, int e) const { return ~((b << 2) | (e - b - 1)); }

    // Returns the child reference for [b, e).
    int build(int b, int e, uint32_t depth) {
        int n = e - b;
        if (depth > max_depth) max_depth = depth;
        const bool must_split = depth == 1;  // the root is always an internal node (see build_root)
        if (n <= 1 && !must_split) return make_leaf(b, e);
        int lo_split = 1, hi_split = n - 1;  // allowed left-side sizes
        if (depth_limit) {
            if (depth >= depth_limit) return make_leaf(b, e);  // n <= leaf_max here by the capacities above
            const int64_t cap = (int64_t)leaf_max << (depth_limit - depth - 1);
            lo_split = (int)std::max<int64_t>(1, n - cap);
            hi_split = (int)std::min<int64_t>(n - 1, cap);
        }
        // Full-sweep SAH over the three centroid axes.
        float best_cost = INFINITY;
        int best_axis = -1, best_split = -1;
        std::vector<int> tmp(order.begin() + b, order.begin() + e);
        std::vector<float> right_area(n);
        for (int axis = 0; axis < 3; axis++) {
            std::stable_sort(tmp.begin(), tmp.end(), [&](int x, int y) {
                return prims[x].centroid[axis] < prims[y].centroid[axis];
            });
            Box acc;
            acc.empty();
            for (int i = n - 1; i > 0; i--) {
                acc.grow(prims[tmp[i]].box);
                right_area[i] = acc.area();
            }
            acc.empty();
            for (int i = 1; i < n; i++) {
                acc.grow(prims[tmp[i - 1]].box);
                if (i < lo_split || i > hi_split) continue;
                float cost = acc.area() * (float)i + right_area[i] * (float)(n - i);
                if (cost < best_cost) { best_cost = cost; best_axis = axis; best_split = i; }
            }
        }
        Box all = range_box(b, e);
        float leaf_cost = all.area() * (float)n;
        if (!must_split && n <= leaf_max && best_cost + traversal * all.area() >= leaf_cost) return make_leaf(b, e);
        if (best_axis < 0) {  // every candidate cost overflowed (boxes at the end of the float range): object median
            best_axis = 0;
            best_split = std::min(std::max(n / 2, lo_split), hi_split);
        }
        std::stable_sort(order.begin() + b, order.begin() + e, [&](int x, int y) {
            return prims[x].centroid[best_axis] < prims[y].centroid[best_axis];
        });
        int mid = b + best_split;
        int id = (int)nodes.size();
        nodes.push_back(Node());
        int l = build(b, mid, depth + 1);
        int r = build(mid, e, depth + 1);
        nodes[id].child[0] = l;
        nodes[id].child[1] = r;
        nodes[id].box[0] = range_box(b, mid);
        nodes[id].box[1] = range_box(mid, e);
        return id;
    }

    void build_root() {
        nodes.clear();
        max_depth = 0;
        int n = (int)prims.size();
        order.resize(n);
        std::iota(order.begin(), order.end(), 0);
        if (n == 0) return;
        if (n == 1) {
            // Root with both children referencing the single leaf (a second test of the same primitive
            // cannot change the closest hit: Sphere::Hit is strict in t_max, rects re-accept the same t).
            nodes.push_back(Node());
            nodes[0].child[0] = nodes[0].child[1] = make_leaf(0, 1);
            nodes[0].box[0] = nodes[0].box[1] = prims[0].box;
            max_depth = 2;
            return;
        }
        max_depth = 1;
        int r = build(0, n, 1);
        (void)r;  // n >= 2 always yields an internal root at index 0
    }
};

// The 32-B primitive record (rt_internal.h).
void pack_prim(const rt_hittable_desc& h, float* o) {
    uint32_t tag = (uint32_t)h.type | ((uint32_t)h.material << 4);
    if (h.type == RT_SPHERE) {
        o[0] = h.center[0]; o[1] = h.center[1]; o[2] = h.center[2]; o[3] = h.radius;
        // o[5]: RN(1/radius) for the kernel's fast normal division (render.hip divs_rn), 0 = IEEE division
        const float ar = std::fabs(h.radius);
        o[4] = h.radius * h.radius; o[5] = (ar >= 0x1p-40f && ar <= 0x1p40f) ? 1.0f / h.radius : 0.0f; o[6] = 0.0f;
    } else {
        RectGeom g = rect_geom(h);
        o[0] = g.k; o[1] = g.a0; o[2] = g.a1; o[3] = g.b0;
        o[4] = g.b1; o[5] = 0.0f; o[6] = 0.0f;
    }
    o[7] = bits_to_float(tag);
}

// The reference BVH over objs[b, e) exactly as the BVHNode constructor builds it (Hittable.cuh:303-385): the range is
// sorted by type; a span of 1 or 2 becomes a node with primitive children (a span-1 node holds its object twice), a
// larger span splits at the end of the first type group (or in the middle) into two node children.  Node boxes are
// the reference's: primitive boxes (Hittable.cuh:112-116, 171-181, 227-237, 283-293, not padded further) merged by
// SurroundingBox (AABB.cuh:53-62).  Children: >= 0 node index, < 0 ~(desc index).  Returns the node index.
struct RefNode {
    float lo[3], hi[3];
    int child[2];
    uint32_t depth;
};
void ref_prim_box(const rt_hittable_desc& h, float lo[3], float hi[3]) {
    if (h.type == RT_SPHERE) {
        for (int i = 0; i < 3; i++) {
            volatile float c = h.center[i], r = h.radius;
            lo[i] = c - r;
            hi[i] = c + r;
        }
        return;
    }
    RectGeom g = rect_geom(h);
    lo[g.ia] = g.a0; hi[g.ia] = g.a1;
    lo[g.ib] = g.b0; hi[g.ib] = g.b1;
    volatile float k = g.k;
    lo[g.ik] = k - 0.0001f;
    hi[g.ik] = k + 0.0001f;
}

// The flat kernels' exactness check (render.hip flat_trace) per flat record: (lo.xyz, kl), (hi.xyz, kh) — the record's
// own reference box, except that a rectangle's plane axis holds 1e30 in lo/hi (its faces are checked through the
// slab distances instead, kl / kh = k -/+ 0.0001f as AABB::Hit has them) and a sphere's kl / kh are NaN (no plane).
void pack_flat_box(const rt_hittable_desc& h, float* o) {
    float lo[3], hi[3];
    ref_prim_box(h, lo, hi);
    float kl = std::numeric_limits<float>::quiet_NaN(), kh = kl;
    if (h.type != RT_SPHERE) {
        const RectGeom g = rect_geom(h);
        kl = lo[g.ik];
        kh = hi[g.ik];
        lo[g.ik] = hi[g.ik] = 1e30f;
    }
    o[0] = lo[0]; o[1] = lo[1]; o[2] = lo[2]; o[3] = kl;
    o[4] = hi[0]; o[5] = hi[1]; o[6] = hi[2]; o[7] = kh;
}
// The BVH kernels' exactness check (render.hip bvh_clear) per BVH-order primitive: (lo.xyz, 0), (hi.xyz, 0) — its own
// reference box as the reference's BoundingBox computes it (the innermost box on its path through the reference tree)
void pack_ref_box(const rt_hittable_desc& h, float* o) {
    float lo[3], hi[3];
    ref_prim_box(h, lo, hi);
    o[0] = lo[0]; o[1] = lo[1]; o[2] = lo[2]; o[3] = 0.0f;
    o[4] = hi[0]; o[5] = hi[1]; o[6] = hi[2]; o[7] = 0.0f;
}
int build_reference_tree(const rt_hittable_desc* h, std::vector<int>& objs, int b, int e, uint32_t depth,
                         std::vector<RefNode>* nodes) {
    const int id = (int)nodes->size();
    nodes->push_back(RefNode());
    // (a range already in type order — every range below the root, whose sort left it so — is its own stable sort:
    // skipped, so a scene of n primitives builds in O(n log n))
    const auto by_type = [&](int x, int y) { return h[x].type < h[y].type; };
    if (!std::is_sorted(objs.begin() + b, objs.begin() + e, by_type))
        std::stable_sort(objs.begin() + b, objs.begin() + e, by_type);
    const int span = e - b;
    int c0, c1;
    if (span <= 2) {
        c0 = ~objs[b];
        c1 = ~objs[span == 1 ? b : b + 1];
    } else {
        int mid = b;
        while (mid < e && h[objs[mid]].type == h[objs[b]].type) mid++;
        if (mid == b || mid == e) mid = b + span / 2;
        c0 = build_reference_tree(h, objs, b, mid, depth + 1, nodes);
        c1 = build_reference_tree(h, objs, mid, e, depth + 1, nodes);
    }
    float lo[2][3], hi[2][3];
    const int ch[2] = {c0, c1};
    for (int k = 0; k < 2; k++) {
        if (ch[k] >= 0) {
            for (int i = 0; i < 3; i++) { lo[k][i] = (*nodes)[ch[k]].lo[i]; hi[k][i] = (*nodes)[ch[k]].hi[i]; }
        } else {
            ref_prim_box(h[~ch[k]], lo[k], hi[k]);
        }
    }
    RefNode& n = (*nodes)[id];
    for (int i = 0; i < 3; i++) {
        n.lo[i] = std::fmin(lo[0][i], lo[1][i]);
        n.hi[i] = std::fmax(hi[0][i], hi[1][i]);
    }
    n.child[0] = c0;
    n.child[1] = c1;
    n.depth = depth;
    return id;
}

// BVHNode::Hit (Hittable.cuh:387-439) pops the right child before the left one: the order in which it tests the
// primitives, box culling aside (culling skips primitives, never reorders them).
void reference_test_order(const std::vector<RefNode>& nodes, int n, std::vector<int>* out) {
    const RefNode& r = nodes[n];
    if (r.child[0] < 0) {
        out->push_back(~r.child[0]);
        if (r.child[1] != r.child[0]) out->push_back(~r.child[1]);
        return;
    }
    reference_test_order(nodes, r.child[1], out);
    reference_test_order(nodes, r.child[0], out);
}

int check_texture(const rt_texture_desc& t, uint32_t num_images, std::string* err) {
    if (t.type < RT_CONSTANT || t.type > RT_IMAGE) {
        *err = "texture type " + std::to_string(t.type) + " is not CONSTANT/CHECKER/IMAGE";
        return RT_ERR_INVALID_SCENE;
    }
    if (t.type == RT_IMAGE && (t.image < -1 || t.image >= (int32_t)num_images)) {
        *err = "image texture index " + std::to_string(t.image) + " out of range";
        return RT_ERR_INVALID_SCENE;
    }
    return RT_OK;
}

}  // namespace

thread_local int g_leaf_max = kLeafMax;
thread_local int g_sah_traversal_x10 = 16;  // 1.6: C3 −4.4 %, C2 −0.4 % against 1.2 (profiles/r02e_ab_sah.txt)
thread_local int g_texel_bytes = 3;

int pack_materials(const rt_material_desc* mats, uint32_t n, uint32_t num_images, std::vector<float>* out,
                   std::string* err) {
    out->assign((size_t)n * 12, 0.0f);
    for (uint32_t i = 0; i < n; i++) {
        const rt_material_desc& m = mats[i];
        if (m.type < RT_LAMBERTIAN || m.type > RT_DIFFUSELIGHT) {
            *err = "material " + std::to_string(i) + ": type " + std::to_string(m.type) + " invalid";
            return RT_ERR_INVALID_SCENE;
        }
        if (m.type != RT_DIELECTRIC) {
            int rc = check_texture(m.albedo, num_images, err);
            if (rc) { *err = "material " + std::to_string(i) + ": " + *err; return rc; }
        }
        float* o = out->data() + (size_t)i * 12;
        uint32_t tex_type = m.type == RT_DIELECTRIC ? 0u : (uint32_t)m.albedo.type;
        o[0] = bits_to_float((uint32_t)m.type | (tex_type << 4));
        o[1] = m.type == RT_METAL ? m.fuzz : (m.type == RT_DIELECTRIC ? m.ir : 0.0f);
        o[2] = (float)m.light_intensity;  // `light_intensity * value`: int → float (Material.cuh:168)
        int32_t img = m.albedo.type == RT_IMAGE ? m.albedo.image : -1;
        o[3] = bits_to_float((uint32_t)img);
        for (int c = 0; c < 3; c++) {
            o[4 + c] = m.albedo.color[c];
            o[8 + c] = m.albedo.color2[c];
        }
        if (m.type == RT_DIELECTRIC) {
            // ir-only terms of Dielectric::Scatter, with the kernel's binary32 operations (this file is
            // compiled -ffp-contract=off): 1.0f / ir (Material.cuh:124) and Reflectance's r0² (:142-143)
            volatile float ir = m.ir;
            volatile float inv = 1.0f / ir;
            volatile float r0 = (1.0f - ir) / (1.0f + ir);
            volatile float r0sq = r0 * r0;
            o[4] = inv;
            o[5] = r0sq;
            o[6] = 0.0f;
        }
    }
    return RT_OK;
}

int build_host_scene(const rt_scene_desc* desc, HostScene* out, std::string* err, bool with_texels) {
    if (!desc) { *err = "scene description is NULL"; return RT_ERR_INVALID_ARGUMENT; }
    if ((desc->num_hittables && !desc->hittables) || (desc->num_materials && !desc->materials) ||
        (desc->num_images && !desc->images)) {
        *err = "scene description has a NULL array with a non-zero count";
        return RT_ERR_INVALID_ARGUMENT;
    }
    *out = HostScene();
    int rc = pack_materials(desc->materials, desc->num_materials, desc->num_images, &out->mats, err);
    if (rc) return rc;
    out->num_mats = desc->num_materials;
    for (uint32_t i = 0; i < desc->num_materials; i++)
        if (desc->materials[i].type != RT_DIELECTRIC && desc->materials[i].albedo.type == RT_IMAGE)
            out->has_image_textures = true;
    for (uint32_t i = 0; i < desc->num_materials; i++)
        if (desc->materials[i].type != RT_DIELECTRIC && desc->materials[i].albedo.type != RT_CONSTANT)
            out->has_textures = true;

    // images: RGB8, 3 bytes per texel (Texture.cuh:76); data == NULL means "no data" (Texture.cuh:83-84)
    size_t off = 0;
    for (uint32_t i = 0; i < desc->num_images; i++) {
        const rt_image_desc& im = desc->images[i];
        if (im.width < 0 || im.height < 0) {
            *err = "image " + std::to_string(i) + ": negative width or height";
            return RT_ERR_INVALID_SCENE;
        }
        const uint64_t texels = (uint64_t)im.width * (uint64_t)im.height;
        if (im.data && texels > (uint64_t)1 << 31) {  // the kernel indexes texel bytes with 64-bit offsets
            *err = "image " + std::to_string(i) + ": more than 2^31 texels";
            return RT_ERR_INVALID_SCENE;
        }
        const int bpt = g_texel_bytes == 4 ? 4 : 3;
        const size_t bytes = im.data ? (size_t)texels * (size_t)bpt : 0;
        if (bytes && off + bytes > (size_t)INT32_MAX) {  // imgs[] holds 32-bit byte offsets
            *err = "images exceed 2 GiB of texels in one scene";
            return RT_ERR_INVALID_SCENE;
        }
        out->imgs.push_back(bytes ? (int32_t)off : -1);
        out->imgs.push_back(im.width);
        out->imgs.push_back(im.height);
        out->imgs.push_back(bpt);
        // (each image is followed by at least 4 spare bytes: the kernels gather a texel as one dword, which for the
        // RGB8 layout's last texel reads one byte past it; then 16-B alignment)
        if (bytes && !with_texels) {
            off = (off + bytes + 4 + 15) & ~(size_t)15;
        } else if (bytes) {
            out->texels.resize(off + bytes);
            uint8_t* dst = out->texels.data() + off;
            if (bpt == 3) {
                std::memcpy(dst, im.data, bytes);
            } else {
                for (size_t t = 0; t < (size_t)texels; t++) {
                    dst[4 * t + 0] = im.data[3 * t + 0];
                    dst[4 * t + 1] = im.data[3 * t + 1];
                    dst[4 * t + 2] = im.data[3 * t + 2];
                    dst[4 * t + 3] = 0;
                }
            }
            off += bytes + 4;
            off = (off + 15) & ~(size_t)15;
            out->texels.resize(off, 0);
        }
    }

    Builder B;
    B.leaf_max = g_leaf_max;
    for (uint32_t i = 0; i < desc->num_hittables; i++) {
        const rt_hittable_desc& h = desc->hittables[i];
        if (!h.is_active) continue;  // thrust::remove_if of inactive objects (Hittable.cuh:311-312)
        if (h.type < RT_SPHERE || h.type > RT_YZRECT) {
            *err = "hittable " + std::to_string(i) + ": type " + std::to_string(h.type) + " invalid";
            return RT_ERR_INVALID_SCENE;
        }
        if (h.material < 0 || (uint32_t)h.material >= desc->num_materials) {
            *err = "hittable " + std::to_string(i) + ": material index " + std::to_string(h.material) +
                   " out of range";
            return RT_ERR_INVALID_SCENE;
        }
        // NaN or infinite geometry has no box (the reference's own AABB would poison every ancestor box)
        const bool sphere = h.type == RT_SPHERE;
        if (!std::isfinite(h.center[0]) || !std::isfinite(h.center[1]) || !std::isfinite(h.center[2]) ||
            (sphere ? !std::isfinite(h.radius) : (!std::isfinite(h.width) || !std::isfinite(h.height)))) {
            *err = "hittable " + std::to_string(i) + ": non-finite centre or size";
            return RT_ERR_INVALID_SCENE;
        }
        // A negative radius turns the reference's sphere box inside out (center - r > center + r,
        // Hittable.cuh:114), which its AABB test (AABB.cuh:30-50) never enters while Sphere::Hit still would: whether
        // the reference draws such a sphere depends on its tree shape.  The reference's editor keeps radii in
        // [0, FLT_MAX] (CudaLayer.cpp:496), so the library rejects the case instead of guessing.
        if (sphere && h.radius < 0.0f) {
            *err = "hittable " + std::to_string(i) + ": negative sphere radius";
            return RT_ERR_INVALID_SCENE;
        }
        out->has_rects = out->has_rects || !sphere;
        BuildPrim p;
        p.box = prim_box(h);
        for (int a = 0; a < 3; a++) p.centroid[a] = 0.5f * (p.box.lo[a] + p.box.hi[a]);
        p.src = (int)i;
        B.prims.push_back(p);
    }
    // the kernels address primitives as 32-B records at 32-bit byte offsets, and leaf references hold
    // first << 2 in a signed 32-bit value
    if (B.prims.size() >= ((size_t)1 << 26)) {
        *err = "more than 2^26 active primitives";
        return RT_ERR_INVALID_SCENE;
    }
    B.traversal = (float)g_sah_traversal_x10 / 10.0f;
    B.build_root();
    // Occupancy guard: a tree deeper than kOccupancyDepth costs the compact v3 kernel its 8th wave per SIMD (its
    // LDS stack grows by 128 B per level; C2's tree at depth 13 renders 8 % slower than at 12,
    // profiles/r02e_ab_sah.txt).  Dearer node visits make the SAH stop splitting earlier: retry with 1.5×, 2×,
    // 3× the cost and keep the first tree that fits; if none does, the first tree stays.
    if (B.max_depth > kOccupancyDepth && B.prims.size() > 1) {
        const float base = B.traversal;
        for (const float f : {1.5f, 2.0f, 3.0f}) {
            Builder T = B;
            T.traversal = base * f;
            T.build_root();
            if (T.max_depth <= kOccupancyDepth) {
                B = std::move(T);
                break;
            }
        }
        // still too deep (thousands of primitives): SAH splits under capacity limits that bound the depth — to
        // kOccupancyDepth when the primitives fit its leaves (8192 at leaf size 4: every 16-bit-reference scene),
        // else to one level above the shallowest tree that holds them (the LDS stack grows with the depth)
        uint32_t dmin = 1;
        while (((size_t)B.leaf_max << (dmin - 1)) < B.prims.size()) dmin++;
        const uint32_t target = std::max<uint32_t>(kOccupancyDepth, dmin + (dmin > kOccupancyDepth ? 1u : 0u));
        if (B.max_depth > target) {
            Builder T = B;
            T.traversal = base;
            T.depth_limit = target;
            T.build_root();
            B = std::move(T);
        }
    }
    out->num_prims = (uint32_t)B.prims.size();
    out->num_nodes = (uint32_t)B.nodes.size();
    out->depth = B.max_depth;

    out->nodes.resize((size_t)out->num_nodes * 16);
    for (uint32_t i = 0; i < out->num_nodes; i++) {
        const Builder::Node& n = B.nodes[i];
        float* o = out->nodes.data() + (size_t)i * 16;
        o[0] = n.box[0].lo[0]; o[1] = n.box[0].hi[0]; o[2] = n.box[0].lo[1]; o[3] = n.box[0].hi[1];
        o[4] = n.box[1].lo[0]; o[5] = n.box[1].hi[0]; o[6] = n.box[1].lo[1]; o[7] = n.box[1].hi[1];
        o[8] = n.box[0].lo[2]; o[9] = n.box[0].hi[2]; o[10] = n.box[1].lo[2]; o[11] = n.box[1].hi[2];
        o[12] = bits_to_float((uint32_t)n.child[0]);
        o[13] = bits_to_float((uint32_t)n.child[1]);
        o[14] = 0.0f;
        o[15] = 0.0f;
    }
    // 16-bit references (internal nodes < 0x7fff, leaves ~(first << 2 | count - 1) with first < 8192) unless the
    // tree is too large: then 32-bit ones (the kernels' WIDE builds, render.hip RefW)
    out->wide_refs = !(out->num_nodes < 0x7fffu && out->num_prims < 8192u);
    out->nodes48.resize((size_t)out->num_nodes * 12);
    out->refs.resize((size_t)out->num_nodes * (out->wide_refs ? 2 : 1));
    for (uint32_t i = 0; i < out->num_nodes; i++) {
        float* o48 = out->nodes48.data() + (size_t)i * 12;
        for (int k = 0; k < 12; k++) o48[k] = out->nodes[(size_t)i * 16 + k];
        const Builder::Node& n = B.nodes[i];
        // The child references also ride in the low bytes of the planes (lo_x, hi_x of each child: bits 0-15;
        // wide: lo_y, hi_y: bits 16-31), so a lane's three 16-B box loads carry them and the vector path needs
        // no fourth load (render.hip).  Each carrier plane moves outward by < 512 ulps (lo down, hi up): the box
        // only grows, and the culling stays conservative.
        for (int c = 0; c < 2; c++) {
            const uint32_t r = (uint32_t)n.child[c];
            float* q = o48 + 4 * c;  // lo_x, hi_x, lo_y, hi_y of child c
            q[0] = with_low_byte(q[0], r & 0xffu, false);
            q[1] = with_low_byte(q[1], (r >> 8) & 0xffu, true);
            if (out->wide_refs) {
                q[2] = with_low_byte(q[2], (r >> 16) & 0xffu, false);
                q[3] = with_low_byte(q[3], r >> 24, true);
            }
        }
        if (out->wide_refs) {
            out->refs[2 * (size_t)i] = (uint32_t)n.child[0];
            out->refs[2 * (size_t)i + 1] = (uint32_t)n.child[1];
        } else {
            out->refs[i] = ((uint32_t)n.child[0] & 0xffffu) | ((uint32_t)n.child[1] << 16);
        }
    }
    // (at least one record: the BVH kernels' shade() loads record 0 for a miss before it knows the ray missed, so an
    // empty scene carries one zero record that no traversal reaches)
    out->prims.assign((size_t)std::max(out->num_prims, 1u) * 8, 0.0f);
    out->prim_source.resize(out->num_prims);
    for (uint32_t i = 0; i < out->num_prims; i++) {
        out->prim_source[i] = B.prims[B.order[i]].src;
        pack_prim(desc->hittables[out->prim_source[i]], out->prims.data() + (size_t)i * 8);
    }
    if (out->num_prims == 0) return RT_OK;
    // The reference's own BVH (its boxes and shape, Hittable.cuh:303-385) over the active primitives in list order.
    std::vector<int> objs;
    for (const BuildPrim& p : B.prims) objs.push_back(p.src);
    std::vector<RefNode> rn;
    build_reference_tree(desc->hittables, objs, 0, (int)objs.size(), 1, &rn);
    uint32_t rdepth = 0;
    for (const RefNode& n : rn) rdepth = std::max(rdepth, n.depth);
    // Every scene: the reference BVH with its primitive children as ~(BVH-order index) and, per BVH-order primitive,
    // its reference box — the BVH kernels' exactness check (render.hip bvh_clear): the rare rays whose closest hit the
    // reference's box culling or an exact tie could change replay the reference BVH over the BVH-order records.
    if (rdepth > kRefTreeMaxDepthBvh) {  // (2^26 primitives give <= 30: not reached within the primitive limit above)
        *err = "reference BVH deeper than " + std::to_string(kRefTreeMaxDepthBvh) + " levels";
        return RT_ERR_INVALID_SCENE;
    }
    {
        std::vector<int> bvh_index(desc->num_hittables, -1);
        for (uint32_t i = 0; i < out->num_prims; i++) bvh_index[out->prim_source[i]] = (int)i;
        out->bvh_boxes.resize((size_t)out->num_prims * 8);
        for (uint32_t i = 0; i < out->num_prims; i++)
            pack_ref_box(desc->hittables[out->prim_source[i]], out->bvh_boxes.data() + (size_t)i * 8);
        out->bvh_ref_nodes.resize(rn.size() * 8);
        for (size_t i = 0; i < rn.size(); i++) {
            float* o = out->bvh_ref_nodes.data() + i * 8;
            for (int k = 0; k < 2; k++) {
                const int c = rn[i].child[k];
                const int enc = c >= 0 ? c : ~bvh_index[~c];
                for (int a = 0; a < 3; a++) o[4 * k + a] = k == 0 ? rn[i].lo[a] : rn[i].hi[a];
                o[4 * k + 3] = bits_to_float((uint32_t)enc);
            }
        }
        // the same tree with each node's children's boxes in the node: (lo.xyz, ref), (hi.xyz, 0) per child, so the
        // replay tests both children of a node from one 64-B record and visits only the nodes whose box accepted
        out->bvh_ref_pairs.assign(rn.size() * 16, 0.0f);
        for (size_t i = 0; i < rn.size(); i++) {
            float* o = out->bvh_ref_pairs.data() + i * 16;
            for (int k = 0; k < 2; k++) {
                const int c = rn[i].child[k];
                const int enc = c >= 0 ? c : ~bvh_index[~c];
                if (c >= 0)
                    for (int a = 0; a < 3; a++) {
                        o[8 * k + a] = rn[c].lo[a];
                        o[8 * k + 4 + a] = rn[c].hi[a];
                    }
                o[8 * k + 3] = bits_to_float((uint32_t)enc);
            }
        }
    }
    // Small scenes: the primitives once more, in the order the reference's own BVH tests them (the flat kernel,
    // render.hip, tests every primitive of every ray in this order, so its closest hit breaks exact ties in t as
    // the reference's does)
    // together with the reference's own BVH (ref_nodes: its boxes and shape), which the flat kernel replays exactly
    // for the rare rays whose closest hit lies on a box face or ties (render.hip, ref_trace)
    if (out->num_prims <= kFlatMaxPrims) {
        if (rdepth <= kRefTreeMaxDepth) {
            std::vector<int> ord;
            reference_test_order(rn, 0, &ord);
            std::vector<int> flat_index(desc->num_hittables, -1);
            out->prims_flat.resize(ord.size() * 8);
            out->flat_boxes.resize(ord.size() * 8);
            for (size_t i = 0; i < ord.size(); i++) {
                flat_index[ord[i]] = (int)i;
                pack_prim(desc->hittables[ord[i]], out->prims_flat.data() + i * 8);
                pack_flat_box(desc->hittables[ord[i]], out->flat_boxes.data() + i * 8);
            }
            // the flat kernels scan one primitive type at a time (no per-primitive type branch): the reference test
            // order keeps each type contiguous (the tree splits at type-group boundaries, BVHNode's type sort); a
            // scene where it would not (never seen) simply does not get the flat kernels
            uint32_t runs[4][2] = {{0u, 0u}, {0u, 0u}, {0u, 0u}, {0u, 0u}};
            bool contiguous = true;
            for (size_t i = 0; i < ord.size();) {
                const int ty = desc->hittables[ord[i]].type;
                size_t j = i;
                while (j < ord.size() && desc->hittables[ord[j]].type == ty) j++;
                if (runs[ty][1] != 0u) contiguous = false;  // a second run of the same type
                runs[ty][0] = (uint32_t)i;
                runs[ty][1] = (uint32_t)j;
                i = j;
            }
            for (int ty = 0; ty < 4; ty++) {
                const uint32_t v = runs[ty][0] | (runs[ty][1] << 8);
                out->flat_runs[ty / 2] |= v << (16 * (ty % 2));
            }
            if (!contiguous) {
                out->prims_flat.clear();
                out->flat_boxes.clear();
                out->flat_runs[0] = out->flat_runs[1] = 0u;
                return RT_OK;
            }
            // per node: (lo.xyz, child 0) (hi.xyz, child 1); a primitive child is ~(its flat index)
            out->ref_nodes.resize(rn.size() * 8);
            for (size_t i = 0; i < rn.size(); i++) {
                float* o = out->ref_nodes.data() + i * 8;
                for (int k = 0; k < 2; k++) {
                    const int c = rn[i].child[k];
                    const int enc = c >= 0 ? c : ~flat_index[~c];
                    for (int a = 0; a < 3; a++) o[4 * k + a] = k == 0 ? rn[i].lo[a] : rn[i].hi[a];
                    o[4 * k + 3] = bits_to_float((uint32_t)enc);
                }
            }
            // ... and as child-pair records (bvh_ref_pairs' layout) for the wave-serial replay (ref_trace_wave)
            out->flat_ref_pairs.assign(rn.size() * 16, 0.0f);
            for (size_t i = 0; i < rn.size(); i++) {
                float* o = out->flat_ref_pairs.data() + i * 16;
                for (int k = 0; k < 2; k++) {
                    const int c = rn[i].child[k];
                    const int enc = c >= 0 ? c : ~flat_index[~c];
                    if (c >= 0)
                        for (int a = 0; a < 3; a++) {
                            o[8 * k + a] = rn[c].lo[a];
                            o[8 * k + 4 + a] = rn[c].hi[a];
                        }
                    o[8 * k + 3] = bits_to_float((uint32_t)enc);
                }
            }
        }
    }
    return RT_OK;
}

}  // namespace rt
