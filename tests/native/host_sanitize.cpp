// host_sanitize.cpp — drives librt_hip.so's host code (scene validation + BVH build, the reference-graph
// flattener, the built-in scenes and textures, the PPM writer, the device-facing entry points' error paths)
// in an AddressSanitizer + UndefinedBehaviorSanitizer build (sanitizers on the host code).
// Built and run by `make -C cudaraytracer_amd/csrc asan` (tests/test_sanitize.py); no GPU is needed: the
// device calls fail cleanly and must come back as status codes.  Exit status 0 = every check held and the
// sanitizers reported nothing (they abort the process on the first report).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt_hip.h"
#include "../../include/rt_reference_graph.h"
#include "../../cudaraytracer_amd/csrc/rt_internal.h"

static int failures = 0;
#define CHECK(cond)                                                                  \
    do {                                                                             \
        if (!(cond)) {                                                               \
            std::fprintf(stderr, "CHECK failed at line %d: %s (%s)\n", __LINE__, #cond, \
                         rt_last_error());                                           \
            failures++;                                                              \
        }                                                                            \
    } while (0)

static std::vector<float> tables(const rt_scene_desc& d, rt_host_tables_info* info, int* rc) {
    *rc = rt_build_host_tables(&d, nullptr, nullptr, nullptr, nullptr, info);
    if (*rc) return {};
    std::vector<float> nodes((size_t)info->num_nodes * 16 + 1), prims((size_t)info->num_prims * 8 + 1),
        mats((size_t)info->num_materials * 12 + 1);
    std::vector<int32_t> src(info->num_prims + 1);
    *rc = rt_build_host_tables(&d, nodes.data(), prims.data(), mats.data(), src.data(), info);
    return nodes;
}

static void builtin_scenes() {
    for (int which = 0; which < 5; which++) {
        uint32_t nh = 0, nm = 0;
        CHECK(rt_builtin_scene(which, 1, nullptr, &nh, nullptr, &nm) == RT_OK);
        std::vector<rt_hittable_desc> h(nh);
        std::vector<rt_material_desc> m(nm);
        uint32_t small = nh ? nh - 1 : 0;  // too-small arrays are refused, never overrun
        if (nh > 1) CHECK(rt_builtin_scene(which, 1, h.data(), &small, m.data(), &nm) == RT_ERR_INVALID_ARGUMENT);
        CHECK(rt_builtin_scene(which, 1, h.data(), &nh, m.data(), &nm) == RT_OK);
        std::vector<std::vector<uint8_t>> px;
        std::vector<rt_image_desc> imgs;
        if (which == 4)
            for (int k = 0; k < 3; k++) {
                px.emplace_back((size_t)64 * 32 * 3);
                CHECK(rt_procedural_texture(k, 64, 32, px.back().data()) == RT_OK);
                imgs.push_back(rt_image_desc{px.back().data(), 64, 32});
            }
        rt_scene_desc d{h.data(), nh, m.data(), nm, imgs.data(), (uint32_t)imgs.size()};
        rt_host_tables_info info{};
        int rc = 0;
        tables(d, &info, &rc);
        CHECK(rc == RT_OK);
        for (uint32_t i = 0; i < nh; i += 3) h[i].is_active = 0;  // drop a third of the objects
        tables(d, &info, &rc);
        CHECK(rc == RT_OK);
        for (uint32_t i = 0; i < nh; i++) h[i].is_active = 0;  // empty scene
        tables(d, &info, &rc);
        CHECK(rc == RT_OK && info.num_nodes == 0);
        rt_scene* s = nullptr;
        CHECK(rt_scene_create(&d, &s) != RT_OK || s != nullptr);  // no device here: a status, not a crash
        if (s) rt_scene_destroy(s);
    }
}

static void invalid_scenes() {
    uint32_t nh = 8, nm = 8;
    rt_hittable_desc h[8];
    rt_material_desc m[8];
    CHECK(rt_builtin_scene(1, 1, h, &nh, m, &nm) == RT_OK);
    uint8_t texel[3] = {1, 2, 3};
    rt_image_desc img{texel, 1, 1};
    rt_scene_desc d{h, nh, m, nm, &img, 1};
    rt_host_tables_info info{};
    int rc = 0;
    img.width = -4;  // negative size
    tables(d, &info, &rc);
    CHECK(rc == RT_ERR_INVALID_SCENE);
    img.width = 1 << 30, img.height = 1 << 30;  // 2^60 texels: refused before any copy
    tables(d, &info, &rc);
    CHECK(rc == RT_ERR_INVALID_SCENE);
    img = rt_image_desc{texel, 1, 1};
    m[0].albedo.type = RT_IMAGE;
    m[0].albedo.image = -5;  // below the "no data" index -1
    tables(d, &info, &rc);
    CHECK(rc == RT_ERR_INVALID_SCENE);
    m[0].albedo.image = -1;  // "no data": valid
    tables(d, &info, &rc);
    CHECK(rc == RT_OK);
    m[0].albedo.image = 1;  // past the image table
    tables(d, &info, &rc);
    CHECK(rc == RT_ERR_INVALID_SCENE);
    m[0].albedo.image = 0;
    h[1].material = 77;
    tables(d, &info, &rc);
    CHECK(rc == RT_ERR_INVALID_SCENE);
    h[1].material = 0;
    h[2].type = 9;
    tables(d, &info, &rc);
    CHECK(rc == RT_ERR_INVALID_SCENE);
    rt_scene_desc nulls{nullptr, 3, m, nm, nullptr, 0};
    tables(nulls, &info, &rc);
    CHECK(rc == RT_ERR_INVALID_ARGUMENT);
    CHECK(rt_build_host_tables(nullptr, nullptr, nullptr, nullptr, nullptr, &info) == RT_ERR_INVALID_ARGUMENT);
}

// A reference graph: BVHNode(left = sphere, right = BVHNode(rect, sphere)), textures of every kind.
static void reference_graph() {
    rtref_constant red{{{0.8f, 0.1f, 0.1f}}, 0.0f}, white{{{0.9f, 0.9f, 0.9f}}, 0.0f};
    rtref_checker chk{&red, &white};
    std::vector<uint8_t> px(16 * 8 * 3, 200);
    rtref_image im{px.data(), "x.jpg", 16, 8, 48};
    void* u_red = &red;
    void* u_chk = &chk;
    void* u_im = &im;
    rtref_texture t_red{RT_CONSTANT, &u_red}, t_chk{RT_CHECKER, &u_chk}, t_im{RT_IMAGE, &u_im};
    rtref_lambertian lam{&t_chk};
    rtref_metal met{&t_red, 0.2f};
    rtref_diffuse_light light{&t_im, 4};
    void* u_lam = &lam;
    void* u_met = &met;
    void* u_light = &light;
    rtref_material m_lam{RT_LAMBERTIAN, &u_lam}, m_met{RT_METAL, &u_met}, m_light{RT_DIFFUSELIGHT, &u_light};
    rtref_sphere s0{{{0, 0, -1}}, 0.5f, &m_lam}, s1{{{1, 0, -1}}, 0.5f, &m_light};
    rtref_rect r0{{{0, -0.5f, 0}}, 10.0f, 10.0f, &m_met};
    void* u_s0 = &s0;
    void* u_s1 = &s1;
    void* u_r0 = &r0;
    rtref_hittable h_s0{RTREF_SPHERE, 1, {}, &u_s0}, h_s1{RTREF_SPHERE, 1, {}, &u_s1}, h_r0{RTREF_XZRECT, 1, {}, &u_r0};
    rtref_bvh_node inner{{}, &h_r0, &h_s1, nullptr};
    void* u_inner = &inner;
    rtref_hittable h_inner{RTREF_BVHNODE, 1, {}, &u_inner};
    rtref_bvh_node root{{}, &h_s0, &h_inner, nullptr};
    void* u_root = &root;
    rtref_hittable world{RTREF_BVHNODE, 1, {}, &u_root};
    uint32_t nh = 0, nm = 0, ni = 0;
    CHECK(rt_reference_graph_flatten(&world, nullptr, &nh, nullptr, &nm, nullptr, &ni) == RT_OK);
    CHECK(nh == 3 && nm == 3 && ni == 1);
    std::vector<rt_hittable_desc> h(nh);
    std::vector<rt_material_desc> m(nm);
    std::vector<rt_image_desc> i(ni);
    uint32_t small = 1;
    CHECK(rt_reference_graph_flatten(&world, h.data(), &small, m.data(), &nm, i.data(), &ni) == RT_ERR_INVALID_ARGUMENT);
    CHECK(rt_reference_graph_flatten(&world, h.data(), &nh, m.data(), &nm, i.data(), &ni) == RT_OK);
    rt_scene_desc d{h.data(), nh, m.data(), nm, i.data(), ni};
    rt_host_tables_info info{};
    int rc = 0;
    tables(d, &info, &rc);
    CHECK(rc == RT_OK && info.num_prims == 3);
    // span-1 leaves reference one object twice (Hittable.cuh:326-327): collected once
    rtref_bvh_node twin{{}, &h_s0, &h_s0, nullptr};
    void* u_twin = &twin;
    rtref_hittable w2{RTREF_BVHNODE, 1, {}, &u_twin};
    CHECK(rt_reference_graph_flatten(&w2, nullptr, &nh, nullptr, &nm, nullptr, &ni) == RT_OK && nh == 1);
    // a cycle (a node that contains itself) terminates
    rtref_bvh_node loop{{}, &h_s0, nullptr, nullptr};
    void* u_loop = &loop;
    rtref_hittable w3{RTREF_BVHNODE, 1, {}, &u_loop};
    loop.right = &w3;
    CHECK(rt_reference_graph_flatten(&w3, nullptr, &nh, nullptr, &nm, nullptr, &ni) == RT_OK && nh == 1);
    // broken graphs are refused: NULL object, NULL material, unknown types, non-BVH world
    void* u_null = nullptr;
    rtref_hittable broken{RTREF_SPHERE, 1, {}, &u_null};
    rtref_bvh_node bad{{}, &broken, &h_s0, nullptr};
    void* u_bad = &bad;
    rtref_hittable w4{RTREF_BVHNODE, 1, {}, &u_bad};
    CHECK(rt_reference_graph_flatten(&w4, nullptr, &nh, nullptr, &nm, nullptr, &ni) == RT_ERR_INVALID_SCENE);
    rtref_sphere nomat{{{0, 0, 0}}, 1.0f, nullptr};
    void* u_nomat = &nomat;
    rtref_hittable h_nomat{RTREF_SPHERE, 1, {}, &u_nomat};
    bad.left = &h_nomat;
    CHECK(rt_reference_graph_flatten(&w4, nullptr, &nh, nullptr, &nm, nullptr, &ni) == RT_ERR_INVALID_SCENE);
    m_lam.type = 42;
    CHECK(rt_reference_graph_flatten(&world, nullptr, &nh, nullptr, &nm, nullptr, &ni) == RT_ERR_INVALID_SCENE);
    m_lam.type = RT_LAMBERTIAN;
    t_chk.type = 7;
    CHECK(rt_reference_graph_flatten(&world, nullptr, &nh, nullptr, &nm, nullptr, &ni) == RT_ERR_INVALID_SCENE);
    t_chk.type = RT_CHECKER;
    CHECK(rt_reference_graph_flatten(&h_s0, nullptr, &nh, nullptr, &nm, nullptr, &ni) == RT_ERR_INVALID_SCENE);
    CHECK(rt_reference_graph_flatten(nullptr, nullptr, &nh, nullptr, &nm, nullptr, &ni) == RT_ERR_INVALID_ARGUMENT);
    // the device paths: no GPU in the sanitizer run, so they must fail with a status (never crash)
    rt_scene* s = nullptr;
    const int rs = rt_scene_from_reference_graph(&world, &s);
    CHECK(rs == RT_OK ? s != nullptr : s == nullptr);
    if (s) rt_scene_destroy(s);
}

static void outputs_and_misc() {
    std::vector<uint32_t> img(7 * 5);
    for (size_t i = 0; i < img.size(); i++) img[i] = 0xff000000u | (uint32_t)(i * 2654435761u & 0xffffffu);
    const std::string path = std::string(std::getenv("TMPDIR") ? std::getenv("TMPDIR") : "/tmp") + "/rt_sanitize.ppm";
    CHECK(rt_write_ppm(path.c_str(), img.data(), 7, 5, 1) == RT_OK);
    FILE* f = std::fopen(path.c_str(), "rb");
    CHECK(f != nullptr);
    if (f) {
        char buf[128];
        const size_t n = std::fread(buf, 1, sizeof(buf), f);
        std::fclose(f);
        CHECK(n == 11 + 7 * 5 * 3);  // "P6\n7 5\n255\n" + pixels
        // first file row = last buffer row (upright image)
        CHECK((uint8_t)buf[11] == (img[4 * 7] & 0xffu));
    }
    std::remove(path.c_str());
    CHECK(rt_write_ppm(nullptr, img.data(), 7, 5, 0) == RT_ERR_INVALID_ARGUMENT);
    CHECK(rt_procedural_texture(3, 8, 8, nullptr) == RT_ERR_INVALID_ARGUMENT);
    rt_glibc_rand g;
    rt_glibc_srand(&g, 1);
    for (int i = 0; i < 1000; i++) CHECK(rt_glibc_rand_next(&g) >= 0);
    float pos[3] = {0, 2, 12}, fwd[3] = {0, 0, -1}, up[3] = {0, 1, 0}, bg[3] = {1, 1, 1};
    rt_input_struct in;
    rt_camera_inputs(pos, fwd, up, 45.0f, 0.1f, 10.0f, bg, bg, &in);
    CHECK(in.up[1] == -1.0f);
    CHECK(rt_set_tuning(99, 1) == RT_ERR_INVALID_ARGUMENT);
    CHECK(rt_set_tuning(RT_TUNE_TEXEL_LAYOUT, 5) == RT_ERR_INVALID_ARGUMENT);
    CHECK(rt_set_tuning(RT_TUNE_QUEUE_CHUNK, 96) == RT_ERR_INVALID_ARGUMENT);
    CHECK(rt_set_tuning(RT_TUNE_QUEUE_STRIDE, 192) == RT_ERR_INVALID_ARGUMENT);
    CHECK(rt_set_tuning(RT_TUNE_QUEUE_STRIDE, 8192) == RT_ERR_INVALID_ARGUMENT);
    CHECK(rt_set_tuning(RT_TUNE_QUEUE_CHUNK, 192) == 128 && rt_set_tuning(RT_TUNE_QUEUE_CHUNK, 128) == 192);
    CHECK(rt_set_tuning(RT_TUNE_QUEUE_STRIDE, 4096) == 128 && rt_set_tuning(RT_TUNE_QUEUE_STRIDE, 128) == 4096);
    CHECK(rt_render(nullptr, nullptr, nullptr) == RT_ERR_INVALID_ARGUMENT);
    const int dev0 = 0;
    rt_tiled_desc td{&dev0, 1, 16, 64, 32, 0, 0, 1984};
    rt_tiled* t = nullptr;
    uint32_t n3 = 8, m3 = 8;
    rt_hittable_desc h[8];
    rt_material_desc m[8];
    CHECK(rt_builtin_scene(1, 1, h, &n3, m, &m3) == RT_OK);
    rt_scene_desc d{h, n3, m, m3, nullptr, 0};
    const int rc = rt_tiled_create(&td, &d, &t);
    CHECK(rc == RT_OK ? t != nullptr : t == nullptr);
    if (t) rt_tiled_destroy(t);
    CHECK(rt_tiled_create(nullptr, &d, &t) == RT_ERR_INVALID_ARGUMENT);
    // creation flags: only the RNG mode; STATE_SOA would make the ranks read their struct states as planes
    rt_tiled_desc bad = td;
    bad.flags = RT_FLAG_STATE_SOA;
    CHECK(rt_tiled_create(&bad, &d, &t) == RT_ERR_INVALID_ARGUMENT);
    bad = td;
    bad.reserved = 1;
    CHECK(rt_tiled_create(&bad, &d, &t) == RT_ERR_INVALID_ARGUMENT);
    CHECK(rt_tiled_render(nullptr, nullptr, nullptr) == RT_ERR_INVALID_ARGUMENT);
    CHECK(rt_gl_register_texture(0, 0x0DE1, nullptr) == RT_ERR_INVALID_ARGUMENT);
}

// The v3 node table carries each node's two 16-bit child references in the low bytes of its x planes
// (scene_build.cpp, render.hip's vector path): the decoded references equal refs16, and every carrier plane
// moved outward (lo down, hi up) by under 512 ulps, so the boxes only grew.
static void node_reference_payload() {
    uint32_t checked = 0;
    for (int which = 0; which < 6; which++) {
        uint32_t nh = 0, nm = 0;
        if (rt_builtin_scene(which, 1, nullptr, &nh, nullptr, &nm) != RT_OK) continue;
        std::vector<rt_hittable_desc> h(nh);
        std::vector<rt_material_desc> m(nm);
        CHECK(rt_builtin_scene(which, 1, h.data(), &nh, m.data(), &nm) == RT_OK);
        rt_scene_desc d{};
        d.hittables = h.data();
        d.num_hittables = nh;
        d.materials = m.data();
        d.num_materials = nm;
        rt::HostScene hs;
        std::string err;
        if (rt::build_host_scene(&d, &hs, &err, false) != RT_OK) continue;  // scenes needing images
        for (uint32_t i = 0; i < hs.num_nodes; i++) {
            const float* o = hs.nodes.data() + (size_t)i * 16;
            const float* q = hs.nodes48.data() + (size_t)i * 12;
            uint32_t b[4];
            std::memcpy(&b[0], &q[0], 4);
            std::memcpy(&b[1], &q[1], 4);
            std::memcpy(&b[2], &q[4], 4);
            std::memcpy(&b[3], &q[5], 4);
            const uint32_t r = (b[0] & 0xffu) | ((b[1] & 0xffu) << 8) | ((b[2] & 0xffu) << 16) | ((b[3] & 0xffu) << 24);
            CHECK(!hs.wide_refs && r == hs.refs[i]);
            for (int k : {0, 4}) CHECK(q[k] <= o[k] && o[k] - q[k] <= 512.0f * std::fabs(o[k]) * 0x1p-23f + 0x1p-140f);
            for (int k : {1, 5}) CHECK(q[k] >= o[k] && q[k] - o[k] <= 512.0f * std::fabs(o[k]) * 0x1p-23f + 0x1p-140f);
            for (int k : {2, 3, 6, 7, 8, 9, 10, 11}) CHECK(q[k] == o[k]);
            checked++;
        }
    }
    CHECK(checked > 250);  // RTIOW alone has 286 nodes
    // a scene beyond 16-bit references (9000 primitives): 32-bit references, bits 16-31 in the y planes
    {
        const int n = 9000;
        std::vector<rt_hittable_desc> h(n);
        rt_material_desc mat{};
        mat.type = RT_LAMBERTIAN;
        mat.albedo.type = RT_CONSTANT;
        mat.albedo.image = -1;
        for (int i = 0; i < n; i++) {
            h[i] = rt_hittable_desc{};
            h[i].type = RT_SPHERE;
            h[i].is_active = 1;
            h[i].center[0] = (float)(i % 100) - 50.0f;
            h[i].center[1] = 0.5f * (float)((i / 100) % 10);
            h[i].center[2] = -(float)(i / 1000);
            h[i].radius = 0.2f;
        }
        rt_scene_desc d{h.data(), (uint32_t)n, &mat, 1, nullptr, 0};
        rt::HostScene hs;
        std::string err;
        CHECK(rt::build_host_scene(&d, &hs, &err, false) == RT_OK);
        CHECK(hs.wide_refs && hs.refs.size() == 2 * (size_t)hs.num_nodes);
        uint32_t leaves_beyond_16bit = 0;
        for (uint32_t i = 0; i < hs.num_nodes; i++) {
            const float* o = hs.nodes.data() + (size_t)i * 16;
            const float* q = hs.nodes48.data() + (size_t)i * 12;
            for (int c = 0; c < 2; c++) {
                uint32_t b[4];
                for (int k = 0; k < 4; k++) std::memcpy(&b[k], &q[4 * c + k], 4);
                const uint32_t r = (b[0] & 0xffu) | ((b[1] & 0xffu) << 8) | ((b[2] & 0xffu) << 16) | ((b[3] & 0xffu) << 24);
                uint32_t want;
                std::memcpy(&want, &o[12 + c], 4);
                CHECK(r == want && r == hs.refs[2 * (size_t)i + c]);
                if ((int32_t)r < 0 && (~r >> 2) >= 8192u) leaves_beyond_16bit++;
                for (int k : {0, 2}) CHECK(q[4 * c + k] <= o[4 * c + k]);
                for (int k : {1, 3}) CHECK(q[4 * c + k] >= o[4 * c + k]);
            }
        }
        CHECK(leaves_beyond_16bit > 0);
    }
    // a box at the end of the float range: carrier planes stay finite
    rt_material_desc m{};
    m.type = RT_LAMBERTIAN;
    m.albedo.type = RT_CONSTANT;
    m.albedo.image = -1;
    rt_hittable_desc h[2] = {};
    for (int k = 0; k < 2; k++) {
        h[k].type = RT_SPHERE;
        h[k].is_active = 1;
        h[k].center[0] = k ? 3.0e38f : -3.0e38f;
        h[k].radius = 3.0e38f;
    }
    rt_scene_desc d{};
    d.hittables = h;
    d.num_hittables = 2;
    d.materials = &m;
    d.num_materials = 1;
    rt::HostScene hs;
    std::string err;
    CHECK(rt::build_host_scene(&d, &hs, &err, false) == RT_OK);
    for (float v : hs.nodes48) CHECK(!std::isnan(v));
    // NaN geometry is rejected
    h[1].center[1] = std::nanf("");
    CHECK(rt::build_host_scene(&d, &hs, &err, false) == RT_ERR_INVALID_SCENE);
}

int main() {
    node_reference_payload();
    builtin_scenes();
    invalid_scenes();
    reference_graph();
    outputs_and_misc();
    if (failures) {
        std::fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    std::printf("host_sanitize: all checks passed\n");
    return 0;
}
