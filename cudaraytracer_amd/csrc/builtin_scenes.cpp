// builtin_scenes.cpp — host-side scene generators and camera set-up (no device needed).
//
// Mirrors the caller side of the boundary: CudaLayer::GenerateWorld (CudaLayer.cpp:103-256), the camera
// → InputStruct fill (CudaLayer.cpp:43-65) and the RND macro (Math.cuh:12, glibc rand()/RAND_MAX).  The
// BASELINE.json configurations that the reference does not ship (3-sphere, RTIOW final scene, Cornell
// box, textured spheres) are expressed in the reference's own types.
//
// Where the reference's C++ leaves the evaluation order of several RND calls in one expression
// unspecified (e.g. `Vec3(a + RND, 0.2f, b + RND)`, CudaLayer.cpp:201), the draws here are taken left to
// right; the generated scenes are inputs, committed as fixtures under tests/golden/.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

#include "rt_internal.h"

extern "C" {

// glibc random_r TYPE_3 (degree 31, separation 3): srand() seeds r[0..30] with 16807·r mod (2^31-1),
// copies r[31..33] = r[0..2], then discards 310 outputs; rand() = (r[i-31] + r[i-3]) >> 1.
void rt_glibc_srand(rt_glibc_rand* g, uint32_t seed) {
    int32_t r[34];
    r[0] = (int32_t)(seed == 0 ? 1 : seed);
    for (int i = 1; i < 31; i++) {
        int64_t hi = r[i - 1] / 127773, lo = r[i - 1] % 127773;
        int64_t word = 16807 * lo - 2836 * hi;
        if (word < 0) word += 2147483647;
        r[i] = (int32_t)word;
    }
    for (int i = 31; i < 34; i++) r[i] = r[i - 31];
    std::memcpy(g->r, r, sizeof(r));
    g->idx = 34;
    for (int i = 0; i < 310; i++) rt_glibc_rand_next(g);
}

int32_t rt_glibc_rand_next(rt_glibc_rand* g) {
    uint32_t i = g->idx;
    uint32_t v = (uint32_t)g->r[(i - 31) % 34] + (uint32_t)g->r[(i - 3) % 34];
    g->r[i % 34] = (int32_t)v;
    g->idx = i + 1 == 68u ? 34u : i + 1;  // idx stays in [34, 68): (idx - 31) and (idx - 3) never wrap
    return (int32_t)(v >> 1);
}

void rt_camera_inputs(const float position[3], const float orientation[3], const float world_up[3],
                      float fov_degrees, float near_plane, float far_plane, const float bg_start[3],
                      const float bg_end[3], rt_input_struct* out) {
    // glm::cross / glm::normalize (v · inversesqrt(dot(v, v))) as CudaLayer.cpp:45-46 calls them.
    auto cross = [](const float* a, const float* b, float* r) {
        r[0] = a[1] * b[2] - b[1] * a[2];
        r[1] = a[2] * b[0] - b[2] * a[0];
        r[2] = a[0] * b[1] - b[0] * a[1];
    };
    auto normalize = [](float* v) {
        float inv = 1.0f / std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        v[0] *= inv; v[1] *= inv; v[2] *= inv;
    };
    float right[3], up[3];
    cross(orientation, world_up, right);
    normalize(right);
    cross(orientation, right, up);
    normalize(up);
    for (int i = 0; i < 3; i++) {
        out->origin[i] = position[i];
        out->orientation[i] = orientation[i];
        out->up[i] = up[i];
        out->background_start[i] = bg_start[i];
        out->background_end[i] = bg_end[i];
    }
    out->far_plane = far_plane;
    out->near_plane = near_plane;
    out->fov = fov_degrees * 0.01745329251994329576923690768489f;  // glm::radians
}

}  // extern "C"

namespace {

struct SceneOut {
    rt_hittable_desc* h;
    uint32_t nh, cap_h;
    rt_material_desc* m;
    uint32_t nm, cap_m;

    int add_material(const rt_material_desc& md) {
        if (m && nm < cap_m) m[nm] = md;
        return (int)nm++;
    }
    void add_hittable(int type, float cx, float cy, float cz, float radius, float w, float hh, int mat) {
        rt_hittable_desc d;
        std::memset(&d, 0, sizeof(d));
        d.type = type;
        d.is_active = 1;
        d.center[0] = cx; d.center[1] = cy; d.center[2] = cz;
        d.radius = radius;
        d.width = w;
        d.height = hh;
        d.material = mat;
        if (h && nh < cap_h) h[nh] = d;
        nh++;
    }
};

rt_material_desc constant_mat(int type, float r, float g, float b) {
    rt_material_desc m;
    std::memset(&m, 0, sizeof(m));
    m.type = type;
    m.albedo.type = RT_CONSTANT;
    m.albedo.image = -1;
    m.albedo.color[0] = r; m.albedo.color[1] = g; m.albedo.color[2] = b;
    return m;
}
rt_material_desc lambertian(float r, float g, float b) { return constant_mat(RT_LAMBERTIAN, r, g, b); }
rt_material_desc metal(float r, float g, float b, float fuzz) {
    rt_material_desc m = constant_mat(RT_METAL, r, g, b);
    m.fuzz = fuzz < 1 ? fuzz : 1;  // Metal ctor clamp, Material.cuh:71
    return m;
}
rt_material_desc dielectric(float ir) {
    rt_material_desc m;
    std::memset(&m, 0, sizeof(m));
    m.type = RT_DIELECTRIC;
    m.ir = ir;
    m.albedo.image = -1;
    return m;
}
rt_material_desc light(float r, float g, float b, int intensity) {
    rt_material_desc m = constant_mat(RT_DIFFUSELIGHT, r, g, b);
    m.light_intensity = intensity;
    return m;
}

struct Rnd {
    rt_glibc_rand g;
    explicit Rnd(uint32_t seed) { rt_glibc_srand(&g, seed); }
    float operator()() { return (float)rt_glibc_rand_next(&g) / (float)2147483647; }  // RND, Math.cuh:12
};

// CudaLayer::GenerateWorld (CudaLayer.cpp:103-256)
void default_world(SceneOut& s, uint32_t seed) {
    Rnd rnd(seed);
    rt_material_desc ground;
    std::memset(&ground, 0, sizeof(ground));
    ground.type = RT_LAMBERTIAN;
    ground.albedo.type = RT_CHECKER;
    ground.albedo.image = -1;
    float odd[3] = {0.2f, 0.3f, 0.1f}, even[3] = {0.9f, 0.9f, 0.9f};
    std::memcpy(ground.albedo.color, odd, sizeof(odd));
    std::memcpy(ground.albedo.color2, even, sizeof(even));
    s.add_hittable(RT_XZRECT, 0.0f, -0.5f, 0.0f, 0.0f, 1000.0f, 1000.0f, s.add_material(ground));
    for (int a = -2; a < 2; a++) {
        for (int b = -2; b < 2; b++) {
            float choose_mat = rnd();
            float cx = a + rnd();
            float cz = b + rnd();
            if (choose_mat < 0.5f) {
                float r = rnd() * rnd(), g = rnd() * rnd(), bb = rnd() * rnd();
                s.add_hittable(RT_SPHERE, cx, 0.2f, cz, 0.2f, 0, 0, s.add_material(lambertian(r, g, bb)));
            } else if (choose_mat < 0.80f) {
                float r = 0.5f * (1.0f + rnd()), g = 0.5f * (1.0f + rnd()), bb = 0.5f * (1.0f + rnd());
                float f = 0.5f * rnd();
                s.add_hittable(RT_SPHERE, cx, 0.2f, cz, 0.2f, 0, 0, s.add_material(metal(r, g, bb, f)));
            } else if (choose_mat < 0.90f) {
                s.add_hittable(RT_SPHERE, cx, 0.2f, cz, 0.3f, 0, 0, s.add_material(dielectric(1.5f)));
            } else {
                s.add_hittable(RT_SPHERE, cx, 0.2f, cz, 0.5f, 0, 0, s.add_material(light(1.0f, 1.0f, 1.0f, 3)));
            }
        }
    }
}

// BASELINE config 1: three Lambertian spheres.
void three_spheres(SceneOut& s) {
    s.add_hittable(RT_SPHERE, 0.0f, 0.0f, -1.0f, 0.5f, 0, 0, s.add_material(lambertian(0.1f, 0.2f, 0.5f)));
    s.add_hittable(RT_SPHERE, 0.0f, -100.5f, -1.0f, 100.0f, 0, 0, s.add_material(lambertian(0.8f, 0.8f, 0.0f)));
    s.add_hittable(RT_SPHERE, 1.0f, 0.0f, -1.0f, 0.5f, 0, 0, s.add_material(lambertian(0.8f, 0.6f, 0.2f)));
}

// BASELINE config 2/4: "Ray Tracing in One Weekend" final scene in the reference's types (488 spheres).
void rtiow_final(SceneOut& s, uint32_t seed) {
    Rnd rnd(seed);
    s.add_hittable(RT_SPHERE, 0.0f, -1000.0f, -1.0f, 1000.0f, 0, 0, s.add_material(lambertian(0.5f, 0.5f, 0.5f)));
    for (int a = -11; a < 11; a++) {
        for (int b = -11; b < 11; b++) {
            float choose_mat = rnd();
            float cx = a + rnd();
            float cz = b + rnd();
            if (choose_mat < 0.8f) {
                float r = rnd() * rnd(), g = rnd() * rnd(), bb = rnd() * rnd();
                s.add_hittable(RT_SPHERE, cx, 0.2f, cz, 0.2f, 0, 0, s.add_material(lambertian(r, g, bb)));
            } else if (choose_mat < 0.95f) {
                float r = 0.5f * (1.0f + rnd()), g = 0.5f * (1.0f + rnd()), bb = 0.5f * (1.0f + rnd());
                float f = 0.5f * rnd();
                s.add_hittable(RT_SPHERE, cx, 0.2f, cz, 0.2f, 0, 0, s.add_material(metal(r, g, bb, f)));
            } else {
                s.add_hittable(RT_SPHERE, cx, 0.2f, cz, 0.2f, 0, 0, s.add_material(dielectric(1.5f)));
            }
        }
    }
    s.add_hittable(RT_SPHERE, 0.0f, 1.0f, 0.0f, 1.0f, 0, 0, s.add_material(dielectric(1.5f)));
    s.add_hittable(RT_SPHERE, -4.0f, 1.0f, 0.0f, 1.0f, 0, 0, s.add_material(lambertian(0.4f, 0.2f, 0.1f)));
    s.add_hittable(RT_SPHERE, 4.0f, 1.0f, 0.0f, 1.0f, 0, 0, s.add_material(metal(0.7f, 0.6f, 0.5f, 0.0f)));
}

// BASELINE config 3: Cornell-style box (555 units) of XY/XZ/YZ rects with an emissive ceiling rect.
void cornell(SceneOut& s) {
    int red = s.add_material(lambertian(0.65f, 0.05f, 0.05f));
    int white = s.add_material(lambertian(0.73f, 0.73f, 0.73f));
    int green = s.add_material(lambertian(0.12f, 0.45f, 0.15f));
    int lamp = s.add_material(light(1.0f, 1.0f, 1.0f, 15));
    int glass = s.add_material(dielectric(1.5f));
    int alu = s.add_material(metal(0.8f, 0.85f, 0.88f, 0.0f));
    s.add_hittable(RT_YZRECT, 555.0f, 277.5f, 277.5f, 0, 555.0f, 555.0f, green);  // x = 555 wall
    s.add_hittable(RT_YZRECT, 0.0f, 277.5f, 277.5f, 0, 555.0f, 555.0f, red);      // x = 0 wall
    s.add_hittable(RT_XZRECT, 278.0f, 554.0f, 279.5f, 0, 130.0f, 105.0f, lamp);   // light
    s.add_hittable(RT_XZRECT, 277.5f, 0.0f, 277.5f, 0, 555.0f, 555.0f, white);    // floor
    s.add_hittable(RT_XZRECT, 277.5f, 555.0f, 277.5f, 0, 555.0f, 555.0f, white);  // ceiling
    s.add_hittable(RT_XYRECT, 277.5f, 277.5f, 555.0f, 0, 555.0f, 555.0f, white);  // back wall
    s.add_hittable(RT_SPHERE, 190.0f, 90.0f, 190.0f, 90.0f, 0, 0, glass);
    s.add_hittable(RT_SPHERE, 370.0f, 120.0f, 370.0f, 120.0f, 0, 0, alu);
}

// BASELINE config 5: textured spheres over a checker ground.  Images 0, 1, 2 are supplied by the caller (the
// reference's 8192×4096 planet textures, assets/textures/8k_*.jpg, or rt_procedural_texture stand-ins):
// an "earth" and a "moon" Lambertian sphere and an emissive "sun" (DiffuseLight with an Image texture).
void textured(SceneOut& s) {
    rt_material_desc ground;
    std::memset(&ground, 0, sizeof(ground));
    ground.type = RT_LAMBERTIAN;
    ground.albedo.type = RT_CHECKER;
    ground.albedo.image = -1;
    ground.albedo.color[0] = 0.2f; ground.albedo.color[1] = 0.3f; ground.albedo.color[2] = 0.1f;
    ground.albedo.color2[0] = 0.9f; ground.albedo.color2[1] = 0.9f; ground.albedo.color2[2] = 0.9f;
    s.add_hittable(RT_XZRECT, 0.0f, -0.5f, 0.0f, 0.0f, 1000.0f, 1000.0f, s.add_material(ground));
    rt_material_desc img;
    std::memset(&img, 0, sizeof(img));
    img.type = RT_LAMBERTIAN;
    img.albedo.type = RT_IMAGE;
    img.albedo.image = 0;
    int earth = s.add_material(img);
    rt_material_desc moon_m = img;
    moon_m.albedo.image = 1;
    int moon = s.add_material(moon_m);
    rt_material_desc glow = img;
    glow.type = RT_DIFFUSELIGHT;
    glow.light_intensity = 2;
    glow.albedo.image = 2;
    int lamp = s.add_material(glow);
    s.add_hittable(RT_SPHERE, 0.0f, 1.0f, 0.0f, 1.5f, 0, 0, earth);
    s.add_hittable(RT_SPHERE, -3.5f, 0.5f, 0.5f, 1.0f, 0, 0, moon);
    s.add_hittable(RT_SPHERE, 3.5f, 0.7f, -0.5f, 1.2f, 0, 0, lamp);
    s.add_hittable(RT_SPHERE, 1.5f, 0.0f, 2.5f, 0.5f, 0, 0, s.add_material(metal(0.8f, 0.8f, 0.8f, 0.05f)));
}

// ---------------------------------------------------------------------------------------------------
// Procedural RGB8 textures standing in for the reference's 8K planet maps (assets/textures/8k_*.jpg; this
// image has no JPEG decoder).  Every texel is a pure function of (kind, x, y, width, height): fractal value
// noise over an integer hash lattice, so tests and benchmarks regenerate identical bytes anywhere.
// ---------------------------------------------------------------------------------------------------
inline uint32_t lattice_hash(uint32_t x, uint32_t y, uint32_t seed) {
    uint32_t h = x * 0x8da6b343u ^ y * 0xd8163841u ^ seed * 0xcb1ab31fu;
    h ^= h >> 15;
    h *= 0x2c1b3c6du;
    h ^= h >> 12;
    h *= 0x297a2d39u;
    h ^= h >> 15;
    return h;
}

float value_noise(float x, float y, uint32_t seed) {
    const float fx0 = std::floor(x), fy0 = std::floor(y);
    const uint32_t ix = (uint32_t)(int32_t)fx0, iy = (uint32_t)(int32_t)fy0;
    float fx = x - fx0, fy = y - fy0;
    fx = fx * fx * (3.0f - 2.0f * fx);
    fy = fy * fy * (3.0f - 2.0f * fy);
    const float k = 1.0f / 16777216.0f;
    const float a = (float)(lattice_hash(ix, iy, seed) >> 8) * k, b = (float)(lattice_hash(ix + 1, iy, seed) >> 8) * k;
    const float c = (float)(lattice_hash(ix, iy + 1, seed) >> 8) * k, d = (float)(lattice_hash(ix + 1, iy + 1, seed) >> 8) * k;
    return (a + (b - a) * fx) + ((c + (d - c) * fx) - (a + (b - a) * fx)) * fy;
}

float fbm(float x, float y, uint32_t seed, int octaves) {
    float sum = 0.0f, amp = 0.5f, norm = 0.0f;
    for (int o = 0; o < octaves; o++) {
        sum += amp * value_noise(x, y, seed + (uint32_t)o * 101u);
        norm += amp;
        amp *= 0.5f;
        x *= 2.03f;
        y *= 2.03f;
    }
    return sum / norm;
}

inline uint8_t to_u8(float v) { return (uint8_t)(v < 0.0f ? 0.0f : (v > 255.0f ? 255.0f : v)); }

void texture_rows(int kind, int32_t w, int32_t h, uint8_t* rgb, int32_t y0, int32_t y1) {
    for (int32_t y = y0; y < y1; y++) {
        const float v = ((float)y + 0.5f) / (float)h;  // 0 at the top row (stb loads top-down)
        const float lat = std::fabs(v - 0.5f) * 2.0f;  // 0 at the equator, 1 at the poles
        for (int32_t x = 0; x < w; x++) {
            const float u = ((float)x + 0.5f) / (float)w;
            uint8_t* px = rgb + ((size_t)y * (size_t)w + (size_t)x) * 3;
            float r, g, b;
            if (kind == 0) {  // earth: oceans, continents, deserts, ice caps
                const float n = fbm(u * 12.0f, v * 6.0f, 7u, 6);
                const float m = fbm(u * 40.0f, v * 20.0f, 19u, 3);
                if (lat > 0.86f + 0.08f * (m - 0.5f)) {
                    r = 235.0f; g = 240.0f; b = 250.0f;
                } else if (n > 0.53f) {
                    const float dry = fbm(u * 25.0f, v * 12.0f, 31u, 4);
                    r = 60.0f + 120.0f * dry; g = 110.0f + 50.0f * (1.0f - dry); b = 40.0f + 30.0f * m;
                } else {
                    r = 15.0f + 20.0f * m; g = 45.0f + 40.0f * n; b = 120.0f + 80.0f * n;
                }
            } else if (kind == 1) {  // moon: grey highlands, dark maria, crater speckle
                const float n = fbm(u * 16.0f, v * 8.0f, 43u, 6);
                const float c = fbm(u * 90.0f, v * 45.0f, 59u, 2);
                float l = 90.0f + 110.0f * n - (n < 0.45f ? 45.0f : 0.0f) - (c > 0.7f ? 50.0f * (c - 0.7f) / 0.3f : 0.0f);
                r = l; g = l; b = l * 1.02f;
            } else {  // sun: orange granulation
                const float n = fbm(u * 30.0f, v * 15.0f, 71u, 5);
                r = 255.0f; g = 120.0f + 110.0f * n; b = 10.0f + 60.0f * n * n;
            }
            px[0] = to_u8(r);
            px[1] = to_u8(g);
            px[2] = to_u8(b);
        }
    }
}

}  // namespace

extern "C" int rt_procedural_texture(int kind, int32_t width, int32_t height, uint8_t* rgb) {
    if (kind < 0 || kind > 2 || width <= 0 || height <= 0 || !rgb) {
        rt::set_error("rt_procedural_texture: kind must be 0..2, width and height positive, rgb non-NULL");
        return RT_ERR_INVALID_ARGUMENT;
    }
    const unsigned hw = std::thread::hardware_concurrency();
    const int32_t nthreads = (int32_t)std::max(1u, std::min(hw ? hw : 1u, 16u));
    const int32_t chunk = (height + nthreads - 1) / nthreads;
    std::vector<std::thread> pool;
    pool.reserve((size_t)nthreads);
    int32_t started_rows = 0;  // rows [0, started_rows) belong to started threads
    for (int32_t t = 0; t < nthreads && started_rows < height; t++) {
        const int32_t y0 = t * chunk, y1 = std::min(height, y0 + chunk);
        try {
            pool.emplace_back(texture_rows, kind, width, height, rgb, y0, y1);
        } catch (const std::exception&) {  // no more threads: the rest on this one
            break;
        }
        started_rows = y1;
    }
    if (started_rows < height) texture_rows(kind, width, height, rgb, started_rows, height);
    for (auto& th : pool) th.join();
    return RT_OK;
}

extern "C" int rt_builtin_scene(int which, uint32_t seed, rt_hittable_desc* hittables, uint32_t* num_hittables,
                                rt_material_desc* materials, uint32_t* num_materials) {
    if (!num_hittables || !num_materials) {
        rt::set_error("rt_builtin_scene: count pointers must not be NULL");
        return RT_ERR_INVALID_ARGUMENT;
    }
    SceneOut s{hittables, 0, hittables ? *num_hittables : 0u, materials, 0, materials ? *num_materials : 0u};
    switch (which) {
    case 0: default_world(s, seed); break;
    case 1: three_spheres(s); break;
    case 2: rtiow_final(s, seed); break;
    case 3: cornell(s); break;
    case 4: textured(s); break;
    default: rt::set_error("rt_builtin_scene: unknown scene " + std::to_string(which)); return RT_ERR_INVALID_ARGUMENT;
    }
    bool fits = (!hittables || s.nh <= s.cap_h) && (!materials || s.nm <= s.cap_m);
    *num_hittables = s.nh;
    *num_materials = s.nm;
    if (!fits) {
        rt::set_error("rt_builtin_scene: output arrays too small");
        return RT_ERR_INVALID_ARGUMENT;
    }
    return RT_OK;
}
