// display.cpp — what happens to the framebuffer after the kernel.
//
// The reference shows each frame by copying the RGBA8 buffer device-to-device into a registered OpenGL
// texture (cudaGraphicsGLRegisterImage, CudaLayer.cpp:89-90; map → cudaGraphicsSubResourceGetMappedArray →
// cudaMemcpy2DToArray → unmap, CudaLayer.cpp:379-386) and displays it flipped (ImGui uv (0,1)→(1,0),
// CudaLayer.cpp:402: row 0 of the buffer is the bottom of the image).  Here:
//   * rt_gl_*: the same interop through HIP (hipGraphicsGLRegisterImage & co.) for a viewer with a GL context;
//   * rt_copy_image_to_host: the host-staging fallback (no GL/HIP interop: copy to host, flip, upload with
//     glTexSubImage2D or write to disk);
//   * rt_write_ppm: headless output (binary PPM, top row first), which the reference lacks (stb_image_write is
//     compiled in, RawStbImage.h:8-9, but never called).
#include <hip/hip_runtime_api.h>
// (after the runtime header: the interop declarations use its types)
#include <hip/hip_gl_interop.h>

#include <cstdio>
#include <exception>
#include <new>
#include <cstring>
#include <string>
#include <vector>

#include "rt_internal.h"

struct rt_gl_target {
    hipGraphicsResource_t resource = nullptr;
    uint32_t gl_texture = 0;
};

namespace {

int hip_status(hipError_t e, const char* what) {
    if (e == hipSuccess) return RT_OK;
    rt::set_error(std::string(what) + ": " + hipGetErrorString(e));
    return RT_ERR_DEVICE;
}

}  // namespace

extern "C" {

int rt_write_ppm(const char* path, const uint32_t* rgba, uint32_t width, uint32_t height, int flip_rows) {
    if (!path || (!rgba && (size_t)width * height) || width == 0 || height == 0) {
        rt::set_error("rt_write_ppm: NULL path/pixels or empty image");
        return RT_ERR_INVALID_ARGUMENT;
    }
    FILE* f = std::fopen(path, "wb");
    if (!f) {
        rt::set_error(std::string("rt_write_ppm: cannot open ") + path);
        return RT_ERR_INVALID_ARGUMENT;
    }
    std::vector<uint8_t> row;
    try {
        row.resize((size_t)width * 3);
    } catch (const std::exception&) {  // nothing may throw through the C ABI
        std::fclose(f);
        rt::set_error("rt_write_ppm: host allocation failed");
        return RT_ERR_OUT_OF_MEMORY;
    }
    std::fprintf(f, "P6\n%u %u\n255\n", width, height);
    bool ok = true;
    for (uint32_t y = 0; y < height && ok; y++) {
        // PPM rows run top to bottom; the framebuffer's row 0 is the bottom of the image (Kernel.cu:157)
        const uint32_t src = flip_rows ? height - 1 - y : y;
        const uint32_t* p = rgba + (size_t)src * width;
        for (uint32_t x = 0; x < width; x++) {  // RGBA8 packs R in the low byte (RgbToInt, Kernel.cu:12-19)
            row[3 * x + 0] = (uint8_t)(p[x] & 0xffu);
            row[3 * x + 1] = (uint8_t)((p[x] >> 8) & 0xffu);
            row[3 * x + 2] = (uint8_t)((p[x] >> 16) & 0xffu);
        }
        ok = std::fwrite(row.data(), 1, row.size(), f) == row.size();
    }
    ok = (std::fclose(f) == 0) && ok;
    if (!ok) {
        rt::set_error(std::string("rt_write_ppm: write failed: ") + path);
        return RT_ERR_DEVICE;
    }
    return RT_OK;
}

int rt_copy_image_to_host(uint32_t* host, const uint32_t* device_pos, uint32_t width, uint32_t height, int flip_rows,
                          rt_stream stream) {
    if (!host || !device_pos) {
        rt::set_error("rt_copy_image_to_host: NULL buffer");
        return RT_ERR_INVALID_ARGUMENT;
    }
    const size_t row = (size_t)width * 4;
    if (row * height == 0) return RT_OK;
    hipStream_t s = (hipStream_t)stream;
    int rc = hip_status(hipMemcpyAsync(host, device_pos, row * height, hipMemcpyDeviceToHost, s),
                        "rt_copy_image_to_host: hipMemcpyAsync");
    if (rc) return rc;
    rc = hip_status(hipStreamSynchronize(s), "rt_copy_image_to_host: hipStreamSynchronize");
    if (rc || !flip_rows) return rc;
    // top row first, as glTexSubImage2D with a top-left origin or an image file expects (CudaLayer.cpp:402)
    std::vector<uint32_t> tmp;
    try {
        tmp.resize(width);
    } catch (const std::exception&) {
        rt::set_error("rt_copy_image_to_host: host allocation failed");
        return RT_ERR_OUT_OF_MEMORY;
    }
    for (uint32_t y = 0; y < height / 2; y++) {
        uint32_t* a = host + (size_t)y * width;
        uint32_t* b = host + (size_t)(height - 1 - y) * width;
        std::memcpy(tmp.data(), a, row);
        std::memcpy(a, b, row);
        std::memcpy(b, tmp.data(), row);
    }
    return RT_OK;
}

int rt_gl_register_texture(uint32_t gl_texture, uint32_t gl_target, rt_gl_target** out) {
    if (!out || gl_texture == 0) {
        rt::set_error("rt_gl_register_texture: NULL out or texture name 0");
        return RT_ERR_INVALID_ARGUMENT;
    }
    *out = nullptr;
    rt_gl_target* t = new (std::nothrow) rt_gl_target();
    if (!t) {
        rt::set_error("rt_gl_register_texture: host allocation failed");
        return RT_ERR_OUT_OF_MEMORY;
    }
    // cudaGraphicsGLRegisterImage(&m_Resource, m_Texture, GL_TEXTURE_2D, WriteDiscard) (CudaLayer.cpp:89-90)
    int rc = hip_status(hipGraphicsGLRegisterImage(&t->resource, gl_texture, gl_target,
                                                   hipGraphicsRegisterFlagsWriteDiscard),
                        "rt_gl_register_texture: hipGraphicsGLRegisterImage");
    if (rc) {
        delete t;
        return rc;
    }
    t->gl_texture = gl_texture;
    *out = t;
    return RT_OK;
}

int rt_gl_copy_image(rt_gl_target* target, const uint32_t* device_pos, uint32_t width, uint32_t height,
                     rt_stream stream) {
    if (!target || !target->resource || !device_pos) {
        rt::set_error("rt_gl_copy_image: NULL target or framebuffer");
        return RT_ERR_INVALID_ARGUMENT;
    }
    hipStream_t s = (hipStream_t)stream;
    // map → mapped array → 2-D device copy of W·4 B × H rows → unmap (CudaLayer.cpp:379-386)
    int rc = hip_status(hipGraphicsMapResources(1, &target->resource, s), "rt_gl_copy_image: hipGraphicsMapResources");
    if (rc) return rc;
    hipArray_t array = nullptr;
    rc = hip_status(hipGraphicsSubResourceGetMappedArray(&array, target->resource, 0, 0),
                    "rt_gl_copy_image: hipGraphicsSubResourceGetMappedArray");
    if (!rc)
        rc = hip_status(hipMemcpy2DToArrayAsync(array, 0, 0, device_pos, (size_t)width * 4, (size_t)width * 4, height,
                                                hipMemcpyDeviceToDevice, s),
                        "rt_gl_copy_image: hipMemcpy2DToArrayAsync");
    const int urc = hip_status(hipGraphicsUnmapResources(1, &target->resource, s),
                               "rt_gl_copy_image: hipGraphicsUnmapResources");
    return rc ? rc : urc;
}

int rt_gl_unregister(rt_gl_target* target) {
    if (!target) return RT_OK;
    int rc = RT_OK;
    if (target->resource)
        rc = hip_status(hipGraphicsUnregisterResource(target->resource), "rt_gl_unregister: hipGraphicsUnregisterResource");
    delete target;
    return rc;
}

}  // extern "C"
