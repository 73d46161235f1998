// tiled.cpp — single-process multi-device image tiling behind the C ABI.
//
// The reference renders on one device (LaunchKernel, Kernel.cu:178-191; findCudaDevice, helper_cuda.h:
// 872-886).  The north star tiles the image across the GPUs of one node with a gather over xGMI: here a C++
// host (the viewer linking librt_hip.so, no torch) gets that from one call.  Every band rank r renders the
// block-cyclic row bands b ≡ r (mod N) of the frame on its own device and stream into a contiguous local
// buffer (rt_tiling; RNG streams keyed by the GLOBAL pixel index, so the image is bit-identical to one
// rank's); then each rank copies its bands straight into their rows of the destination framebuffer with one
// strided 2-D peer copy over xGMI (band k of rank r → global band k·N + r), the gather and the row unshuffle
// in a single transfer per rank.  Ranks run concurrently; several ranks may share a device (one stream each).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "rt_internal.h"
#include "rt_scene_device.h"

namespace rt {
namespace {

int hip_err(hipError_t e, const std::string& what) {
    if (e == hipSuccess) return RT_OK;
    set_error("rt_tiled: " + what + ": " + hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? RT_ERR_OUT_OF_MEMORY : RT_ERR_DEVICE;
}

// Restores the calling thread's current device on scope exit.
struct DeviceGuard {
    int saved = 0;
    bool ok = false;
    DeviceGuard() { ok = hipGetDevice(&saved) == hipSuccess; }
    ~DeviceGuard() {
        if (ok) (void)hipSetDevice(saved);
    }
};

uint32_t rows_of_rank(uint32_t height, uint32_t band, uint32_t n, uint32_t r) {
    uint32_t rows = 0;
    for (uint64_t b = r; b * band < height; b += n) rows += (uint32_t)std::min<uint64_t>(band, height - b * band);
    return rows;
}

}  // namespace
}  // namespace rt

struct rt_tiled {
    struct Rank {
        int device = 0;
        uint32_t local_rows = 0;
        hipStream_t stream = nullptr;
        uint32_t* pos = nullptr;
        rt_curand_state* state = nullptr;
        uint64_t* counters = nullptr;
        hipEvent_t ev[3] = {nullptr, nullptr, nullptr};  // start, rendered, gathered
    };
    rt_tiled_desc desc{};
    std::vector<int> devices;
    std::vector<Rank> ranks;
    std::map<int, rt_scene*> scenes;  // one device scene per distinct device
    uint32_t frame = 0;

    ~rt_tiled() {
        rt::DeviceGuard g;
        for (Rank& k : ranks) {
            if (hipSetDevice(k.device) != hipSuccess) continue;
            if (k.stream) (void)hipStreamSynchronize(k.stream);
            for (hipEvent_t& e : k.ev)
                if (e) (void)hipEventDestroy(e);
            if (k.pos) (void)hipFree(k.pos);
            if (k.state) (void)hipFree(k.state);
            if (k.counters) (void)hipFree(k.counters);
            if (k.stream) (void)hipStreamDestroy(k.stream);
        }
        for (auto& kv : scenes) {
            if (hipSetDevice(kv.first) == hipSuccess) rt_scene_destroy(kv.second);
        }
    }
};

using namespace rt;

extern "C" {

int rt_tiled_create(const rt_tiled_desc* desc, const rt_scene_desc* scene, rt_tiled** out) {
    if (!desc || !scene || !out || !desc->devices || desc->num_ranks == 0) {
        set_error("rt_tiled_create: NULL argument or no ranks");
        return RT_ERR_INVALID_ARGUMENT;
    }
    *out = nullptr;
    if (desc->width == 0 || desc->height == 0) {
        set_error("rt_tiled_create: empty image");
        return RT_ERR_INVALID_ARGUMENT;
    }
    if ((desc->flags & ~(uint32_t)RT_FLAG_RNG_PHILOX) || desc->reserved != 0) {
        set_error("rt_tiled_create: flags other than RT_FLAG_RNG_PHILOX, or reserved != 0");
        return RT_ERR_INVALID_ARGUMENT;
    }
    int ndev = 0;
    if (int rc = hip_err(hipGetDeviceCount(&ndev), "hipGetDeviceCount")) return rc;
    for (uint32_t r = 0; r < desc->num_ranks; r++)
        if (desc->devices[r] < 0 || desc->devices[r] >= ndev) {
            set_error("rt_tiled_create: device ordinal " + std::to_string(desc->devices[r]) + " out of range");
            return RT_ERR_INVALID_ARGUMENT;
        }
    DeviceGuard guard;
    std::unique_ptr<rt_tiled> t;
    try {
        t.reset(new rt_tiled());
        t->desc = *desc;
        t->desc.band_rows = desc->band_rows ? desc->band_rows : 16;
        t->devices.assign(desc->devices, desc->devices + desc->num_ranks);
        t->desc.devices = t->devices.data();
        t->ranks.resize(desc->num_ranks);
    } catch (const std::bad_alloc&) {
        set_error("rt_tiled_create: host allocation failed");
        return RT_ERR_OUT_OF_MEMORY;
    }
    const bool philox = (desc->flags & RT_FLAG_RNG_PHILOX) != 0;
    const uint32_t W = desc->width, H = desc->height, B = t->desc.band_rows, N = desc->num_ranks;
    for (uint32_t r = 0; r < N; r++) {
        rt_tiled::Rank& k = t->ranks[r];
        k.device = desc->devices[r];
        k.local_rows = rows_of_rank(H, B, N, r);
        if (int rc = hip_err(hipSetDevice(k.device), "hipSetDevice")) return rc;
        if (!t->scenes.count(k.device)) {
            rt_scene* s = nullptr;
            if (int rc = rt_scene_create(scene, &s)) return rc;
            t->scenes[k.device] = s;
        }
        if (int rc = hip_err(hipStreamCreateWithFlags(&k.stream, hipStreamNonBlocking), "hipStreamCreate")) return rc;
        for (hipEvent_t& e : k.ev)
            if (int rc = hip_err(hipEventCreate(&e), "hipEventCreate")) return rc;
        if (int rc = hip_err(hipMalloc((void**)&k.counters, RT_COUNTERS_WORDS * sizeof(uint64_t)), "counter allocation")) return rc;
        if (k.local_rows == 0) continue;
        const size_t px = (size_t)W * k.local_rows;
        if (int rc = hip_err(hipMalloc((void**)&k.pos, px * 4), "framebuffer allocation")) return rc;
        if (!philox) {
            if (int rc = hip_err(hipMalloc((void**)&k.state, px * sizeof(rt_curand_state)), "RNG state allocation"))
                return rc;
            const rt_tiling tiling{B, N, r, k.local_rows};
            if (int rc = rt_render_init(k.state, W, H, &tiling, desc->seed, k.stream)) return rc;
        }
    }
    for (rt_tiled::Rank& k : t->ranks) {
        (void)hipSetDevice(k.device);
        if (int rc = hip_err(hipStreamSynchronize(k.stream), "RNG seeding")) return rc;
    }
    *out = t.release();
    return RT_OK;
}

int rt_tiled_render(rt_tiled* t, const rt_tiled_frame* f, rt_tiled_timing* timing) {
    if (!t || !f || !f->pos) {
        set_error("rt_tiled_render: NULL argument");
        return RT_ERR_INVALID_ARGUMENT;
    }
    // Frame flags the band ranks can honour: each rank's state buffer is rt_curand_state structs seeded by
    // rt_render_init (so RT_FLAG_STATE_SOA would read them as planes, past their end for short ranks), the
    // RNG mode is fixed at creation and there is no per-rank accumulation buffer.
    constexpr uint32_t kFrameFlags = RT_FLAG_FAITHFUL_GRID | RT_FLAG_NO_STATE_WRITEBACK | RT_FLAG_COUNT_TESTS |
                                     RT_FLAG_RIUS_LEFT_TO_RIGHT;
    if (f->flags & ~kFrameFlags) {
        set_error("rt_tiled_render: frame flags outside FAITHFUL_GRID | NO_STATE_WRITEBACK | COUNT_TESTS | "
                  "RIUS_LEFT_TO_RIGHT");
        return RT_ERR_INVALID_ARGUMENT;
    }
    if (f->reserved != 0 || (f->rng_frame_set != 0 && f->rng_frame_set != 1)) {
        set_error("rt_tiled_render: reserved fields must be 0 and rng_frame_set 0 or 1");
        return RT_ERR_INVALID_ARGUMENT;
    }
    const auto t0 = std::chrono::steady_clock::now();
    DeviceGuard guard;
    const uint32_t W = t->desc.width, H = t->desc.height, B = t->desc.band_rows, N = t->desc.num_ranks;
    const bool philox = (t->desc.flags & RT_FLAG_RNG_PHILOX) != 0;
    int dst_device = 0;
    {
        hipPointerAttribute_t attr;
        if (hipPointerGetAttributes(&attr, f->pos) != hipSuccess || attr.type != hipMemoryTypeDevice) {
            (void)hipGetLastError();
            set_error("rt_tiled_render: pos must be device memory (the gathered W·H RGBA8 frame)");
            return RT_ERR_INVALID_ARGUMENT;
        }
        dst_device = attr.device;
    }
    const uint32_t frame = f->rng_frame_set ? f->rng_frame : t->frame;
    // An error after some ranks have been launched returns only once their streams are idle: the caller may
    // free `pos` (or the scene) as soon as the call fails, and an in-flight render or gather would write into it.
    auto drain = [t](int rc) {
        std::string msg = rt_last_error();
        for (rt_tiled::Rank& k : t->ranks)
            if (k.stream && hipSetDevice(k.device) == hipSuccess) (void)hipStreamSynchronize(k.stream);
        (void)hipGetLastError();
        set_error(msg);
        return rc;
    };
    // 1. every rank renders its bands on its own stream (concurrently)
    for (uint32_t r = 0; r < N; r++) {
        rt_tiled::Rank& k = t->ranks[r];
        if (int rc = hip_err(hipSetDevice(k.device), "hipSetDevice")) return drain(rc);
        if (int rc = hip_err(hipEventRecord(k.ev[0], k.stream), "hipEventRecord")) return drain(rc);
        if (int rc = hip_err(hipMemsetAsync(k.counters, 0, RT_COUNTERS_WORDS * sizeof(uint64_t), k.stream), "counter reset"))
            return drain(rc);
        if (k.local_rows) {
            rt_render_args a{};
            a.pos = k.pos;
            a.state = k.state;
            a.counters = k.counters;
            a.width = W;
            a.height = H;
            a.samples_per_pixel = f->samples_per_pixel;
            a.max_depth = f->max_depth;
            a.flags = f->flags | (philox ? (uint32_t)RT_FLAG_RNG_PHILOX : 0u);
            a.tiling = rt_tiling{B, N, r, k.local_rows};
            a.inputs = f->inputs;
            a.rng_seed = t->desc.seed;
            a.rng_frame = frame;
            if (int rc = rt_render(t->scenes[k.device], &a, k.stream)) return drain(rc);
        }
        if (int rc = hip_err(hipEventRecord(k.ev[1], k.stream), "hipEventRecord")) return drain(rc);
    }
    // 2. gather + unshuffle: rank r's local band k → global band k·N + r of the destination frame, one
    //    strided 2-D copy per rank over the peer link (the last global band may be partial: copied apart)
    for (uint32_t r = 0; r < N; r++) {
        rt_tiled::Rank& k = t->ranks[r];
        (void)hipSetDevice(k.device);
        if (k.device != dst_device) {
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, k.device, dst_device) == hipSuccess && can) {
                const hipError_t e = hipDeviceEnablePeerAccess(dst_device, 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
                    return drain(hip_err(e, "hipDeviceEnablePeerAccess"));
                (void)hipGetLastError();
            }
        }
        if (k.local_rows) {
            const uint32_t full = k.local_rows / B;  // whole bands of this rank
            const size_t band_bytes = (size_t)B * W * 4;
            uint32_t* dst0 = f->pos + (size_t)r * B * W;
            if (full > 0) {
                if (int rc = hip_err(hipMemcpy2DAsync(dst0, band_bytes * N, k.pos, band_bytes, band_bytes, full,
                                                      hipMemcpyDefault, k.stream),
                                     "gather (hipMemcpy2DAsync)"))
                    return drain(rc);
            }
            const uint32_t tail = k.local_rows - full * B;
            if (tail) {
                uint32_t* dst = f->pos + ((size_t)full * N + r) * B * W;
                if (int rc = hip_err(hipMemcpyAsync(dst, k.pos + (size_t)full * B * W, (size_t)tail * W * 4,
                                                    hipMemcpyDefault, k.stream),
                                     "gather (hipMemcpyAsync)"))
                    return drain(rc);
            }
        }
        if (int rc = hip_err(hipEventRecord(k.ev[2], k.stream), "hipEventRecord")) return drain(rc);
    }
    // 3. wait for every rank (the call is synchronous, as LaunchKernel is, Kernel.cu:190)
    float render_ms = 0.0f, gather_ms = 0.0f;
    uint64_t rays = 0;
    for (rt_tiled::Rank& k : t->ranks) {
        (void)hipSetDevice(k.device);
        if (int rc = hip_err(hipStreamSynchronize(k.stream), "hipStreamSynchronize")) return drain(rc);
        float a = 0.0f, b = 0.0f;
        (void)hipEventElapsedTime(&a, k.ev[0], k.ev[1]);
        (void)hipEventElapsedTime(&b, k.ev[1], k.ev[2]);
        render_ms = std::max(render_ms, a);
        gather_ms = std::max(gather_ms, b);
        uint64_t c = 0;
        if (int rc = hip_err(hipMemcpy(&c, k.counters, sizeof(c), hipMemcpyDeviceToHost), "counter readback"))
            return drain(rc);
        rays += c;
    }
    if (!f->rng_frame_set && !(f->flags & RT_FLAG_NO_STATE_WRITEBACK)) t->frame++;
    if (timing) {
        timing->render_ms = render_ms;
        timing->gather_ms = gather_ms;
        timing->total_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
        timing->rays = rays;
    }
    return RT_OK;
}

int rt_tiled_destroy(rt_tiled* t) {
    delete t;
    return RT_OK;
}

}  // extern "C"
