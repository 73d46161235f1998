// Device (gfx950) build of the Random() fill-order probe (probe.h): one lane evaluates the expression in a kernel
// and writes x, y, z; the host prints the order.  The device IR (hipcc --cuda-device-only -emit-llvm) shows the
// same order statically: run.sh records it without a GPU.
#include <hip/hip_runtime.h>
#include <cstdio>
#define PROBE_QUAL __host__ __device__
#include "probe.h"
__global__ void probe_kernel(float* out) {
    Draws s{0};
    Vec3p v = random_vec(&s);
    out[0] = v.e[0];
    out[1] = v.e[1];
    out[2] = v.e[2];
}
int main() {
    float* d = nullptr;
    float h[3] = {0, 0, 0};
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) { std::printf("no device\n"); return 2; }
    hipLaunchKernelGGL(probe_kernel, dim3(1), dim3(1), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) { std::printf("copy failed\n"); return 3; }
    (void)hipFree(d);
    std::printf("gfx950 device: x=%g y=%g z=%g -> %s\n", h[0], h[1], h[2],
                h[0] == 1.0f ? "left-to-right" : (h[2] == 1.0f ? "right-to-left" : "other"));
    return 0;
}
