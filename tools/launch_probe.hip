// Launch-floor microbenchmark: back-to-back dependent launches of a trivial kernel on one stream,
// with a small kernarg, with a 1.5 KB by-value struct (the size of BatchCtx + BaArgs), and with a
// pointer to that struct in device memory.  hipcc --offload-arch=gfx950 -O3 tools/launch_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

struct Big { double v[188]; int n; };   // 1,512 B

__global__ void k_small(int* out, int n) { if (threadIdx.x == 0 && blockIdx.x == 0 && n < 0) out[0] = n; }
__global__ void k_big(Big b, int* out) { if (threadIdx.x == 0 && blockIdx.x == 0 && b.n < 0) out[0] = (int)b.v[3]; }
__global__ void k_ptr(const Big* b, int* out) { if (threadIdx.x == 0 && blockIdx.x == 0 && b->n < 0) out[0] = (int)b->v[3]; }
__global__ void k_bigread(Big b, int* out) {   // every wave reads several kernarg fields
    double s = b.v[threadIdx.x & 63] + b.v[64 + (threadIdx.x & 63)];
    if (s < -1.0) out[0] = 1;
}

int main() {
    int* out; hipMalloc(&out, 4);
    Big h{}; h.n = 1;
    Big* d; hipMalloc(&d, sizeof(Big)); hipMemcpy(d, &h, sizeof(Big), hipMemcpyHostToDevice);
    hipStream_t s; hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const int N = 400;
    for (int grid : {1, 64, 256}) {
        for (int kind = 0; kind < 4; ++kind) {
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(e0, s);
                for (int i = 0; i < N; ++i) {
                    if (kind == 0) hipLaunchKernelGGL(k_small, dim3(grid), dim3(256), 0, s, out, 1);
                    if (kind == 1) hipLaunchKernelGGL(k_big, dim3(grid), dim3(256), 0, s, h, out);
                    if (kind == 2) hipLaunchKernelGGL(k_ptr, dim3(grid), dim3(256), 0, s, d, out);
                    if (kind == 3) hipLaunchKernelGGL(k_bigread, dim3(grid), dim3(256), 0, s, h, out);
                }
                hipEventRecord(e1, s);
                hipEventSynchronize(e1);
                float ms; hipEventElapsedTime(&ms, e0, e1);
                if (rep) printf("grid %4d %-9s %6.2f us per launch\n", grid,
                                kind == 0 ? "small" : kind == 1 ? "big" : kind == 2 ? "ptr" : "bigread", 1000.0f * ms / N);
            }
        }
    }
    return 0;
}
