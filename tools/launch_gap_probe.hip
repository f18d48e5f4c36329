// GPU-side cost of a dependent kernel boundary by kernarg size (profiling aid): a spin kernel holds
// the stream ~3 ms while the host enqueues N launches behind it, so the launches then run back to
// back from a full queue; HIP events after the spin and after the last launch give the GPU time
// per launch.  Kernargs: 16 B, a 1,608-B struct by value (the size class of BatchCtx + BaArgs),
// and the same struct read through a device pointer.
// hipcc --offload-arch=gfx950 -O3 tools/launch_gap_probe.hip -o tools/launch_gap_probe.bin
#include <hip/hip_runtime.h>
#include <cstdio>

struct Big { double v[200]; int n; };   // 1,608 B

__global__ void k_spin(uint64_t ticks) {
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
}
__global__ void k_small(int* out, int n) { if (threadIdx.x == 0 && blockIdx.x == 0 && n < 0) out[0] = n; }
__global__ void k_big(Big b, int* out) { if (threadIdx.x == 0 && blockIdx.x == 0 && b.n < 0) out[0] = (int)b.v[3]; }
__global__ void k_ptr(const Big* b, int* out) { if (threadIdx.x == 0 && blockIdx.x == 0 && b->n < 0) out[0] = (int)b->v[3]; }

int main() {
    int* out;
    Big* dbig;
    (void)hipMalloc(&out, 4);
    (void)hipMalloc(&dbig, sizeof(Big));
    Big h{};
    h.n = 1;
    (void)hipMemcpy(dbig, &h, sizeof(Big), hipMemcpyHostToDevice);
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    int rate_khz = 0;
    (void)hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0);
    const uint64_t spin = (uint64_t)rate_khz * 3;   // 3 ms
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int N = 200;
    const char* names[3] = {"16 B kernarg", "1608 B kernarg", "pointer to 1608 B"};
    for (int grid : {1, 64, 256}) {
        for (int kind = 0; kind < 3; ++kind) {
            float best = 1e9f;
            for (int rep = 0; rep < 3; ++rep) {
                hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, spin);
                (void)hipEventRecord(e0, s);
                for (int i = 0; i < N; ++i) {
                    if (kind == 0) hipLaunchKernelGGL(k_small, dim3(grid), dim3(256), 0, s, out, 1);
                    else if (kind == 1) hipLaunchKernelGGL(k_big, dim3(grid), dim3(256), 0, s, h, out);
                    else hipLaunchKernelGGL(k_ptr, dim3(grid), dim3(256), 0, s, (const Big*)dbig, out);
                }
                (void)hipEventRecord(e1, s);
                (void)hipStreamSynchronize(s);
                float ms = 0.0f;
                (void)hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            printf("grid %3d  %-18s %6.2f us per launch (GPU, queue full)\n", grid, names[kind], best * 1e3f / N);
        }
    }
    return 0;
}
