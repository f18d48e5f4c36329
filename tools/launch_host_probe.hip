// Host submission cost of dependent launches (the C4 BA enqueues ~24 per keyframe): wall-clock of
// the enqueue loop alone (before any wait) and end to end, for a small kernarg, a 1.6 KB by-value
// struct (BatchCtx + BaArgs) and a 24-node captured hipGraph replay.
// hipcc --offload-arch=gfx950 -O3 tools/launch_host_probe.hip -o /tmp/lhp
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

struct Big { double v[200]; int n; };   // 1,608 B

__global__ void k_small(int* out, int n) { if (threadIdx.x == 0 && blockIdx.x == 0 && n < 0) out[0] = n; }
__global__ void k_big(Big b, int* out) { if (threadIdx.x == 0 && blockIdx.x == 0 && b.n < 0) out[0] = (int)b.v[3]; }

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    int* out; (void)hipMalloc(&out, 4);
    Big h{}; h.n = 1;
    hipStream_t s; (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    const int N = 480;
    for (int kind = 0; kind < 2; ++kind) {
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipStreamSynchronize(s);
            const double t0 = now_us();
            for (int i = 0; i < N; ++i) {
                if (kind == 0) hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, s, out, 1);
                else hipLaunchKernelGGL(k_big, dim3(64), dim3(256), 0, s, h, out);
            }
            const double t1 = now_us();
            (void)hipStreamSynchronize(s);
            const double t2 = now_us();
            if (rep == 2) printf("%-5s enqueue %6.2f us/launch, end to end %6.2f us/launch\n", kind ? "big" : "small",
                                 (t1 - t0) / N, (t2 - t0) / N);
        }
    }
    // 24-node graph of big launches, replayed N / 24 times
    hipGraph_t g; hipGraphExec_t ge;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    for (int i = 0; i < 24; ++i) hipLaunchKernelGGL(k_big, dim3(64), dim3(256), 0, s, h, out);
    (void)hipStreamEndCapture(s, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipStreamSynchronize(s);
        const double t0 = now_us();
        for (int i = 0; i < N / 24; ++i) {
            hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, out, 1);   // the per-keyframe args launch
            (void)hipGraphLaunch(ge, s);
        }
        const double t1 = now_us();
        (void)hipStreamSynchronize(s);
        const double t2 = now_us();
        if (rep == 2) printf("graph enqueue %6.2f us/node, end to end %6.2f us/node (24 nodes + 1 launch per replay)\n",
                             (t1 - t0) / N, (t2 - t0) / N);
    }
    return 0;
}
