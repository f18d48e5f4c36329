// mfma_hamming_probe.hip — checks the FP4 block-scaled MFMA Hamming tile used by k_match
// against a CPU popcount, for random 256-bit descriptors (profiling / bring-up aid, not the
// product).  Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_hamming_probe.hip -o /tmp/mhp
//
// Encoding (k_match.hip): lane l = (r = l & 31, h = l >> 5); MFMA step s (0..3) of the 32x32x64
// instruction takes, in register j (0..3) of lane l, bit s of every nibble of descriptor word
// 4h + j.  Train side (B): the bits in place, w & (0x11111111 << s) (step 3: (w >> 1) & 0x44444444),
// fp4 values 0.5 / 1 / 2 / 2 -> E8M0 scales 2, 1, 0.5, 0.5.  Query side (A): +-1 (0b0010 / 0b1010)
// = 1 - 2q.  C = popcount(q_row): D = |q| + |t| - 2|q & t| = Hamming(q, t).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int mfma_row(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

__global__ void k_probe(const uint32_t* q, const uint32_t* t, float* out) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    const uint4 qw = reinterpret_cast<const uint4*>(q + 8 * r)[h];
    const uint4 tw = reinterpret_cast<const uint4*>(t + 8 * r)[h];
    v16f acc;
    for (int reg = 0; reg < 16; ++reg) {
        const int row = mfma_row(reg, h);
        int pc = 0;
        for (int w = 0; w < 8; ++w) pc += __popc(q[8 * row + w]);
        acc[reg] = (float)pc;
    }
    const uint32_t qa[4] = {qw.x, qw.y, qw.z, qw.w}, tb[4] = {tw.x, tw.y, tw.z, tw.w};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        v8i a = {}, b = {};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            a[j] = (int)(0x22222222u | (((qa[j] >> s) & 0x11111111u) << 3));
            b[j] = (int)(s < 3 ? (tb[j] & (0x11111111u << s)) : ((tb[j] >> 1) & 0x44444444u));
        }
        const int sb = s == 0 ? 128 : s == 1 ? 127 : 126;
        acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc, 4, 4, 0, 127, 0, sb);
    }
    for (int reg = 0; reg < 16; ++reg) out[mfma_row(reg, h) * 32 + r] = acc[reg];
}

int main() {
    uint32_t hq[256], ht[256];
    srand(7);
    for (int i = 0; i < 256; ++i) {
        hq[i] = (uint32_t)rand() ^ ((uint32_t)rand() << 16);
        ht[i] = (uint32_t)rand() ^ ((uint32_t)rand() << 16);
    }
    for (int w = 0; w < 8; ++w) { hq[8 * 3 + w] = 0; ht[8 * 5 + w] = ~0u; hq[8 * 9 + w] = ht[8 * 9 + w]; }
    uint32_t *dq, *dt;
    float* dout;
    (void)hipMalloc(&dq, 1024);
    (void)hipMalloc(&dt, 1024);
    (void)hipMalloc(&dout, 4096);
    (void)hipMemcpy(dq, hq, 1024, hipMemcpyHostToDevice);
    (void)hipMemcpy(dt, ht, 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, dq, dt, dout);
    float out[1024];
    (void)hipMemcpy(out, dout, 4096, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
            int d = 0;
            for (int w = 0; w < 8; ++w) d += __builtin_popcount(hq[8 * i + w] ^ ht[8 * j + w]);
            if (out[i * 32 + j] != (float)d) {
                if (bad < 5) printf("mismatch q%d t%d: mfma %g cpu %d\n", i, j, out[i * 32 + j], d);
                ++bad;
            }
        }
    printf("fp4 mfma hamming tile: %d / 1024 mismatches\n", bad);
    return bad != 0;
}
