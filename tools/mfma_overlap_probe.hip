// mfma_overlap_probe.hip — does v_mfma_scale_f32_32x32x64_f8f6f4 give the right result when its
// destination shares registers with a source?  (diagnostic for k_match; not the product)
//
// The toolchain does not keep vdst of the block-scaled MFMA apart from its sources: the assembler
// rejects "source 2 operand must not partially overlap with dst" for v_mfma_f32_32x32x16_bf16 but
// accepts the same operands for v_mfma_scale_*, and under register pressure the allocator emits
// such operands (a spilling k_match build: vdst v[16:31] with srcC v[4:19] and srcA v[20:23]).
// Each kernel below runs ONE FP4 MFMA with the registers pinned in inline asm — a disjoint
// reference and the overlap layouts seen in builds — on the same random operands, and the host
// compares every layout's 16 accumulators per lane with the reference's.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mfma_overlap_probe.hip -o /tmp/mop && /tmp/mop
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CLOB8(a, b, c, d, e, f, g, h) "v" #a, "v" #b, "v" #c, "v" #d, "v" #e, "v" #f, "v" #g, "v" #h
#define CLOBBERS                                                                                        \
    CLOB8(0, 1, 2, 3, 4, 5, 6, 7), CLOB8(8, 9, 10, 11, 12, 13, 14, 15), CLOB8(16, 17, 18, 19, 20, 21, 22, 23), \
    CLOB8(24, 25, 26, 27, 28, 29, 30, 31), CLOB8(32, 33, 34, 35, 36, 37, 38, 39),                        \
    CLOB8(40, 41, 42, 43, 44, 45, 46, 47), CLOB8(48, 49, 50, 51, 52, 53, 54, 55),                        \
    CLOB8(56, 57, 58, 59, 60, 61, 62, 63), CLOB8(64, 65, 66, 67, 68, 69, 70, 71), "v100", "v101"

// D, A, B, C: register ranges; C0..C3 / D0..D3: their 4-register quarters
#define PROBE(NAME, D, A, B, C, C0, C1, C2, C3, D0, D1, D2, D3)                                           \
    __global__ void NAME(const uint4* pa, const uint4* pb, const uint4* pc, uint4* po) {                 \
        const int l = threadIdx.x;                                                                     \
        const uint4* a = pa + l;                                                                       \
        const uint4* b = pb + l;                                                                       \
        const uint4* c = pc + 4 * l;                                                                   \
        uint4* o = po + 4 * l;                                                                         \
        asm volatile("global_load_dwordx4 " C0 ", %2, off\n"                                           \
                     "global_load_dwordx4 " C1 ", %2, off offset:16\n"                                 \
                     "global_load_dwordx4 " C2 ", %2, off offset:32\n"                                 \
                     "global_load_dwordx4 " C3 ", %2, off offset:48\n"                                 \
                     "global_load_dwordx4 " A ", %0, off\n"                                            \
                     "global_load_dwordx4 " B ", %1, off\n"                                            \
                     "v_mov_b32 v100, 127\n"                                                           \
                     "v_mov_b32 v101, 128\n"                                                           \
                     "s_waitcnt vmcnt(0)\n"                                                            \
                     "v_mfma_scale_f32_32x32x64_f8f6f4 " D ", " A ", " B ", " C                          \
                     ", v100, v101 op_sel_hi:[0,0,0] cbsz:4 blgp:4\n"                                   \
                     "s_nop 7\ns_nop 7\ns_nop 7\ns_nop 7\n"                                             \
                     "global_store_dwordx4 %3, " D0 ", off\n"                                          \
                     "global_store_dwordx4 %3, " D1 ", off offset:16\n"                                \
                     "global_store_dwordx4 %3, " D2 ", off offset:32\n"                                \
                     "global_store_dwordx4 %3, " D3 ", off offset:48\n"                                \
                     "s_waitcnt vmcnt(0)\n" ::"v"(a), "v"(b), "v"(c), "v"(o)                           \
                     : "memory", CLOBBERS);                                                            \
    }

#define Q(x, y) "v[" #x ":" #y "]"
// reference: nothing shared
PROBE(k_ref, Q(32, 47), Q(20, 23), Q(24, 27), Q(0, 15), Q(0, 3), Q(4, 7), Q(8, 11), Q(12, 15), Q(32, 35), Q(36, 39), Q(40, 43), Q(44, 47))
// srcC partially overlaps vdst (low end of D / high end of D)
PROBE(k_c_lo, Q(16, 31), Q(32, 35), Q(36, 39), Q(4, 19), Q(4, 7), Q(8, 11), Q(12, 15), Q(16, 19), Q(16, 19), Q(20, 23), Q(24, 27), Q(28, 31))
PROBE(k_c_hi, Q(16, 31), Q(48, 51), Q(52, 55), Q(24, 39), Q(24, 27), Q(28, 31), Q(32, 35), Q(36, 39), Q(16, 19), Q(20, 23), Q(24, 27), Q(28, 31))
// srcA inside vdst (first / last quarter)
PROBE(k_a_lo, Q(16, 31), Q(16, 19), Q(36, 39), Q(0, 15), Q(0, 3), Q(4, 7), Q(8, 11), Q(12, 15), Q(16, 19), Q(20, 23), Q(24, 27), Q(28, 31))
PROBE(k_a_hi, Q(16, 31), Q(28, 31), Q(36, 39), Q(0, 15), Q(0, 3), Q(4, 7), Q(8, 11), Q(12, 15), Q(16, 19), Q(20, 23), Q(24, 27), Q(28, 31))
// srcB inside vdst (first quarter = the shipped k_match build's layout / last quarter)
PROBE(k_b_lo, Q(16, 31), Q(40, 43), Q(16, 19), Q(0, 15), Q(0, 3), Q(4, 7), Q(8, 11), Q(12, 15), Q(16, 19), Q(20, 23), Q(24, 27), Q(28, 31))
PROBE(k_b_hi, Q(16, 31), Q(40, 43), Q(28, 31), Q(0, 15), Q(0, 3), Q(4, 7), Q(8, 11), Q(12, 15), Q(16, 19), Q(20, 23), Q(24, 27), Q(28, 31))
// the spilling build's two MFMAs (spill_kmatch.s): A + partial C, and A + B inside D
PROBE(k_spill1, Q(16, 31), Q(20, 23), Q(0, 3), Q(4, 19), Q(4, 7), Q(8, 11), Q(12, 15), Q(16, 19), Q(16, 19), Q(20, 23), Q(24, 27), Q(28, 31))
PROBE(k_spill2, Q(16, 31), Q(20, 23), Q(16, 19), Q(56, 71), Q(56, 59), Q(60, 63), Q(64, 67), Q(68, 71), Q(16, 19), Q(20, 23), Q(24, 27), Q(28, 31))
// srcC == vdst exactly (the accumulate form: legal)
PROBE(k_mac, Q(0, 15), Q(20, 23), Q(24, 27), Q(0, 15), Q(0, 3), Q(4, 7), Q(8, 11), Q(12, 15), Q(0, 3), Q(4, 7), Q(8, 11), Q(12, 15))

typedef void (*probe_fn)(const uint4*, const uint4*, const uint4*, uint4*);

int main() {
    const int lanes = 64;
    uint32_t ha[lanes * 4], hb[lanes * 4];
    float hc[lanes * 16];
    srand(11);
    for (int i = 0; i < lanes * 4; ++i) {
        // A: +-1 per nibble (k_match's query side), B: arbitrary nibbles 0 / 0.5 (bit 0 of a nibble)
        const uint32_t r = (uint32_t)rand() ^ ((uint32_t)rand() << 16);
        ha[i] = 0x22222222u | ((r & 0x11111111u) << 3);
        hb[i] = ((uint32_t)rand() ^ ((uint32_t)rand() << 16)) & 0x11111111u;
    }
    for (int i = 0; i < lanes * 16; ++i) hc[i] = (float)(rand() % 257);
    uint4 *da, *db, *dc, *dout;
    (void)hipMalloc(&da, sizeof ha);
    (void)hipMalloc(&db, sizeof hb);
    (void)hipMalloc(&dc, sizeof hc);
    (void)hipMalloc(&dout, sizeof hc);
    (void)hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
    (void)hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
    (void)hipMemcpy(dc, hc, sizeof hc, hipMemcpyHostToDevice);
    const struct {
        const char* name;
        probe_fn fn;
    } probes[] = {{"ref (disjoint)", k_ref},      {"srcC partial, D low", k_c_lo}, {"srcC partial, D high", k_c_hi},
                  {"srcA in D, first quarter", k_a_lo}, {"srcA in D, last quarter", k_a_hi},
                  {"srcB in D, first quarter", k_b_lo}, {"srcB in D, last quarter", k_b_hi},
                  {"spill build mfma 1 (A + partial C)", k_spill1}, {"spill build mfma 2 (A + B in D)", k_spill2},
                  {"srcC == D (accumulate)", k_mac}};
    static float ref[lanes * 16], out[lanes * 16];
    int rc = 0;
    for (size_t v = 0; v < sizeof probes / sizeof probes[0]; ++v) {
        (void)hipMemset(dout, 0xFF, sizeof hc);
        hipLaunchKernelGGL(probes[v].fn, dim3(1), dim3(lanes), 0, 0, da, db, dc, dout);
        if (hipDeviceSynchronize() != hipSuccess) {
            printf("%s: launch failed\n", probes[v].name);
            return 2;
        }
        (void)hipMemcpy(v == 0 ? ref : out, dout, sizeof hc, hipMemcpyDeviceToHost);
        if (v == 0) {
            printf("%-36s reference\n", probes[v].name);
            continue;
        }
        int bad = 0;
        for (int i = 0; i < lanes * 16; ++i) bad += memcmp(&ref[i], &out[i], 4) != 0;
        printf("%-36s %4d / %d accumulators differ from the reference\n", probes[v].name, bad, lanes * 16);
        if (bad && v != 0) rc = 1;
    }
    return rc;
}
