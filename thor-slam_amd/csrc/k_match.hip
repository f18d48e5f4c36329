// k_match.hip — row A6 of SURVEY.md §8a: brute-force Hamming matching (stereo L<->R with a row
// band and positive disparity; temporal L(t)<->L(t-1) with a window), ratio test, mutual check,
// and the integer-SAD sub-pixel refinements (A6b stereo disparity, A7a temporal position).
// Bit-exact with oracle.match / oracle.stereo_subpixel / oracle.temporal_subpixel.
//
// k_match: the Hamming distances come from the matrix cores.  A block holds 128 y-sorted queries
// of one level, one 32-query MFMA row tile per wave (temporal blocks first re-deal their queries
// by x, so each wave holds an x-quartile and its column box admits about half of the trains).
// Each wave walks the train rows its queries can reach in chunks of 64 y-sorted positions,
// compacts the trains inside its column box into an LDS ring (ballot + mbcnt), and scores every
// full ring tile of 32 trains with four FP4 block-scaled MFMAs:
//   Hamming(q, t) = |q| + sum_k (1 - 2 q_k) t_k
// The query side is +-1 (e2m1 0b0010 / 0b1010), the train side the descriptor bits in place
// (w & (0x11111111 << s): fp4 0.5 / 1 / 2, step 3 shifted to 2), undone by the E8M0 block scales
// 2 / 1 / 0.5 / 0.5, and C starts at |q| of the row — every partial sum is a small integer, so
// the f32 result is the exact distance (tools/mfma_hamming_probe.hip checks the encoding).
// One tile costs 4 MFMAs + ~20 VALU of bit unpacking per lane where the VALU kernel spent 16
// v_xor/v_bcnt per lane and pair; the remaining per-pair VALU is the geometric gate and the
// best / second / mutual bookkeeping (9 ops).
//
// Keys.  A non-negative integer-valued f32 orders like its bits and leaves the low 15 mantissa
// bits zero, so (distance, index) keys are bits(H) | index (index < 8192): the query side's best
// is a v_min, its second a v_med3; an ineligible pair gets +inf bits (0x7F800000), above every
// eligible key.  The train side's (distance, query) minimum for the mutual check uses the wave
// slot (0..31) as the index: a wave's queries take their slots in keypoint-index order, so slot
// order is query order.  Slot 2 * reg + h is MFMA row (reg & 3) + 8 (reg >> 2) + 4 h, i.e. the
// row accumulator register reg of lane half h holds, so the slot's low bit is the lane half (ORed
// in after the register minimum).  One global atomicMin per train and wave tile publishes it
// in the (distance << 16 | query) format the refinement kernels read.
#include "tslam_common.h"

#define TS_MQ 128          // queries per k_match block (4 waves x one 32-row MFMA tile)
#define TS_MRED_PITCH 33   // (best, second) rows of the final per-slot reduction, padded
#define TS_MRING 1024      // compacted trains per walk round (the ring shares the reduction's LDS)
#define TS_MCHUNKS 6       // 64-position chunks whose record loads are in flight together

typedef int v8i_t __attribute__((ext_vector_type(8)));
typedef float v16f_t __attribute__((ext_vector_type(16)));
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t med3_u32(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// the geometric gate of one (query row, train column) pair: both 16-bit halves of
// (query gate word - train xy) within the spans (v_pk_sub_u16, v_pk_min_u16, v_cmp)
__device__ __forceinline__ bool gate_ok(uint32_t qgate, uint32_t txy, uint32_t span) {
    const u16x2_t d = __builtin_bit_cast(u16x2_t, qgate) - __builtin_bit_cast(u16x2_t, txy);
    const u16x2_t m = __builtin_elementwise_min(d, __builtin_bit_cast(u16x2_t, span));
    return __builtin_bit_cast(uint32_t, m) == __builtin_bit_cast(uint32_t, d);
}

__device__ __forceinline__ uint32_t key_dist(uint32_t key) {   // distance of a finite key
    return (uint32_t)__uint_as_float(key & 0xFFFF8000u);
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_match(BatchCtx c) {
    TS_BACK_PRIO;
    // per wave: the compacted-train ring during the walk, then the (best, second) reduction
    __shared__ __attribute__((aligned(16))) uint2 s_red[4][32 * TS_MRED_PITCH];
    __shared__ __attribute__((aligned(16))) uint32_t s_key[2][TS_MQ];  // temporal: (x, thread) sort keys, then the dealt positions
    __shared__ __attribute__((aligned(16))) uint32_t s_wk[4][32];   // per wave: query-index sort keys
    // the block's query records and descriptors (one load round), in the ring's LDS: they are dead
    // once every wave has built its A operand (the barrier before the walk)
    uint4* const s_qrec = reinterpret_cast<uint4*>(&s_red[0][0]);
    uint4* const s_qdesc = s_qrec + TS_MQ;
    __shared__ uint32_t s_sq[4][32];      // per wave slot: query keypoint index (~0: empty slot)
    __shared__ uint32_t s_si[4][32];      // ... its block-local index
    // ... gate word (qy + gy_tol) << 16 | (qx - gx_lo) and |q| (popcount of the descriptor), by
    // [wave][slot & 1][slot >> 1]: lane half h reads its 16 accumulator rows as four 16-byte words
    __shared__ __attribute__((aligned(16))) uint32_t s_sg[4][2][16];
    __shared__ __attribute__((aligned(16))) float s_spc[4][2][16];
    // blockIdx.y: the temporal blocks (the heavy ones: a window of rows, not a row band) of every
    // frame first, then the stereo blocks, so the short stereo blocks fill the launch's tail
    // (stereo-only launches, match_modes == 1: blockIdx.y = f * P + p, all stereo)
    const int nfp = c.match_modes == 1 ? 0 : c.n * c.npair;
    const int z = blockIdx.y;
    const int mode = z < nfp ? 1 : 0;
    const int fl = z < nfp ? z : z - nfp;     // f * npair + (p - pair0)
    const int p = c.pair0 + fl % c.npair;
    const int f = fl / c.npair;
    const int64_t g = c.g0 + f;
    if (mode == 1 && g == 0) return;          // no previous frame
    if (mode == 0 && c.rgbd) return;          // RGB-D: depth replaces stereo matching
    int l = 0;
    while (l + 1 < c.g.n_levels && (int)blockIdx.x >= c.g.qtile_start[l + 1]) ++l;
    const int tile = blockIdx.x - c.g.qtile_start[l];
    const int slot = ring_slot(c, g);
    const int qcam = c.cpp * p;
    const int tslot = mode == 0 ? slot : ring_slot(c, g - 1);
    const int tcam = mode == 0 ? qcam + 1 : qcam;
    const int K = c.g.K;
    const int qn = c.kcount[((size_t)slot * c.C + qcam) * c.g.n_levels + l];
    const int tn = c.kcount[((size_t)tslot * c.C + tcam) * c.g.n_levels + l];
    const int q0 = tile * TS_MQ;
    if (q0 >= qn || tn == 0) return;          // block-uniform
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int ci = lane & 31, h = lane >> 5;  // MFMA column / row index, lane half (k half)
    const size_t qbase = ((size_t)slot * c.C + qcam) * K;
    const size_t tbase = ((size_t)tslot * c.C + tcam) * K;
    const size_t mbase = (((size_t)f * c.P + p) * 2 + mode) * K;
    const uint4* qys = c.ys + qbase + c.g.koff[l];           // y-sorted records of the level
    const uint4* tys = c.ys + tbase + c.g.koff[l];
    const uint4* qdesc = reinterpret_cast<const uint4*>(c.desc_ys + (qbase + c.g.koff[l]) * 8);
    const uint4* tdesc = reinterpret_cast<const uint4*>(c.desc_ys + (tbase + c.g.koff[l]) * 8);
    const uint16_t* trs = c.rowstart + ((size_t)tslot * c.C + tcam) * c.g.rs_total + c.g.rs_off[l];
    const int Hl = c.g.H[l];
    const int row_tol = c.mp.row_tol, dmax = c.mp.max_disp >> l, win = c.mp.window >> l;
    // the geometric gate as one box: stereo 1 <= x_q - x_t <= max_disp and |y_q - y_t| <= row_tol;
    // temporal |x_q - x_t| <= window and |y_q - y_t| <= window
    const int gx_lo = mode == 0 ? 1 : -win, gx_hi = mode == 0 ? dmax : win, gy_tol = mode == 0 ? row_tol : win;
    const uint32_t span = (uint32_t)(2 * gy_tol) << 16 | (uint32_t)(gx_hi - gx_lo);

    // The block's 128 query records and descriptors land in LDS in one round of global loads, so
    // every later setup step reads LDS; the records are y-sorted, so each wave's train rows (and
    // the row-start loads for them) are known at once.
    const int nq = min(TS_MQ, qn - q0);
    {
        const int t = threadIdx.x & (TS_MQ - 1), half = threadIdx.x >> 7;
        const int pos = q0 + min(t, nq - 1);   // past nq: a clamped duplicate, never active
        if (half == 0) s_qrec[t] = qys[pos];
        s_qdesc[2 * t + half] = qdesc[2 * pos + half];
    }
    __syncthreads();
    // this wave's 32 queries (block-local indices): 32 wave + i (stereo: y order), or the block's
    // x-ranks 32 wave .. 32 wave + 31 (temporal); active ones come first in either order
    const bool wave_active = 32 * wave < nq;
    const int reach = mode == 0 ? row_tol : win;
    int wt0 = 0, wt1 = 0;
    {
        // train rows: the wave's own (stereo) or the block's (temporal: an x-quartile spans them)
        const int i0 = mode == 1 ? 0 : min(32 * wave, nq - 1), i1 = mode == 1 ? nq - 1 : min(32 * wave + 31, nq - 1);
        const int wy0 = (int)(s_qrec[i0].x >> 16), wy1 = (int)(s_qrec[i1].x >> 16);
        if (wave_active) {
            wt0 = (int)trs[max(0, wy0 - reach)];
            wt1 = (int)trs[min(Hl - 1, wy1 + reach) + 1];
        }
    }
    int bi = 32 * wave + ci;
    if (mode == 1) {
        if (threadIdx.x < TS_MQ) {
            const int t = threadIdx.x;
            s_key[0][t] = t < nq ? (s_qrec[t].x & 0xFFFF) << 8 | (uint32_t)t : 0x1000000u | (uint32_t)t;
        }
        __syncthreads();
        if (threadIdx.x < TS_MQ) {
            const uint32_t key = s_key[0][threadIdx.x];
            int rank = 0;
            const uint4* k4 = reinterpret_cast<const uint4*>(s_key[0]);
#pragma unroll 4
            for (int i = 0; i < TS_MQ / 4; ++i) {
                const uint4 v = k4[i];
                rank += (v.x < key) + (v.y < key) + (v.z < key) + (v.w < key);
            }
            s_key[1][rank] = threadIdx.x;   // keys are distinct: a permutation
        }
        __syncthreads();
        bi = (int)s_key[1][32 * wave + ci];
    }
    const bool active = bi < nq;
    int qx = 0, qy = 0;
    uint32_t qi = 0, pc = 0;
    if (active) {
        const uint4 rec = s_qrec[bi];
        const uint4 d = s_qdesc[2 * bi + h];
        qi = rec.z;
        qx = rec.x & 0xFFFF;
        qy = rec.x >> 16;
        pc = __popc(d.x) + __popc(d.y) + __popc(d.z) + __popc(d.w);
    }
    pc += (uint32_t)__shfl_xor((int)pc, 32, 64);
    // slots in query-index order (the mutual check's tie-break): rank among the wave's 32
    if (h == 0) s_wk[wave][ci] = active ? qi : 0x10000u | (uint32_t)ci;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    {
        const uint32_t key = active ? qi : 0x10000u | (uint32_t)ci;
        int rank = 0;
        const uint4* k4 = reinterpret_cast<const uint4*>(s_wk[wave]);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint4 v = k4[i];
            rank += (v.x < key) + (v.y < key) + (v.z < key) + (v.w < key);
        }
        if (h == 0) {
            s_sq[wave][rank] = active ? qi : 0xFFFFFFFFu;
            s_si[wave][rank] = (uint32_t)bi;
            // inactive: 0xFFFF halves fail every gate
            s_sg[wave][rank & 1][rank >> 1] = active ? ((uint32_t)(qy + gy_tol) << 16 | ((uint32_t)(qx - gx_lo) & 0xFFFFu)) : 0xFFFFFFFFu;
            s_spc[wave][rank & 1][rank >> 1] = (float)pc;
        }
    }
    // the columns of this wave's queries
    int wx0, wx1;
    {
        int ax = active ? qx : (1 << 20), bx = active ? qx : -1;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            ax = min(ax, __shfl_xor(ax, o, 64));
            bx = max(bx, __shfl_xor(bx, o, 64));
        }
        wx0 = __builtin_amdgcn_readfirstlane(ax);   // equal in every lane: make it provably uniform
        wx1 = __builtin_amdgcn_readfirstlane(bx);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (gx_hi < gx_lo) wt1 = wt0;   // empty disparity range at this level: nothing is eligible
    // a train column some query of the wave can reach: qx - tx in [gx_lo, gx_hi] for a wave qx
    const uint32_t bx0 = (uint32_t)(wx0 - gx_hi), bx_span = (uint32_t)(wx1 - gx_lo - (wx0 - gx_hi));

    // A operand (rows = slots): lane (row ci, half h) holds, for MFMA step s, bit s of every nibble
    // of descriptor words 4h .. 4h+3 of the query in slot(ci), as +-1
    uint32_t qa[4][4];
    {
        const int srow = 2 * ((ci & 3) + 4 * (ci >> 3)) + ((ci >> 2) & 1);
        uint4 d = {0u, 0u, 0u, 0u};
        if (s_sq[wave][srow] != 0xFFFFFFFFu) d = s_qdesc[2 * (int)s_si[wave][srow] + h];
        const uint32_t w4[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int j = 0; j < 4; ++j) qa[s][j] = 0x22222222u | (((w4[j] >> s) & 0x11111111u) << 3);
    }
    __syncthreads();   // every wave's A operand is built: s_qrec / s_qdesc become ring space
    // per accumulator register: the slot's |q| (the MFMA's C) and gate word, re-read from LDS per
    // tile (32 VGPRs fewer across the walk: 4 waves per SIMD instead of 3)
    const float4* const spc4 = reinterpret_cast<const float4*>(s_spc[wave][h]);
    const uint4* const sg4 = reinterpret_cast<const uint4*>(s_sg[wave][h]);
    uint32_t best[16], second[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) best[r] = second[r] = 0xFFFFFFFFu;

    // The walk in rounds: compact the trains inside the wave's column box into the ring (chunks of
    // 64 y-sorted positions, TS_MCHUNKS chunks' record loads in flight at a time) until it holds
    // TS_MRING - 64 TS_MCHUNKS or more (every round but a rare last one: all of them), then score
    // the ring's 32-train tiles, each tile's entries and descriptors loaded one tile ahead (two
    // tiles per loop trip measured slower: 173 VGPRs, 2 waves/SIMD).
    // Every load is unconditional (indices clamped into the ring; a padding column only gets the
    // gate-failing xy) and the train-side minima go back into the ring entries (the flush's global
    // atomics come after the round's last tile), so the loop body is straight-line code whose
    // vmcnt waits cover exactly the tile being scored.
    uint2* ring = s_red[wave];   // {txy, tidx << 16 | position}; after scoring {tmin, ...}
    auto score = [&](const uint4& d, const uint2& e, uint32_t k, uint32_t n) {
        const uint32_t w4[4] = {d.x, d.y, d.z, d.w};
        v16f_t acc;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float4 v = spc4[i];
            acc[4 * i] = v.x;
            acc[4 * i + 1] = v.y;
            acc[4 * i + 2] = v.z;
            acc[4 * i + 3] = v.w;
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            v8i_t a, b;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                a[j] = (int)qa[s][j];
                b[j] = (int)(s < 3 ? (w4[j] & (0x11111111u << s)) : ((w4[j] >> 1) & 0x44444444u));
                a[j + 4] = 0;
                b[j + 4] = 0;
            }
            acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc, 4, 4, 0, 127, 0, s == 0 ? 128 : s == 1 ? 127 : 126);
            // b stays live past the MFMA, so the destination never lands on it: the compiler does
            // not keep vdst of the block-scaled MFMA apart from its sources (no early-clobber), and
            // a build that spilled put vdst over srcA and half of srcC — wrong stereo matches
            // (DESIGN.md §5).  isa_guard.py checks every build's MFMA operands.
            asm volatile("" ::"v"(b));
        }
        const uint32_t txy = k < n ? e.x : 0x80008000u;   // padding fails every gate
        const uint32_t tidx = e.y >> 16;
        uint32_t tmin = 0xFFFFFFFFu;
        uint32_t qgate[16];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint4 v = sg4[i];
            qgate[4 * i] = v.x;
            qgate[4 * i + 1] = v.y;
            qgate[4 * i + 2] = v.z;
            qgate[4 * i + 3] = v.w;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t hb = gate_ok(qgate[r], txy, span) ? __float_as_uint(acc[r]) : 0x7F800000u;
            const uint32_t key = hb | tidx;
            second[r] = med3_u32(best[r], second[r], key);   // = min(second, max(best, key)): best <= second
            best[r] = min(best[r], key);
            tmin = min(tmin, hb | (uint32_t)(2 * r));
        }
        tmin |= (uint32_t)h;
        tmin = min(tmin, (uint32_t)__shfl_xor((int)tmin, 32, 64));
        if (h == 0 && k < n) ring[k].x = tmin;
    };
    for (int jt = wt0; jt < wt1;) {
        uint32_t n = 0;
        for (; jt < wt1 && n <= TS_MRING - 64 * TS_MCHUNKS; jt += 64 * TS_MCHUNKS) {
            uint4 r4[TS_MCHUNKS];
#pragma unroll
            for (int u = 0; u < TS_MCHUNKS; ++u) r4[u] = tys[min(jt + 64 * u + lane, wt1 - 1)];
#pragma unroll
            for (int u = 0; u < TS_MCHUNKS; ++u) {
                const int j = jt + 64 * u + lane;
                const bool inbox = j < wt1 && (uint32_t)((int)(r4[u].x & 0xFFFF) - (int)bx0) <= bx_span;
                const uint64_t m = __ballot(inbox);
                if (inbox)
                    ring[n + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] =
                        uint2{r4[u].x, r4[u].z << 16 | (uint32_t)j};
                n += (uint32_t)__popcll(m);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (n > 0) {
            const uint32_t last = n - 1;
            uint2 e0 = ring[min((uint32_t)ci, last)];
            uint4 d0 = tdesc[2 * (int)(e0.y & 0xFFFFu) + h];
            for (uint32_t k = (uint32_t)ci; k - (uint32_t)ci < n; k += 32u) {
                const uint2 e1 = ring[min(k + 32u, last)];
                const uint4 d1 = tdesc[2 * (int)(e1.y & 0xFFFFu) + h];
                score(d0, e0, k, n);
                e0 = e1;
                d0 = d1;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // flush: each train's (distance, query) minimum over the wave's queries
            for (uint32_t k = (uint32_t)lane; k < n; k += 64) {
                const uint2 e = ring[k];
                if (e.x < 0x7F800000u) atomicMin(&c.tbest[mbase + (e.y >> 16)], key_dist(e.x & ~31u) << 16 | s_sq[wave][e.x & 31u]);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // the ring is refilled by the next round
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }

    // per slot: merge the 32 columns' (best, second) — best = min, second = min(s1, s2, max(b1, b2))
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint2* red = s_red[wave];
#pragma unroll
    for (int r = 0; r < 16; ++r) red[(2 * r + h) * TS_MRED_PITCH + ci] = uint2{best[r], second[r]};
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t b = 0xFFFFFFFFu, s2 = 0xFFFFFFFFu;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint2 v = red[ci * TS_MRED_PITCH + 16 * h + i];
        s2 = min(min(s2, v.y), max(b, v.x));
        b = min(b, v.x);
    }
    {
        const uint32_t ob = (uint32_t)__shfl_xor((int)b, 32, 64), os = (uint32_t)__shfl_xor((int)s2, 32, 64);
        s2 = min(min(s2, os), max(b, ob));
        b = min(b, ob);
    }
    // stored by the query's y-sorted position (the refinement kernels load them beside its record)
    const uint32_t qk = s_sq[wave][ci];
    if (h == 0 && qk != 0xFFFFFFFFu) {
        const size_t qp = mbase + c.g.koff[l] + q0 + s_si[wave][ci];
        c.qbest[qp] = b < 0x7F800000u ? key_dist(b) << 16 | (b & 0x7FFFu) : 0xFFFFFFFFu;
        c.qsecond[qp] = s2 < 0x7F800000u ? key_dist(s2) : 256u;
    }
}

// Sub-pixel offset of a discrete minimum from three integer costs (exact double division).
__device__ __forceinline__ double parabola(int sm, int s0, int sp) {
    const int den = sm - 2 * s0 + sp;
    return den > 0 ? (double)(sm - sp) / (2.0 * (double)den) : 0.0;
}

// The 11 bytes of row `y` starting at column `x0` as three dwords (byte 12 zeroed), from aligned
// dword loads + v_alignbyte (any alignment of the level base, row pitch and x0).
__device__ __forceinline__ void row11(const uint8_t* img, int W, int y, int x0, uint32_t* w) {
    const uint8_t* a = img + (size_t)y * W + x0;
    const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(a) & 3u);
    const uint32_t* p = reinterpret_cast<const uint32_t*>(a - sh);   // pointer arithmetic keeps global loads
    const uint32_t d0 = p[0], d1 = p[1], d2 = p[2], d3 = p[3];
    w[0] = __builtin_amdgcn_alignbyte(d1, d0, sh);
    w[1] = __builtin_amdgcn_alignbyte(d2, d1, sh);
    w[2] = __builtin_amdgcn_alignbyte(d3, d2, sh) & 0x00FFFFFFu;
}

// The match of the query at y-sorted position `pos` (keypoint qi): k_match stores (qbest, qsecond)
// by position, so they load beside the query's record, and the train side's best query and the
// train's keypoint word {x | y << 16} (image base tkb) load together once the best train j is
// known — two dependent rounds instead of three.  Returns j when the match passes max distance,
// ratio and the mutual check (and `ok`), else -1.
__device__ __forceinline__ int match_lookup(const BatchCtx& c, size_t mbase, int pos, int qi, bool ok, size_t tkb,
                                            uint32_t* tkp) {
    const uint32_t qb = c.qbest[mbase + pos];
    const uint32_t sd = c.qsecond[mbase + pos];
    const int j = qb == 0xFFFFFFFFu ? 0 : (int)(qb & 0xFFFF);
    const uint32_t tb = c.tbest[mbase + j];
    *tkp = c.kps[(tkb + j) * 2];
    const int bd = (int)(qb >> 16);
    return (ok && qb != 0xFFFFFFFFu && bd <= c.mp.max_hamming && bd * 100 < c.mp.ratio_pct * (int)sd &&
            (int)(tb & 0xFFFF) == qi) ? j : -1;
}

// Stereo refinement (A6b): validity + disparity by 5-offset SAD + parabola.  Eight queries per
// wave, 8 lanes each (lane = query slot * 8 + sub), as the temporal refinement: the query's 11x11
// left patch and the 15x11 right window (offsets -2..+2 around the matched x) are staged in LDS,
// 22 rows dealt over the 8 lanes, so a query costs ~27 row loads instead of 5 x 88 scattered
// dword gathers (the texture-address path, not the VALU, bound the per-lane version); sub-lanes
// 0..4 score the 5 offsets from LDS; the first minimum is an xor-shuffle over the 8 lanes.
// grid xcd_grid(n*P, ceil(K/32)), block 256.
#define TS_RS_QPB 32   // queries per block
__global__ __launch_bounds__(256) void k_refine_stereo(BatchCtx c) {
    TS_BACK_PRIO;
    __shared__ uint4 s_a[TS_RS_QPB][11];   // left patch rows: 11 bytes used
    __shared__ uint4 s_b[TS_RS_QPB][11];   // right window rows: 15 bytes used
    __shared__ int s_cost[TS_RS_QPB][5];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int K = c.g.K;
    int z, local;
    if (!xcd_image_block(blockIdx.x, c.n * c.npair, (K + TS_RS_QPB - 1) / TS_RS_QPB, &z, &local)) return;
    const int p = c.pair0 + z % c.npair, f = z / c.npair;
    const int64_t g = c.g0 + f;
    const int slot = ring_slot(c, g);
    const int sub = lane & 7;
    const int qslot = wave * 8 + (lane >> 3);
    const int pos = local * TS_RS_QPB + qslot;
    const bool live = pos < K;
    const size_t mbase = (((size_t)f * c.P + p) * 2 + 0) * K;
    const int qcam = c.cpp * p;
    const size_t qkb = ((size_t)slot * c.C + qcam) * K;
    int l = 0, qi = 0, j = -1;
    uint32_t qxy = 0, tkp = 0;
    if (live) {
        const uint4 rec = c.ys[qkb + pos];
        qi = (int)rec.z;
        l = (int)(rec.y & 0xFFu);
        qxy = rec.x;
        j = match_lookup(c, mbase, pos, qi, rec.w != 0, ((size_t)slot * c.C + qcam + 1) * K, &tkp);
    }
    const double nanv = __builtin_nan("");
    if (live && sub == 0 && j < 0) {
        c.stereo[((size_t)slot * c.P + p) * K + qi] = -1;
        c.disp[((size_t)slot * c.P + p) * K + qi] = nanv;
    }
    int qx = 0, xr = 0;
    if (j >= 0) {
        const int W = c.g.W[l];
        qx = qxy & 0xFFFF;
        const int qy = qxy >> 16;
        xr = tkp & 0xFFFF;
        const uint8_t* Lp = c.pyr + ((size_t)slot * c.C + qcam) * c.g.pyr_bytes + c.g.pyr_off[l];
        const uint8_t* Rp = c.pyr + ((size_t)slot * c.C + qcam + 1) * c.g.pyr_bytes + c.g.pyr_off[l];
        for (int hl = sub; hl < 22; hl += 8) {
            if (hl < 11) {
                uint32_t w3[3];
                row11(Lp, W, qy - TS_SAD_HALF + hl, qx - TS_SAD_HALF, w3);
                s_a[qslot][hl] = uint4{w3[0], w3[1], w3[2], 0u};
            } else {
                const int r = hl - 11;
                const uint8_t* a = Rp + (size_t)(qy - TS_SAD_HALF + r) * W + (xr - TS_SAD_HALF - TS_SAD_RANGE);
                const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(a) & 3u);
                const uint32_t* q = reinterpret_cast<const uint32_t*>(a - sh);
                const uint32_t d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3], d4 = q[4];
                s_b[qslot][r] = uint4{__builtin_amdgcn_alignbyte(d1, d0, sh), __builtin_amdgcn_alignbyte(d2, d1, sh),
                                      __builtin_amdgcn_alignbyte(d3, d2, sh), __builtin_amdgcn_alignbyte(d4, d3, sh) & 0x00FFFFFFu};
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");   // staged rows before the reads (own wave)
    uint32_t key = 0xFFFFFFFFu;
    if (j >= 0 && sub < 5) {
        const int kx = sub;   // window bytes kx .. kx+10: right patch centred at xr + kx - 2
        // kx == 4: start one word later with no byte shift (the 4th word is then unused)
        const int kh = kx >> 2;
        const uint32_t sh = (uint32_t)(kx & 3);
        const uint32_t* wb = reinterpret_cast<const uint32_t*>(&s_b[qslot][0]);
        uint32_t s = 0;
#pragma unroll
        for (int dy = 0; dy < 11; ++dy) {
            const uint4 ra = s_a[qslot][dy];
            const uint32_t d0 = wb[4 * dy + kh], d1 = wb[4 * dy + kh + 1], d2 = wb[4 * dy + kh + 2], d3 = wb[4 * dy + 3 - kh];
            const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
            const uint32_t w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
            const uint32_t w2 = __builtin_amdgcn_alignbyte(d3, d2, sh) & 0x00FFFFFFu;
            s = __builtin_amdgcn_sad_u8(ra.x, w0, s);
            s = __builtin_amdgcn_sad_u8(ra.y, w1, s);
            s = __builtin_amdgcn_sad_u8(ra.z, w2, s);
        }
        s_cost[qslot][sub] = (int)s;
        key = (s << 5) | (uint32_t)sub;
    }
#pragma unroll
    for (int m = 1; m < 8; m <<= 1) key = min(key, (uint32_t)__shfl_xor((int)key, m, 64));
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");   // costs of the 5 lanes before the reads
    if (j >= 0 && sub == 0) {
        const int ks = (int)(key & 31u);
        double d0 = nanv;
        if (ks > 0 && ks < 4) {
            const double delta = parabola(s_cost[qslot][ks - 1], s_cost[qslot][ks], s_cost[qslot][ks + 1]);
            const double sc = (double)(1 << l);
            const double v = ((double)qx - ((double)(xr + (ks - TS_SAD_RANGE)) + delta)) * sc;
            if (v > 0.0) d0 = v;
        }
        c.stereo[((size_t)slot * c.P + p) * K + qi] = j;
        c.disp[((size_t)slot * c.P + p) * K + qi] = d0;
    }
}

// Temporal refinement (A7a): validity + position by 5x5 SAD search + 2-D parabola.  Eight queries
// per wave, 8 lanes each (lane = query slot * 8 + sub), so the dependent chain of loads (record ->
// match validity -> previous keypoint -> image rows) is paid once per 8 queries, not per 2.  The
// query's 11x11 patch at t-1 and its 15x15 search window at t are staged in LDS (sub-lane s loads
// rows s, s+8, .. of the 26), rows padded to 16 bytes and read back as ds_read_b128; sub-lane s
// scores offsets s, s+8, s+16, s+24 of the 25; the first minimum is an xor-shuffle over the 8
// lanes.  grid xcd_grid(n*P, ceil(K/32)), block 256.
#define TS_RT_AROWS 11
#define TS_RT_BROWS 15
#define TS_RT_QPB 32   // queries per block
__global__ __launch_bounds__(256) void k_refine_temporal(BatchCtx c) {
    TS_BACK_PRIO;
    __shared__ uint4 s_a[TS_RT_QPB][TS_RT_AROWS];   // [query slot][row]: 11 bytes used (+ zero pad)
    __shared__ uint4 s_b[TS_RT_QPB][TS_RT_BROWS];   // 15 bytes used
    __shared__ int s_cost[TS_RT_QPB][25];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int K = c.g.K;
    int z, local;
    if (!xcd_image_block(blockIdx.x, c.n * c.npair, (K + TS_RT_QPB - 1) / TS_RT_QPB, &z, &local)) return;
    const int p = c.pair0 + z % c.npair, f = z / c.npair;
    const int64_t g = c.g0 + f;
    const int slot = ring_slot(c, g);
    const int sub = lane & 7;
    const int qslot = wave * 8 + (lane >> 3);
    const int pos = local * TS_RT_QPB + qslot;
    const bool live = pos < K;
    const size_t mbase = (((size_t)f * c.P + p) * 2 + 1) * K;
    const int qcam = c.cpp * p;
    const size_t qkb = ((size_t)slot * c.C + qcam) * K;
    int l = 0, qi = 0, j = -1;
    uint32_t qxy = 0, pxy = 0;
    const int pslot = g > 0 ? ring_slot(c, g - 1) : slot;   // frame 0: nothing matches
    if (live) {
        const uint4 rec = c.ys[qkb + pos];
        qi = (int)rec.z;
        l = (int)(rec.y & 0xFFu);
        qxy = rec.x;
        j = match_lookup(c, mbase, pos, qi, rec.w != 0 && g > 0, ((size_t)pslot * c.C + qcam) * K, &pxy);
    }
    int32_t* out_idx = c.temporal + ((size_t)slot * c.P + p) * K;
    double* out_uv = c.tuv + (((size_t)f * c.P + p) * K + qi) * 2;
    const double nanv = __builtin_nan("");
    if (live && sub == 0) out_idx[qi] = j;
    if (live && sub == 0 && j < 0) {
        out_uv[0] = nanv;
        out_uv[1] = nanv;
    }
    int qx = 0, qy = 0;
    if (j >= 0) {
        const int W = c.g.W[l];
        qx = qxy & 0xFFFF;
        qy = qxy >> 16;
        const int px = pxy & 0xFFFF, py = pxy >> 16;
        const uint8_t* A = c.pyr + ((size_t)pslot * c.C + qcam) * c.g.pyr_bytes + c.g.pyr_off[l];
        const uint8_t* B = c.pyr + ((size_t)slot * c.C + qcam) * c.g.pyr_bytes + c.g.pyr_off[l];
        // stage: rows 0..10 the patch (3 dwords via row11), rows 11..25 the window (15 bytes from
        // 5 aligned dwords + alignbyte); row r by sub-lane r % 8
        for (int hl = sub; hl < TS_RT_AROWS + TS_RT_BROWS; hl += 8) {
            if (hl < TS_RT_AROWS) {
                uint32_t w3[3];
                row11(A, W, py - TS_SAD_HALF + hl, px - TS_SAD_HALF, w3);
                s_a[qslot][hl] = uint4{w3[0], w3[1], w3[2], 0u};
            } else {
                const int r = hl - TS_RT_AROWS;
                const uint8_t* a = B + (size_t)(qy - TS_SAD_HALF - TS_SAD_RANGE + r) * W + (qx - TS_SAD_HALF - TS_SAD_RANGE);
                const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(a) & 3u);
                const uint32_t* q = reinterpret_cast<const uint32_t*>(a - sh);
                const uint32_t d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3], d4 = q[4];
                s_b[qslot][r] = uint4{__builtin_amdgcn_alignbyte(d1, d0, sh), __builtin_amdgcn_alignbyte(d2, d1, sh),
                                      __builtin_amdgcn_alignbyte(d3, d2, sh), __builtin_amdgcn_alignbyte(d4, d3, sh) & 0x00FFFFFFu};
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");   // staged rows before the reads (own wave)
    // sub-lane kx < 5 scores the 5 offsets (kx, ky = 0..4) of its column shift: each window row is
    // realigned once (its 11 bytes from kx on) and serves every ky it meets (patch row dy = r - ky);
    // the sums are integers, so the costs equal a per-offset loop's
    uint32_t key = 0xFFFFFFFFu;   // first minimum of (cost << 5 | offset) over this lane's offsets
    if (j >= 0 && sub < 5) {
        const int kx = sub, kh = kx >> 2;
        const uint32_t sh = (uint32_t)(kx & 3);
        const uint32_t* wb = reinterpret_cast<const uint32_t*>(&s_b[qslot][0]);
        uint32_t s[5] = {0u, 0u, 0u, 0u, 0u};
#pragma unroll
        for (int r = 0; r < TS_RT_BROWS; ++r) {
            // kx == 4: start one word later with no byte shift (the 4th word is then unused)
            const uint32_t d0 = wb[4 * r + kh], d1 = wb[4 * r + kh + 1], d2 = wb[4 * r + kh + 2], d3 = wb[4 * r + 3 - kh];
            const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
            const uint32_t w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
            const uint32_t w2 = __builtin_amdgcn_alignbyte(d3, d2, sh) & 0x00FFFFFFu;
#pragma unroll
            for (int ky = 0; ky < 5; ++ky) {
                const int dy = r - ky;
                if (dy < 0 || dy >= TS_RT_AROWS) continue;   // compile-time
                const uint4 ra = s_a[qslot][dy];
                s[ky] = __builtin_amdgcn_sad_u8(ra.x, w0, s[ky]);
                s[ky] = __builtin_amdgcn_sad_u8(ra.y, w1, s[ky]);
                s[ky] = __builtin_amdgcn_sad_u8(ra.z, w2, s[ky]);
            }
        }
#pragma unroll
        for (int ky = 0; ky < 5; ++ky) {
            const int o = ky * 5 + kx;
            s_cost[qslot][o] = (int)s[ky];
            key = min(key, (s[ky] << 5) | (uint32_t)o);
        }
    }
#pragma unroll
    for (int m = 1; m < 8; m <<= 1) key = min(key, (uint32_t)__shfl_xor((int)key, m, 64));
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");   // costs of the 8 lanes before the reads
    if (j >= 0 && sub == 0) {
        const int a = (int)(key & 31u);
        const int* cq = s_cost[qslot];
        const int c0 = cq[a];
        const int cl = cq[max(a - 1, 0)], cr = cq[min(a + 1, 24)];
        const int cu = cq[max(a - 5, 0)], cd = cq[min(a + 5, 24)];
        const int ky = a / 5, kx = a % 5;
        double u = nanv, v = nanv;
        if (kx > 0 && kx < 4 && ky > 0 && ky < 4) {
            const double ddx = parabola(cl, c0, cr);
            const double ddy = parabola(cu, c0, cd);
            const double sc = (double)(1 << l);
            u = (((double)(qx + (kx - TS_SAD_RANGE)) + ddx) + 0.5) * sc - 0.5;
            v = (((double)(qy + (ky - TS_SAD_RANGE)) + ddy) + 0.5) * sc - 0.5;
        }
        out_uv[0] = u;
        out_uv[1] = v;
    }
}

void launch_match(const BatchCtx& c, hipStream_t s) {
    (void)hipMemsetAsync(c.tbest, 0xFF, sizeof(uint32_t) * (size_t)c.n * c.P * 2 * c.g.K, s);
    (void)hipMemsetAsync(c.qbest, 0xFF, sizeof(uint32_t) * (size_t)c.n * c.P * 2 * c.g.K, s);
    dim3 grid(c.g.total_qtiles, c.n * c.npair * (c.match_modes == 1 ? 1 : 2));
    hipLaunchKernelGGL(k_match, grid, dim3(256), 0, s, c);
}

// Stereo matching + refinement only (the sharded rig's pre-pass for the frame before a rank's
// range, whose disparities the range's first frame triangulates from).
void launch_match_stereo(const BatchCtx& c, hipStream_t s) {
    BatchCtx st = c;
    st.match_modes = 1;
    (void)hipMemsetAsync(st.tbest, 0xFF, sizeof(uint32_t) * (size_t)st.n * st.P * 2 * st.g.K, s);
    (void)hipMemsetAsync(st.qbest, 0xFF, sizeof(uint32_t) * (size_t)st.n * st.P * 2 * st.g.K, s);
    hipLaunchKernelGGL(k_match, dim3(st.g.total_qtiles, st.n * st.npair), dim3(256), 0, s, st);
    hipLaunchKernelGGL(k_refine_stereo, dim3(xcd_grid(st.n * st.npair, (st.g.K + TS_RS_QPB - 1) / TS_RS_QPB)), dim3(256), 0, s, st);
}

void launch_match_refine(const BatchCtx& c, hipStream_t s) {
    const int K = c.g.K;
    if (c.rgbd)
        launch_rgbd_depth(c, s);
    else
        hipLaunchKernelGGL(k_refine_stereo, dim3(xcd_grid(c.n * c.npair, (K + TS_RS_QPB - 1) / TS_RS_QPB)), dim3(256), 0, s, c);
    hipLaunchKernelGGL(k_refine_temporal, dim3(xcd_grid(c.n * c.npair, (K + TS_RT_QPB - 1) / TS_RT_QPB)), dim3(256), 0, s, c);
}
