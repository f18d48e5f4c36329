// k_match.hip — row A6 of SURVEY.md §8a: brute-force Hamming matching (stereo L<->R with a row
// band and positive disparity; temporal L(t)<->L(t-1) with a window), ratio test, mutual check,
// and the integer-SAD sub-pixel refinements (A6b stereo disparity, A7a temporal position).
// Bit-exact with oracle.match / oracle.stereo_subpixel / oracle.temporal_subpixel.
//
// k_match: one thread per query, 256 queries per block, 4 waves.  Temporal blocks re-deal their
// 256 y-sorted queries by x (one rank sort in LDS, the only block barrier), so each wave holds an
// x-quartile: its queries' gate box then admits about half of the train columns, and each 64-train
// tile is compacted by a ballot of the box test before any Hamming work (stereo blocks keep the
// y order: their row band is what limits them).
// The train side of a pair is wave-uniform, so its record and descriptor come through SCALAR
// loads (constant address space, s_load_dwordx4/x8 into SGPRs, served by the scalar cache) and
// feed the VALU as SGPR operands: each pair costs 8 v_xor + 8 v_bcnt and a few compares, with no
// LDS read (an LDS broadcast of a 32-byte descriptor still returns 2 KiB per wave at 128 B/clk).
// The train side's best query (for the mutual check) comes from a per-wave distance tile read
// transposed (lane = train) and one global atomicMin per train descriptor per wave tile: min is
// order-independent, so the result is deterministic.
#include "tslam_common.h"

// Distances enter the mutual check as bytes: the train side's best query only matters when its
// distance is <= the query's best <= max_hamming <= 253 (validated), so min(d, 254) keeps every
// decision exact; 255 marks "not eligible".  Rows padded to 68 B for conflict-free transposed
// reads.  LDS 18 KiB per block.
#define TS_TILE_PITCH 68

// popcount(x) + acc as one v_bcnt_u32_b32 (the compiler would re-associate a chain of
// __popc(x) + acc into bcnt + v_add3 trees)
__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc) {
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}

__device__ __forceinline__ uint32_t med3_u32(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_match(BatchCtx c) {
    __shared__ uint8_t s_tile[4][64][TS_TILE_PITCH];   // per wave: min(distance, 254)[train jj][query lane]
    __shared__ __attribute__((aligned(16))) uint32_t s_qi[4][64];
    __shared__ uint32_t s_tr[4][64];    // per wave: the compacted tile's train keypoint indices
    __shared__ uint32_t s_key[256];     // temporal: (x, slot) sort keys, then the dealt positions
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
    const int q0 = tile * 256;
    if (q0 >= qn || tn == 0) return;          // block-uniform
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t qbase = ((size_t)slot * c.C + qcam) * K;
    const size_t tbase = ((size_t)tslot * c.C + tcam) * K;
    const size_t mbase = (((size_t)f * c.P + p) * 2 + mode) * K;
    const uint4* qys = c.ys + qbase + c.g.koff[l];           // y-sorted records of the level
    const uint4* tys = c.ys + tbase + c.g.koff[l];
    const uint4* qdesc = reinterpret_cast<const uint4*>(c.desc_ys + (qbase + c.g.koff[l]) * 8);
    const uint4* tdesc = reinterpret_cast<const uint4*>(c.desc_ys + (tbase + c.g.koff[l]) * 8);
    const uint16_t* trs = c.rowstart + ((size_t)tslot * c.C + tcam) * c.g.rs_total + c.g.rs_off[l];
    const int Hl = c.g.H[l];

    // queries in y-sorted order: this block holds positions q0 .. q0+255 of the level
    int qpos = q0 + threadIdx.x;
    if (mode == 1) {
        // deal the block's queries by x: thread t takes the query of x-rank t (inactive slots,
        // keyed past every x, stay last); keys are distinct, so the ranks are a permutation
        const uint32_t key = qpos < qn ? (uint32_t)(qys[qpos].x & 0xFFFF) << 8 | threadIdx.x
                                       : 0x1000000u | threadIdx.x;
        s_key[threadIdx.x] = key;
        __syncthreads();
        int rank = 0;
        const uint4* k4 = reinterpret_cast<const uint4*>(s_key);
#pragma unroll 4
        for (int i = 0; i < 64; ++i) {
            const uint4 v = k4[i];
            rank += (v.x < key) + (v.y < key) + (v.z < key) + (v.w < key);
        }
        __syncthreads();
        s_key[rank] = (uint32_t)qpos;
        __syncthreads();
        qpos = (int)s_key[threadIdx.x];
    }
    const bool active = qpos < qn;
    uint32_t q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int qx = 0, qy = 0, qi = 0;
    if (active) {
        const uint4 rec = qys[qpos];
        const uint4 a = qdesc[2 * qpos], b = qdesc[2 * qpos + 1];
        q[0] = a.x; q[1] = a.y; q[2] = a.z; q[3] = a.w; q[4] = b.x; q[5] = b.y; q[6] = b.z; q[7] = b.w;
        qi = (int)rec.z;
        qx = rec.x & 0xFFFF;
        qy = rec.x >> 16;
    }
    s_qi[wave][lane] = (uint32_t)qi;
    const int row_tol = c.mp.row_tol, dmax = c.mp.max_disp >> l, win = c.mp.window >> l;
    const int reach = mode == 0 ? row_tol : win;
    // the box of this wave's queries: rows any of them can match (the train range) and columns
    int wy0, wy1, wx0, wx1;
    {
        int a = active ? qy : (1 << 20), b = active ? qy : -1;
        int ax = active ? qx : (1 << 20), bx = active ? qx : -1;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            a = min(a, __shfl_xor(a, o, 64));
            b = max(b, __shfl_xor(b, o, 64));
            ax = min(ax, __shfl_xor(ax, o, 64));
            bx = max(bx, __shfl_xor(bx, o, 64));
        }
        wy0 = __builtin_amdgcn_readfirstlane(a);   // equal in every lane: make it provably uniform
        wy1 = __builtin_amdgcn_readfirstlane(b);
        wx0 = __builtin_amdgcn_readfirstlane(ax);
        wx1 = __builtin_amdgcn_readfirstlane(bx);
    }
    const bool wave_active = wy1 >= 0;
    const int wt0 = wave_active ? (int)trs[max(0, wy0 - reach)] : 0;
    int wt1 = wave_active ? (int)trs[min(Hl - 1, wy1 + reach) + 1] : 0;

    // (distance << 16 | train index) keys: the lexicographic (distance, index) minimum is one
    // v_min_u32, and the second-best distance is the minimum over every key but the best one,
    // min(second, max(best, key)) (keys are distinct: train indices are) — the oracle's rule
    uint32_t best_key = 0xFFFFFFFFu, second_key = 0xFFFFFFFFu;
    // the geometric gate as one box, branch-free: stereo 1 <= x_q - x_t <= max_disp and
    // |y_q - y_t| <= row_tol; temporal |x_q - x_t| <= window and |y_q - y_t| <= window
    const int gx_lo = mode == 0 ? 1 : -win, gx_hi = mode == 0 ? dmax : win, gy_tol = mode == 0 ? row_tol : win;
    const uint32_t gx_span = (uint32_t)(gx_hi - gx_lo), gy_span = (uint32_t)(2 * gy_tol);
    // a train column some query of the wave can reach: qx - tx in [gx_lo, gx_hi] for a wave qx
    const uint32_t bx0 = (uint32_t)(wx0 - gx_hi), bx_span = (uint32_t)(wx1 - gx_lo - (wx0 - gx_hi));
    if (!active) qx = -(1 << 24);   // an inactive lane fails the x range test
    if (gx_hi < gx_lo) wt1 = wt0;   // empty disparity range at this level: nothing is eligible
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    typedef const __attribute__((address_space(4))) v4u cv4u;       // uniform address -> s_load
    cv4u* ctys = (cv4u*)(uintptr_t)tys;
    cv4u* ctdesc = (cv4u*)(uintptr_t)tdesc;
    // The 4 waves are independent (no block barrier): each walks its own train range in tiles of
    // 64 and publishes each train descriptor's best query with one global atomicMin per tile
    // (min is order-independent, so the result is deterministic).
    for (int jt = wt0; jt < wt1; jt += 64) {
        // compaction: the tile's trains inside the wave's column box, in index order
        bool inbox = false;
        uint32_t tz = 0;
        if (jt + lane < wt1) {
            const uint4 r = tys[jt + lane];
            inbox = (uint32_t)((int)(r.x & 0xFFFF) - (int)bx0) <= bx_span;
            tz = r.z;
        }
        uint64_t tm = __ballot(inbox);
        if (tm == 0) continue;
        const int jcount = __popcll(tm);
        if (inbox) s_tr[wave][__builtin_amdgcn_mbcnt_hi((uint32_t)(tm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)tm, 0u))] = tz;
        const int jlast = jt + 63 - __builtin_clzll(tm);
        // phase 1: this lane's query against the compacted trains, each a wave-uniform record +
        // descriptor in SGPRs (index from the mask's lowest set bit); unrolled by 8 so 8
        // descriptors' scalar loads are in flight together
        for (int jj0 = 0; jj0 < jcount; jj0 += 8) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int jj = jj0 + u;
                const int j = tm ? jt + __builtin_ctzll(tm) : jlast;
                tm &= tm - 1;
                const v4u rec = ctys[j];
                const v4u a = ctdesc[2 * j], b = ctdesc[2 * j + 1];
                // gate as two unsigned range tests (one v_sub + one v_cmp each; the train's
                // offsets are scalar): gx_lo <= qx - tx <= gx_hi, -gy_tol <= qy - ty <= gy_tol
                const int tx = rec.x & 0xFFFF, ty = rec.x >> 16;
                const bool elig = (uint32_t)(qx - (tx + gx_lo)) <= gx_span && (uint32_t)(qy - (ty - gy_tol)) <= gy_span &&
                                  jj < jcount;
                uint32_t dd = __popc(q[0] ^ a.x);   // v_bcnt accumulate chain (8 v_xor + 8 v_bcnt)
                dd = bcnt_acc(q[1] ^ a.y, dd);
                dd = bcnt_acc(q[2] ^ a.z, dd);
                dd = bcnt_acc(q[3] ^ a.w, dd);
                dd = bcnt_acc(q[4] ^ b.x, dd);
                dd = bcnt_acc(q[5] ^ b.y, dd);
                dd = bcnt_acc(q[6] ^ b.z, dd);
                dd = bcnt_acc(q[7] ^ b.w, dd);
                const uint32_t key = elig ? ((dd << 16) | rec.z) : 0xFFFFFFFFu;
                second_key = med3_u32(best_key, second_key, key);   // = min(second, max(best, key)): best <= second
                best_key = min(best_key, key);
                s_tile[wave][jj][lane] = (uint8_t)(elig ? min(dd, 254u) : 255u);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        // phase 2: transposed read, lane = compacted train: (distance, query) minimum over
        // the wave's 64 queries, 4 queries per dword read (row pitch 68 B = 17 dwords, an
        // odd stride, so the 64 lanes hit 64 different banks), no cross-lane reduction
        if (lane < jcount) {
            const uint32_t my_train = s_tr[wave][lane];
            // an ineligible pair's key (255 << 16 | query) exceeds every eligible one (distance
            // <= 254), so a plain minimum is exact and "no eligible query" is best >= 255 << 16
            uint32_t best = 0xFFFFFFFFu;
            const uint32_t* row = reinterpret_cast<const uint32_t*>(&s_tile[wave][lane][0]);
            const uint4* qi4 = reinterpret_cast<const uint4*>(&s_qi[wave][0]);
#pragma unroll 2
            for (int r4 = 0; r4 < 16; ++r4) {
                const uint32_t d4 = row[r4];
                const uint4 qq = qi4[r4];
                best = min(best, __builtin_amdgcn_ubfe(d4, 0, 8) << 16 | qq.x);
                best = min(best, __builtin_amdgcn_ubfe(d4, 8, 8) << 16 | qq.y);
                best = min(best, __builtin_amdgcn_ubfe(d4, 16, 8) << 16 | qq.z);
                best = min(best, (d4 >> 24) << 16 | qq.w);
            }
            if (best < (255u << 16)) atomicMin(&c.tbest[mbase + my_train], best);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
    }
    if (active) {
        const int qk = (int)s_qi[wave][lane];   // re-read: one VGPR less through the train loop
        c.qbest[mbase + qk] = best_key;
        c.qsecond[mbase + qk] = second_key == 0xFFFFFFFFu ? 256u : (second_key >> 16);
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

// Validity of the match of query keypoint qi (max distance, ratio, mutual); returns the train
// index or -1.
__device__ __forceinline__ int match_valid(const BatchCtx& c, size_t mbase, int qi) {
    const uint32_t qb = c.qbest[mbase + qi];
    if (qb == 0xFFFFFFFFu) return -1;
    const int bd = qb >> 16, j = qb & 0xFFFF;
    const int sd = c.qsecond[mbase + qi];
    const uint32_t tb = c.tbest[mbase + j];
    return (bd <= c.mp.max_hamming && bd * 100 < c.mp.ratio_pct * sd && (int)(tb & 0xFFFF) == qi) ? j : -1;
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
    uint32_t qxy = 0;
    if (live) {
        const uint4 rec = c.ys[qkb + pos];
        qi = (int)rec.z;
        l = (int)(rec.y & 0xFFu);
        qxy = rec.x;
        if (rec.w) j = match_valid(c, mbase, qi);
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
        xr = c.kps[(((size_t)slot * c.C + qcam + 1) * K + j) * 2] & 0xFFFF;
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
    uint32_t qxy = 0;
    if (live) {
        const uint4 rec = c.ys[qkb + pos];
        qi = (int)rec.z;
        l = (int)(rec.y & 0xFFu);
        qxy = rec.x;
        if (rec.w && g > 0) j = match_valid(c, mbase, qi);
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
        const int pslot = ring_slot(c, g - 1);
        const uint32_t pxy = c.kps[(((size_t)pslot * c.C + qcam) * K + j) * 2];
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
