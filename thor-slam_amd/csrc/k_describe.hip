// k_describe.hip — row A5 of SURVEY.md §8a: intensity-centroid orientation + rotated BRIEF-256.
//
// Tile-staged: a block owns a 128 x 64 tile of one level.  It copies the tile plus halo of the
// raw level (orientation) and of the smoothed level (BRIEF) into LDS with 16-byte LDS-DMA loads,
// then serves every keypoint inside the tile from LDS, one wave per keypoint.  A wave-per-
// keypoint design that fetched each 37x37 patch from L2 issued ~10 cache-line requests per
// wave-load and ran L2-request-bound; staging reads every line of the tile once (the patches of
// neighbouring keypoints overlap ~3-4x).
//  * keypoints of the tile: the y-sorted records of the tile's rows (rowstart), 64 at a time,
//    filtered by x with a ballot;
//  * orientation: lane (row, word) holds the realigned word at dx = 4w - 15 .. 4w - 12 of disc
//    row dy = row - 15; m10 = dot4(wx, I) - 15 dot4(mask, I), m01 = dy dot4(mask, I) with
//    per-lane constant byte weights (3 ops per word); bin by 30 wedge tests in parallel lanes;
//  * BRIEF: the rotated pattern is a table of byte offsets for the tile pitch (built by the host),
//    2 ds_read_u8 + 1 compare per test, four wave ballots per descriptor.
// Bit-exact with oracle.orientation_bins / oracle.brief.
#include "tslam_common.h"

// shared with the host (tslam_api.cpp builds the BRIEF offset table for TS_DT_P)
#include "tslam_describe.h"

#define TS_DT_G 1   // keypoints per orientation / table-load group (1 / 2 / 4 / 8: 461 / 467 / 480 / 567 us)

// 16-byte async global -> LDS copy; `wave_dst` is the wave-uniform LDS base, lane k lands at +16k
__device__ __forceinline__ void glds16d(const void* src, void* wave_dst) {
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)wave_dst, 16, 0, 0);
}

// Copy rows [r0, r0 + nrows) x the first NLD of the NCH 16-byte chunks of columns [cs, cs + 16 NCH)
// of a level (pitch W, H rows) into an LDS image of pitch 16 NCH (lane-linear: the LDS-DMA lands a
// wave's 64 chunks contiguously; chunks NLD.. of a row are LDS pitch padding).  Rows outside the
// level and chunks outside [0, W) are skipped (the keypoint margin guarantees no keypoint reads
// them).
template <int NCH, int NLD = NCH>
__device__ __forceinline__ void stage_tile(const uint8_t* level, int W, int H, int r0, int cs, int nrows,
                                           uint8_t* lds, bool wide16) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (wide16) {
        const int n = nrows * NCH;
        for (int i0 = wave * 64; i0 < n; i0 += TS_DT_THREADS) {
            const int i = i0 + lane;
            if (i < n) {
                const int r = i / NCH, q = i - r * NCH;
                const int y = r0 + r, x = cs + 16 * q;
                if (q < NLD && y >= 0 && y < H && x >= 0 && x + 16 <= W) glds16d(level + (size_t)y * W + x, lds + 16 * i0);
            }
        }
    } else {
        for (int i = threadIdx.x; i < nrows * 16 * NCH; i += TS_DT_THREADS) {
            const int r = i / (16 * NCH), q = i - r * (16 * NCH);
            const int y = r0 + r, x = cs + q;
            if (y >= 0 && y < H && x >= 0 && x < W) lds[i] = level[(size_t)y * W + x];
        }
    }
}

// Per-lane orientation disc constants of slot s = lane + 64 i (i < 5): byte weights dx + 15,
// dy + 15 and the 0/1 mask of the 4 pixels of dword w = s % 9 in disc row r = s / 9 (pixel
// dx = 4w - 15 + j, dy = r - 15, inside the radius-15 disc), and the word's LDS offset in the raw
// tile.  Built at compile time: one 16-byte load per slot instead of the per-block disc
// arithmetic.  The offset weights keep all three moment sums on v_dot4_u32_u8 (no 32-bit
// multiplies): m10 = sum (dx + 15) I - 15 sum I, m01 = sum (dy + 15) I - 15 sum I.
struct DiscSlot {
    uint32_t wx, mk, wy;
    int32_t rofs;
};
struct DiscTable {
    DiscSlot e[320];
};
constexpr DiscTable make_disc_table() {
    DiscTable t{};
    for (int s = 0; s < 320; ++s) {
        const int r = s / 9, w = s - 9 * r;
        uint32_t a = 0, m = 0, b = 0;
        for (int j = 0; j < 4; ++j) {
            const int dx = 4 * w - 15 + j, dy = r - 15;
            if (r < 31 && dx <= 15 && dx * dx + dy * dy <= 225) {
                a |= (uint32_t)(dx + 15) << (8 * j);
                m |= 1u << (8 * j);
                b |= (uint32_t)(dy + 15) << (8 * j);
            }
        }
        t.e[s] = DiscSlot{a, m, b, (r < 30 ? r : 30) * TS_DT_RAW_P + 4 * w};
    }
    return t;
}
__constant__ DiscTable c_disc = make_disc_table();

__global__ __launch_bounds__(TS_DT_THREADS) void k_describe(BatchCtx c) {
    // raw tile: the orientation discs' columns [x0 - 16, x0 + 144) only (10 chunks), + 1 row of
    // slack for the masked bytes the last disc row's dword window reads past the row end
    __shared__ __attribute__((aligned(16))) uint8_t s_raw[(TS_DT_RAW_ROWS + 1) * TS_DT_RAW_P];
    __shared__ __attribute__((aligned(16))) uint8_t s_smo[TS_DT_SMO_ROWS * TS_DT_P];
    __shared__ uint16_t s_list[TS_DT_W * TS_DT_H / 4];   // NMS keeps at most one per 2x2
    __shared__ uint32_t s_n;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // block -> (image, level, tile); all tiles of one image on one XCD (tile geometry from the
    // host: no scalar divisions per block beyond the tile's row)
    int img, local;
    if (!xcd_image_block(blockIdx.x, c.n * c.ncam, c.g.dt_total, &img, &local)) return;
    int l = 0;
    while (l + 1 < c.g.n_levels && local >= c.g.dt_start[l + 1]) ++l;
    local -= c.g.dt_start[l];
    const int nx = c.g.dt_nx[l];
    const int ty = local / nx, tx = local - ty * nx;
    const int W = c.g.W[l], H = c.g.H[l];
    const int x0 = tx * TS_DT_W, y0 = ty * TS_DT_H;
    int cam, f;
    view_image(c, img, &f, &cam);
    const int slot = ring_slot(c, c.g0 + f);
    const size_t ib = (size_t)slot * c.C + cam;
    const uint8_t* raw = c.pyr + ib * c.g.pyr_bytes + c.g.pyr_off[l];
    const uint8_t* smo = c.smo + ((size_t)f * c.C + cam) * c.g.pyr_bytes + c.g.pyr_off[l];
    uint32_t* kps = c.kps + ib * c.g.K * 2;
    uint32_t* desc = c.desc + ib * c.g.K * 8;
    uint32_t* desc_ys = c.desc_ys + ib * c.g.K * 8;
    const uint4* ys = c.ys + ib * c.g.K + c.g.koff[l];
    const uint16_t* rs = c.rowstart + ib * c.g.rs_total + c.g.rs_off[l];
    const int kn = c.kcount[ib * c.g.n_levels + l];

    // padding slots of the level get zero descriptors (first tile of the level does it)
    if (local == 0) {
        const int Kl = c.g.Kq[l];
        for (int i = kn * 8 + threadIdx.x; i < Kl * 8; i += TS_DT_THREADS) {
            desc[(size_t)(c.g.koff[l] + i / 8) * 8 + (i & 7)] = 0u;
            desc_ys[(size_t)(c.g.koff[l] + i / 8) * 8 + (i & 7)] = 0u;
        }
    }
    const int pa = rs[y0], pb = rs[min(y0 + TS_DT_H, H)];
    if (pa >= pb) return;   // no keypoint in the tile's rows (block-uniform)
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();

    const bool wide16 = ((W & 15) == 0) && ((c.g.pyr_off[l] & 15) == 0) && ((c.g.pyr_bytes & 15) == 0);
    const int c0 = x0 - TS_DT_HX;        // smoothed tile's column origin (pitch TS_DT_P)
    const int cr = x0 - 16;              // raw tile's column origin (pitch TS_DT_RAW_P)
    stage_tile<TS_DT_RAW_P / 16>(raw, W, H, y0 - 15, cr, TS_DT_RAW_ROWS, s_raw, wide16);
    // smoothed tile: BRIEF reads columns [x0 - 18, x0 + 146): chunks 0..11; chunk 12 is the pad
    stage_tile<TS_DT_P / 16, (TS_DT_W + 2 * TS_DT_HX) / 16>(smo, W, H, y0 - 18, c0, TS_DT_SMO_ROWS, s_smo, wide16);

    // per-lane disc constants (slot s = lane + 64 i; see DiscTable)
    uint32_t wx[5], mk[5], wy[5];
    int rofs[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const uint4 d = reinterpret_cast<const uint4*>(&c_disc)[lane + 64 * i];
        wx[i] = d.x;
        mk[i] = d.y;
        wy[i] = d.z;
        rofs[i] = (int)d.w;
    }
    // wedge directions as doubles: |u| < 2^25 and |m| < 2^23, so every product and difference
    // below is an exact integer in f64 (< 2^53) and the sign tests equal the int64 ones
    const double wa0 = lane < 30 ? (double)c.wedges[2 * lane] : 0.0, wa1 = lane < 30 ? (double)c.wedges[2 * lane + 1] : 0.0;
    const double wb0 = lane < 30 ? (double)c.wedges[2 * lane + 2] : 0.0, wb1 = lane < 30 ? (double)c.wedges[2 * lane + 3] : 0.0;

    // keypoints of the tile: the records of its rows filtered by x, compacted into an LDS list
    // so the 4 waves get equal shares (order is irrelevant: every keypoint is independent)
    for (int p = pa + threadIdx.x; p < pb; p += TS_DT_THREADS) {
        const int x = ys[p].x & 0xFFFF;
        if (x >= x0 && x < x0 + TS_DT_W) s_list[atomicAdd(&s_n, 1u)] = (uint16_t)p;
    }
    __syncthreads();   // tiles landed (drains the LDS-DMA) and the list is complete
    const int n = (int)s_n;
    // groups of TS_DT_G keypoints per wave: all orientations, then all table rows (one exposed
    // latency per group), then the descriptors
    for (int g0 = wave * TS_DT_G; g0 < n; g0 += (TS_DT_THREADS / 64) * TS_DT_G) {
        int bin[TS_DT_G], pos[TS_DT_G];
        uint4 rec[TS_DT_G];
#pragma unroll
        for (int g = 0; g < TS_DT_G; ++g) {
            pos[g] = g0 + g < n ? (int)s_list[g0 + g] : -1;
            rec[g] = pos[g] >= 0 ? ys[pos[g]] : uint4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int g = 0; g < TS_DT_G; ++g) {
            bin[g] = 0;
            if (pos[g] < 0) continue;
            const int x = rec[g].x & 0xFFFF, y = rec[g].x >> 16;
            // orientation: disc origin (x - 15, y - 15) in the raw tile
            const int ob = (y - y0) * TS_DT_RAW_P + (x - 15 - cr);
            const uint32_t sh = (uint32_t)ob & 3u;
            const uint8_t* obase = s_raw + (ob & ~3);
            uint32_t sx = 0, s1 = 0, sy = 0;
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                const uint32_t* wp = reinterpret_cast<const uint32_t*>(obase + rofs[i]);
                const uint32_t v = __builtin_amdgcn_alignbyte(wp[1], wp[0], sh);
                s1 = __builtin_amdgcn_udot4(mk[i], v, s1, false);
                sx = __builtin_amdgcn_udot4(wx[i], v, sx, false);
                sy = __builtin_amdgcn_udot4(wy[i], v, sy, false);
            }
            // per-lane sums < 2^17: 15 * s1 as one full-rate 24-bit multiply
            const int s15 = (int)__umul24(s1, 15u);
            const int m10 = wave_sum_dpp((int)sx - s15);
            const int m01 = wave_sum_dpp((int)sy - s15);
            const double d01 = (double)m01, d10 = (double)m10;
            const bool hit = lane < 30 && (wa0 * d01 - wa1 * d10) >= 0.0 && (wb0 * d01 - wb1 * d10) < 0.0;
            const uint64_t hm = __ballot(hit);
            bin[g] = hm ? (int)__builtin_ctzll(hm) : 0;
        }
        uint32_t t[TS_DT_G][4];
#pragma unroll
        for (int g = 0; g < TS_DT_G; ++g)
#pragma unroll
            for (int j = 0; j < 4; ++j) t[g][j] = pos[g] >= 0 ? c.brief_table[bin[g] * 256 + 64 * j + lane] : 0u;
#pragma unroll
        for (int g = 0; g < TS_DT_G; ++g) {
            if (pos[g] < 0) continue;
            const int x = rec[g].x & 0xFFFF, y = rec[g].x >> 16;
            // BRIEF: patch origin (x - 18, y - 18) in the smoothed tile
            const uint8_t* pbase = s_smo + (y - y0) * TS_DT_P + (x - 18 - c0);
            uint32_t words[8];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int a = pbase[t[g][j] & 0xFFFFu];
                const int b = pbase[t[g][j] >> 16];
                const uint64_t bm = __ballot(a < b);
                words[2 * j] = (uint32_t)bm;
                words[2 * j + 1] = (uint32_t)(bm >> 32);
            }
            const int kidx = (int)rec[g].z;
            // word j (wave-uniform) into lane j: 8 v_writelane
            uint32_t w = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(w) : "s"(words[j]), "i"(j));
            if (lane < 8) {
                desc[(size_t)kidx * 8 + lane] = w;
                desc_ys[(size_t)(c.g.koff[l] + pos[g]) * 8 + lane] = w;
            }
            if (lane == 0) kps[(size_t)kidx * 2 + 1] = (rec[g].y & ~0xFF00u) | ((uint32_t)bin[g] << 8);
        }
    }
}

void launch_describe(const BatchCtx& c, hipStream_t s) {
    hipLaunchKernelGGL(k_describe, dim3(xcd_grid(c.n * c.ncam, c.g.dt_total)), dim3(TS_DT_THREADS), 0, s, c);
}
