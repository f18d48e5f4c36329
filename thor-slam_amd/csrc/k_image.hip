// k_image.hip — rows A2-A4 of SURVEY.md §8a on gfx950: rectify + pyramid, FAST-9 detect with
// smoothing and NMS, exact per-level top-K.  Integer only; bit-exact with oracle/numpy_slam.py
// (remap, pyramid, smooth, fast_scores, nms_keys, select_topk).
//
// Roofline: HBM-bound streaming (1 B/px in, 1.33 B/px pyramid out, 1.33 B/px smoothed out);
// the per-pixel FAST arithmetic (~180 int ops) is far below the VALU ceiling.  Each block owns a
// row band, stages it with its halo in LDS once (coalesced row loads), and does every stencil
// (5x5 smoothing, 16-tap circle, 3x3 NMS) out of LDS.
#include "tslam_common.h"

// ---------------------------------------------------------------------------------------------
// A2 + A3: rectify (fixed-point bilinear remap) and build all pyramid levels for a 32-row band.
// grid (ceil(H/32), n*C), block 256.  32 = 2^5 keeps every level's rows of the band inside the
// block (2x2 boxes never straddle bands) for up to 6 levels.
// ---------------------------------------------------------------------------------------------
// Bilinear sample of the source at a 1/32-px fixed-point map position (oracle.remap).
__device__ __forceinline__ int remap_px(const uint8_t* src, int W, int H, int2 m) {
    const int sx = m.x >> 5, sy = m.y >> 5;
    const int fx = m.x & 31, fy = m.y & 31;
    const int xa = min(max(sx, 0), W - 1), xb = min(max(sx + 1, 0), W - 1);
    const int ya = min(max(sy, 0), H - 1), yb = min(max(sy + 1, 0), H - 1);
    const int p00 = src[ya * W + xa], p01 = src[ya * W + xb];
    const int p10 = src[yb * W + xa], p11 = src[yb * W + xb];
    const int acc = p00 * (32 - fx) * (32 - fy) + p01 * fx * (32 - fy) + p10 * (32 - fx) * fy + p11 * fx * fy;
    return (acc + 512) >> 10;
}

// 2x2 box of 8 bytes of two rows -> 4 output bytes: (a + b + c + d + 2) >> 2 per output, on u16
// pairs (even / odd byte lanes), exact.
__device__ __forceinline__ uint32_t box4(uint32_t r0a, uint32_t r0b, uint32_t r1a, uint32_t r1b) {
    auto pairsum = [](uint32_t v) { return (v & 0x00FF00FFu) + ((v >> 8) & 0x00FF00FFu); };   // (b0+b1, b2+b3)
    const uint32_t sa = pairsum(r0a) + pairsum(r1a) + 0x00020002u;   // outputs 0, 1 (u16 lanes)
    const uint32_t sb = pairsum(r0b) + pairsum(r1b) + 0x00020002u;   // outputs 2, 3
    const uint32_t qa = (sa >> 2) & 0x00FF00FFu, qb = (sb >> 2) & 0x00FF00FFu;
    return __builtin_amdgcn_perm(qb, qa, 0x06040200u);   // bytes: qa.lo, qa.hi, qb.lo, qb.hi
}

__global__ __launch_bounds__(256) void k_rectify_pyramid(BatchCtx c) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int img = blockIdx.y;             // f * ncam + view camera
    int f, cam;
    view_image(c, img, &f, &cam);
    const int W = c.W, H = c.H;
    const int y0 = blockIdx.x * TS_RECT_BAND;
    const int rows0 = min(TS_RECT_BAND, H - y0);
    const uint8_t* src = c.images + view_src(c, img) * W * H;
    uint8_t* pyr = c.pyr + ((size_t)ring_slot(c, c.g0 + f) * c.C + cam) * c.g.pyr_bytes;
    const bool has_map = (c.map_mask >> cam) & 1u;
    const int32_t* map = c.maps + (size_t)cam * W * H * 2;
    // 16-byte rows everywhere (W % 64 == 0 keeps every level's rows 16-byte aligned for 4 levels;
    // the configs in BASELINE.json have W = 640 / 1280): wide path; byte path otherwise
    bool wide = (W & 63) == 0 && (c.g.pyr_bytes & 15) == 0;
    for (int l = 1; l < c.g.n_levels; ++l) wide = wide && (c.g.pyr_off[l] & 15) == 0 && (c.g.W[l] & 15) == 0;

    uint8_t* l0 = lds;
    if (wide) {
        // level 0: 16 pixels per thread item
        const int W16 = W >> 4, n16 = rows0 * W16;
        for (int i = threadIdx.x; i < n16; i += blockDim.x) {
            const int r = i / W16, x16 = i - r * W16;
            const size_t off = (size_t)(y0 + r) * W + 16 * x16;
            uint4 v;
            if (has_map) {
                uint32_t w[4];
                const int2* mp = reinterpret_cast<const int2*>(map) + off;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    uint32_t acc = 0;
#pragma unroll
                    for (int b = 0; b < 4; ++b) acc |= (uint32_t)remap_px(src, W, H, mp[4 * q + b]) << (8 * b);
                    w[q] = acc;
                }
                v = {w[0], w[1], w[2], w[3]};
            } else {
                v = *reinterpret_cast<const uint4*>(src + off);
            }
            reinterpret_cast<uint4*>(l0)[i] = v;
            *reinterpret_cast<uint4*>(pyr + off) = v;
        }
        __syncthreads();
        // levels 1..: 4 output bytes per item from two 8-byte row pieces of the previous level
        const uint8_t* prev = l0;
        int prevW = W;
        uint8_t* cur = l0 + TS_RECT_BAND * W;
        for (int l = 1; l < c.g.n_levels; ++l) {
            const int Wl = c.g.W[l], Hl = c.g.H[l];
            const int ly0 = y0 >> l;
            const int lrows = min(TS_RECT_BAND >> l, Hl - ly0);
            const int W4 = Wl >> 2;
            uint8_t* out = pyr + c.g.pyr_off[l];
            for (int i = threadIdx.x; i < lrows * W4; i += blockDim.x) {
                const int r = i / W4, x4 = i - r * W4;
                const uint2 a = *reinterpret_cast<const uint2*>(prev + (2 * r) * prevW + 8 * x4);
                const uint2 b = *reinterpret_cast<const uint2*>(prev + (2 * r + 1) * prevW + 8 * x4);
                const uint32_t v = box4(a.x, a.y, b.x, b.y);
                reinterpret_cast<uint32_t*>(cur)[i] = v;
                *reinterpret_cast<uint32_t*>(out + (size_t)(ly0 + r) * Wl + 4 * x4) = v;
            }
            __syncthreads();
            prev = cur;
            prevW = Wl;
            cur = cur + (TS_RECT_BAND >> l) * Wl;
        }
        return;
    }

    // byte path (any geometry)
    for (int idx = threadIdx.x; idx < rows0 * W; idx += blockDim.x) {
        const int r = idx / W;
        const int x = idx - r * W;
        const int y = y0 + r;
        const int v = has_map ? remap_px(src, W, H, *reinterpret_cast<const int2*>(map + ((size_t)y * W + x) * 2))
                              : src[y * W + x];
        l0[r * W + x] = (uint8_t)v;
        pyr[(size_t)y * W + x] = (uint8_t)v;
    }
    __syncthreads();
    const uint8_t* prev = l0;
    int prevW = W;
    uint8_t* cur = l0 + TS_RECT_BAND * W;
    for (int l = 1; l < c.g.n_levels; ++l) {
        const int Wl = c.g.W[l], Hl = c.g.H[l];
        const int ly0 = y0 >> l;
        const int lrows = min(TS_RECT_BAND >> l, Hl - ly0);
        uint8_t* out = pyr + c.g.pyr_off[l];
        for (int idx = threadIdx.x; idx < lrows * Wl; idx += blockDim.x) {
            const int r = idx / Wl;
            const int x = idx - r * Wl;
            const int a = prev[(2 * r) * prevW + 2 * x] + prev[(2 * r) * prevW + 2 * x + 1] +
                          prev[(2 * r + 1) * prevW + 2 * x] + prev[(2 * r + 1) * prevW + 2 * x + 1];
            const uint8_t v = (uint8_t)((a + 2) >> 2);
            cur[r * Wl + x] = v;
            out[(size_t)(ly0 + r) * Wl + x] = v;
        }
        __syncthreads();
        prev = cur;
        prevW = Wl;
        cur = cur + (TS_RECT_BAND >> l) * Wl;
    }
}

// ---------------------------------------------------------------------------------------------
// FAST-9 score of the centre pixel at LDS row r, column x (image pitch W).  Exact integer
// definition: max over the 16 arcs of 9 contiguous circle pixels of
// max(min(I_c - I_p), min(I_p - I_c)); callers only keep it when > threshold.
// ---------------------------------------------------------------------------------------------
typedef short s16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ s16x2 pk_min(s16x2 a, s16x2 b) { return __builtin_elementwise_min(a, b); }
__device__ __forceinline__ s16x2 pk_max(s16x2 a, s16x2 b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ s16x2 swp(s16x2 a) { return __builtin_shufflevector(a, a, 1, 0); }

__device__ __forceinline__ int fast9_core(const uint8_t* p, int W, int thr, bool pretest) {
    const int c0 = p[0];
    int d[16];
    d[0] = p[-3 * W] - c0;      d[1] = p[-3 * W + 1] - c0; d[2] = p[-2 * W + 2] - c0; d[3] = p[-W + 3] - c0;
    d[4] = p[3] - c0;           d[5] = p[W + 3] - c0;      d[6] = p[2 * W + 2] - c0;  d[7] = p[3 * W + 1] - c0;
    d[8] = p[3 * W] - c0;       d[9] = p[3 * W - 1] - c0;  d[10] = p[2 * W - 2] - c0; d[11] = p[W - 3] - c0;
    d[12] = p[-3] - c0;         d[13] = p[-W - 3] - c0;    d[14] = p[-2 * W - 2] - c0; d[15] = p[-3 * W - 1] - c0;
    // every 9-arc contains circle index 0 or 8, and 4 or 12: a pixel is not a corner when
    // both of either pair are within the threshold (score irrelevant then: it becomes 0).
    if (pretest) {
        const bool rej = (abs(d[0]) <= thr && abs(d[8]) <= thr) || (abs(d[4]) <= thr && abs(d[12]) <= thr);
        if (rej) return 0;
    }
    // packed pairs P[k] = (d[k], d[k+8]); circle index k+8 (k < 8) is the swapped pair.
    s16x2 P[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) P[k] = (s16x2){(short)d[k], (short)d[k + 8]};
    // S(v, k) = pair for circle index k of a packed 16-array v
#define SEL(v, k) ((k) < 8 ? (v)[(k)] : swp((v)[(k) - 8]))
    s16x2 A2[8], B2[8], A4[8], B4[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        A2[k] = pk_min(P[k], SEL(P, k + 1));
        B2[k] = pk_max(P[k], SEL(P, k + 1));
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        A4[k] = pk_min(A2[k], SEL(A2, k + 2));
        B4[k] = pk_max(B2[k], SEL(B2, k + 2));
    }
    s16x2 br = (s16x2){-1024, -1024}, dk = (s16x2){1024, 1024};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const s16x2 a8 = pk_min(A4[k], SEL(A4, k + 4));
        const s16x2 b8 = pk_max(B4[k], SEL(B4, k + 4));
        br = pk_max(br, pk_min(a8, swp(P[k])));   // a9 = min(a8, d[k+8])
        dk = pk_min(dk, pk_max(b8, swp(P[k])));
    }
#undef SEL
    const int bright = max((int)br.x, (int)br.y);
    const int darkmin = min((int)dk.x, (int)dk.y);
    return max(max(bright, -darkmin), 0);
}

__device__ __forceinline__ int fast9_score(const uint8_t* t, int W, int r, int x, int thr) {
    return fast9_core(t + r * W + x, W, thr, true);
}

// FAST-9 scores of the 4 pixels x0..x0+3 of tile row `rc` (pitch W), thresholded (score > thr,
// else 0), as 4 bytes.  Straight-line packed f16: the pixels travel as (x0, x0+2) / (x0+1, x0+3)
// pairs; a byte b becomes the f16 1024 + b (0x64 as its high byte, one v_perm per pair), so
// every difference, min and max below is exact.  The 16 circle windows come from 3 dword LDS reads per
// circle row + v_alignbyte; each 9-arc minimum is min3(min3 of 3, 3, 3) (v_pk_minimum3_f16).
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ h16x2 hmin3(h16x2 a, h16x2 b, h16x2 c) {
    return __builtin_elementwise_minimum(a, __builtin_elementwise_minimum(b, c));
}
__device__ __forceinline__ h16x2 hmax3(h16x2 a, h16x2 b, h16x2 c) {
    return __builtin_elementwise_maximum(a, __builtin_elementwise_maximum(b, c));
}

// Exact FAST-9 scores of the 4 pixels x0..x0+3 of tile row `rc` (pitch W), thresholded (score >
// thr, else 0), as 4 bytes.  Straight-line packed f16: the pixels travel as (x0, x0+2) / (x0+1,
// x0+3) pairs; a byte b becomes the f16 1024 + b (0x64 as its high byte, one v_perm per pair), so
// every difference, min and max below is exact.  The 16 circle windows come from 3 dword LDS reads
// per circle row + v_alignbyte; each 9-arc minimum is min3(min3 of 3, 3, 3) (v_pk_minimum3_f16).
// SIDE: 1 = bright arcs only (max over arcs of min(I_p) - I_c), 2 = dark only, 3 = both (the
// score).  A pixel whose other side cannot reach thr + 1 (phase A's test) has its score on one side.
template <int SIDE>
__device__ __forceinline__ uint32_t fast4s(const uint8_t* rc, int W, int x0, int thr) {
    // circle index k -> (dx, dy): 0 (0,-3) 1 (1,-3) 2 (2,-2) 3 (3,-1) 4 (3,0) 5 (3,1) 6 (2,2)
    // 7 (1,3) 8 (0,3) 9 (-1,3) 10 (-2,2) 11 (-3,1) 12 (-3,0) 13 (-3,-1) 14 (-2,-2) 15 (-1,-3)
    uint32_t win[16], cen;
    {
        const uint32_t* p = (const uint32_t*)(rc - 3 * W + x0);   // rows walked by adding W
        const int Wd = W >> 2;
        uint32_t a, b, c;
        auto rd = [&]() {
            a = p[-1];
            b = p[0];
            c = p[1];
            p += Wd;
        };
        rd();   // dy = -3
        win[15] = __builtin_amdgcn_alignbyte(b, a, 3); win[0] = b; win[1] = __builtin_amdgcn_alignbyte(c, b, 1);
        rd();   // dy = -2
        win[14] = __builtin_amdgcn_alignbyte(b, a, 2); win[2] = __builtin_amdgcn_alignbyte(c, b, 2);
        rd();   // dy = -1
        win[13] = __builtin_amdgcn_alignbyte(b, a, 1); win[3] = __builtin_amdgcn_alignbyte(c, b, 3);
        rd();   // dy = 0
        win[12] = __builtin_amdgcn_alignbyte(b, a, 1); win[4] = __builtin_amdgcn_alignbyte(c, b, 3); cen = b;
        rd();   // dy = 1
        win[11] = __builtin_amdgcn_alignbyte(b, a, 1); win[5] = __builtin_amdgcn_alignbyte(c, b, 3);
        rd();   // dy = 2
        win[10] = __builtin_amdgcn_alignbyte(b, a, 2); win[6] = __builtin_amdgcn_alignbyte(c, b, 2);
        rd();   // dy = 3
        win[9] = __builtin_amdgcn_alignbyte(b, a, 3); win[8] = b; win[7] = __builtin_amdgcn_alignbyte(c, b, 1);
    }
    // Arc extrema are taken on the raw values (min over an arc of (p - c) = (min over it of p) - c),
    // so the centre is subtracted once: score = max(max_k min9_k - c, c - min_k max9_k, 0).
    uint32_t out = 0;
    constexpr uint32_t k64 = 0x64646464u;
#pragma unroll
    for (int h = 0; h < 2; ++h) {   // h = 0: pixels x0, x0+2; h = 1: pixels x0+1, x0+3
        // v_perm: bytes (h, 2+h) of the window into the low bytes of two f16 lanes, 0x64 above
        const uint32_t sel = h ? 0x00070005u : 0x00060004u;
        auto toh = [sel](uint32_t v) { return __builtin_bit_cast(h16x2, __builtin_amdgcn_perm(v, k64, sel)); };
        h16x2 p[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) p[k] = toh(win[k]);
        const h16x2 cc = toh(cen);
        const h16x2 zero = {(_Float16)0, (_Float16)0};
        h16x2 sb = zero, sd = zero;
        if (SIDE & 1) {
            h16x2 a3[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) a3[k] = hmin3(p[k], p[(k + 1) & 15], p[(k + 2) & 15]);
            h16x2 a9[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) a9[k] = hmin3(a3[k], a3[(k + 3) & 15], a3[(k + 6) & 15]);
            h16x2 br = hmax3(a9[0], a9[1], a9[2]);
#pragma unroll
            for (int k = 3; k < 15; k += 2) br = hmax3(br, a9[k], a9[k + 1]);
            br = __builtin_elementwise_maximum(br, a9[15]);
            sb = br - cc;
        }
        if (SIDE & 2) {
            h16x2 b3[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) b3[k] = hmax3(p[k], p[(k + 1) & 15], p[(k + 2) & 15]);
            h16x2 b9[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) b9[k] = hmax3(b3[k], b3[(k + 3) & 15], b3[(k + 6) & 15]);
            h16x2 dk = hmin3(b9[0], b9[1], b9[2]);
#pragma unroll
            for (int k = 3; k < 15; k += 2) dk = hmin3(dk, b9[k], b9[k + 1]);
            dk = __builtin_elementwise_minimum(dk, b9[15]);
            sd = cc - dk;
        }
        const h16x2 sc = hmax3(sb, sd, zero) + (h16x2){(_Float16)1024, (_Float16)1024};
        const uint32_t bits = __builtin_bit_cast(uint32_t, sc) & 0x03FF03FFu;   // (score, score) as u16
        const uint32_t s0 = bits & 0xFFFFu, s1 = bits >> 16;
        out |= (s0 > (uint32_t)thr ? s0 : 0u) << (8 * h);
        out |= (s1 > (uint32_t)thr ? s1 : 0u) << (8 * h + 16);
    }
    return out;
}


// Phase A of FAST at the speculative threshold te: every 9-arc of the circle holds one of circle
// indices {0, 8} and one of {4, 12}, so score >= te needs max(p0, p8) and max(p4, p12) >= c + te
// (bright) or min(p0, p8) and min(p4, p12) <= c - te (dark).  4 pixels x0..x0+3 of tile row `rc`
// (pitch W) from 5 dword LDS reads, on f16 pairs 1024 + byte (exact): bit j = pixel x0 + j may
// reach te on the bright side, bit 4 + j on the dark side (~25 VALU per quad against ~270 for the
// exact scores of both sides).
__device__ __forceinline__ uint32_t fast4_maybe(const uint8_t* rc, int W, int x0, h16x2 te2) {
    const uint32_t* p = (const uint32_t*)(rc + x0);
    const int Wd = W >> 2;
    const uint32_t up = p[-3 * Wd], dn = p[3 * Wd];
    const uint32_t a = p[-1], b = p[0], cc = p[1];
    const uint32_t w4 = __builtin_amdgcn_alignbyte(cc, b, 3), w12 = __builtin_amdgcn_alignbyte(b, a, 1);
    constexpr uint32_t k64 = 0x64646464u;
    uint32_t bits = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {   // h = 0: pixels x0, x0+2; h = 1: pixels x0+1, x0+3
        const uint32_t sel = h ? 0x00070005u : 0x00060004u;
        auto toh = [sel](uint32_t v) { return __builtin_bit_cast(h16x2, __builtin_amdgcn_perm(v, k64, sel)); };
        const h16x2 p0 = toh(up), p8 = toh(dn), p4 = toh(w4), p12 = toh(w12), c = toh(b);
        const h16x2 bmin = __builtin_elementwise_minimum(__builtin_elementwise_maximum(p0, p8),
                                                         __builtin_elementwise_maximum(p4, p12));
        const h16x2 dmax = __builtin_elementwise_maximum(__builtin_elementwise_minimum(p0, p8),
                                                         __builtin_elementwise_minimum(p4, p12));
        const uint32_t vb = ~__builtin_bit_cast(uint32_t, bmin - (c + te2));   // sign clear: bright candidate
        const uint32_t vd = ~__builtin_bit_cast(uint32_t, (c - te2) - dmax);   // dark candidate
        bits |= ((vb >> 15) & 1u) << h;
        bits |= ((vb >> 31) & 1u) << (h + 2);
        bits |= ((vd >> 15) & 1u) << (h + 4);
        bits |= ((vd >> 31) & 1u) << (h + 6);
    }
    return bits;   // bit j: pixel x0 + j may reach te bright; bit 4 + j: dark
}

// fast4_maybe reduced to the quad's two queue decisions: bit 0 = some pixel may reach te on the
// bright side, bit 1 = on the dark side (a sign bit clear in either f16 pair), without the per-pixel
// bits (~20 VALU fewer per item).  Valid where no pixel of the quad needs the x / y border masks.
__device__ __forceinline__ uint32_t fast4_any(const uint8_t* rc, int W, int x0, h16x2 te2) {
    const uint32_t* p = (const uint32_t*)(rc + x0);
    const int Wd = W >> 2;
    const uint32_t up = p[-3 * Wd], dn = p[3 * Wd];
    const uint32_t a = p[-1], b = p[0], cc = p[1];
    const uint32_t w4 = __builtin_amdgcn_alignbyte(cc, b, 3), w12 = __builtin_amdgcn_alignbyte(b, a, 1);
    constexpr uint32_t k64 = 0x64646464u;
    uint32_t ab = 0xFFFFFFFFu, ad = 0xFFFFFFFFu;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint32_t sel = h ? 0x00070005u : 0x00060004u;
        auto toh = [sel](uint32_t v) { return __builtin_bit_cast(h16x2, __builtin_amdgcn_perm(v, k64, sel)); };
        const h16x2 p0 = toh(up), p8 = toh(dn), p4 = toh(w4), p12 = toh(w12), c = toh(b);
        const h16x2 bmin = __builtin_elementwise_minimum(__builtin_elementwise_maximum(p0, p8),
                                                         __builtin_elementwise_maximum(p4, p12));
        const h16x2 dmax = __builtin_elementwise_maximum(__builtin_elementwise_minimum(p0, p8),
                                                         __builtin_elementwise_minimum(p4, p12));
        ab &= __builtin_bit_cast(uint32_t, bmin - (c + te2));   // sign clear: bright candidate
        ad &= __builtin_bit_cast(uint32_t, (c - te2) - dmax);   // dark candidate
    }
    return ((~ab & 0x80008000u) != 0u ? 1u : 0u) | ((~ad & 0x80008000u) != 0u ? 2u : 0u);
}

// Phase B: exact scores (>= te, else 0) of the `cnt` (<= 64) candidate quads at q (entries
// r << 9 | quad: score row r, columns 4 quad .. 4 quad + 3), one quad per lane with the dense
// aligned-dword fast4s of one side, combined by a byte-wise max into the quad's score word (zeroed
// by phase A; a quad with candidates on both sides is in both queues).  92 % of the candidate quads
// have candidates on one side only, so splitting the queue by side skips half the arc work.
// Wave-local (no block barrier).
#define TS_DET_Q 128   // per-wave, per-side candidate queue (quads): flushed at 64, + <= 64 per append
#ifndef TS_DET_U
#define TS_DET_U 2     // phase-A items per lane per iteration: 2 / 3 / 4 -> 71 / 79 / 80+5 spilled VGPRs;
                       // 467 / 466 / 478 us alone, 931 / 957 / 978 us beside the back end, C2 bench
                       // 145.0k / 143.1k / 141.6k frames/s (round 2)
#endif
__device__ __forceinline__ uint32_t bytes_max(uint32_t a, uint32_t b) {
    typedef unsigned short u16v2 __attribute__((ext_vector_type(2)));
    const u16v2 ae = __builtin_bit_cast(u16v2, a & 0x00FF00FFu), ao = __builtin_bit_cast(u16v2, (a >> 8) & 0x00FF00FFu);
    const u16v2 be = __builtin_bit_cast(u16v2, b & 0x00FF00FFu), bo = __builtin_bit_cast(u16v2, (b >> 8) & 0x00FF00FFu);
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(ae, be)) |
           (__builtin_bit_cast(uint32_t, __builtin_elementwise_max(ao, bo)) << 8);
}
template <int SIDE>
__device__ __forceinline__ void fast_flush(const uint16_t* q, int cnt, const uint8_t* tile, uint32_t* score32, int W,
                                           int te, bool border) {
    const int lane = threadIdx.x & 63;
    if (lane >= cnt) return;
    const uint32_t e = q[lane];
    const int r = (int)(e >> 9), x4 = (int)(e & 511u), x0 = 4 * x4;
    uint32_t sc4 = fast4s<SIDE>(tile + (r + TS_DET_HALO - 1) * W, W, x0, te - 1);
    if (border) {   // margin < 7 only: a quad may hold pixels outside [3, W-3)
        if (x0 < 3) sc4 &= 0xFFFFFFFFu << (8 * (3 - x0));                  // x >= 3
        if (x0 + 4 > W - 3) {                                              // x < W-3
            const int keep = max(W - 3 - x0, 0);
            sc4 &= keep >= 4 ? 0xFFFFFFFFu : ((1u << (8 * keep)) - 1u);
        }
    }
    uint32_t* w = score32 + r * (W >> 2) + x4;
    *w = bytes_max(*w, sc4);
}

// 3x3 NMS of the `cnt` (<= 64) queued nonzero score quads at q (entries r << 9 | quad: score row
// r = y - y0 + 1, pixels 4 quad .. 4 quad + 3), one quad per lane; survivors inside the margin
// M <= x < W - M are appended to `cand` (one LDS atomic per wave) and counted in `hist`.
// Wave-local (no block barrier).
__device__ __forceinline__ void nms_flush(const uint16_t* q, int cnt, const uint32_t* sc32, int W4, int W, int M, int y0,
                                          uint32_t* cand, uint32_t* count, uint32_t* hist) {
    const int lane = threadIdx.x & 63;
    constexpr uint32_t k64 = 0x64646464u;
    const h16x2 half = {(_Float16)0.5, (_Float16)0.5};
    uint32_t kbits = 0;   // bit j: pixel x0 + j survives
    uint32_t P = 0;
    int y = 0, x0 = 0;
    if (lane < cnt) {
        const uint32_t e = q[lane];
        const int r = (int)(e >> 9), qq = (int)(e & 511u);
        y = y0 - 1 + r;
        x0 = 4 * qq;
        const uint32_t* pm = sc32 + r * W4 + qq;
        const uint32_t* pu = pm - W4;
        const uint32_t* pd = pm + W4;
        P = pm[0];
        const uint32_t ua = pu[-1], ub = pu[0], uc = pu[1];
        const uint32_t ma = pm[-1], mc = pm[1];
        const uint32_t da = pd[-1], db = pd[0], dc = pd[1];
        const uint32_t ul = __builtin_amdgcn_alignbyte(ub, ua, 3), ur = __builtin_amdgcn_alignbyte(uc, ub, 1);
        const uint32_t ml = __builtin_amdgcn_alignbyte(P, ma, 3), mr = __builtin_amdgcn_alignbyte(mc, P, 1);
        const uint32_t dl = __builtin_amdgcn_alignbyte(db, da, 3), dr = __builtin_amdgcn_alignbyte(dc, db, 1);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t sel = h ? 0x00070005u : 0x00060004u;
            auto toh = [sel](uint32_t v) { return __builtin_bit_cast(h16x2, __builtin_amdgcn_perm(v, k64, sel)); };
            const h16x2 pp = toh(P);
            const h16x2 before = hmax3(hmax3(toh(ul), toh(ub), toh(ur)), toh(ml), toh(ml));
            const h16x2 after = hmax3(hmax3(toh(dl), toh(db), toh(dr)), toh(mr), toh(mr));
            const h16x2 k = __builtin_elementwise_minimum((pp - before) - half, pp - after);
            const uint32_t nb = ~__builtin_bit_cast(uint32_t, k);
            kbits |= ((nb >> 15) & 1u) << h;
            kbits |= ((nb >> 31) & 1u) << (h + 2);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (x0 + j < M || x0 + j >= W - M) kbits &= ~(1u << j);
    }
    uint64_t bm[4];
    uint32_t tot = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        bm[j] = __ballot((kbits >> j) & 1u);
        tot += (uint32_t)__popcll(bm[j]);
    }
    if (tot == 0) return;   // wave-uniform
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(count, tot);
    base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if ((kbits >> j) & 1u) {
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(bm[j] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm[j], 0u));
            const uint32_t pv = (P >> (8 * j)) & 0xFFu;
            cand[base + rank] = ((255u - pv) << 22) | ((uint32_t)y << 11) | (uint32_t)(x0 + j);
            atomicAdd(&hist[255 - pv], 1u);
        }
        base += (uint32_t)__popcll(bm[j]);
    }
}

// ---------------------------------------------------------------------------------------------
// A3 smoothing + A4 FAST/NMS candidates for one band of BR = g.band_rows rows of one level.
// grid (total_bands, n*C), block 512 (8 waves).  LDS: image rows [y0-4, y0+BR+4) (row-clamped),
// scores of rows [y0-1, y0+BR+1): (2 BR + 10) W bytes.  BR = 32 at W <= 640 (47 KiB, 3 blocks per
// CU = the VGPR limit at 70 registers; 1.25x halo rows instead of 1.5x at BR = 16: 778 -> 725 us
// per 256-frame batch), 24 at W = 1280 (74 KiB, 2 blocks per CU as at 16: 611 -> 575 us per
// 50-frame C4 batch).  Work inside each phase is dealt
// to the 8 waves in equal (row, 64-lane chunk) items.
// ---------------------------------------------------------------------------------------------
#define TS_DET_THREADS 512
#define TS_DET_WAVES (TS_DET_THREADS / 64)

// 16-byte async global -> LDS copy; `wave_dst` is the wave-uniform LDS base, lane k lands at +16k
__device__ __forceinline__ void glds16(const uint4* src, uint4* wave_dst) {
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)wave_dst, 16, 0, 0);
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// Horizontal 1-4-6-4-1 of the 4 pixels x0..x0+3 of one tile row as two u16 pairs:
// ev = (h[x0], h[x0+2]), od = (h[x0+1], h[x0+3]).  Byte windows D_k = row[x0-2+k .. x0+1+k].
// Column clamp (x-2 < 0, x+2 > W-1) only for the first and last quad of a row.
__device__ __forceinline__ void hsum4(const uint8_t* row, int x0, int W, u16x2* ev, u16x2* od) {
    uint32_t D[5];
    if (x0 >= 4 && x0 + 8 <= W) {
        const uint32_t a = *(const uint32_t*)(row + x0 - 4), b = *(const uint32_t*)(row + x0),
                       c2 = *(const uint32_t*)(row + x0 + 4);
        D[0] = __builtin_amdgcn_alignbyte(b, a, 2);
        D[1] = __builtin_amdgcn_alignbyte(b, a, 3);
        D[2] = b;
        D[3] = __builtin_amdgcn_alignbyte(c2, b, 1);
        D[4] = __builtin_amdgcn_alignbyte(c2, b, 2);
    } else {
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            uint32_t w = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) w |= (uint32_t)row[min(max(x0 - 2 + k + j, 0), W - 1)] << (8 * j);
            D[k] = w;
        }
    }
    // pixel x0 + j: taps row[x0-2+j .. x0+1+j] = bytes of D_j against weights (1, 4, 6, 4), plus
    // row[x0+2+j] = byte 3 of D_{j+1}: one v_dot4_u32_u8 with that byte as the accumulator
    uint32_t hj[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) hj[j] = __builtin_amdgcn_udot4(D[j], 0x04060401u, D[j + 1] >> 24, false);
    *ev = __builtin_bit_cast(u16x2, hj[0] | (hj[2] << 16));   // sums <= 16 * 255: u16 lanes
    *od = __builtin_bit_cast(u16x2, hj[1] | (hj[3] << 16));
}

// Horizontal 1-4-6-4-1 of an interior quad (4 <= x0, x0 + 8 <= W: no column clamp), `p` = row + x0.
__device__ __forceinline__ void hsum4_in(const uint8_t* p, u16x2* ev, u16x2* od) {
    const uint32_t a = *(const uint32_t*)(p - 4), b = *(const uint32_t*)p, c2 = *(const uint32_t*)(p + 4);
    const uint32_t D0 = __builtin_amdgcn_alignbyte(b, a, 2), D1 = __builtin_amdgcn_alignbyte(b, a, 3);
    const uint32_t D3 = __builtin_amdgcn_alignbyte(c2, b, 1), D4 = __builtin_amdgcn_alignbyte(c2, b, 2);
    const uint32_t h0 = __builtin_amdgcn_udot4(D0, 0x04060401u, D1 >> 24, false);
    const uint32_t h1 = __builtin_amdgcn_udot4(D1, 0x04060401u, b >> 24, false);
    const uint32_t h2 = __builtin_amdgcn_udot4(b, 0x04060401u, D3 >> 24, false);
    const uint32_t h3 = __builtin_amdgcn_udot4(D3, 0x04060401u, D4 >> 24, false);
    *ev = __builtin_bit_cast(u16x2, h0 | (h2 << 16));
    *od = __builtin_bit_cast(u16x2, h1 | (h3 << 16));
}

// Vertical 1-4-6-4-1 of five horizontal sums (rows o-2 .. o+2) + rounding, packed to 4 bytes: the
// rounded sums stay below 2^16, so byte 1 of each u16 lane is the result (one v_perm picks the
// four: ev lanes -> bytes 0 / 2, od lanes -> bytes 1 / 3).
__device__ __forceinline__ uint32_t vsum4(u16x2 e0, u16x2 e1, u16x2 e2, u16x2 e3, u16x2 e4, u16x2 d0, u16x2 d1,
                                          u16x2 d2, u16x2 d3, u16x2 d4) {
    const u16x2 four = {4, 4}, six = {6, 6}, rnd = {128, 128};
    const u16x2 ve = six * e2 + (four * (e1 + e3) + ((e0 + e4) + rnd));
    const u16x2 vo = six * d2 + (four * (d1 + d3) + ((d0 + d4) + rnd));
    return __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, vo), __builtin_bit_cast(uint32_t, ve), 0x07030501u);
}

// MODE 0: speculative threshold (k_detect); MODE 1: exact fallback at t + 1 for the flagged
// images (k_detect_fallback, its own symbol so profiles keep the two launches apart)
// (bx: the band over all levels, img: the view image; the fallback runs only flagged image-levels)
template <int MODE>
__device__ __forceinline__ void detect_body(const BatchCtx& c, int bx, int img) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    __shared__ uint32_t s_hist[256];
    __shared__ uint32_t s_count;
    __shared__ uint16_t s_q[TS_DET_WAVES][2][TS_DET_Q];   // per wave: bright, dark candidate quads
    int f, cam;
    view_image(c, img, &f, &cam);
    int l = 0;
    while (l + 1 < c.g.n_levels && bx >= c.g.band_start[l + 1]) ++l;
    // speculative threshold: scores below te cannot reach the level's top K (select checks it)
    const int te = MODE == 1 ? c.fast_threshold + 1
                                   : max(c.fast_threshold + 1, (int)c.det_thr[(size_t)cam * c.g.n_levels + l]);
    const int band = bx - c.g.band_start[l];
    const int W = c.g.W[l], H = c.g.H[l];
    const int BR = c.g.band_rows[l];
    const int y0 = band * BR;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t img_off = ((size_t)ring_slot(c, c.g0 + f) * c.C + cam) * c.g.pyr_bytes + c.g.pyr_off[l];
    const uint8_t* src = c.pyr + img_off;
    uint8_t* smo = c.smo + ((size_t)f * c.C + cam) * c.g.pyr_bytes + c.g.pyr_off[l];
    const int NR = BR + 2 * TS_DET_HALO;
    uint8_t* tile = lds;
    uint8_t* score = lds + NR * W;
    const int thr = c.fast_threshold;
    // dword rows (W % 4 == 0: every config in BASELINE.json) take the packed paths; byte rows
    // the scalar ones
    const bool wide = ((W & 3) == 0) && ((img_off & 3) == 0);
    const int rows_here = min(BR, H - y0);

    for (int i = threadIdx.x; i < 256; i += TS_DET_THREADS) s_hist[i] = 0;
    if (threadIdx.x == 0) s_count = 0;
    if (((W & 15) == 0) && ((img_off & 15) == 0)) {
        // LDS-DMA: each wave-instruction lands 1 KiB of the lane-linear tile, no VGPRs
        const int W16 = W >> 4, n16 = NR * W16;
        const uint4* s16 = (const uint4*)src;
        // (row, chunk) of i = i0 + lane stepped without a division per chunk
        const int dr = TS_DET_THREADS / W16, dx = TS_DET_THREADS - dr * W16;
        int r = (wave * 64 + lane) / W16, x = wave * 64 + lane - r * W16;
        for (int i0 = wave * 64; i0 < n16; i0 += TS_DET_THREADS) {
            if (i0 + lane < n16)
                glds16(s16 + (size_t)min(max(y0 - TS_DET_HALO + r, 0), H - 1) * W16 + x, (uint4*)tile + i0);
            r += dr;
            x += dx;
            if (x >= W16) {
                x -= W16;
                ++r;
            }
        }
    } else {
        for (int i = threadIdx.x; i < NR * W; i += TS_DET_THREADS) {
            const int r = i / W, x = i - r * W;
            tile[i] = src[(size_t)min(max(y0 - TS_DET_HALO + r, 0), H - 1) * W + x];
        }
    }
    __syncthreads();

    // 5x5 binomial smoothing of the band rows (column clamp; rows already clamped in LDS).
    if (wide) {
        // item = (4-pixel quad, row group): the horizontal sums (3 dword LDS reads + 4 v_dot4
        // each) slide through 5 register pairs, rotated by unrolling 5 rows (no moves); u16 pairs
        // cannot overflow (16 * 16 * 255 + 128 < 2^16).  Interior quads (1 .. W4 - 2) need no
        // column clamp and run without divergence; the two edge quads of each row group follow.
        const int W4 = W >> 2;
        const int groups = c.g.smooth_groups[l];
        const int SR = (BR + groups - 1) / groups;
        const int NQ = W4 - 2;
        for (int it = threadIdx.x; it < groups * NQ; it += TS_DET_THREADS) {
            const int half = it / NQ, q = 1 + (it - half * NQ), x0 = 4 * q;
            const int o0 = SR * half, o1 = min(o0 + SR, rows_here);   // output rows (band-relative)
            if (o0 >= o1) continue;
            const uint8_t* rp = tile + (TS_DET_HALO - 2 + o0) * W + x0;
            u16x2 e0, e1, e2, e3, e4, d0, d1, d2, d3, d4;
            hsum4_in(rp, &e0, &d0);
            hsum4_in(rp + W, &e1, &d1);
            hsum4_in(rp + 2 * W, &e2, &d2);
            hsum4_in(rp + 3 * W, &e3, &d3);
            rp += 4 * W;
            uint32_t off = (uint32_t)((y0 + o0) * W + x0);
            int o = o0;
#define TS_SMOOTH_ROW(A, B, C, D, N, a, b, cc, d, n)                            \
    {                                                                         \
        hsum4_in(rp, &N, &n);                                                 \
        *(uint32_t*)(smo + off) = vsum4(A, B, C, D, N, a, b, cc, d, n);       \
        rp += W;                                                              \
        off += (uint32_t)W;                                                   \
        if (++o == o1) break;                                                 \
    }
            for (;;) {
                TS_SMOOTH_ROW(e0, e1, e2, e3, e4, d0, d1, d2, d3, d4)
                TS_SMOOTH_ROW(e1, e2, e3, e4, e0, d1, d2, d3, d4, d0)
                TS_SMOOTH_ROW(e2, e3, e4, e0, e1, d2, d3, d4, d0, d1)
                TS_SMOOTH_ROW(e3, e4, e0, e1, e2, d3, d4, d0, d1, d2)
                TS_SMOOTH_ROW(e4, e0, e1, e2, e3, d4, d0, d1, d2, d3)
            }
#undef TS_SMOOTH_ROW
        }
        for (int it = threadIdx.x; it < groups * 2; it += TS_DET_THREADS) {   // the edge quads (clamped)
            const int half = it >> 1, x0 = (it & 1) ? 4 * (W4 - 1) : 0;
            const int o0 = SR * half, o1 = min(o0 + SR, rows_here);
            if (o0 >= o1) continue;
            u16x2 e[5], d[5];
#pragma unroll
            for (int k = 0; k < 4; ++k) hsum4(tile + (TS_DET_HALO - 2 + o0 + k) * W, x0, W, &e[k], &d[k]);
            for (int o = o0; o < o1; ++o) {
                hsum4(tile + (TS_DET_HALO + 2 + o) * W, x0, W, &e[4], &d[4]);
                *(uint32_t*)(smo + (size_t)(y0 + o) * W + x0) = vsum4(e[0], e[1], e[2], e[3], e[4], d[0], d[1], d[2], d[3], d[4]);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    e[k] = e[k + 1];
                    d[k] = d[k + 1];
                }
            }
        }
    } else {
        for (int x = threadIdx.x; x < W; x += TS_DET_THREADS) {
            const int xm2 = max(x - 2, 0), xm1 = max(x - 1, 0), xp1 = min(x + 1, W - 1), xp2 = min(x + 2, W - 1);
            int h0 = 0, h1 = 0, h2 = 0, h3 = 0;
            for (int r = TS_DET_HALO - 2; r < TS_DET_HALO + rows_here + 2; ++r) {
                const uint8_t* row = tile + r * W;
                const int h4 = row[xm2] + 4 * row[xm1] + 6 * row[x] + 4 * row[xp1] + row[xp2];
                if (r >= TS_DET_HALO + 2) {
                    const int acc = h0 + 4 * h1 + 6 * h2 + 4 * h3 + h4;
                    smo[(size_t)(y0 + r - 2 - TS_DET_HALO) * W + x] = (uint8_t)((acc + 128) >> 8);
                }
                h0 = h1; h1 = h2; h2 = h3; h3 = h4;
            }
        }
    }

    // FAST scores (>= te, else 0) for rows y0-1 .. y0+BR
    if (wide) {
        // phase A over (row, quad) items: the four compass points of 4 pixels per lane; quads
        // with a candidate pixel (~30 % at a learnt te against ~90 % at t) go to the wave's LDS
        // queue (ballot + mbcnt) and get the exact scores, one quad per lane, in rounds of 64
        // (phase B, the dense fast4); the others keep a zero score word
        uint32_t* score32 = (uint32_t*)score;
        const int W4 = W >> 2;
        // only where the NMS reads: rows y in [M-1, H-M], columns [M-1, W-M] (keypoints lie in
        // [M, W-M) x [M, H-M)); the margin is ~20 % of a 640x400 pyramid's pixels.  Score words
        // outside are never read for a pixel inside the margin.
        const int Mg = c.margin;
        const int ra = max(0, Mg - y0), rb = min(BR + 2, H - Mg + 2 - y0);
        const int qa = (Mg - 1) >> 2, nq = ((W - Mg) >> 2) + 1 - qa;
        // with Mg >= 7 every scored pixel lies in rows [Mg-1, H-Mg] and columns [4 qa, W-Mg+3]
        // inside [3, H-3) x [3, W-3): the FAST border tests are needed only below that
        const bool border = Mg < 7;
        const _Float16 tef = (_Float16)te;
        const h16x2 te2 = {tef, tef};
        uint16_t* qb = s_q[wave][0];
        uint16_t* qd = s_q[wave][1];
        int nqb = 0, nqd = 0;   // wave-uniform
        const int nitems = max(rb - ra, 0) * nq;
        // (row, quad) of item it = wave * 64 + lane + k * TS_DET_THREADS, stepped without a division;
        // TS_DET_U items per lane per iteration, so their 5 LDS reads each are in flight together
        // (one item per iteration left phase A waiting on LDS latency)
        const int dr = TS_DET_THREADS / nq, dq = TS_DET_THREADS - dr * nq;
        int r = ra + (wave * 64 + lane) / nq, x4 = qa + (wave * 64 + lane) % nq;
        for (int i0 = wave * 64; i0 < nitems; i0 += TS_DET_U * TS_DET_THREADS) {
            int ru[TS_DET_U], xu[TS_DET_U];
            bool cb[TS_DET_U], cd[TS_DET_U];
#pragma unroll
            for (int u = 0; u < TS_DET_U; ++u) {
                ru[u] = r;
                xu[u] = x4;
                r += dr;
                x4 += dq;
                if (x4 >= qa + nq) {
                    x4 -= nq;
                    ++r;
                }
            }
#pragma unroll
            for (int u = 0; u < TS_DET_U; ++u) {
                const bool active = i0 + u * TS_DET_THREADS + lane < nitems;
                const int y = y0 - 1 + ru[u], x0 = 4 * xu[u];
                cb[u] = cd[u] = false;
                if (active) {
                    if (!border) {
                        const uint32_t m = fast4_any(tile + (ru[u] + TS_DET_HALO - 1) * W, W, x0, te2);
                        cb[u] = (m & 1u) != 0u;
                        cd[u] = (m & 2u) != 0u;
                    } else if (y >= 3 && y < H - 3) {
                        uint32_t c4 = fast4_maybe(tile + (ru[u] + TS_DET_HALO - 1) * W, W, x0, te2);
                        if (x0 < 3) c4 &= 0x11u * ((0xFu << (3 - x0)) & 0xFu);          // x >= 3 (both nibbles)
                        if (x0 + 4 > W - 3) c4 &= 0x11u * ((1u << max(W - 3 - x0, 0)) - 1u);   // x < W-3
                        cb[u] = (c4 & 0xFu) != 0;
                        cd[u] = (c4 >> 4) != 0;
                    }
                    score32[ru[u] * W4 + xu[u]] = 0;   // the flushes max their scores into it
                }
            }
#pragma unroll
            for (int u = 0; u < TS_DET_U; ++u) {
                const uint32_t ent = ((uint32_t)ru[u] << 9) | (uint32_t)xu[u];
                const uint64_t bb = __ballot(cb[u]), bd = __ballot(cd[u]);
                if (cb[u]) qb[nqb + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bb, 0u))] = (uint16_t)ent;
                if (cd[u]) qd[nqd + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bd >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bd, 0u))] = (uint16_t)ent;
                nqb += (int)__popcll(bb);
                nqd += (int)__popcll(bd);
                // a wave's LDS operations complete in issue order, and the queues are wave-private:
                // no fence between its entries' stores and the flush's loads
                if (nqb >= 64) {
                    fast_flush<1>(qb + nqb - 64, 64, tile, score32, W, te, border);
                    nqb -= 64;
                }
                if (nqd >= 64) {
                    fast_flush<2>(qd + nqd - 64, 64, tile, score32, W, te, border);
                    nqd -= 64;
                }
            }
        }
        if (nqb > 0) fast_flush<1>(qb, nqb, tile, score32, W, te, border);
        if (nqd > 0) fast_flush<2>(qd, nqd, tile, score32, W, te, border);
    } else {
        for (int i = threadIdx.x; i < (BR + 2) * W; i += TS_DET_THREADS) {
            const int r = i / W, x = i - r * W;
            const int y = y0 - 1 + r;
            int sc = 0;
            if (y >= 3 && y < H - 3 && x >= 3 && x < W - 3) {
                sc = fast9_score(tile, W, r + TS_DET_HALO - 1, x, thr);
                if (sc < te) sc = 0;
            }
            score[i] = (uint8_t)sc;
        }
    }
    __syncthreads();

    // 3x3 NMS (ties -> earlier raster position) inside the margin; emit keys.
    const int M = c.margin;
    uint32_t* cand = c.cand + ((size_t)f * c.C + cam) * c.g.cand_total + c.g.cand_off[l] + (size_t)band * c.g.cand_cap[l];
    const int ylo = max(y0, M), yhi = min(y0 + BR, H - M);
    if (wide) {
        // Only quads with a nonzero score word can hold a survivor (~10 % of them at a learnt te),
        // but a wave of 64 quads almost always has one, so a dense pass ran the whole test for
        // every quad.  A scan over the score words (one LDS read + a ballot per quad) queues the
        // nonzero quads in the wave's (now idle) phase-B queue; each 64 queued quads get the test:
        // 4 pixels per lane, keep = p > max(4 earlier neighbours) && p >= max(4 later ones), on the
        // two f16 pixel pairs (1024 + score, exact); survivors are appended with one LDS atomic
        // per wave and pixel slot.  The candidate order in `cand` never mattered (select sorts by
        // key, and the LDS atomics already made it arrival order).
        const int W4 = W >> 2;
        const uint32_t* sc32 = (const uint32_t*)score;
        uint16_t* nq = s_q[wave][0];   // 2 * TS_DET_Q contiguous entries: phase B is done (barrier)
        int nn = 0;                    // wave-uniform
        const int dr = TS_DET_THREADS / W4, dq = TS_DET_THREADS - dr * W4;
        int yy = (wave * 64 + lane) / W4, q = wave * 64 + lane - yy * W4;   // stepped without a division
        for (int i0 = wave * 64; i0 < (yhi - ylo) * W4;
             i0 += TS_DET_THREADS, yy += dr, q += dq, (q >= W4 ? (q -= W4, ++yy) : 0)) {
            bool nz = false;
            const int r = ylo + yy - y0 + 1;
            if (i0 + lane < (yhi - ylo) * W4) nz = sc32[r * W4 + q] != 0u && 4 * q + 4 > M && 4 * q < W - M;
            const uint64_t bm = __ballot(nz);
            if (nz) nq[nn + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u))] =
                        (uint16_t)(((uint32_t)r << 9) | (uint32_t)q);
            nn += (int)__popcll(bm);
            if (nn >= 64) {
                nms_flush(nq + nn - 64, 64, sc32, W4, W, M, y0, cand, &s_count, s_hist);
                nn -= 64;
            }
        }
        if (nn > 0) nms_flush(nq, nn, sc32, W4, W, M, y0, cand, &s_count, s_hist);
    } else {
        const int xspan = W - 2 * M, nchx = (xspan + 63) >> 6;
        for (int it = wave; it < (yhi - ylo) * nchx; it += TS_DET_WAVES) {
            const int yy = it / nchx, ch = it - yy * nchx;
            const int y = ylo + yy, x = M + ch * 64 + lane;
            if (x >= W - M) continue;
            const int r = y - y0 + 1;
            const int p = score[r * W + x];
            if (p == 0) continue;
            const uint8_t* up = score + (r - 1) * W + x;
            const uint8_t* mid = score + r * W + x;
            const uint8_t* dn = score + (r + 1) * W + x;
            const bool keep = up[-1] < p && up[0] < p && up[1] < p && mid[-1] < p &&
                              mid[1] <= p && dn[-1] <= p && dn[0] <= p && dn[1] <= p;
            if (keep) {
                const uint32_t key = ((uint32_t)(255 - p) << 22) | ((uint32_t)y << 11) | (uint32_t)x;
                const uint32_t slot = atomicAdd(&s_count, 1u);
                cand[slot] = key;
                atomicAdd(&s_hist[255 - p], 1u);
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) c.ccount[((size_t)f * c.C + cam) * c.g.total_bands + bx] = s_count;
    uint32_t* gh = c.hist + (((size_t)f * c.C + cam) * c.g.n_levels + l) * 256;
    for (int i = threadIdx.x; i < 256; i += TS_DET_THREADS)
        if (s_hist[i]) atomicAdd(&gh[i], s_hist[i]);
}

// 6 waves per SIMD (VGPRs <= 80; 71 without spills at TS_DET_U = 2): three 512-thread blocks per CU, as the LDS
// allows, instead of two at 84 VGPRs (567 -> 528 us per 256-frame batch alone)
__global__ __launch_bounds__(TS_DET_THREADS) __attribute__((amdgpu_waves_per_eu(6))) void k_detect(BatchCtx c) {
    detect_body<0>(c, blockIdx.x, blockIdx.y);
}

// The exact fallback at t + 1 for the image-levels whose speculative select came short (rare):
// TS_FB_BLOCKS persistent blocks scan the (image, level) flags, one per thread and a block-wide OR,
// and run every band of a flagged image-level (detect) or its top-K (select) in turn.  With no
// flag set a launch is one flag load per thread; the per-band / per-level grids of the
// speculative kernels had cost ~55 us of empty blocks per 1024-frame batch on the critical path.
#define TS_FB_BLOCKS 32
template <typename F>
__device__ __forceinline__ void for_flagged_levels(const BatchCtx& c, int nthreads, F&& fn) {
    __shared__ int s_items[1024];
    __shared__ int s_n;
    const int L = c.g.n_levels, total = c.n * c.ncam * L;
    for (int i0 = blockIdx.x * nthreads; i0 < total; i0 += gridDim.x * nthreads) {
        if (threadIdx.x == 0) s_n = 0;
        __syncthreads();
        const int i = i0 + (int)threadIdx.x;
        if (i < total) {
            int f, cam;
            view_image(c, i / L, &f, &cam);
            if (c.det_fail[((size_t)f * c.C + cam) * L + i % L]) s_items[atomicAdd(&s_n, 1)] = i;
        }
        __syncthreads();
        const int n = s_n;
        for (int k = 0; k < n; ++k) {
            fn(s_items[k] / L, s_items[k] % L);
            __syncthreads();   // LDS reuse by the next item
        }
    }
}

__global__ __launch_bounds__(TS_DET_THREADS) void k_detect_fallback(BatchCtx c) {
    for_flagged_levels(c, TS_DET_THREADS, [&](int img, int l) {
        for (int b = 0; b < c.g.nbands[l]; ++b) {
            detect_body<1>(c, c.g.band_start[l] + b, img);
            __syncthreads();
        }
    });
}

// ---------------------------------------------------------------------------------------------
// A4 top-K: exact K_l smallest keys of an image level, sorted ascending.
// Radix select on (score bin, y, x) histograms, then counting sorts (bitonic fallback) in LDS.
// grid (n*C, n_levels), block 1024: blockIdx.y = level, so every level-0 block (the ~10k-
// candidate sweeps) is dispatched in the first round and the short upper-level blocks follow;
// LDS (42 KiB) and wave slots allow 2 such blocks per CU = 512 at once.
// ---------------------------------------------------------------------------------------------
#define SEL_THREADS 1024
#define SEL_MAX 8192

// smallest bin b with sum(h[0..b]) >= need; returns b and the count strictly before it.
// Inclusive scan of one value per thread over the block (SEL_THREADS = 16 waves): a 6-step
// shuffle scan inside each wave, the 16 wave totals through LDS, two barriers in all (a
// Hillis-Steele scan through LDS took 20).  s_w: 2 x 16 words, alternated by `phase` so that
// back-to-back scans need no barrier between them.
__device__ __forceinline__ uint32_t block_inclusive_scan(uint32_t v, uint32_t* s_w, int phase) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)v, o, 64);
        if (lane >= o) v += t;
    }
    uint32_t* w = s_w + 16 * (phase & 1);
    if (lane == 63) w[wave] = v;
    __syncthreads();
    uint32_t add = 0;
    for (int k = 0; k < wave; ++k) add += w[k];
    return v + add;
}

__device__ void block_find_crossing(const uint32_t* h, int nbins, uint32_t need, uint32_t* s_part,
                                    int* out_bin, uint32_t* out_before) {
    const int per = (nbins + SEL_THREADS - 1) / SEL_THREADS;
    const int b0 = threadIdx.x * per;
    uint32_t local = 0;
    for (int b = b0; b < min(b0 + per, nbins); ++b) local += h[b];
    const uint32_t incl = block_inclusive_scan(local, s_part, 0);
    const uint32_t excl = incl - local;
    if (excl < need && incl >= need) {
        uint32_t cum = excl;
        for (int b = b0; b < min(b0 + per, nbins); ++b) {
            if (cum + h[b] >= need) {
                *out_bin = b;
                *out_before = cum;
                break;
            }
            cum += h[b];
        }
    }
    __syncthreads();
}

#define TS_SEL_BUCKET_MAX 256   // larger score buckets -> bitonic fallback (O(n^2) ranking)

// In-place exclusive scan of a[0..n) (n <= 8 * SEL_THREADS) by the whole block; ends synchronised.
__device__ void block_exclusive_scan(uint32_t* a, int n, uint32_t* s_part) {
    const int per = (n + SEL_THREADS - 1) / SEL_THREADS;
    const int b0 = threadIdx.x * per;
    uint32_t local = 0;
    for (int b = b0; b < min(b0 + per, n); ++b) local += a[b];
    uint32_t run = block_inclusive_scan(local, s_part, 1) - local;
    for (int b = b0; b < min(b0 + per, n); ++b) {
        const uint32_t v = a[b];
        a[b] = run;
        run += v;
    }
    __syncthreads();
}

// Ascending bitonic sort of a[0..n) in place (pads to a power of two with 0xFFFFFFFF; n <= SEL_MAX).
__device__ void bitonic_sort(uint32_t* a, int n) {
    int np2 = 1;
    while (np2 < n) np2 <<= 1;
    for (int i = n + threadIdx.x; i < np2; i += SEL_THREADS) a[i] = 0xFFFFFFFFu;
    __syncthreads();
    for (int k = 2; k <= np2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < np2; i += SEL_THREADS) {
                const int p = i ^ j;
                if (p > i) {
                    const uint32_t x = a[i], y = a[p];
                    const bool up = (i & k) == 0;
                    if ((x > y) == up) {
                        a[i] = y;
                        a[p] = x;
                    }
                }
            }
            __syncthreads();
        }
    }
}

template <int MODE>
__device__ __forceinline__ void select_body(const BatchCtx& c, int img, int l) {
    __shared__ uint32_t s_keys[SEL_MAX];
    __shared__ uint32_t s_h[2048];
    __shared__ uint32_t s_part[SEL_THREADS];
    __shared__ uint32_t s_pref[SEL_THREADS + 1];
    __shared__ int s_bin;
    __shared__ uint32_t s_before, s_nsel, s_flag;
    int f, cam;
    view_image(c, img, &f, &cam);
    const size_t fcl = ((size_t)f * c.C + cam) * c.g.n_levels + l;
    const int Kl = c.g.Kq[l];
    const uint32_t* cand = c.cand + ((size_t)f * c.C + cam) * c.g.cand_total + c.g.cand_off[l];
    const uint32_t* cnt = c.ccount + ((size_t)f * c.C + cam) * c.g.total_bands + c.g.band_start[l];
    uint32_t* gh = c.hist + (((size_t)f * c.C + cam) * c.g.n_levels + l) * 256;
    const int nb = c.g.nbands[l];
    const int cap = c.g.cand_cap[l];

    // band counts -> exclusive prefix (flat candidate index i lives in band b with
    // s_pref[b] <= i < s_pref[b+1]); every pass below is then one flat, independent-load sweep
    // over the level's candidates (a per-band loop serialised ~25 dependent global round trips)
    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
        s_h[i] = gh[i];
        gh[i] = 0u;   // back to zero for the next detect of this image-level (fallback or next batch)
    }
    {
        const uint32_t bc = (int)threadIdx.x < nb ? cnt[threadIdx.x] : 0u;
        const uint32_t incl = block_inclusive_scan(bc, s_part, 1);
        if (threadIdx.x == 0) s_pref[0] = 0u;
        if ((int)threadIdx.x < nb) s_pref[threadIdx.x + 1] = incl;
    }
    __syncthreads();
    const int ncand = (int)s_pref[nb];
    // sweep(fn): fn(key) for every candidate, 4 independent loads in flight per thread.  A
    // thread's indices only grow along a sweep, so its band (the b with s_pref[b] <= i <
    // s_pref[b+1]; s_pref[nb] = ncand ends the walk) is found by walking forward from the
    // previous candidate's band (no per-candidate search); band * cap < 2^21 (W, H <= 2047, tslam_create), so the address
    // is a full-rate 24-bit multiply
    auto sweep = [&](auto&& fn) {
        int lo = 0;
        for (int i0 = threadIdx.x; i0 < ncand; i0 += 4 * SEL_THREADS) {
            uint32_t k[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = i0 + u * SEL_THREADS;
                k[u] = 0u;
                if (i < ncand) {
                    while ((int)s_pref[lo + 1] <= i) ++lo;
                    k[u] = cand[__umul24((uint32_t)lo, (uint32_t)cap) + (uint32_t)(i - (int)s_pref[lo])];
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i0 + u * SEL_THREADS < ncand) fn(k[u]);
        }
    };
    uint32_t total = 0;
    for (int i = 0; i < 256; ++i) total += s_h[i];   // uniform per thread (LDS broadcast)

    uint32_t thresh = 0xFFFFFFFFu;  // inclusive max key taken
    if (total > (uint32_t)Kl) {
        block_find_crossing(s_h, 256, (uint32_t)Kl, s_part, &s_bin, &s_before);
        const uint32_t sbin = (uint32_t)s_bin;  // = 255 - s*
        const uint32_t need = (uint32_t)Kl - s_before;
        const uint32_t eq = s_h[sbin];
        thresh = (sbin << 22) | 0x3FFFFFu;
        if (need < eq) {
            // radix on y among keys of this score
            __syncthreads();
            for (int i = threadIdx.x; i < 2048; i += blockDim.x) s_h[i] = 0;
            __syncthreads();
            sweep([&](uint32_t k) {
                if ((k >> 22) == sbin) atomicAdd(&s_h[(k >> 11) & 2047u], 1u);
            });
            __syncthreads();
            block_find_crossing(s_h, 2048, need, s_part, &s_bin, &s_before);
            const uint32_t ystar = (uint32_t)s_bin;
            const uint32_t need2 = need - s_before;
            const uint32_t eq2 = s_h[ystar];
            thresh = (sbin << 22) | (ystar << 11) | 2047u;
            if (need2 < eq2) {
                __syncthreads();
                for (int i = threadIdx.x; i < 2048; i += blockDim.x) s_h[i] = 0;
                __syncthreads();
                sweep([&](uint32_t k) {
                    if ((k >> 11) == ((sbin << 11) | ystar)) atomicAdd(&s_h[k & 2047u], 1u);
                });
                __syncthreads();
                block_find_crossing(s_h, 2048, need2, s_part, &s_bin, &s_before);
                thresh = (sbin << 22) | (ystar << 11) | (uint32_t)s_bin;
            }
        }
    }
    // collect survivors
    if (threadIdx.x == 0) s_nsel = 0;
    __syncthreads();
    sweep([&](uint32_t k) {
        if (k <= thresh) {
            const uint32_t slot = atomicAdd(&s_nsel, 1u);
            if (slot < SEL_MAX) s_keys[slot] = k;
        }
    });
    __syncthreads();
    const int nsel = min((int)s_nsel, Kl);
    const int slot = ring_slot(c, c.g0 + f);
    uint32_t* kp = c.kps + (((size_t)slot * c.C + cam) * c.g.K + c.g.koff[l]) * 2;
    const int Hl = c.g.H[l];
    // Counting sorts (few barriers) when the level fits a quarter of s_keys and no score
    // bucket is huge; a bitonic network otherwise (66 barrier stages at 2048 keys).  Keys are
    // unique, so "rank = bucket offset + #smaller keys in the bucket" is the sorted position.
    uint32_t* s_tmp = s_keys + SEL_MAX / 2;
    if (threadIdx.x == 0) s_flag = 0;
    for (int i = threadIdx.x; i < 512; i += SEL_THREADS) s_h[i] = 0;
    __syncthreads();
    const bool counting = nsel <= SEL_MAX / 4;   // s_tmp = [4096, 6144), row fill = [6144, 8192)
    if (counting) {
        for (int i = threadIdx.x; i < nsel; i += SEL_THREADS) atomicAdd(&s_h[s_keys[i] >> 22], 1u);
        __syncthreads();
        if (threadIdx.x < 256 && s_h[threadIdx.x] > TS_SEL_BUCKET_MAX) s_flag = 1;   // one score bucket per thread
        block_exclusive_scan(s_h, 256, s_part);      // s_h[b] = bucket offset
    }
    __syncthreads();
    if (counting && s_flag == 0) {
        uint32_t* fill = s_h + 256;
        for (int i = threadIdx.x; i < nsel; i += SEL_THREADS) {
            const uint32_t k = s_keys[i], b = k >> 22;
            s_tmp[s_h[b] + atomicAdd(&fill[b], 1u)] = k;
        }
        __syncthreads();
        for (int i = threadIdx.x; i < nsel; i += SEL_THREADS) {
            const uint32_t k = s_tmp[i], b = k >> 22;
            const int lo = (int)s_h[b], n = (int)fill[b];
            int r = 0;
            for (int j = lo; j < lo + n; ++j) r += s_tmp[j] < k;
            s_keys[lo + r] = k;
        }
        __syncthreads();
    } else {
        bitonic_sort(s_keys, nsel);
    }
    for (int i = threadIdx.x; i < Kl; i += SEL_THREADS) {
        uint32_t xy = 0, meta = (uint32_t)l;   // padding entries keep their level
        if (i < nsel) {
            const uint32_t k = s_keys[i];
            xy = (k & 2047u) | (((k >> 11) & 2047u) << 16);
            meta = (uint32_t)l | ((255u - (k >> 22)) << 16);
        }
        kp[2 * i] = xy;
        kp[2 * i + 1] = meta;
    }
    if (threadIdx.x == 0) {
        c.kcount[((size_t)slot * c.C + cam) * c.g.n_levels + l] = nsel;
        // speculative threshold: the candidates are the NMS survivors with score >= te; the top K
        // is exact iff at least K of them exist (a pixel below te can neither be selected nor
        // suppress one at or above it) or te = t + 1.  Otherwise flag the image for the
        // fallback pass.  Next batch's te for this (camera, level): 2 below the K-th score (the
        // minimum over the batch's frames; a fallback costs ~2 us per image-level, so a tight
        // margin pays: 4 -> 2 -> 0 gave 492 / 483 / 464 us per 256-frame detect alone, 2 kept
        // against real sequences drifting faster than a replay), t + 1 when the level had fewer
        // than K.
        const int tfull = c.fast_threshold + 1;
        const int te = MODE == 1 ? tfull : max(tfull, (int)c.det_thr[(size_t)cam * c.g.n_levels + l]);
        const bool short_k = (int)total < Kl;
        if (MODE == 0) c.det_fail[fcl] = (short_k && te > tfull) ? 1u : 0u;
        int next = tfull;
        if (!short_k && nsel > 0) {
            const int sk = 255 - (int)(s_keys[nsel - 1] >> 22);   // the K-th score (keys sorted ascending)
            next = max(tfull, sk - 2);
        }
        atomicMin(&c.det_thr_acc[(size_t)cam * c.g.n_levels + l], (uint32_t)next);
    }

    // y-sorted order of this level (by y, then rank) + row-start table, for band-limited matching
    uint4* ys = c.ys + ((size_t)slot * c.C + cam) * c.g.K + c.g.koff[l];
    uint16_t* rs = c.rowstart + ((size_t)slot * c.C + cam) * c.g.rs_total + c.g.rs_off[l];
    auto record = [&](int rank) -> uint4 {
        const uint32_t k = s_keys[rank];
        return {(k & 2047u) | (((k >> 11) & 2047u) << 16), (uint32_t)l | ((255u - (k >> 22)) << 16),
                (uint32_t)(c.g.koff[l] + rank), 1u};
    };
    for (int i = nsel + threadIdx.x; i < Kl; i += SEL_THREADS) ys[i] = {0u, (uint32_t)l, (uint32_t)(c.g.koff[l] + i), 0u};
    if (counting) {
        // rows: counts -> exclusive offsets (= rowstart), bucket ranks by row, order by rank
        uint32_t* fill = s_keys + SEL_MAX / 2 + SEL_MAX / 4;   // [2048] row fill counters
        __syncthreads();
        for (int i = threadIdx.x; i < 2048; i += SEL_THREADS) {
            s_h[i] = 0;
            fill[i] = 0;
        }
        __syncthreads();
        for (int i = threadIdx.x; i < nsel; i += SEL_THREADS) atomicAdd(&s_h[(s_keys[i] >> 11) & 2047u], 1u);
        __syncthreads();
        block_exclusive_scan(s_h, 2048, s_part);
        for (int y = threadIdx.x; y <= Hl; y += SEL_THREADS) rs[y] = (uint16_t)s_h[y];
        for (int i = threadIdx.x; i < nsel; i += SEL_THREADS) {
            const uint32_t y = (s_keys[i] >> 11) & 2047u;
            s_tmp[s_h[y] + atomicAdd(&fill[y], 1u)] = (uint32_t)i;
        }
        __syncthreads();
        for (int p = threadIdx.x; p < nsel; p += SEL_THREADS) {
            const uint32_t i = s_tmp[p], y = (s_keys[i] >> 11) & 2047u;
            const int lo = (int)s_h[y], n = (int)fill[y];
            int r = 0;
            for (int j = lo; j < lo + n; ++j) r += s_tmp[j] < i;
            ys[lo + r] = record((int)i);
        }
    } else {
        // bitonic on (y << 13 | rank) in the scratch half is not possible here (nsel > half):
        // sort in place after the records are taken
        __syncthreads();
        uint32_t* yk = s_keys;   // reuse: keys are re-derived from kp[] below
        for (int i = threadIdx.x; i < nsel; i += SEL_THREADS) yk[i] = (((yk[i] >> 11) & 2047u) << 13) | (uint32_t)i;
        __syncthreads();
        bitonic_sort(yk, nsel);
        for (int i = threadIdx.x; i < nsel; i += SEL_THREADS) {
            const int rank = (int)(yk[i] & 8191u);
            const uint2 e = *reinterpret_cast<const uint2*>(kp + 2 * rank);
            ys[i] = {e.x, e.y, (uint32_t)(c.g.koff[l] + rank), 1u};
        }
        for (int y = threadIdx.x; y <= Hl; y += SEL_THREADS) {
            const uint32_t target = (uint32_t)y << 13;
            int lo = 0, hi = nsel;  // first position with key >= target
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (yk[mid] < target) lo = mid + 1; else hi = mid;
            }
            rs[y] = (uint16_t)lo;
        }
    }
}

__global__ __launch_bounds__(SEL_THREADS) void k_select(BatchCtx c) { select_body<0>(c, blockIdx.x, blockIdx.y); }
__global__ __launch_bounds__(SEL_THREADS) void k_select_fallback(BatchCtx c) {
    for_flagged_levels(c, SEL_THREADS, [&](int img, int l) { select_body<1>(c, img, l); });
}

// ---------------------------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------------------------
void launch_rectify_pyramid(const BatchCtx& c, hipStream_t s) {
    size_t lds = 0;
    for (int l = 0; l < c.g.n_levels; ++l) lds += (size_t)(TS_RECT_BAND >> l) * c.g.W[l];
    const int imgs = c.peer_S ? (c.C / c.peer_S - 1) * c.n * c.peer_S : c.n * c.ncam;
    dim3 grid((c.H + TS_RECT_BAND - 1) / TS_RECT_BAND, imgs);
    hipLaunchKernelGGL(k_rectify_pyramid, grid, dim3(256), lds, s, c);
}

void launch_detect(const BatchCtx& c, hipStream_t s) {
    const size_t lds = (size_t)c.g.det_lds;
    dim3 grid(c.g.total_bands, c.n * c.ncam);
    // hist [B][C][L][256] is zero here: zeroed at allocation, and every select (speculative or
    // fallback) zeroes its image-level's histogram once it has read it
    hipLaunchKernelGGL(k_detect, grid, dim3(TS_DET_THREADS), lds, s, c);
}

// next batch's te <- this batch's running minimum; the minimum restarts (view cameras)
__global__ void k_det_thr_commit(BatchCtx c) {
    const int i = threadIdx.x;
    if (i >= c.ncam * c.g.n_levels) return;
    const size_t k = (size_t)c.cam0 * c.g.n_levels + i;
    const_cast<uint32_t*>(c.det_thr)[k] = c.det_thr_acc[k];
    c.det_thr_acc[k] = 0xFFFFFFFFu;
}

void launch_select(const BatchCtx& c, hipStream_t s) {
    dim3 grid(c.n * c.ncam, c.g.n_levels);
    hipLaunchKernelGGL(k_select, grid, dim3(SEL_THREADS), 0, s, c);
    // fallback for images whose speculative threshold left fewer than K candidates: detect and
    // select again at t + 1, gated on the device flags (near-empty launches when none is set)
    hipLaunchKernelGGL(k_detect_fallback, dim3(TS_FB_BLOCKS), dim3(TS_DET_THREADS), (size_t)c.g.det_lds, s, c);
    hipLaunchKernelGGL(k_select_fallback, dim3(TS_FB_BLOCKS), dim3(SEL_THREADS), 0, s, c);
    hipLaunchKernelGGL(k_det_thr_commit, dim3(1), dim3(256), 0, s, c);
}
