// k_match.hip — row A6 of SURVEY.md §8a: brute-force Hamming matching (stereo L<->R with a row
// band and positive disparity; temporal L(t)<->L(t-1) with a window), ratio test, mutual check,
// and the integer-SAD sub-pixel refinements (A6b stereo disparity, A7a temporal position).
// Bit-exact with oracle.match / oracle.stereo_subpixel / oracle.temporal_subpixel.
//
// k_match: one thread per query, 256 queries per block; the train descriptors of the same level
// are staged in LDS in chunks of 1024 (32 KiB) and read as LDS broadcasts, so each pair costs
// 8 v_xor + 8 v_bcnt (popcount with accumulate) and a compare.  The train side's best query
// (for the mutual check) is a wave min-reduction of (dist<<16 | query) per train descriptor,
// an LDS atomicMin per wave, and one global atomicMin per train descriptor per block: min is
// order-independent, so the result is deterministic.
#include "tslam_common.h"

__global__ __launch_bounds__(256) void k_match(BatchCtx c) {
    __shared__ uint4 s_desc[TS_MATCH_CHUNK * 2];
    __shared__ uint32_t s_xy[TS_MATCH_CHUNK];
    __shared__ uint32_t s_tmin[TS_MATCH_CHUNK];
    const int z = blockIdx.y;                 // (f * P + p) * 2 + mode
    const int mode = z & 1;
    const int fp = z >> 1;
    const int p = fp % c.P;
    const int f = fp / c.P;
    const int64_t g = c.g0 + f;
    if (mode == 1 && g == 0) return;          // no previous frame
    int l = 0;
    while (l + 1 < c.g.n_levels && (int)blockIdx.x >= c.g.qtile_start[l + 1]) ++l;
    const int tile = blockIdx.x - c.g.qtile_start[l];
    const int slot = ring_slot(c, g);
    const int qcam = 2 * p;
    const int tslot = mode == 0 ? slot : ring_slot(c, g - 1);
    const int tcam = mode == 0 ? 2 * p + 1 : 2 * p;
    const int K = c.g.K;
    const int qn = c.kcount[((size_t)slot * c.C + qcam) * c.g.n_levels + l];
    const int tn = c.kcount[((size_t)tslot * c.C + tcam) * c.g.n_levels + l];
    const int qlocal = tile * 256 + threadIdx.x;
    const bool active = qlocal < qn;
    const int qi = c.g.koff[l] + qlocal;
    const size_t qbase = ((size_t)slot * c.C + qcam) * K;
    const size_t tbase = ((size_t)tslot * c.C + tcam) * K;
    const size_t mbase = (((size_t)f * c.P + p) * 2 + mode) * K;

    uint32_t q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int qx = 0, qy = 0;
    if (active) {
        const uint4* d = reinterpret_cast<const uint4*>(c.desc + (qbase + qi) * 8);
        const uint4 a = d[0], b = d[1];
        q[0] = a.x; q[1] = a.y; q[2] = a.z; q[3] = a.w; q[4] = b.x; q[5] = b.y; q[6] = b.z; q[7] = b.w;
        const uint32_t xy = c.kps[(qbase + qi) * 2];
        qx = xy & 0xFFFF;
        qy = xy >> 16;
    }
    const int row_tol = c.mp.row_tol, dmax = c.mp.max_disp >> l, win = c.mp.window >> l;
    int best_d = 1 << 20, best_j = -1, second_d = 1 << 20;

    for (int j0 = 0; j0 < tn; j0 += TS_MATCH_CHUNK) {
        const int jn = min(TS_MATCH_CHUNK, tn - j0);
        __syncthreads();
        for (int i = threadIdx.x; i < jn; i += blockDim.x) {
            const size_t tj = tbase + c.g.koff[l] + j0 + i;
            const uint4* d = reinterpret_cast<const uint4*>(c.desc + tj * 8);
            s_desc[2 * i] = d[0];
            s_desc[2 * i + 1] = d[1];
            s_xy[i] = c.kps[tj * 2];
            s_tmin[i] = 0xFFFFFFFFu;
        }
        __syncthreads();
        for (int j = 0; j < jn; ++j) {
            const uint32_t txy = s_xy[j];
            const int tx = txy & 0xFFFF, ty = txy >> 16;
            bool elig;
            if (mode == 0) {
                const int dd = qx - tx;
                elig = abs(qy - ty) <= row_tol && dd >= 1 && dd <= dmax;
            } else {
                elig = abs(qx - tx) <= win && abs(qy - ty) <= win;
            }
            elig = elig && active;
            if (__any(elig)) {
                const uint4 a = s_desc[2 * j], b = s_desc[2 * j + 1];
                int dist = __popc(q[0] ^ a.x) + __popc(q[1] ^ a.y) + __popc(q[2] ^ a.z) + __popc(q[3] ^ a.w) +
                           __popc(q[4] ^ b.x) + __popc(q[5] ^ b.y) + __popc(q[6] ^ b.z) + __popc(q[7] ^ b.w);
                if (elig) {
                    if (dist < best_d) {
                        second_d = best_d;
                        best_d = dist;
                        best_j = j0 + j;
                    } else if (dist < second_d) {
                        second_d = dist;
                    }
                }
                uint32_t packed = elig ? (((uint32_t)dist << 16) | (uint32_t)qi) : 0xFFFFFFFFu;
                packed = wave_min_u32(packed);
                if ((threadIdx.x & 63) == 0 && packed != 0xFFFFFFFFu) atomicMin(&s_tmin[j], packed);
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < jn; i += blockDim.x)
            if (s_tmin[i] != 0xFFFFFFFFu) atomicMin(&c.tbest[mbase + c.g.koff[l] + j0 + i], s_tmin[i]);
    }
    if (active) {
        c.qbest[mbase + qi] = best_j >= 0 ? (((uint32_t)best_d << 16) | (uint32_t)(c.g.koff[l] + best_j)) : 0xFFFFFFFFu;
        c.qsecond[mbase + qi] = second_d >= (1 << 20) ? 256u : (uint32_t)second_d;
    }
}

// Sub-pixel offset of a discrete minimum from three integer costs (exact double division).
__device__ __forceinline__ double parabola(int sm, int s0, int sp) {
    const int den = sm - 2 * s0 + sp;
    return den > 0 ? (double)(sm - sp) / (2.0 * (double)den) : 0.0;
}

// 11x11 integer SAD between patch a (centre ax, ay) and patch b (centre bx, by), pitch W.
__device__ __forceinline__ int sad11(const uint8_t* a, int ax, int ay, const uint8_t* b, int bx, int by, int W) {
    int s = 0;
    for (int dy = -TS_SAD_HALF; dy <= TS_SAD_HALF; ++dy) {
        const uint8_t* ra = a + (size_t)(ay + dy) * W + ax - TS_SAD_HALF;
        const uint8_t* rb = b + (size_t)(by + dy) * W + bx - TS_SAD_HALF;
#pragma unroll
        for (int t = 0; t < 2 * TS_SAD_HALF + 1; ++t) s += abs((int)ra[t] - (int)rb[t]);
    }
    return s;
}

// k_match_refine: validity (max distance, ratio, mutual) + sub-pixel refinement, one wave per
// query keypoint (4 per block), one search offset per lane, costs gathered by shuffles (no LDS,
// no barriers).  grid (ceil(K/4), n*P*2).
__global__ __launch_bounds__(256) void k_match_refine(BatchCtx c) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int qi = blockIdx.x * 4 + wave;
    const int z = blockIdx.y;
    const int mode = z & 1;
    const int fp = z >> 1;
    const int p = fp % c.P;
    const int f = fp / c.P;
    const int64_t g = c.g0 + f;
    const int K = c.g.K;
    if (qi >= K) return;
    const int slot = ring_slot(c, g);
    const size_t mbase = (((size_t)f * c.P + p) * 2 + mode) * K;
    int32_t* out_idx = mode == 0 ? c.stereo + ((size_t)slot * c.P + p) * K : c.temporal + ((size_t)f * c.P + p) * K;
    const int qcam = 2 * p;
    const size_t qkb = ((size_t)slot * c.C + qcam) * K;
    const uint32_t meta = c.kps[(qkb + qi) * 2 + 1];
    const int l = meta & 0xFF;
    const int qn = c.kcount[((size_t)slot * c.C + qcam) * c.g.n_levels + l];
    bool valid = (qi - c.g.koff[l]) < qn && !(mode == 1 && g == 0);
    int j = -1;
    if (valid) {
        const uint32_t qb = c.qbest[mbase + qi];
        if (qb == 0xFFFFFFFFu) {
            valid = false;
        } else {
            const int bd = qb >> 16;
            j = qb & 0xFFFF;
            const int sd = c.qsecond[mbase + qi];
            const uint32_t tb = c.tbest[mbase + j];
            valid = bd <= c.mp.max_hamming && bd * 100 < c.mp.ratio_pct * sd && (int)(tb & 0xFFFF) == qi;
        }
    }
    if (lane == 0) out_idx[qi] = valid ? j : -1;
    double* out_val = mode == 0 ? c.disp + ((size_t)slot * c.P + p) * K + qi
                                : c.tuv + (((size_t)f * c.P + p) * K + qi) * 2;
    const double nanv = __builtin_nan("");
    if (!valid) {
        if (lane == 0) {
            out_val[0] = nanv;
            if (mode == 1) out_val[1] = nanv;
        }
        return;
    }
    const int W = c.g.W[l];
    const uint32_t qxy = c.kps[(qkb + qi) * 2];
    const int qx = qxy & 0xFFFF, qy = qxy >> 16;
    const int BIG = 0x7FFFFFFF;
    if (mode == 0) {
        // left patch at (qx, qy) vs right row qy at xr + k, k in [-2, 2]
        const size_t rkb = ((size_t)slot * c.C + qcam + 1) * K;
        const int xr = c.kps[(rkb + j) * 2] & 0xFFFF;
        const uint8_t* L = c.pyr + ((size_t)slot * c.C + qcam) * c.g.pyr_bytes + c.g.pyr_off[l];
        const uint8_t* R = c.pyr + ((size_t)slot * c.C + qcam + 1) * c.g.pyr_bytes + c.g.pyr_off[l];
        int cost = BIG;
        if (lane < 2 * TS_SAD_RANGE + 1) cost = sad11(L, qx, qy, R, xr + lane - TS_SAD_RANGE, qy, W);
        int cs[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) cs[k] = __shfl(cost, k, 64);
        if (lane == 0) {
            int ks = 0;
            for (int k = 1; k < 5; ++k)
                if (cs[k] < cs[ks]) ks = k;
            double d0 = nanv;
            if (ks > 0 && ks < 4) {
                const double delta = parabola(cs[ks - 1], cs[ks], cs[ks + 1]);
                const double sc = (double)(1 << l);
                const double v = ((double)qx - ((double)(xr + (ks - TS_SAD_RANGE)) + delta)) * sc;
                if (v > 0.0) d0 = v;
            }
            out_val[0] = d0;
        }
    } else {
        // left(t-1) patch at kp j vs left(t) at (qx + kx, qy + ky), kx, ky in [-2, 2]
        const int pslot = ring_slot(c, g - 1);
        const size_t pkb = ((size_t)pslot * c.C + qcam) * K;
        const uint32_t pxy = c.kps[(pkb + j) * 2];
        const int px = pxy & 0xFFFF, py = pxy >> 16;
        const uint8_t* A = c.pyr + ((size_t)pslot * c.C + qcam) * c.g.pyr_bytes + c.g.pyr_off[l];
        const uint8_t* B = c.pyr + ((size_t)slot * c.C + qcam) * c.g.pyr_bytes + c.g.pyr_off[l];
        int cost = BIG;
        if (lane < 25) cost = sad11(A, px, py, B, qx + lane % 5 - TS_SAD_RANGE, qy + lane / 5 - TS_SAD_RANGE, W);
        int cs[25];
#pragma unroll
        for (int o = 0; o < 25; ++o) cs[o] = __shfl(cost, o, 64);
        if (lane == 0) {
            int a = 0;
            for (int o = 1; o < 25; ++o)
                if (cs[o] < cs[a]) a = o;
            const int ky = a / 5, kx = a % 5;
            double u = nanv, v = nanv;
            if (kx > 0 && kx < 4 && ky > 0 && ky < 4) {
                const double ddx = parabola(cs[ky * 5 + kx - 1], cs[ky * 5 + kx], cs[ky * 5 + kx + 1]);
                const double ddy = parabola(cs[(ky - 1) * 5 + kx], cs[ky * 5 + kx], cs[(ky + 1) * 5 + kx]);
                const double sc = (double)(1 << l);
                u = (((double)(qx + (kx - TS_SAD_RANGE)) + ddx) + 0.5) * sc - 0.5;
                v = (((double)(qy + (ky - TS_SAD_RANGE)) + ddy) + 0.5) * sc - 0.5;
            }
            out_val[0] = u;
            out_val[1] = v;
        }
    }
}

void launch_match(const BatchCtx& c, hipStream_t s) {
    (void)hipMemsetAsync(c.tbest, 0xFF, sizeof(uint32_t) * (size_t)c.n * c.P * 2 * c.g.K, s);
    (void)hipMemsetAsync(c.qbest, 0xFF, sizeof(uint32_t) * (size_t)c.n * c.P * 2 * c.g.K, s);
    dim3 grid(c.g.total_qtiles, c.n * c.P * 2);
    hipLaunchKernelGGL(k_match, grid, dim3(256), 0, s, c);
}

void launch_match_refine(const BatchCtx& c, hipStream_t s) {
    dim3 grid((c.g.K + 3) / 4, c.n * c.P * 2);
    hipLaunchKernelGGL(k_match_refine, grid, dim3(256), 0, s, c);
}
