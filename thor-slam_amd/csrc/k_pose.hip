// k_pose.hip — row A7 of SURVEY.md §8a: correspondences (t-1 stereo 3D <-> t refined 2D),
// P3P-RANSAC with a counter-based RNG, Gauss-Newton refinement, pose chaining.
//
// FP64 throughout, compiled with -ffp-contract=off, and written operation-for-operation like
// oracle/numpy_slam.py (p3p, _roots, count_inliers, refine, solve6, cayley): only IEEE +,-,*,/
// and sqrt are used, so the hypotheses, their inlier counts and the winning hypothesis are
// bit-identical to the oracle; the refined pose differs only by the summation order of the
// normal equations (~1e-16 relative).
//
// One 256-thread block per (frame, pair).  Phase A: thread h solves P3P for hypothesis h and
// parks its <= 4 poses in LDS.  Phase B: every thread scores 4H/256 poses against all
// correspondences (wave-uniform addresses -> broadcast loads).  Phase C: block argmax, then
// Gauss-Newton with a block reduction of the 6x6 normal equations per iteration.
#include "tslam_common.h"

#define P3P_VMAX 1000.0
#define P3P_BISECT 60

struct V3 {
    double x, y, z;
};

__device__ __forceinline__ double dot3(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ V3 sub3(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ V3 cross3(V3 a, V3 b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ V3 norm3(V3 a) {
    const double n = sqrt(dot3(a, a));
    return {a.x / n, a.y / n, a.z / n};
}
__device__ __forceinline__ void frame3(V3 p1, V3 p2, V3 p3, V3* e) {
    e[0] = norm3(sub3(p2, p1));
    e[2] = norm3(cross3(e[0], sub3(p3, p1)));
    e[1] = cross3(e[2], e[0]);
}
__device__ __forceinline__ double comp(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

template <int N>
__device__ __forceinline__ double horner(const double* c, double v) {
    double p = c[N];
#pragma unroll
    for (int k = N - 1; k >= 0; --k) p = p * v + c[k];
    return p;
}

// Real roots in (lo, hi) of sum c_k v^k, ascending, NaN-padded (mirrors oracle._roots).
template <int N>
__device__ void real_roots(const double* c, double lo, double hi, double* out) {
    if constexpr (N == 1) {
        const double r = -c[0] / c[1];
        out[0] = (c[1] != 0.0 && r > lo && r < hi) ? r : __builtin_nan("");
    } else {
        double dc[N];
#pragma unroll
        for (int k = 0; k < N; ++k) dc[k] = c[k + 1] * (double)(k + 1);
        double crit[N - 1];
        real_roots<N - 1>(dc, lo, hi, crit);
        double pts[N + 1];
        pts[0] = lo;
#pragma unroll
        for (int i = 0; i < N - 1; ++i) pts[i + 1] = __builtin_isnan(crit[i]) ? hi : crit[i];
        pts[N] = hi;
#pragma unroll
        for (int i = 0; i < N; ++i) out[i] = __builtin_nan("");
        int nr = 0;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            double a = pts[i], b = pts[i + 1];
            const bool sa = horner<N>(c, a) > 0.0;
            const bool sb = horner<N>(c, b) > 0.0;
            const bool has = sa != sb && b > a;
            if (has) {
                for (int it = 0; it < P3P_BISECT; ++it) {
                    const double m = 0.5 * (a + b);
                    const bool sm = horner<N>(c, m) > 0.0;
                    if (sm == sa) a = m; else b = m;
                }
            }
            const double root = 0.5 * (a + b);
            // compaction with compile-time register indices (no scratch)
#pragma unroll
            for (int k = 0; k < N; ++k)
                if (has && nr == k) out[k] = root;
            nr += has ? 1 : 0;
        }
    }
}

struct Pose {
    double r[9];
    double t[3];
};

// Grunert P3P (oracle.p3p): up to 4 poses ordered by ascending v = s3/s1; returns validity mask.
__device__ int p3p_solve(const V3* pw, const V3* f, Pose* out) {
    const V3 d12 = sub3(pw[1], pw[2]), d02 = sub3(pw[0], pw[2]), d01 = sub3(pw[0], pw[1]);
    const double a2 = dot3(d12, d12), b2 = dot3(d02, d02), c2 = dot3(d01, d01);
    const double ca = dot3(f[1], f[2]), cb = dot3(f[0], f[2]), cg = dot3(f[0], f[1]);
    const double kk = (a2 - c2) / b2;
    const double kc = c2 / b2;
    const double n0 = 1.0 + kk, n1 = (-2.0 * kk) * cb, n2 = kk - 1.0;
    const double d0 = cg, d1 = -ca;
    const double g0 = 1.0 - kc, g1 = (2.0 * kc) * cb, g2 = -kc;
    double q[5];
    q[4] = n2 * n2;
    q[3] = (2.0 * n1) * n2;
    q[2] = n1 * n1 + (2.0 * n0) * n2;
    q[1] = (2.0 * n0) * n1;
    q[0] = n0 * n0;
    const double m = -4.0 * cg;
    q[3] = q[3] + m * (n2 * d1);
    q[2] = q[2] + m * (n1 * d1 + n2 * d0);
    q[1] = q[1] + m * (n0 * d1 + n1 * d0);
    q[0] = q[0] + m * (n0 * d0);
    const double e0 = d0 * d0, e1 = (2.0 * d0) * d1, e2 = d1 * d1;
    q[4] = q[4] + 4.0 * (e2 * g2);
    q[3] = q[3] + 4.0 * (e1 * g2 + e2 * g1);
    q[2] = q[2] + 4.0 * ((e0 * g2 + e1 * g1) + e2 * g0);
    q[1] = q[1] + 4.0 * (e0 * g1 + e1 * g0);
    q[0] = q[0] + 4.0 * (e0 * g0);
    double roots[4];
    real_roots<4>(q, 0.0, P3P_VMAX, roots);
    V3 fw[3];
    frame3(pw[0], pw[1], pw[2], fw);
    int mask = 0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const double v = roots[s];
        const double num = (n0 + n1 * v) + n2 * (v * v);
        const double den = 2.0 * (cg - ca * v);
        const double u = num / den;
        const double s1sq = b2 / ((1.0 + v * v) - (2.0 * cb) * v);
        bool good = !__builtin_isnan(v) && u > 0.0 && s1sq > 0.0 && __builtin_isfinite(u) && __builtin_isfinite(s1sq);
        const double s1 = sqrt(good ? s1sq : 1.0);
        const double s2 = u * s1, s3 = v * s1;
        const V3 pc0 = {f[0].x * s1, f[0].y * s1, f[0].z * s1};
        const V3 pc1 = {f[1].x * s2, f[1].y * s2, f[1].z * s2};
        const V3 pc2 = {f[2].x * s3, f[2].y * s3, f[2].z * s3};
        V3 fc[3];
        frame3(pc0, pc1, pc2, fc);
        Pose& P = out[s];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j)
                P.r[3 * i + j] = (comp(fc[0], i) * comp(fw[0], j) + comp(fc[1], i) * comp(fw[1], j)) + comp(fc[2], i) * comp(fw[2], j);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const double rp = (P.r[3 * i] * pw[0].x + P.r[3 * i + 1] * pw[0].y) + P.r[3 * i + 2] * pw[0].z;
            P.t[i] = comp(pc0, i) - rp;
        }
#pragma unroll
        for (int i = 0; i < 9; ++i) good = good && __builtin_isfinite(P.r[i]);
#pragma unroll
        for (int i = 0; i < 3; ++i) good = good && __builtin_isfinite(P.t[i]);
        if (good) mask |= 1 << s;
    }
    return mask;
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x = x + 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// inlier test (oracle.count_inliers / count_inliers_mask)
__device__ __forceinline__ bool is_inlier(const double* R, const double* t, const double* cr, double fx, double fy, double thr2) {
    const double X = cr[0], Y = cr[1], Z = cr[2], du = cr[3], dv = cr[4];
    const double xc = ((R[0] * X + R[1] * Y) + R[2] * Z) + t[0];
    const double yc = ((R[3] * X + R[4] * Y) + R[5] * Z) + t[1];
    const double zc = ((R[6] * X + R[7] * Y) + R[8] * Z) + t[2];
    const double ex = fx * xc + du * zc;
    const double ey = fy * yc + dv * zc;
    const double e2 = ex * ex + ey * ey;
    const double lim = thr2 * (zc * zc);
    return zc > 0.0 && e2 < lim;
}

// The same decision from an f32 evaluation with a rigorous error bound: +1 inlier, 0 outlier,
// -1 undecided (the exact f64 test decides).  With u = 2^-24, each of xc, yc, zc (three f32
// FMAs over inputs rounded to f32) is within 5u a (a = the sum of the term magnitudes), ex and ey
// within 8u (f a_x + |du| a_z), and D = thr2 zc^2 - (ex^2 + ey^2) within
// 16u [|ex| (fx a_x + |du| a_z) + |ey| (fy a_y + |dv| a_z) + thr2 |zc| a_z + ex^2 + ey^2 + thr2 zc^2]
// to first order; the test uses twice that, which also covers the second-order terms, the f32
// evaluation of the bound and the f64 reference's own rounding (~2^-53 of the same sum).  So
// D > E and zc > E_z mean the f64 test says inlier, D < -E or zc < -E_z outlier.
// The bound is taken with one magnitude for all three rows, a = rmax S + tmax >= a_x, a_y, a_z
// (rmax = max |R_ij|, S = |X| + |Y| + |Z|, tmax = max |t_i|), which turns it into
// a [|ex| (fx + |du|) + |ey| (fy + |dv|) + thr2 |zc|] + ex^2 + ey^2 + thr2 zc^2: per test 8
// operations instead of 20, with fx + |du|, fy + |dv| and S per correspondence.
// pf: the pose's f32 record (R 9, t 3, rmax, tmax; k_p3p); q: X Y Z du dv S fx+|du| fy+|dv|.
typedef float f32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ int inlier_f32(const f32x16& pf, const float* q, float fx, float fy, float thr2) {
    const float X = q[0], Y = q[1], Z = q[2], du = q[3], dv = q[4];
    const float xc = fmaf(pf[0], X, fmaf(pf[1], Y, fmaf(pf[2], Z, pf[9])));
    const float yc = fmaf(pf[3], X, fmaf(pf[4], Y, fmaf(pf[5], Z, pf[10])));
    const float zc = fmaf(pf[6], X, fmaf(pf[7], Y, fmaf(pf[8], Z, pf[11])));
    const float ex = fmaf(fx, xc, du * zc);
    const float ey = fmaf(fy, yc, dv * zc);
    const float e2 = fmaf(ex, ex, ey * ey);
    const float lim = thr2 * (zc * zc);
    const float D = lim - e2;
    const float a = fmaf(pf[12], q[5], pf[13]);
    const float inner = fmaf(fabsf(ex), q[6], fmaf(fabsf(ey), q[7], thr2 * fabsf(zc)));
    const float bsum = fmaf(a, inner, e2 + lim);
    const float E = bsum * (32.0f / 16777216.0f);
    const float Ez = a * (32.0f / 16777216.0f);
    if (zc < -Ez || D < -E) return 0;
    if (zc > Ez && D > E) return 1;
    return -1;
}

// Cholesky solve of H x = g (oracle.solve6); returns false when H is not positive definite.
// One reciprocal per pivot and multiplications after it: the thread-0 solve of every
// Gauss-Newton step is a serial chain, and an f64 division is ~10 dependent instructions (27 of
// them before, 6 now).  The pose stays within 1e-9 of the oracle's solve (parity tests).
__device__ bool solve6(const double* Hm, const double* g, double* x, double* L) {
    double inv[6];
    for (int j = 0; j < 6; ++j) {
        double s = Hm[j * 6 + j];
        for (int k = 0; k < j; ++k) s = s - L[j * 6 + k] * L[j * 6 + k];
        if (!(s > 0.0)) return false;
        const double d = sqrt(s);
        L[j * 6 + j] = d;
        inv[j] = 1.0 / d;
        for (int i = j + 1; i < 6; ++i) {
            double t = Hm[i * 6 + j];
            for (int k = 0; k < j; ++k) t = t - L[i * 6 + k] * L[j * 6 + k];
            L[i * 6 + j] = t * inv[j];
        }
    }
    double y[6];
    for (int i = 0; i < 6; ++i) {
        double s = g[i];
        for (int k = 0; k < i; ++k) s = s - L[i * 6 + k] * y[k];
        y[i] = s * inv[i];
    }
    for (int i = 5; i >= 0; --i) {
        double s = y[i];
        for (int k = i + 1; k < 6; ++k) s = s - L[k * 6 + i] * x[k];
        x[i] = s * inv[i];
    }
    return true;
}

#define POSE_THREADS 256
#define TS_RS_CPT 4            // correspondences per thread per scoring pass (k_ransac_all)
#define TS_MAX_HYP_SPLIT 256   // hypotheses per k_ransac_all block (n_hyp <= 256)
#define N_ACC 29   // 21 (upper H) + 6 (g) + 1 (sq) + 1 (count)

__device__ __forceinline__ void write_stats(int32_t* so, int status, int n, int n_in, int best_cnt, int best_idx, int64_t g) {
    so[0] = status; so[1] = n; so[2] = n_in; so[3] = best_cnt; so[4] = best_idx; so[5] = (int)g; so[6] = 0; so[7] = 0;
}

// ---- k_corr: correspondences of one (frame, pair), ordered by the current keypoint index ------
__global__ __launch_bounds__(POSE_THREADS) void k_corr(BatchCtx c) {
    TS_BACK_PRIO;
    __shared__ int s_scan[2 * (POSE_THREADS / 64)];
    const int p = c.pair0 + (int)blockIdx.x % c.npair;   // (frame, pair) of the pair view
    const int f = (int)blockIdx.x / c.npair;
    const int fp = f * c.P + p;
    const int64_t g = c.g0 + f;
    const int tid = threadIdx.x;
    const int K = c.g.K;
    double* pout = c.pose + (size_t)fp * TS_POSE_DOUBLES;
    int32_t* sout = c.stats + (size_t)fp * TS_STATS_INTS;
    for (int i = tid; i < TS_POSE_DOUBLES; i += POSE_THREADS) pout[i] = (i < 16 && (i % 5) == 0) ? 1.0 : 0.0;
    if (g == 0) {
        if (tid == 0) write_stats(sout, 2, 0, 0, 0, -1, g);
        return;
    }
    const PairCalib cal = c.calib[p];
    const double fx = cal.fx, fy = cal.fy, cx = cal.cx, cy = cal.cy;
    const int pslot = ring_slot(c, g - 1);
    const int32_t* tm = c.temporal + ((size_t)ring_slot(c, g) * c.P + p) * K;
    const double* tuv = c.tuv + ((size_t)f * c.P + p) * K * 2;
    const double* dprev = c.disp + ((size_t)pslot * c.P + p) * K;
    const uint32_t* kprev = c.kps + ((size_t)pslot * c.C + c.cpp * p) * K * 2;
    double* corr = c.corr + ((size_t)f * c.P + p) * K * TS_CORR_DOUBLES;
    int n = 0;
    for (int base = 0; base < K; base += POSE_THREADS) {
        const int j = base + tid;
        int flag = 0, i = -1;
        double u = 0.0, v = 0.0, d = 0.0;
        if (j < K) {
            i = tm[j];
            if (i >= 0) {
                d = dprev[i];
                u = tuv[2 * j];
                v = tuv[2 * j + 1];
                flag = __builtin_isfinite(d) && __builtin_isfinite(u) && __builtin_isfinite(v);
            }
        }
        // stream compaction in keypoint order: wave ballots + the 4 wave counts (double-buffered,
        // one barrier per chunk of 256)
        const uint64_t bm = __ballot(flag != 0);
        const int lane = tid & 63, wave = tid >> 6;
        int* wc = s_scan + ((base / POSE_THREADS) & 1) * 4;
        if (lane == 0) wc[wave] = __popcll(bm);
        __syncthreads();
        int before = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < POSE_THREADS / 64; ++w) {
            before += w < wave ? wc[w] : 0;
            tot += wc[w];
        }
        const int pos = n + before + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
        if (flag) {
            const uint32_t xy = kprev[2 * i], meta = kprev[2 * i + 1];
            const double sc = (double)(1 << (meta & 0xFF));
            const double ul = ((double)(xy & 0xFFFF) + 0.5) * sc - 0.5;
            const double vl = ((double)(xy >> 16) + 0.5) * sc - 0.5;
            const double z = cal.fxb / d;
            const double x = (ul - cx) * z / fx;
            const double y = (vl - cy) * z / fy;
            const double bx = (u - cx) / fx;
            const double by = (v - cy) / fy;
            const double nn = sqrt((bx * bx + by * by) + 1.0);
            double* cr = corr + (size_t)pos * TS_CORR_DOUBLES;
            cr[0] = x; cr[1] = y; cr[2] = z; cr[3] = cx - u; cr[4] = cy - v;
            cr[5] = bx / nn; cr[6] = by / nn; cr[7] = 1.0 / nn;
        }
        n += tot;
    }
    if (tid == 0) write_stats(sout, n < max(6, c.pp.min_inliers) ? 1 : 3, n, 0, 0, -1, g);  // 3 = "to be solved"
}

// ---- k_p3p: one thread per (frame, pair, hypothesis) -------------------------------------
// Draws the hypothesis' 3 correspondences (splitmix64 of (seed, frame, h)), solves P3P and writes
// its 4 candidate poses to c.hyp ([R 9 | t 3] f64 + their f32 scoring copies, TS_HYP_DOUBLES;
// first element NaN = no solution).
__global__ __launch_bounds__(POSE_THREADS) void k_p3p(BatchCtx c) {
    TS_BACK_PRIO;
    const int H = c.pp.n_hyp;
    const int gid = blockIdx.x * POSE_THREADS + threadIdx.x;
    if (gid >= c.n * c.npair * H) return;
    const int fl = gid / H, h = gid - fl * H;
    const int p = c.pair0 + fl % c.npair;
    const int f = fl / c.npair;
    const int fp = f * c.P + p;
    const int64_t g = c.g0 + f;
    const int32_t* sout = c.stats + (size_t)fp * TS_STATS_INTS;
    if (sout[0] != 3) return;
    const int n = sout[1];
    const double* corr = c.corr + ((size_t)f * c.P + p) * c.g.K * TS_CORR_DOUBLES;
    const uint64_t base_rng = splitmix64(c.pp.seed ^ ((uint64_t)g * 0x9E3779B97F4A7C15ull));
    uint32_t r[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) r[k] = (uint32_t)(splitmix64(base_rng ^ ((uint64_t)h * 4ull + (uint64_t)k)) >> 32);
    const uint32_t un = (uint32_t)n;
    int i0 = (int)(r[0] % un);
    int i1 = (int)(r[1] % (un - 1));
    i1 += (i1 >= i0);
    int i2 = (int)(r[2] % (un - 2));
    const int lo = min(i0, i1), hi = max(i0, i1);
    i2 += (i2 >= lo);
    i2 += (i2 >= hi);
    const int idx[3] = {i0, i1, i2};
    V3 pw[3], fb[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double* cr = corr + (size_t)idx[k] * TS_CORR_DOUBLES;
        pw[k] = {cr[0], cr[1], cr[2]};
        fb[k] = {cr[5], cr[6], cr[7]};
    }
    Pose sol[4];
    const int mask = p3p_solve(pw, fb, sol);
    double* out = c.hyp + ((size_t)fp * 4 * H + 4 * h) * TS_HYP_DOUBLES;
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
        double* dst = out + s2 * TS_HYP_DOUBLES;
        if ((mask >> s2) & 1) {
            float* df = reinterpret_cast<float*>(dst + 12);
            float rmax = 0.0f, tmax = 0.0f;
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                dst[k] = sol[s2].r[k];
                df[k] = (float)sol[s2].r[k];
                rmax = fmaxf(rmax, fabsf(df[k]));
            }
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                dst[9 + k] = sol[s2].t[k];
                df[9 + k] = (float)sol[s2].t[k];
                tmax = fmaxf(tmax, fabsf(df[9 + k]));
            }
            df[12] = rmax;
            df[13] = tmax;
        } else {
            dst[0] = __builtin_nan("");
            reinterpret_cast<float*>(dst + 12)[0] = __builtin_nanf("");
        }
    }
}

// ---- k_ransac_all: exhaustive scoring of one split (small launches) ------------------------
// grid (n*P*S): block (fp, split) scores the 4*(h1-h0) candidate poses of hypotheses [h0, h1):
// correspondences stay in registers (TS_RS_CPT per thread); a pose is wave-uniform, so it comes
// through scalar loads (SGPR operands of the f64 VALU ops — an LDS broadcast of its 96 bytes
// returned 6 KiB per wave and bound the loop); inlier counts are wave ballots (integer sums:
// order-independent).  Writes its best (count+1)<<12 | (4095 - pose index) key and that pose.
// Every pose is scored against every correspondence by the whole block: with few frames per
// launch (B = 1 latency, C4's 50) the per-pose latency of k_ransac's one-wave scans would be the
// launch's critical path, so those launches take this kernel (same keys, same winner).
__global__ __launch_bounds__(POSE_THREADS) void k_ransac_all(BatchCtx c, int S) {
    TS_BACK_PRIO;
    __shared__ int s_cnt[4 * TS_MAX_HYP_SPLIT];
    __shared__ uint32_t s_wbest[4];
    const int fl = blockIdx.x / S;
    const int split = blockIdx.x % S;
    const int p = c.pair0 + fl % c.npair;
    const int f = fl / c.npair;
    const int fp = f * c.P + p;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int32_t* sout = c.stats + (size_t)fp * TS_STATS_INTS;
    uint32_t* kout = reinterpret_cast<uint32_t*>(c.ransac) + ((size_t)fp * S + split) * TS_RANSAC_WORDS;
    if (sout[0] != 3) {
        if (tid == 0) kout[0] = 0u;
        return;
    }
    const int n = sout[1];
    const int H = c.pp.n_hyp;
    const int Hs = (H + S - 1) / S;
    const int h0 = split * Hs, h1 = min(H, h0 + Hs);
    const int nh = max(0, h1 - h0);
    const PairCalib cal = c.calib[p];
    const double fx = cal.fx, fy = cal.fy;
    const double* corr = c.corr + ((size_t)f * c.P + p) * c.g.K * TS_CORR_DOUBLES;
    const double* hyp = c.hyp + ((size_t)fp * 4 * H + 4 * h0) * TS_HYP_DOUBLES;   // this split's poses
    typedef const __attribute__((address_space(4))) double cdouble;   // uniform address -> s_load
    cdouble* chyp = (cdouble*)(uintptr_t)hyp;
    const int npose = 4 * nh;
    for (int i = tid; i < npose; i += POSE_THREADS) s_cnt[i] = 0;
    __syncthreads();
    const double thr2 = c.pp.thr2;
    const float fxf = (float)fx, fyf = (float)fy, thr2f = (float)thr2;
    for (int c0 = 0; c0 < n; c0 += POSE_THREADS * TS_RS_CPT) {
        float cf[TS_RS_CPT][8];   // X Y Z du dv, |X| + |Y| + |Z|, fx + |du|, fy + |dv|
        bool have[TS_RS_CPT];
#pragma unroll
        for (int k = 0; k < TS_RS_CPT; ++k) {
            const int ci = c0 + k * POSE_THREADS + tid;
            have[k] = ci < n;
            const double* cr = corr + (size_t)(have[k] ? ci : 0) * TS_CORR_DOUBLES;
#pragma unroll
            for (int q = 0; q < 5; ++q) cf[k][q] = (float)cr[q];
            cf[k][5] = fabsf(cf[k][0]) + fabsf(cf[k][1]) + fabsf(cf[k][2]);
            cf[k][6] = fxf + fabsf(cf[k][3]);
            cf[k][7] = fyf + fabsf(cf[k][4]);
        }
        // correspondence slots no lane of this wave has are skipped (wave-uniform)
        const int kmax = min(TS_RS_CPT, (n - c0 - wave * 64 + POSE_THREADS - 1) / POSE_THREADS);
        for (int pi = 0; pi < npose; ++pi) {
            cdouble* ps = chyp + (size_t)pi * TS_HYP_DOUBLES;
            // the f32 record in one scalar load (SGPR operands of the test)
            const f32x16 pf = *(const __attribute__((address_space(4))) f32x16*)(ps + 12);
            if (__builtin_isnan(pf[0])) continue;   // uniform
            int cnt = 0;
#pragma unroll
            for (int k = 0; k < TS_RS_CPT; ++k) {
                if (k >= kmax) break;   // uniform
                int v = have[k] ? inlier_f32(pf, cf[k], fxf, fyf, thr2f) : 0;
                if (v < 0) {   // near the threshold: the exact f64 test (rare, divergent)
                    double R[9], t[3];
                    const double* cr = corr + (size_t)(c0 + k * POSE_THREADS + tid) * TS_CORR_DOUBLES;
#pragma unroll
                    for (int q = 0; q < 9; ++q) R[q] = ps[q];
                    t[0] = ps[9]; t[1] = ps[10]; t[2] = ps[11];
                    v = is_inlier(R, t, cr, fx, fy, thr2) ? 1 : 0;
                }
                cnt += __popcll(__ballot(v != 0));
            }
            if (lane == 0 && cnt) atomicAdd(&s_cnt[pi], cnt);
        }
    }
    __syncthreads();
    uint32_t my_best = 0;
    for (int pi = tid; pi < npose; pi += POSE_THREADS) {
        const bool valid = !__builtin_isnan(hyp[(size_t)pi * TS_HYP_DOUBLES]);
        const int gidx = 4 * h0 + pi;
        const uint32_t key = valid ? ((uint32_t)(s_cnt[pi] + 1) << 12) | (uint32_t)(4095 - gidx) : (uint32_t)(4095 - gidx);
        my_best = key > my_best ? key : my_best;
    }
    uint32_t wb = my_best;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t other = (uint32_t)__shfl_xor((int)wb, o, 64);
        wb = other > wb ? other : wb;
    }
    if (lane == 0) s_wbest[wave] = wb;
    __syncthreads();
    uint32_t best = s_wbest[0];
    for (int w = 1; w < 4; ++w) best = s_wbest[w] > best ? s_wbest[w] : best;
    if (tid == 0) kout[0] = best;
    if (tid < 12 && best != 0u) {
        const int gidx = 4095 - (int)(best & 4095u);
        const double v = hyp[(size_t)(gidx - 4 * h0) * TS_HYP_DOUBLES + tid];
        reinterpret_cast<double*>(kout + 2)[tid] = v;
    }
}

// ---- k_ransac: score one split of the poses of one (frame, pair) ---------------------------
// grid (n*P*S): block (fp, split) finds the best (count+1)<<12 | (4095 - pose index) key over the
// 4*(h1-h0) candidate poses of hypotheses [h0, h1) and writes it with that pose.
//
// Bounded scoring: each wave takes its own poses (wave w: poses w, w+4, ...) and scans the frame's
// correspondences 64 at a time (one per lane, inlier decisions by ballot), while the block keeps
// the best key of the poses it has scored completely in LDS.  A pose whose count cannot reach that
// key any more — count + unscanned < best count, or equal with a larger pose index — is dropped
// mid-scan, and a pose that could not reach it with every correspondence an inlier is never
// loaded.  The best key only grows and is always an exactly scored pose's, so every dropped pose
// has a smaller key than the winner: the winner, its count and the pose are those of the
// exhaustive scoring (the oracle's), only the work differs.  A wave first tests a pose on the
// misses of the best pose it has scored itself (correct poses share their outliers), so a pose
// that cannot win usually drops after that one chunk; with no outliers at all the first correct
// root saturates the count and the remaining poses are not loaded.
//
// Correspondences are staged once per block in LDS as f32 (X Y Z du dv, |X|+|Y|+|Z|), the first
// TS_RS_LDS_CAP of them (beyond that the f64 records are read from global memory); a pose is
// wave-uniform, its f32 record in SGPR operands.
#define TS_RS_LDS_CAP 2048
#ifndef TS_RS_UNROLL
#define TS_RS_UNROLL 4
#endif
__global__ __launch_bounds__(POSE_THREADS) void k_ransac(BatchCtx c, int S) {
    TS_BACK_PRIO;
    extern __shared__ float4 s_corr[];   // [cap] (X, Y, Z, du) then [cap] float2 (dv, S)
    __shared__ uint32_t s_best;
    __shared__ int s_wout[POSE_THREADS / 64][64];   // a wave's misses of the pose it is scanning
    const int fl = blockIdx.x / S;
    const int split = blockIdx.x % S;
    const int p = c.pair0 + fl % c.npair;
    const int f = fl / c.npair;
    const int fp = f * c.P + p;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int32_t* sout = c.stats + (size_t)fp * TS_STATS_INTS;
    uint32_t* kout = reinterpret_cast<uint32_t*>(c.ransac) + ((size_t)fp * S + split) * TS_RANSAC_WORDS;
    if (sout[0] != 3) {
        if (tid == 0) kout[0] = 0u;
        return;
    }
    const int n = sout[1];
    const int H = c.pp.n_hyp;
    const int Hs = (H + S - 1) / S;
    const int h0 = split * Hs, h1 = min(H, h0 + Hs);
    const int nh = max(0, h1 - h0);
    const PairCalib cal = c.calib[p];
    const double fx = cal.fx, fy = cal.fy;
    const double* corr = c.corr + ((size_t)f * c.P + p) * c.g.K * TS_CORR_DOUBLES;
    const double* hyp = c.hyp + ((size_t)fp * 4 * H + 4 * h0) * TS_HYP_DOUBLES;   // this split's poses
    const int npose = 4 * nh;
    const int cap = min(c.g.K, TS_RS_LDS_CAP);
    const int nl = min(n, cap);
    float2* s_cd = reinterpret_cast<float2*>(s_corr + cap);
    for (int i = tid; i < nl; i += POSE_THREADS) {
        const double* cr = corr + (size_t)i * TS_CORR_DOUBLES;
        const float X = (float)cr[0], Y = (float)cr[1], Z = (float)cr[2];
        s_corr[i] = make_float4(X, Y, Z, (float)cr[3]);
        s_cd[i] = make_float2((float)cr[4], fabsf(X) + fabsf(Y) + fabsf(Z));
    }
    if (tid == 0) s_best = 0u;
    __syncthreads();
    const double thr2 = c.pp.thr2;
    const float fxf = (float)fx, fyf = (float)fy, thr2f = (float)thr2;
    volatile uint32_t* vbest = &s_best;
    // Per wave: the misses (first 64) of the best pose this wave has scored completely, one index
    // per lane (-1: none).  The next pose is tested on those first: correct poses share their
    // outliers, so a pose that cannot beat the block's best usually drops after one chunk.
    int my_out = -1;
    uint32_t my_key = 0u;
    auto test = [&](const double* ps, const f32x16& pf, int i) -> int {
        float q[8];
        if (i < cap) {
            const float4 a = s_corr[i];
            const float2 b = s_cd[i];
            q[0] = a.x; q[1] = a.y; q[2] = a.z; q[3] = a.w; q[4] = b.x; q[5] = b.y;
        } else {
            const double* cr = corr + (size_t)i * TS_CORR_DOUBLES;
#pragma unroll
            for (int k = 0; k < 5; ++k) q[k] = (float)cr[k];
            q[5] = fabsf(q[0]) + fabsf(q[1]) + fabsf(q[2]);
        }
        q[6] = fxf + fabsf(q[3]);
        q[7] = fyf + fabsf(q[4]);
        int v = inlier_f32(pf, q, fxf, fyf, thr2f);
        if (v < 0) {   // near the threshold: the exact f64 test (rare, divergent)
            double R[9], t[3];
#pragma unroll
            for (int k = 0; k < 9; ++k) R[k] = ps[k];
            t[0] = ps[9]; t[1] = ps[10]; t[2] = ps[11];
            v = is_inlier(R, t, corr + (size_t)i * TS_CORR_DOUBLES, fx, fy, thr2) ? 1 : 0;
        }
        return v;
    };
    // Poses go in groups of RS_GROUP per wave step: lane (k = lane / 8, j = lane % 8) holds pose
    // k's f32 record and tests it on entry j of the wave's outlier list, so the NaN checks and
    // the outlier pre-tests of 8 poses cost one chunk; only poses that survive them are scanned,
    // one at a time, with the record moved to SGPRs by readlane.
    constexpr int RS_GROUP = 8;
    bool done = false;
    const int k = lane >> 3, j = lane & 7;
    constexpr int GSTEP = (POSE_THREADS / 64) * RS_GROUP;
    for (int g0 = wave; g0 < npose && !done; g0 += GSTEP) {
        const uint32_t bnd0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)*vbest);
        if ((((uint32_t)(n + 1) << 12) | (uint32_t)(4095 - (4 * h0 + g0))) < bnd0) break;   // no later pose can win
        const int pk = g0 + (POSE_THREADS / 64) * k;
        const double* psk = hyp + (size_t)(pk < npose ? pk : 0) * TS_HYP_DOUBLES;
        f32x16 pl;   // this lane's pose record
        {
            const float4* r4 = reinterpret_cast<const float4*>(psk + 12);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 w = r4[q];
                pl[4 * q] = w.x; pl[4 * q + 1] = w.y; pl[4 * q + 2] = w.z; pl[4 * q + 3] = w.w;
            }
        }
        const bool valid = pk < npose && !__builtin_isnan(pl[0]);
        if (pk < npose && !valid && j == 0) atomicMax(&s_best, (uint32_t)(4095 - (4 * h0 + pk)));   // key without a count
        uint64_t pre = 0;   // lanes of the poses the outlier pre-test rules out
        if (my_key != 0u) {   // uniform
            const int idx = __shfl(my_out, j, 64);
            const int v = (valid && idx >= 0) ? test(psk, pl, idx) : 1;
            const uint64_t mm = __ballot(v == 0);
            const int miss = __popcll((mm >> (8 * k)) & 0xFFull);
            const uint32_t up = ((uint32_t)(n - miss + 1) << 12) | (uint32_t)(4095 - (4 * h0 + pk));
            pre = __ballot(up < bnd0);
        }
        const uint64_t live = __ballot(valid && j == 0) & ~pre;   // bit 8k: pose k still to be scanned
        for (int kk = 0; kk < RS_GROUP; ++kk) {
            if (!((live >> (8 * kk)) & 1ull)) continue;   // uniform
            const int pi = g0 + (POSE_THREADS / 64) * kk;
            const uint32_t tag = (uint32_t)(4095 - (4 * h0 + pi));
            // the block's best when this pose starts: it only grows, so a stale copy is still a
            // bound (an LDS read per chunk would put a round trip in the scan's dependency chain)
            const uint32_t bnd = (uint32_t)__builtin_amdgcn_readfirstlane((int)*vbest);
            if ((((uint32_t)(n + 1) << 12) | tag) < bnd) {
                done = true;
                break;
            }
            const bool list_ok = (my_key >> 12) + 2u >= (bnd >> 12);
            const double* ps = hyp + (size_t)pi * TS_HYP_DOUBLES;
            f32x16 pf;
#pragma unroll
            for (int q = 0; q < 16; ++q) pf[q] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pl[q]), 8 * kk));
            int cnt = 0, nm = 0;
            bool dropped = false;
            for (int c0 = 0; c0 < n; c0 += 64 * TS_RS_UNROLL) {
                // TS_RS_UNROLL independent chunks between two drop tests: a test per chunk puts the
                // whole LDS -> VALU -> ballot -> branch chain of every chunk on the critical path
    #pragma unroll
                for (int u = 0; u < TS_RS_UNROLL; ++u) {
                    const int cu = c0 + 64 * u;
                    const int i = cu + lane;
                    const int v = i < n ? test(ps, pf, i) : 1;
                    const uint64_t mm = __ballot(v == 0);
                    if (v == 0) {
                        const int pos = nm + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
                        if (pos < 64) s_wout[wave][pos] = i;
                    }
                    nm += __popcll(mm);
                    cnt += max(0, min(64, n - cu)) - __popcll(mm);
                }
                const int rest = max(0, n - (c0 + 64 * TS_RS_UNROLL));
                // drop only once the wave's own outlier list is nearly as good as the block's
                // best: a wave that kept dropping would keep a useless list (and pre-test nothing)
                if (list_ok && (((uint32_t)(cnt + rest + 1) << 12) | tag) < bnd) {   // uniform
                    dropped = true;
                    break;
                }
            }
            if (!dropped) {
                const uint32_t key = ((uint32_t)(cnt + 1) << 12) | tag;
                if (lane == 0) atomicMax(&s_best, key);
                if (key > my_key) {
                    my_key = key;
                    __builtin_amdgcn_wave_barrier();
                    my_out = lane < nm ? s_wout[wave][lane] : -1;
                    __builtin_amdgcn_wave_barrier();
                }
            }
        }
    }
    __syncthreads();
    const uint32_t best = s_best;
    if (tid == 0) kout[0] = best;
    if (tid < 12 && best != 0u) {
        const int gidx = 4095 - (int)(best & 4095u);
        const double v = hyp[(size_t)(gidx - 4 * h0) * TS_HYP_DOUBLES + tid];
        reinterpret_cast<double*>(kout + 2)[tid] = v;
    }
}

// ---- k_refine: pick the best split, Gauss-Newton on the inliers, covariance -----------------
// k_refine's block is RF_THREADS = 128 (2 waves) for large launches: its 222 VGPRs allow 2 waves
// per SIMD, so 4 such blocks fit a CU and 1024 frames run in one round instead of two (C2: 147
// against 160 us; 64 threads: 185); small launches keep 256 threads per frame.
// The normal-equation sums do not depend on the block size: they always follow the partition of
// RF_VIRT = 256 virtual threads (virtual thread v sums correspondences v, v + 256, ...; virtual
// wave w = v >> 6 is reduced by wave_multi_sum; the 4 wave sums are added in order).  A 128-thread
// block runs the virtual threads in two passes (tid, then tid + 128), so the pose, covariance and
// inlier decisions are bit-identical whatever the launch size (batch-size invariance, and the
// sharded ranks' smaller launches against one device's).
#define RF_VIRT 256
template <int RF_THREADS>
__global__ __launch_bounds__(RF_THREADS) void k_refine(BatchCtx c, int S) {
    TS_BACK_PRIO;
    static_assert(RF_VIRT % RF_THREADS == 0, "virtual partition");
    __shared__ int s_scan[RF_THREADS / 64];
    __shared__ double s_red[RF_VIRT / 64][N_ACC];
    __shared__ double s_tot[N_ACC];
    __shared__ double s_R[9], s_t[3], s_H[36], s_misc[4];
    __shared__ int s_flag, s_best;
    const int p = c.pair0 + (int)blockIdx.x % c.npair;
    const int f = (int)blockIdx.x / c.npair;
    const int fp = f * c.P + p;
    const int64_t g = c.g0 + f;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int32_t* sout = c.stats + (size_t)fp * TS_STATS_INTS;
    if (sout[0] != 3) return;
    const int n = sout[1];
    double* pout = c.pose + (size_t)fp * TS_POSE_DOUBLES;
    const PairCalib cal = c.calib[p];
    const double fx = cal.fx, fy = cal.fy, cx = cal.cx, cy = cal.cy;
    const double thr2 = c.pp.thr2;
    const double* corr = c.corr + ((size_t)f * c.P + p) * c.g.K * TS_CORR_DOUBLES;
    const uint32_t* kin = reinterpret_cast<const uint32_t*>(c.ransac) + (size_t)fp * S * TS_RANSAC_WORDS;
    if (tid == 0) {
        uint32_t best = 0;
        int bs = 0;
        for (int s2 = 0; s2 < S; ++s2)
            if (kin[s2 * TS_RANSAC_WORDS] > best) {
                best = kin[s2 * TS_RANSAC_WORDS];
                bs = s2;
            }
        s_best = bs;
    }
    __syncthreads();
    const uint32_t bkey = kin[s_best * TS_RANSAC_WORDS];
    const int best_cnt = (int)(bkey >> 12) - 1;
    const int best_idx = 4095 - (int)(bkey & 4095u);
    if (best_cnt < 3) {
        if (tid == 0) write_stats(sout, 1, n, 0, best_cnt, best_idx, g);
        return;
    }
    if (tid < 12) {
        const double v = reinterpret_cast<const double*>(kin + s_best * TS_RANSAC_WORDS + 2)[tid];
        if (tid < 9) s_R[tid] = v; else s_t[tid - 9] = v;
    }
    __syncthreads();

    bool fail = false;
    double sq_last = 0.0;
    for (int it = 0; it < c.pp.iters; ++it) {
        double R[9], t[3];
#pragma unroll
        for (int k = 0; k < 9; ++k) R[k] = s_R[k];
        t[0] = s_t[0]; t[1] = s_t[1]; t[2] = s_t[2];
        for (int pass = 0; pass < RF_VIRT / RF_THREADS; ++pass) {
        double acc[N_ACC];
#pragma unroll
        for (int k = 0; k < N_ACC; ++k) acc[k] = 0.0;
        for (int ci = tid + pass * RF_THREADS; ci < n; ci += RF_VIRT) {
            const double* cr = corr + (size_t)ci * TS_CORR_DOUBLES;
            if (!is_inlier(R, t, cr, fx, fy, thr2)) continue;
            const double X = cr[0], Y = cr[1], Z = cr[2];
            const double u = cx - cr[3], v = cy - cr[4];
            const double xc = ((R[0] * X + R[1] * Y) + R[2] * Z) + t[0];
            const double yc = ((R[3] * X + R[4] * Y) + R[5] * Z) + t[1];
            const double zc = ((R[6] * X + R[7] * Y) + R[8] * Z) + t[2];
            const double iz = 1.0 / zc;
            const double rx = (((fx * xc) * iz) + cx) - u;
            const double ry = (((fy * yc) * iz) + cy) - v;
            const double a = fx * iz, b = fy * iz;
            const double cc = (-(fx * xc)) * (iz * iz);
            const double dd = (-(fy * yc)) * (iz * iz);
            const double jx[6] = {a, 0.0, cc, cc * yc, a * zc - cc * xc, -a * yc};
            const double jy[6] = {0.0, b, dd, -b * zc + dd * yc, -dd * xc, b * xc};
            int k = 0;
#pragma unroll
            for (int r0 = 0; r0 < 6; ++r0)
#pragma unroll
                for (int c0 = r0; c0 < 6; ++c0) acc[k++] += jx[r0] * jx[c0] + jy[r0] * jy[c0];
#pragma unroll
            for (int r0 = 0; r0 < 6; ++r0) acc[21 + r0] += jx[r0] * rx + jy[r0] * ry;
            acc[27] += rx * rx + ry * ry;
            acc[28] += 1.0;
        }
        {
            const double w = wave_multi_sum(acc);   // the sum of acc[lane >> 1]
            if ((lane & 1) == 0 && (lane >> 1) < N_ACC) s_red[wave + pass * (RF_THREADS / 64)][lane >> 1] = w;
        }
        }
        __syncthreads();
        // lanes 0..28 of wave 0 add the virtual waves' sums of one accumulator each (the order the
        // single thread used), then thread 0 reads the 29 totals
        if (tid < N_ACC) {
            double v = s_red[0][tid];
#pragma unroll
            for (int w = 1; w < RF_VIRT / 64; ++w) v += s_red[w][tid];
            s_tot[tid] = v;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (tid == 0) {
            double tot[N_ACC];
            for (int k = 0; k < N_ACC; ++k) tot[k] = s_tot[k];
            const int n_in = (int)tot[28];
            s_flag = 0;
            if (n_in < 6) {
                s_flag = 1;
            } else {
                double Hm[36], gv[6], x[6], L[36];
                int k = 0;
                for (int r0 = 0; r0 < 6; ++r0)
                    for (int c0 = r0; c0 < 6; ++c0) {
                        Hm[r0 * 6 + c0] = tot[k];
                        Hm[c0 * 6 + r0] = tot[k];
                        ++k;
                    }
                for (int r0 = 0; r0 < 6; ++r0) gv[r0] = -tot[21 + r0];
                if (c.prior) {   // IMU rotation prior (weight W, px^2 / rad^2): W/2 |w - delta|^2
                    const double* pr = c.prior + (size_t)fp * TS_PRIOR_DOUBLES;
                    const double W = pr[9];
                    if (W > 0.0) {
                        double Mq[9];
                        for (int i = 0; i < 3; ++i)
                            for (int j = 0; j < 3; ++j)
                                Mq[3 * i + j] = (pr[3 * i] * s_R[3 * j] + pr[3 * i + 1] * s_R[3 * j + 1]) + pr[3 * i + 2] * s_R[3 * j + 2];
                        const double dl[3] = {0.5 * (Mq[7] - Mq[5]), 0.5 * (Mq[2] - Mq[6]), 0.5 * (Mq[3] - Mq[1])};
                        for (int i = 0; i < 3; ++i) {
                            Hm[(3 + i) * 6 + 3 + i] += W;
                            gv[3 + i] += W * dl[i];
                        }
                    }
                    // accelerometer translation prior (weight W_t, px^2 / m^2): W_t/2 |t + rho - t_prior|^2
                    const double Wt = pr[13];
                    if (Wt > 0.0) {
                        for (int i = 0; i < 3; ++i) {
                            Hm[i * 6 + i] += Wt;
                            gv[i] += Wt * (pr[10 + i] - s_t[i]);
                        }
                    }
                }
                for (int q = 0; q < 36; ++q) L[q] = 0.0;
                if (!solve6(Hm, gv, x, L)) {
                    s_flag = 1;
                } else {
                    const double w0 = x[3], w1 = x[4], w2 = x[5];
                    const double A[9] = {0.0, -w2, w1, w2, 0.0, -w0, -w1, w0, 0.0};
                    double A2[9];
                    for (int i = 0; i < 3; ++i)
                        for (int j = 0; j < 3; ++j)
                            A2[3 * i + j] = (A[3 * i] * A[j] + A[3 * i + 1] * A[3 + j]) + A[3 * i + 2] * A[6 + j];
                    const double n2 = (w0 * w0 + w1 * w1) + w2 * w2;
                    const double sc = 4.0 / (4.0 + n2);
                    double RU[9];
                    for (int q = 0; q < 9; ++q) RU[q] = ((q % 4) == 0 ? 1.0 : 0.0) + sc * (A[q] + 0.5 * A2[q]);
                    double Rn[9], tn[3];
                    for (int i = 0; i < 3; ++i) {
                        for (int j = 0; j < 3; ++j)
                            Rn[3 * i + j] = (RU[3 * i] * s_R[j] + RU[3 * i + 1] * s_R[3 + j]) + RU[3 * i + 2] * s_R[6 + j];
                        tn[i] = ((RU[3 * i] * s_t[0] + RU[3 * i + 1] * s_t[1]) + RU[3 * i + 2] * s_t[2]) + x[i];
                    }
                    for (int q = 0; q < 9; ++q) s_R[q] = Rn[q];
                    for (int q = 0; q < 3; ++q) s_t[q] = tn[q];
                    for (int q = 0; q < 36; ++q) s_H[q] = Hm[q];
                    s_misc[0] = tot[27];
                }
            }
        }
        __syncthreads();
        if (s_flag) {
            fail = true;
            break;
        }
        sq_last = s_misc[0];
    }
    int cnt_local = 0;
    if (!fail) {
        double R[9], t[3];
#pragma unroll
        for (int k = 0; k < 9; ++k) R[k] = s_R[k];
        t[0] = s_t[0]; t[1] = s_t[1]; t[2] = s_t[2];
        for (int ci = tid; ci < n; ci += RF_THREADS)
            cnt_local += is_inlier(R, t, corr + (size_t)ci * TS_CORR_DOUBLES, fx, fy, thr2) ? 1 : 0;
    }
    cnt_local = wave_sum_i32(cnt_local);
    if (lane == 0) s_scan[wave] = cnt_local;
    __syncthreads();
    int n_in = 0;
    for (int w = 0; w < RF_THREADS / 64; ++w) n_in += s_scan[w];
    const bool ok = !fail && n_in >= c.pp.min_inliers;
    const double sigma2 = sq_last / (double)max(1, 2 * n_in - 6);
    if (tid == 0) {
        write_stats(sout, ok ? 0 : 1, n, fail ? 0 : n_in, best_cnt, best_idx, g);
        if (ok) {
            for (int i = 0; i < 3; ++i) {
                for (int j = 0; j < 3; ++j) pout[4 * i + j] = s_R[3 * i + j];
                pout[4 * i + 3] = s_t[i];
            }
            // stats[6..7]: sigma^2 (f64), so the host can take a motion prior back out of the
            // covariance (the vision-only motion for the IMU filter's bias update)
            *reinterpret_cast<double*>(sout + 6) = sigma2;
        }
    }
    if (ok && tid < 6) {   // covariance column k = tid: H^-1 e_k sigma^2, the six columns side by side
        double L[36], e[6], col[6];
        for (int q = 0; q < 36; ++q) L[q] = 0.0;
        for (int q = 0; q < 6; ++q) e[q] = q == tid ? 1.0 : 0.0;
        if (solve6(s_H, e, col, L))
            for (int q = 0; q < 6; ++q) pout[32 + q * 6 + tid] = col[q] * sigma2;
    }
}

// Pose chaining: T_abs(g) = T_abs(g-1) * F(g), F(g) = inv(T_rel(g)) for a tracked frame (the IMU's
// motion for an IMU-propagated one), the identity otherwise.  The association of the products is
// fixed by the global frame index, so results do not depend on how frames are batched (nor on a
// sharded rig's ranges): frames form global blocks of TS_CHAIN_BLK, and
//   T_abs(g) = A(j) * Q(g),  Q(g) = Q(g-1) * F(g) inside block j (Q = I before its first frame),
//   A(j) = A(j-1) * Q(last frame of block j-1).
// The chain state is (A, Q) of the last chained frame (32 doubles); a batch whose first frame opens
// a block first folds Q into A.  One block per chain (blocks 0 .. P-1 the pairs, block P the rig's
// body motion), rounds of up to TS_CHAIN_SEGS global blocks: the round's factors are inverted in
// parallel into LDS, the blocks' prefixes run side by side (16 lanes each, one element of Q per lane:
// a row of Q by 4 quad-DPP broadcasts, its element of the product by a 4-term dot product, written
// back over the factor in LDS), one 16-lane group chains the round's A's, and every element of
// every A * Q is one parallel pass.  A launch of n frames costs about TS_CHAIN_BLK + n / TS_CHAIN_BLK
// dependent steps instead of n (C2, 1,024 frames: 164 -> see DESIGN.md §5).
#define TS_CHAIN_BLK 64
#define TS_CHAIN_SEGS 4
#define TS_CHAIN_ROUND (TS_CHAIN_BLK * TS_CHAIN_SEGS)

// a * b of two row-major 4x4 matrices, element (i, j), the oracle's operation order
__device__ __forceinline__ double mul4_elem(const double* a, const double* b, int i, int j) {
    return ((a[4 * i] * b[j] + a[4 * i + 1] * b[4 + j]) + a[4 * i + 2] * b[8 + j]) + a[4 * i + 3] * b[12 + j];
}

__global__ __launch_bounds__(256) void k_chain(BatchCtx c) {
    TS_BACK_PRIO;
    __shared__ double s_f[TS_CHAIN_ROUND][16];   // the round's factors, then its prefixes Q(f)
    __shared__ int s_keep[TS_CHAIN_ROUND];        // 1: the frame does not move the chain
    __shared__ double s_A[TS_CHAIN_SEGS + 1][16];  // A of each segment of the round (+ the next)
    __shared__ double s_Qin[16];                    // the round's first segment's starting prefix
    __shared__ double s_Ql[TS_CHAIN_SEGS][16];     // each segment's last prefix
    const int tid = threadIdx.x;
    const bool rig = (int)blockIdx.x >= c.P;   // the rig's chain (k_rig_pose's body motions)
    const int P = rig ? 1 : c.P, p = rig ? 0 : (int)blockIdx.x;
    double* pose = rig ? c.rig_pose : c.pose;
    const int32_t* stats = rig ? c.rig_stats : c.stats;
    double* state = rig ? c.rig_state : c.state + 32 * p;
    const double* prior = rig ? (c.prior ? c.rig_prior : nullptr) : c.prior;
    const int off = (int)(c.g0 % TS_CHAIN_BLK);
    if (tid < 16) {
        const double A = state[tid], Q = state[16 + tid];
        s_A[0][tid] = A;
        s_Qin[tid] = Q;
    }
    __syncthreads();
    if (off == 0 && tid < 16) {   // the batch opens a block: A = A * Q, Q = I
        const int i = tid >> 2, j = tid & 3;
        const double A = mul4_elem(s_A[0], s_Qin, i, j);
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");   // every lane has read A, Q
        s_A[0][tid] = A;
        s_Qin[tid] = i == j ? 1.0 : 0.0;
    }
    __syncthreads();
    // segments of the batch: [0, len0), then whole global blocks, the last one possibly partial
    const int len0 = min(c.n, TS_CHAIN_BLK - off);
    const int nseg = 1 + (c.n - len0 + TS_CHAIN_BLK - 1) / TS_CHAIN_BLK;
    for (int s0 = 0; s0 < nseg; s0 += TS_CHAIN_SEGS) {
        const int ns = min(TS_CHAIN_SEGS, nseg - s0);
        const int f0 = s0 == 0 ? 0 : len0 + (s0 - 1) * TS_CHAIN_BLK;   // the round's first frame
        const int f1 = min(c.n, len0 + (s0 + ns - 1) * TS_CHAIN_BLK);  // one past its last
        const int nf = f1 - f0;
        // 1. factors F(f) = inv(T_rel(f)) into LDS; an untracked frame with an accelerometer
        // prediction (W_t > 0) moves by the IMU's T_rel = [R_prior | t_prior] (its pose record's
        // T_rel becomes that prediction); other untracked frames keep the chain
        for (int fl = tid; fl < nf; fl += blockDim.x) {
            const size_t fp = (size_t)(f0 + fl) * P + p;
            const int st = stats[fp * TS_STATS_INTS];
            const bool imu = st != 0 && prior && prior[fp * TS_PRIOR_DOUBLES + 13] > 0.0;
            s_keep[fl] = (st == 0 || imu) ? 0 : 1;
        }
        __syncthreads();
        for (int i = tid; i < nf * 16; i += blockDim.x) {
            const int fl = i / 16, e = i % 16, r = e / 4, q = e % 4;
            const size_t fp = (size_t)(f0 + fl) * P + p;
            const double* rel = pose + fp * TS_POSE_DOUBLES;
            const bool imu = stats[fp * TS_STATS_INTS] != 0 && !s_keep[fl];
            double v;
            if (imu) {
                const double* pr = prior + fp * TS_PRIOR_DOUBLES;
                if (r == 3) v = q == 3 ? 1.0 : 0.0;
                else if (q < 3) v = pr[3 * q + r];
                else v = -((pr[r] * pr[10] + pr[3 + r] * pr[11]) + pr[6 + r] * pr[12]);
                pose[fp * TS_POSE_DOUBLES + e] = r == 3 ? (q == 3 ? 1.0 : 0.0) : (q < 3 ? pr[3 * r + q] : pr[10 + r]);
            } else {
                if (r == 3) v = q == 3 ? 1.0 : 0.0;
                else if (q < 3) v = rel[4 * q + r];
                else v = -((rel[r] * rel[3] + rel[4 + r] * rel[7]) + rel[8 + r] * rel[11]);
            }
            s_f[fl][e] = v;
        }
        __syncthreads();
        // 2. the prefixes: segment s0 + q by lanes 16q .. 16q + 15 of wave 0
        if (tid < 16 * ns) {
            const int q = tid >> 4, e = tid & 15, i = e >> 2, j = e & 3;
            const int sg = s0 + q;
            const int a = (sg == 0 ? 0 : len0 + (sg - 1) * TS_CHAIN_BLK) - f0;
            const int b = min(c.n, sg == 0 ? len0 : len0 + sg * TS_CHAIN_BLK) - f0;
            double Q = sg == 0 ? s_Qin[e] : (i == j ? 1.0 : 0.0);
            double i0 = s_f[a][j], i1 = s_f[a][4 + j], i2 = s_f[a][8 + j], i3 = s_f[a][12 + j];
            int keep = s_keep[a];
            for (int fl = a; fl < b; ++fl) {
                const int fn = min(fl + 1, b - 1);   // the next frame's operands, off the critical path
                const double n0 = s_f[fn][j], n1 = s_f[fn][4 + j], n2 = s_f[fn][8 + j], n3 = s_f[fn][12 + j];
                const int keep_n = s_keep[fn];
                // row i of Q lives in this lane's quad: quad_perm broadcasts
                const double t0 = dpp_f64c<0x00>(Q), t1 = dpp_f64c<0x55>(Q);
                const double t2 = dpp_f64c<0xAA>(Q), t3 = dpp_f64c<0xFF>(Q);
                const double nq = ((t0 * i0 + t1 * i1) + t2 * i2) + t3 * i3;
                Q = keep ? Q : nq;
                s_f[fl][e] = Q;   // every lane of the group read this frame's column above
                keep = keep_n;
                i0 = n0;
                i1 = n1;
                i2 = n2;
                i3 = n3;
            }
            s_Ql[q][e] = Q;
        }
        __syncthreads();
        // 3. the round's A's, in order: A(s + 1) = A(s) * Q_last(s)
        if (tid < 16) {
            const int i = tid >> 2, j = tid & 3;
            for (int q = 0; q < ns; ++q) {
                const double An = mul4_elem(s_A[q], s_Ql[q], i, j);
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                s_A[q + 1][tid] = An;
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            }
        }
        __syncthreads();
        // 4. T_abs(f) = A(segment of f) * Q(f)
        for (int i = tid; i < nf * 16; i += blockDim.x) {
            const int fl = i / 16, e = i % 16;
            const int f = f0 + fl;
            const int q = (f < len0 ? 0 : 1 + (f - len0) / TS_CHAIN_BLK) - s0;
            pose[((size_t)f * P + p) * TS_POSE_DOUBLES + 16 + e] = mul4_elem(s_A[q], s_f[fl], e >> 2, e & 3);
        }
        __syncthreads();
        // the new state: (A, Q) of the round's last segment; the next round starts from A(ns)
        if (tid < 16) {
            const double Al = s_A[ns - 1][tid], Ql = s_Ql[ns - 1][tid], An = s_A[ns][tid];
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            if (s0 + ns == nseg) {
                state[tid] = Al;
                state[16 + tid] = Ql;
            }
            s_A[0][tid] = An;
        }
        __syncthreads();
    }
}

// ---- rig pose: generalised PnP over every pair of the rig ---------------
// One block per frame.  Candidates: each tracked pair's motion moved to the body frame,
// M_p = (E_p T_p) E_p^-1 with E_p = base_T_rect-left of pair p.  Each candidate is scored on the
// correspondences of ALL pairs (pair q sees T_q = (E_q^-1 M) E_q, A7's inlier test in its own
// camera); the most inliers wins (ties: lowest pair).  Gauss-Newton then refines M on the inliers
// of all pairs together (re-selected every iteration, A7's left-multiplied Cayley update applied to
// the body motion): with Y = E_q Xc the body point, d(res)/d(rho, omega) = [q, Y x q] where
// q = dpi/dXc R_e^T.  Covariance sigma^2 H^-1 in the body frame.
__device__ __forceinline__ void mul4_fixed(const double* A, const double* B, double* out) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            out[4 * i + j] = ((A[4 * i] * B[j] + A[4 * i + 1] * B[4 + j]) + A[4 * i + 2] * B[8 + j]) + A[4 * i + 3] * B[12 + j];
}

#define TS_RIG_MAXP 8
// 512 threads (8 waves) per frame: the kernel is a per-frame latency chain (scoring, then 8
// Gauss-Newton sweeps over every pair's correspondences with a block reduction and a 6x6 solve
// each); 198 VGPRs fit 2 waves per SIMD, and each thread's share of the sweeps halves
#define RIG_THREADS 512
#define RIG_WAVES (RIG_THREADS / 64)
__global__ __launch_bounds__(RIG_THREADS) void k_rig_pose(BatchCtx c) {
    TS_BACK_PRIO;
    __shared__ double s_M[TS_RIG_MAXP][16];                  // candidates (body motions)
    __shared__ double s_T[TS_RIG_MAXP][TS_RIG_MAXP][12];     // [candidate][pair] R | t
    __shared__ int s_cnt[RIG_WAVES][TS_RIG_MAXP];
    __shared__ double s_red[RIG_WAVES][N_ACC];
    __shared__ double s_tot[N_ACC];
    __shared__ double s_H[36], s_misc[2];
    __shared__ int s_nc, s_flag, s_best;
    const int f = blockIdx.x;
    const int64_t g = c.g0 + f;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int P = c.P, K = c.g.K;
    double* pout = c.rig_pose + (size_t)f * TS_POSE_DOUBLES;
    int32_t* sout = c.rig_stats + (size_t)f * TS_STATS_INTS;
    for (int i = tid; i < TS_POSE_DOUBLES; i += RIG_THREADS) pout[i] = (i < 16 && (i % 5) == 0) ? 1.0 : 0.0;
    if (g == 0 && !c.reloc) {
        if (tid == 0) write_stats(sout, 2, 0, 0, 0, -1, g);
        return;
    }
#ifdef TS_RIG_STAMPS   // experiment builds: phase durations of block 0 (s_memrealtime, 100 MHz)
    uint64_t ts_prev = wall_clock64(), ts_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define RSTAMP(i)                                    \
    do {                                             \
        const uint64_t n_ = wall_clock64();          \
        ts_acc[i] += n_ - ts_prev;                   \
        ts_prev = n_;                                \
    } while (0)
#else
#define RSTAMP(i) \
    do {          \
    } while (0)
#endif
    if (tid == 0) {
        int nc = 0;
        for (int p = 0; p < P; ++p) {
            if (c.stats[(size_t)(f * P + p) * TS_STATS_INTS] != 0) continue;
            double Tp[16], ET[16];
            const double* rel = c.pose + (size_t)(f * P + p) * TS_POSE_DOUBLES;
            for (int e = 0; e < 16; ++e) Tp[e] = rel[e];
            mul4_fixed(c.rig_E + 16 * p, Tp, ET);
            mul4_fixed(ET, c.rig_Einv + 16 * p, s_M[nc]);
            ++nc;
        }
        s_nc = nc;
    }
    __syncthreads();
    RSTAMP(0);
    const int nc = s_nc;
    int n_total = 0;
    for (int q = 0; q < P; ++q) n_total += c.stats[(size_t)(f * P + q) * TS_STATS_INTS + 1];
    if (nc == 0) {
        if (tid == 0) write_stats(sout, 1, n_total, 0, 0, -1, g);
        return;
    }
    // per (candidate, pair): T_q = (E_q^-1 M) E_q
    for (int i = tid; i < nc * P; i += RIG_THREADS) {
        const int m = i / P, q = i % P;
        double A[16], T[16];
        mul4_fixed(c.rig_Einv + 16 * q, s_M[m], A);
        mul4_fixed(A, c.rig_E + 16 * q, T);
        for (int r = 0; r < 3; ++r) {
            for (int k = 0; k < 3; ++k) s_T[m][q][3 * r + k] = T[4 * r + k];
            s_T[m][q][9 + r] = T[4 * r + 3];
        }
    }
    __syncthreads();
    RSTAMP(1);
    // scoring: every candidate on every pair's correspondences (integer counts, order-free)
    int cnt[TS_RIG_MAXP];
    for (int m = 0; m < TS_RIG_MAXP; ++m) cnt[m] = 0;
    const double thr2 = c.pp.thr2;
    for (int q = 0; q < P; ++q) {
        const int nq = c.stats[(size_t)(f * P + q) * TS_STATS_INTS + 1];
        const double* corr = c.corr + ((size_t)f * P + q) * K * TS_CORR_DOUBLES;
        const double fx = c.calib[q].fx, fy = c.calib[q].fy;
        for (int ci = tid; ci < nq; ci += RIG_THREADS) {
            const double* cr = corr + (size_t)ci * TS_CORR_DOUBLES;
            for (int m = 0; m < nc; ++m) cnt[m] += is_inlier(s_T[m][q], s_T[m][q] + 9, cr, fx, fy, thr2) ? 1 : 0;
        }
    }
    for (int m = 0; m < TS_RIG_MAXP; ++m) {
        const int w = wave_sum_i32(cnt[m]);
        if (lane == 0) s_cnt[wave][m] = w;
    }
    __syncthreads();
    RSTAMP(2);
    if (tid == 0) {
        int best = 0, bc = -1;
        for (int m = 0; m < nc; ++m) {
            int t = 0;
            for (int w = 0; w < RIG_WAVES; ++w) t += s_cnt[w][m];
            if (t > bc) {
                bc = t;
                best = m;
            }
        }
        s_best = best;
        s_misc[1] = (double)bc;
    }
    __syncthreads();
    const int best_cnt = (int)s_misc[1], best_idx = s_best;
    // Gauss-Newton on the body motion (s_M[0] holds the current estimate)
    if (tid < 16) s_M[0][tid] = s_M[best_idx][tid];
    __syncthreads();
    RSTAMP(3);
    bool fail = false;
    double sq_last = 0.0;
    for (int it = 0; it < c.pp.iters; ++it) {
        for (int q = tid; q < P; q += RIG_THREADS) {
            double A[16], T[16];
            mul4_fixed(c.rig_Einv + 16 * q, s_M[0], A);
            mul4_fixed(A, c.rig_E + 16 * q, T);
            for (int r = 0; r < 3; ++r) {
                for (int k = 0; k < 3; ++k) s_T[0][q][3 * r + k] = T[4 * r + k];
                s_T[0][q][9 + r] = T[4 * r + 3];
            }
        }
        __syncthreads();
        RSTAMP(4);
        double acc[N_ACC];
#pragma unroll
        for (int k = 0; k < N_ACC; ++k) acc[k] = 0.0;
        for (int q = 0; q < P; ++q) {
            const int nq = c.stats[(size_t)(f * P + q) * TS_STATS_INTS + 1];
            const double* corr = c.corr + ((size_t)f * P + q) * K * TS_CORR_DOUBLES;
            const PairCalib cal = c.calib[q];
            const double fx = cal.fx, fy = cal.fy, cx = cal.cx, cy = cal.cy;
            const double* R = s_T[0][q];
            const double* t = R + 9;
            const double* E = c.rig_E + 16 * q;
            for (int ci = tid; ci < nq; ci += RIG_THREADS) {
                const double* cr = corr + (size_t)ci * TS_CORR_DOUBLES;
                if (!is_inlier(R, t, cr, fx, fy, thr2)) continue;
                const double X = cr[0], Y = cr[1], Z = cr[2];
                const double u = cx - cr[3], v = cy - cr[4];
                const double xc = ((R[0] * X + R[1] * Y) + R[2] * Z) + t[0];
                const double yc = ((R[3] * X + R[4] * Y) + R[5] * Z) + t[1];
                const double zc = ((R[6] * X + R[7] * Y) + R[8] * Z) + t[2];
                const double iz = 1.0 / zc;
                const double rx = (((fx * xc) * iz) + cx) - u;
                const double ry = (((fy * yc) * iz) + cy) - v;
                const double a = fx * iz, b = fy * iz;
                const double cc = (-(fx * xc)) * (iz * iz);
                const double dd = (-(fy * yc)) * (iz * iz);
                const double by0 = ((E[0] * xc + E[1] * yc) + E[2] * zc) + E[3];
                const double by1 = ((E[4] * xc + E[5] * yc) + E[6] * zc) + E[7];
                const double by2 = ((E[8] * xc + E[9] * yc) + E[10] * zc) + E[11];
                // q = dpi/dXc R_e^T: q_j = sum_i p_i R_e[j][i]
                const double qx0 = a * E[0] + cc * E[2], qx1 = a * E[4] + cc * E[6], qx2 = a * E[8] + cc * E[10];
                const double qy0 = b * E[1] + dd * E[2], qy1 = b * E[5] + dd * E[6], qy2 = b * E[9] + dd * E[10];
                const double jx[6] = {qx0, qx1, qx2, by1 * qx2 - by2 * qx1, by2 * qx0 - by0 * qx2, by0 * qx1 - by1 * qx0};
                const double jy[6] = {qy0, qy1, qy2, by1 * qy2 - by2 * qy1, by2 * qy0 - by0 * qy2, by0 * qy1 - by1 * qy0};
                int k = 0;
#pragma unroll
                for (int r0 = 0; r0 < 6; ++r0)
#pragma unroll
                    for (int c0 = r0; c0 < 6; ++c0) acc[k++] += jx[r0] * jx[c0] + jy[r0] * jy[c0];
#pragma unroll
                for (int r0 = 0; r0 < 6; ++r0) acc[21 + r0] += jx[r0] * rx + jy[r0] * ry;
                acc[27] += rx * rx + ry * ry;
                acc[28] += 1.0;
            }
        }
        {
            const double w = wave_multi_sum(acc);   // the sum of acc[lane >> 1]
            if ((lane & 1) == 0 && (lane >> 1) < N_ACC) s_red[wave][lane >> 1] = w;
        }
        __syncthreads();
        RSTAMP(5);
        // lanes 0..28 of wave 0 add the 8 wave sums of one accumulator each (the same order the
        // single thread used), then thread 0 reads the 29 totals
        if (tid < N_ACC) {
            double v = s_red[0][tid];
#pragma unroll
            for (int w = 1; w < RIG_WAVES; ++w) v += s_red[w][tid];
            s_tot[tid] = v;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (tid == 0) {
            double tot[N_ACC];
            for (int k = 0; k < N_ACC; ++k) tot[k] = s_tot[k];
            s_flag = 0;
            double Hm[36], gv[6], x[6], L[36];
            int k = 0;
            for (int r0 = 0; r0 < 6; ++r0)
                for (int c0 = r0; c0 < 6; ++c0) {
                    Hm[r0 * 6 + c0] = tot[k];
                    Hm[c0 * 6 + r0] = tot[k];
                    ++k;
                }
            for (int r0 = 0; r0 < 6; ++r0) gv[r0] = -tot[21 + r0];
            for (int q = 0; q < 36; ++q) L[q] = 0.0;
            if ((int)tot[28] < 6 || !solve6(Hm, gv, x, L)) {
                s_flag = 1;
            } else {
                const double w0 = x[3], w1 = x[4], w2 = x[5];
                const double A[9] = {0.0, -w2, w1, w2, 0.0, -w0, -w1, w0, 0.0};
                double A2[9];
                for (int i = 0; i < 3; ++i)
                    for (int j = 0; j < 3; ++j) A2[3 * i + j] = (A[3 * i] * A[j] + A[3 * i + 1] * A[3 + j]) + A[3 * i + 2] * A[6 + j];
                const double n2 = (w0 * w0 + w1 * w1) + w2 * w2;
                const double sc = 4.0 / (4.0 + n2);
                double RU[9];
                for (int q = 0; q < 9; ++q) RU[q] = ((q % 4) == 0 ? 1.0 : 0.0) + sc * (A[q] + 0.5 * A2[q]);
                double* M = s_M[0];
                double Rn[9], tn[3];
                for (int i = 0; i < 3; ++i) {
                    for (int j = 0; j < 3; ++j) Rn[3 * i + j] = (RU[3 * i] * M[j] + RU[3 * i + 1] * M[4 + j]) + RU[3 * i + 2] * M[8 + j];
                    tn[i] = ((RU[3 * i] * M[3] + RU[3 * i + 1] * M[7]) + RU[3 * i + 2] * M[11]) + x[i];
                }
                for (int i = 0; i < 3; ++i) {
                    for (int j = 0; j < 3; ++j) M[4 * i + j] = Rn[3 * i + j];
                    M[4 * i + 3] = tn[i];
                }
                for (int q = 0; q < 36; ++q) s_H[q] = Hm[q];
                s_misc[0] = tot[27];
            }
        }
        __syncthreads();
        RSTAMP(6);
        if (s_flag) {
            fail = true;
            break;
        }
        sq_last = s_misc[0];
    }
    // final inliers of all pairs under M
    for (int q = tid; q < P; q += RIG_THREADS) {
        double A[16], T[16];
        mul4_fixed(c.rig_Einv + 16 * q, s_M[0], A);
        mul4_fixed(A, c.rig_E + 16 * q, T);
        for (int r = 0; r < 3; ++r) {
            for (int k = 0; k < 3; ++k) s_T[0][q][3 * r + k] = T[4 * r + k];
            s_T[0][q][9 + r] = T[4 * r + 3];
        }
    }
    __syncthreads();
    int cnt_local = 0;
    if (!fail)
        for (int q = 0; q < P; ++q) {
            const int nq = c.stats[(size_t)(f * P + q) * TS_STATS_INTS + 1];
            const double* corr = c.corr + ((size_t)f * P + q) * K * TS_CORR_DOUBLES;
            for (int ci = tid; ci < nq; ci += RIG_THREADS)
                cnt_local += is_inlier(s_T[0][q], s_T[0][q] + 9, corr + (size_t)ci * TS_CORR_DOUBLES, c.calib[q].fx,
                                       c.calib[q].fy, thr2) ? 1 : 0;
        }
    cnt_local = wave_sum_i32(cnt_local);
    if (lane == 0) s_cnt[wave][0] = cnt_local;
    __syncthreads();
    int n_in = 0;
    for (int w = 0; w < RIG_WAVES; ++w) n_in += s_cnt[w][0];
    const bool ok = !fail && n_in >= c.pp.min_inliers;
    if (tid == 0) {
        write_stats(sout, ok ? 0 : 1, n_total, fail ? 0 : n_in, best_cnt, best_idx, g);
        if (ok)
            for (int e = 0; e < 12; ++e) pout[e] = s_M[0][e];
    }
    if (ok && tid < 6) {   // covariance column k = tid, the six columns side by side
        const double sigma2 = sq_last / (double)max(1, 2 * n_in - 6);
        double L[36], e6[6], col[6];
        for (int q = 0; q < 36; ++q) L[q] = 0.0;
        for (int q = 0; q < 6; ++q) e6[q] = q == tid ? 1.0 : 0.0;
        if (solve6(s_H, e6, col, L))
            for (int q = 0; q < 6; ++q) pout[32 + q * 6 + tid] = col[q] * sigma2;
    }
#ifdef TS_RIG_STAMPS
    __syncthreads();
    RSTAMP(7);
    if (tid == 0 && (f == 0 || f == (int)gridDim.x - 1))
        printf("rig_stamps f=%d cand %lu candT %lu score %lu best %lu gnT %lu gnAcc %lu gnSolve %lu final %lu (x10ns)\n", f,
               ts_acc[0], ts_acc[1], ts_acc[2], ts_acc[3], ts_acc[4], ts_acc[5], ts_acc[6], ts_acc[7]);
#endif
#undef RSTAMP
}

void launch_rig_pose(const BatchCtx& c, hipStream_t s) {
    hipLaunchKernelGGL(k_rig_pose, dim3(c.n), dim3(RIG_THREADS), 0, s, c);
}


// The rig chain's IMU prediction per frame: the first pair with a translation prior (W_t > 0),
// moved to the body frame, M = (E_p [R | t]) E_p^-1, in the prior record layout; weights kept.
__global__ __launch_bounds__(256) void k_rig_prior(BatchCtx c) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= c.n) return;
    double* out = c.rig_prior + (size_t)f * TS_PRIOR_DOUBLES;
    int p = 0;
    while (p < c.P && !(c.prior[((size_t)f * c.P + p) * TS_PRIOR_DOUBLES + 13] > 0.0)) ++p;
    if (p == c.P) {
        for (int i = 0; i < TS_PRIOR_DOUBLES; ++i) out[i] = 0.0;
        return;
    }
    const double* pr = c.prior + ((size_t)f * c.P + p) * TS_PRIOR_DOUBLES;
    double T[16], A[16], M[16];
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) T[4 * i + j] = pr[3 * i + j];
        T[4 * i + 3] = pr[10 + i];
        T[12 + i] = 0.0;
    }
    T[15] = 1.0;
    mul4_fixed(c.rig_E + 16 * p, T, A);
    mul4_fixed(A, c.rig_Einv + 16 * p, M);
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) out[3 * i + j] = M[4 * i + j];
        out[10 + i] = M[4 * i + 3];
    }
    out[9] = pr[9];
    out[13] = pr[13];
    out[14] = out[15] = 0.0;
}

static size_t ransac_lds(const BatchCtx& c) { return (size_t)min(c.g.K, TS_RS_LDS_CAP) * (16 + 8); }

// Bounded scoring (k_ransac) from 256 frames per launch; below that the exhaustive block-wide
// kernel (k_ransac_all) has the shorter critical path (C4, B = 50: 82 against 117 us).
static bool ransac_bounded(const BatchCtx& c) {
    return c.pp.mode == 2 || (c.pp.mode == 0 && c.n * c.npair >= 256);
}

int ransac_splits(const BatchCtx& c) {
    if (c.pp.splits > 0) return min(min(c.pp.splits, c.pp.n_hyp), TS_MAX_SPLITS);
    // bounded: >= 1024 blocks (4 per CU) - fewer splits let one block's best key bound more poses;
    // exhaustive: >= 4096 blocks (measured at B = 256: S = 4 / 8 / 16 -> 325 / 295 / 283 us for the
    // pose stage).  At least 8 hypotheses per split either way.
    const int frames = c.n * c.npair;
    const int target = ransac_bounded(c) ? 1024 : 4096;
    int S = (target + frames - 1) / frames;
    S = max(1, min(S, max(1, c.pp.n_hyp / 8)));
    return min(S, TS_MAX_SPLITS);
}

static void launch_refine(const BatchCtx& c, int S, hipStream_t s) {
    // the block size changes only the speed (RF_VIRT partition above), never the results: 128
    // threads from 1024 problems up (the C2 step: its VGPR-heavy waves then finish in one round
    // beside detect), 256 below (a sharded rank's 512-problem range: pose 305 -> 269 us, probe r4w)
    if (c.pp.refine_block == 128 || (c.pp.refine_block == 0 && c.n * c.npair >= 1024))
        hipLaunchKernelGGL(k_refine<128>, dim3(c.n * c.npair), dim3(128), 0, s, c, S);
    else
        hipLaunchKernelGGL(k_refine<256>, dim3(c.n * c.npair), dim3(256), 0, s, c, S);
}

static void launch_ransac(const BatchCtx& c, int S, hipStream_t s) {
    if (ransac_bounded(c))
        hipLaunchKernelGGL(k_ransac, dim3(c.n * c.npair * S), dim3(POSE_THREADS), ransac_lds(c), s, c, S);
    else
        hipLaunchKernelGGL(k_ransac_all, dim3(c.n * c.npair * S), dim3(POSE_THREADS), 0, s, c, S);
}

void launch_pose(const BatchCtx& c, hipStream_t s) {
    const int S = ransac_splits(c);
    hipLaunchKernelGGL(k_corr, dim3(c.n * c.npair), dim3(POSE_THREADS), 0, s, c);
    hipLaunchKernelGGL(k_p3p, dim3((c.n * c.npair * c.pp.n_hyp + POSE_THREADS - 1) / POSE_THREADS), dim3(POSE_THREADS), 0, s, c);
    launch_ransac(c, S, s);
    launch_refine(c, S, s);
}

// Benchmark hook (never on the product path): moves `percent` % of the batch's refined temporal
// positions by 8..40 px per axis in a random direction — outliers to every pose, the regime of
// tests/test_gpu_parity.py::test_ransac_bounded_scoring_with_outliers — decided per (frame, pair,
// keypoint) by a counter hash of `seed`, so the pose stage can be timed where the bounded RANSAC
// scoring (k_ransac) ends late.  Runs between MATCH_REFINE and POSE.
__global__ __launch_bounds__(256) void k_perturb_uv(BatchCtx c, int percent, uint64_t seed) {
    const int K = c.g.K;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)c.n * c.P * K) return;
    const int k = (int)(i % K), fp = (int)(i / K), p = fp % c.P, f = fp / c.P;
    double* uv = c.tuv + i * 2;
    if (!(uv[0] == uv[0])) return;   // no refined position
    const uint64_t h = splitmix64(seed ^ splitmix64(((uint64_t)(c.g0 + f) << 24) ^ ((uint64_t)p << 16) ^ (uint64_t)k));
    if ((int)(h % 100u) >= percent) return;
    const double du = 8.0 + (double)((h >> 8) % 33u), dv = 8.0 + (double)((h >> 16) % 33u);
    uv[0] += ((h >> 40) & 1u) ? du : -du;
    uv[1] += ((h >> 41) & 1u) ? dv : -dv;
}

void launch_perturb_uv(const BatchCtx& c, int percent, uint64_t seed, hipStream_t s) {
    const int64_t n = (int64_t)c.n * c.P * c.g.K;
    hipLaunchKernelGGL(k_perturb_uv, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, c, percent, seed);
}

// RANSAC + refinement only, on correspondences another kernel wrote (relocalisation).
void launch_pose_solve(const BatchCtx& c, hipStream_t s) {
    const int S = ransac_splits(c);
    hipLaunchKernelGGL(k_p3p, dim3((c.n * c.npair * c.pp.n_hyp + POSE_THREADS - 1) / POSE_THREADS), dim3(POSE_THREADS), 0, s, c);
    launch_ransac(c, S, s);
    launch_refine(c, S, s);
}

// Every pair's chain and, with `rig`, the rig's (after k_rig_prior moves the IMU prediction to
// the body frame), one block each in one launch.
void launch_chains(const BatchCtx& c, bool rig, hipStream_t s) {
    if (rig && c.prior && c.rig_prior)
        hipLaunchKernelGGL(k_rig_prior, dim3((c.n + 255) / 256), dim3(256), 0, s, c);
    hipLaunchKernelGGL(k_chain, dim3(c.P + (rig ? 1 : 0)), dim3(256), 0, s, c);
}
