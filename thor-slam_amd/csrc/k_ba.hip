// k_ba.hip — row A8 of SURVEY.md §8a: sliding-window local bundle adjustment (config C4).
//
// Follows oracle/numpy_ba.py (the spec: keyframes, association by chained temporal matches,
// landmark homes slot*K + k with re-homing on eviction, stereo reprojection residuals, Schur
// complement on the cameras, Gauss-Newton with Levenberg damping, gauge = oldest keyframe).
//
// Per window solve and iteration:
//   k_ba_lin     one thread per landmark: Jacobians of its (<= window) observations, V_i, g_p,i,
//                the Cholesky factor L_i of V_i, and the landmark's Schur columns
//                Q_i = [W_o L_i^-T] (camera rows) with y_i = L_i^-1 g_p,i appended as row 60;
//   k_ba_camred  one block per camera: U_c = sum J_c^T J_c, g_c = sum J_c^T r (fixed order);
//   k_ba_gemm    the dense part of the Schur complement, C = Qe Qe^T over all 3L landmark columns,
//                on the FP64 matrix cores (v_mfma_f64_16x16x4f64), split over blocks in K;
//                C[0:60,0:60] = sum_i W V^-1 W^T and C[0:60, 60] = sum_i W V^-1 g_p;
//   k_ba_solve   one block: fixed-order sum of the split partials, S = blockdiag(U + lam) - C,
//                b = -g_c + C[:,60], camera 0 removed, Cholesky, camera updates (Cayley);
//   k_ba_backsub one thread per landmark: dp = V^-1 (-g_p - sum W_o^T dc), X += dp.
// Every reduction has a fixed order, so a solve is deterministic run to run.  Floating-point
// results differ from the oracle's (LU solves, numpy summation order) at the 1e-12 level.
#include "tslam_ba.h"

// ---------------------------------------------------------------------------------------------
// small dense helpers (f64)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void inv_rigid(const double* T, double* out) {   // 4x4 rigid inverse
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) out[4 * i + j] = T[4 * j + i];
        out[4 * i + 3] = -((T[i] * T[3] + T[4 + i] * T[7]) + T[8 + i] * T[11]);
    }
    out[12] = out[13] = out[14] = 0.0;
    out[15] = 1.0;
}
__device__ __forceinline__ void mul4(const double* A, const double* B, double* out) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            out[4 * i + j] = ((A[4 * i] * B[j] + A[4 * i + 1] * B[4 + j]) + A[4 * i + 2] * B[8 + j]) + A[4 * i + 3] * B[12 + j];
}

// Level-0 observation and validity of keypoint k of image (slot, cam); mirrors oracle.level0_coords.
__device__ __forceinline__ bool kp_obs(const BatchCtx& c, int slot, int cam, int k, double* u, double* v) {
    const uint32_t* kp = c.kps + (((size_t)slot * c.C + cam) * c.g.K + k) * 2;
    const int l = (int)(kp[1] & 0xFF);
    const int cnt = c.kcount[((size_t)slot * c.C + cam) * c.g.n_levels + l];
    if (k - c.g.koff[l] >= cnt) return false;
    const double sc = (double)(1 << l);
    *u = ((double)(kp[0] & 0xFFFF) + 0.5) * sc - 0.5;
    *v = ((double)(kp[0] >> 16) + 0.5) * sc - 0.5;
    return true;
}

// ---------------------------------------------------------------------------------------------
// keyframe insertion (after the batch that contains frame g) and eviction
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_ba_evict(BatchCtx c, BaArgs a) {
    const int K = c.g.K;
    BaPair q = ba_pair(c, a, a.pair);
    const int lo = a.slot * K;
    for (int k = threadIdx.x; k < K; k += blockDim.x) q.remap[k] = -1;
    __syncthreads();
    for (int r = 0; r < a.n_order; ++r) {          // remaining keyframes, oldest first
        const int s = a.order[r];
        for (int k = threadIdx.x; k < K; k += blockDim.x) {
            const int id = q.lm[(size_t)s * K + k];
            if (id >= lo && id < lo + K && q.remap[id - lo] < 0) {   // ids are unique per keyframe
                q.remap[id - lo] = s * K + k;
                for (int e = 0; e < 3; ++e) q.X[(size_t)(s * K + k) * 3 + e] = q.X[(size_t)id * 3 + e];
            }
        }
        __syncthreads();
    }
    for (int r = 0; r < a.n_order; ++r) {
        const int s = a.order[r];
        for (int k = threadIdx.x; k < K; k += blockDim.x) {
            const int id = q.lm[(size_t)s * K + k];
            if (id >= lo && id < lo + K) q.lm[(size_t)s * K + k] = q.remap[id - lo];
        }
    }
    for (int k = threadIdx.x; k < K; k += blockDim.x) q.lm[(size_t)a.slot * K + k] = -1;
}

__global__ __launch_bounds__(1024) void k_ba_insert(BatchCtx c, BaArgs a) {
    __shared__ double s_T[16];   // new keyframe's cam_T_world
    const int K = c.g.K, p = a.pair;
    BaPair q = ba_pair(c, a, p);
    const int64_t g = a.frame;
    const int f = (int)(g - c.g0);                  // frame of the current batch
    const int rslot = ring_slot(c, g);
    if (threadIdx.x == 0) {
        const double* Tfe = c.pose + (size_t)(f * c.P + p) * TS_POSE_DOUBLES + 16;   // world_T_cam
        double Twc[16];
        if (a.prev < 0) {
            for (int e = 0; e < 16; ++e) Twc[e] = Tfe[e];
        } else {
            // W_ba(prev) * inv(W_fe(prev)) * W_fe(g)
            double Wba[16], ifp[16], tmp[16];
            inv_rigid(q.T + (size_t)a.prev * 16, Wba);
            inv_rigid(q.Tfe + (size_t)a.prev * 16, ifp);
            mul4(Wba, ifp, tmp);
            mul4(tmp, Tfe, Twc);
        }
        for (int e = 0; e < 16; ++e) q.Tfe[(size_t)a.slot * 16 + e] = Tfe[e];
        double Tcw[16];
        inv_rigid(Twc, Tcw);
        for (int e = 0; e < 16; ++e) {
            s_T[e] = Tcw[e];
            q.T[(size_t)a.slot * 16 + e] = Tcw[e];
        }
    }
    __syncthreads();
    const PairCalib cal = c.calib[p];
    const double* disp = c.disp + ((size_t)rslot * c.P + p) * K;
    for (int k = threadIdx.x; k < K; k += blockDim.x) {
        double u = __builtin_nan(""), v = __builtin_nan("");
        const bool valid = kp_obs(c, rslot, 2 * p, k, &u, &v);
        const double dd = disp[k];
        const bool has_d = __builtin_isfinite(dd) && dd > 0.0;
        int lm = -1;
        if (valid && a.prev >= 0) {
            int j = k;   // chain the temporal matches back to the previous keyframe
            for (int st = 0; st < a.interval && j >= 0; ++st)
                j = c.temporal[((size_t)ring_slot(c, g - st) * c.P + p) * K + j];
            if (j >= 0) lm = q.lm[(size_t)a.prev * K + j];
        }
        if (valid && lm < 0 && has_d) {
            lm = a.slot * K + k;
            const double z = cal.fxb / dd;
            const double xc[3] = {(u - cal.cx) * z / cal.fx, (v - cal.cy) * z / cal.fy, z};
            for (int e = 0; e < 3; ++e)   // R^T (xc - t)
                q.X[(size_t)lm * 3 + e] = ((s_T[e] * (xc[0] - s_T[3]) + s_T[4 + e] * (xc[1] - s_T[7])) + s_T[8 + e] * (xc[2] - s_T[11]));
        }
        const size_t o = (size_t)a.slot * K + k;
        q.u[o] = valid ? u : __builtin_nan("");
        q.v[o] = valid ? v : __builtin_nan("");
        q.d[o] = has_d ? dd : __builtin_nan("");
        q.lm[o] = lm;
    }
}

// ---------------------------------------------------------------------------------------------
// observation set of a solve (one block): gate at the initial estimate, >= 2 observations per
// landmark, compact landmark index (sorted ids), landmark -> observations CSR, camera ranges
// ---------------------------------------------------------------------------------------------
__device__ int block_scan_excl(int v, int* s_tmp, int* total) {
    // exclusive scan of one int per thread over the block (1024 threads)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_tmp[wave] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        int run = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
            const int t = s_tmp[w];
            s_tmp[w] = run;
            run += t;
        }
        s_tmp[31] = run;
    }
    __syncthreads();
    const int r = s_tmp[wave] + x - v;
    *total = s_tmp[31];
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(1024) void k_ba_gather(BatchCtx c, BaArgs a) {
    __shared__ int s_tmp[32];
    __shared__ double s_T[TS_BA_MAXW][12];
    const int K = c.g.K, p = a.pair;
    BaPair q = ba_pair(c, a, p);
    const PairCalib cal = c.calib[p];
    const int NID = a.W * K;
    for (int i = threadIdx.x; i < NID; i += blockDim.x) q.cnt[i] = 0;
    for (int i = threadIdx.x; i < a.n_order * 12; i += blockDim.x) {
        const int ci = i / 12, e = i % 12;
        s_T[ci][e] = q.T[(size_t)a.order[ci] * 16 + e];
    }
    __syncthreads();
    const double lim = a.outlier_px * a.outlier_px;
    // pass 1: gated candidates in (camera, keypoint) order -> obs arrays, counts per landmark
    int n1 = 0;
    const int total1 = a.n_order * K;
    for (int base = 0; base < total1; base += blockDim.x) {
        const int i = base + threadIdx.x;
        int keep = 0, id = -1, ci = 0, k = 0;
        if (i < total1) {
            ci = i / K;
            k = i - ci * K;
            const size_t o = (size_t)a.order[ci] * K + k;
            id = q.lm[o];
            if (id >= 0) {
                const double* T = s_T[ci];
                const double* X = q.X + (size_t)id * 3;
                const double xc = ((T[0] * X[0] + T[1] * X[1]) + T[2] * X[2]) + T[3];
                const double yc = ((T[4] * X[0] + T[5] * X[1]) + T[6] * X[2]) + T[7];
                const double zc = ((T[8] * X[0] + T[9] * X[1]) + T[10] * X[2]) + T[11];
                const double pu = cal.fx * xc / zc + cal.cx, pv = cal.fy * yc / zc + cal.cy;
                const double du = pu - q.u[o], dv = pv - q.v[o];
                keep = zc > 0.0 && du * du + dv * dv <= lim;
            }
        }
        int tot;
        const int pos = n1 + block_scan_excl(keep, s_tmp, &tot);
        if (keep) {
            q.obs_cam[pos] = ci;
            q.obs_k[pos] = k;
            q.obs_id[pos] = id;
            atomicAdd(&q.cnt[id], 1);
        }
        n1 += tot;
    }
    __syncthreads();
    // pass 2: keep observations of landmarks seen >= 2 times (stable, in place)
    int n2 = 0;
    for (int base = 0; base < n1; base += blockDim.x) {
        const int i = base + threadIdx.x;
        int keep = 0, ci = 0, k = 0, id = 0;
        if (i < n1) {
            ci = q.obs_cam[i];
            k = q.obs_k[i];
            id = q.obs_id[i];
            keep = q.cnt[id] >= 2;
        }
        int tot;
        const int pos = n2 + block_scan_excl(keep, s_tmp, &tot);
        __syncthreads();   // every read of this chunk before any in-place write
        if (keep) {
            q.obs_cam[pos] = ci;
            q.obs_k[pos] = k;
            q.obs_id[pos] = id;
        }
        n2 += tot;
        __syncthreads();
    }
    // compact landmark index = rank among the ids with >= 2 observations (sorted ids)
    int L = 0;
    for (int base = 0; base < NID; base += blockDim.x) {
        const int i = base + threadIdx.x;
        const int fl = i < NID && q.cnt[i] >= 2;
        int tot;
        const int r = L + block_scan_excl(fl, s_tmp, &tot);
        if (i < NID) q.li[i] = fl ? r : -1;
        if (fl) q.lm_id[r] = i;
        L += tot;
    }
    __syncthreads();
    // CSR offsets (counts per compact landmark, exclusive scan)
    int run = 0;
    for (int base = 0; base < L; base += blockDim.x) {
        const int r = base + threadIdx.x;
        const int cn = r < L ? q.cnt[q.lm_id[r]] : 0;
        int tot;
        const int off = run + block_scan_excl(cn, s_tmp, &tot);
        if (r < L) {
            q.lm_off[r] = off;
            q.fill[r] = 0;
        }
        run += tot;
    }
    if (threadIdx.x == 0) q.lm_off[L] = run;
    __syncthreads();
    for (int i = threadIdx.x; i < n2; i += blockDim.x) {
        const int r = q.li[q.obs_id[i]];
        q.lm_obs[q.lm_off[r] + atomicAdd(&q.fill[r], 1)] = i;
    }
    __syncthreads();
    for (int r = threadIdx.x; r < L; r += blockDim.x) {   // each segment in observation order
        const int o0 = q.lm_off[r], o1 = q.lm_off[r + 1];
        for (int x = o0 + 1; x < o1; ++x)
            for (int y = x; y > o0 && q.lm_obs[y - 1] > q.lm_obs[y]; --y) {
                const int t = q.lm_obs[y];
                q.lm_obs[y] = q.lm_obs[y - 1];
                q.lm_obs[y - 1] = t;
            }
    }
    // camera ranges of the (camera-ordered) observations
    for (int ci = threadIdx.x; ci <= a.n_order; ci += blockDim.x) {
        int lo = 0, hi = n2;   // first observation with camera >= ci
        while (lo < hi) {
            const int m = (lo + hi) >> 1;
            if (q.obs_cam[m] < ci) lo = m + 1; else hi = m;
        }
        q.cam_off[ci] = lo;
    }
    if (threadIdx.x == 0) {
        q.counts[0] = n2;
        q.counts[1] = L;
    }
}

// ---------------------------------------------------------------------------------------------
// one Gauss-Newton step
// ---------------------------------------------------------------------------------------------
// Jacobians and residual of one observation (3 rows; the stereo row is zero without disparity).
__device__ __forceinline__ void ba_obs_jac(const double* T, const double* X, double u, double v, double d,
                                           const PairCalib& cal, double Jc[3][6], double Jp[3][3], double r[3]) {
    const double xc = ((T[0] * X[0] + T[1] * X[1]) + T[2] * X[2]) + T[3];
    const double yc = ((T[4] * X[0] + T[5] * X[1]) + T[6] * X[2]) + T[7];
    const double zc = ((T[8] * X[0] + T[9] * X[1]) + T[10] * X[2]) + T[11];
    const double iz = 1.0 / zc;
    const double base = cal.fxb / cal.fx;
    const bool st = __builtin_isfinite(d);
    double dpi[3][3] = {{cal.fx * iz, 0.0, -cal.fx * xc * iz * iz},
                        {0.0, cal.fy * iz, -cal.fy * yc * iz * iz},
                        {st ? cal.fx * iz : 0.0, 0.0, st ? -cal.fx * (xc - base) * iz * iz : 0.0}};
    r[0] = cal.fx * xc * iz + cal.cx - u;
    r[1] = cal.fy * yc * iz + cal.cy - v;
    r[2] = st ? cal.fx * (xc - base) * iz + cal.cx - (u - d) : 0.0;
    // J_c = dpi [I | -[Xc]x];  -[Xc]x = [[0, zc, -yc], [-zc, 0, xc], [yc, -xc, 0]]
    for (int i = 0; i < 3; ++i) {
        Jc[i][0] = dpi[i][0];
        Jc[i][1] = dpi[i][1];
        Jc[i][2] = dpi[i][2];
        Jc[i][3] = -dpi[i][1] * zc + dpi[i][2] * yc;
        Jc[i][4] = dpi[i][0] * zc - dpi[i][2] * xc;
        Jc[i][5] = -dpi[i][0] * yc + dpi[i][1] * xc;
        for (int j = 0; j < 3; ++j) Jp[i][j] = (dpi[i][0] * T[j] + dpi[i][1] * T[4 + j]) + dpi[i][2] * T[8 + j];
    }
}

__global__ __launch_bounds__(256) void k_ba_lin(BatchCtx c, BaArgs a) {
    const int K = c.g.K;
    BaPair q = ba_pair(c, a, a.pair);
    const int L = q.counts[1];
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    const int kpad = (3 * L + 3) & ~3;
    if (r >= L) {
        // zero the padding columns up to a multiple of 4 (the MFMA k-step)
        const int col = 3 * L + (r - L);
        if (col < kpad)
            for (int e = 0; e < 64; ++e) q.Qt[(size_t)col * 64 + e] = 0.0;
        return;
    }
    const PairCalib cal = c.calib[a.pair];
    const int id = q.lm_id[r];
    const double X[3] = {q.X[(size_t)id * 3], q.X[(size_t)id * 3 + 1], q.X[(size_t)id * 3 + 2]};
    double V[3][3] = {{a.lam, 0.0, 0.0}, {0.0, a.lam, 0.0}, {0.0, 0.0, a.lam}}, gp[3] = {0.0, 0.0, 0.0};
    const int o0 = q.lm_off[r], o1 = q.lm_off[r + 1];
    for (int oi = o0; oi < o1; ++oi) {
        const int o = q.lm_obs[oi];
        const int ci = q.obs_cam[o], k = q.obs_k[o];
        const int s = a.order[ci];
        const size_t so = (size_t)s * K + k;
        double Jc[3][6], Jp[3][3], res[3];
        ba_obs_jac(q.T + (size_t)s * 16, X, q.u[so], q.v[so], q.d[so], cal, Jc, Jp, res);
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) V[i][j] += (Jp[0][i] * Jp[0][j] + Jp[1][i] * Jp[1][j]) + Jp[2][i] * Jp[2][j];
            gp[i] += (Jp[0][i] * res[0] + Jp[1][i] * res[1]) + Jp[2][i] * res[2];
        }
        double* W = q.obs_W + (size_t)o * 18;
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 3; ++j) W[3 * i + j] = (Jc[0][i] * Jp[0][j] + Jc[1][i] * Jp[1][j]) + Jc[2][i] * Jp[2][j];
        double* Ug = q.obs_Ug + (size_t)o * 27;   // upper-triangular J_c^T J_c (21) + J_c^T r (6)
        int e = 0;
        for (int i = 0; i < 6; ++i)
            for (int j = i; j < 6; ++j) Ug[e++] = (Jc[0][i] * Jc[0][j] + Jc[1][i] * Jc[1][j]) + Jc[2][i] * Jc[2][j];
        for (int i = 0; i < 6; ++i) Ug[21 + i] = (Jc[0][i] * res[0] + Jc[1][i] * res[1]) + Jc[2][i] * res[2];
    }
    // Cholesky V = L L^T
    double Lm[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    for (int j = 0; j < 3; ++j) {
        double sd = V[j][j];
        for (int k = 0; k < j; ++k) sd -= Lm[j][k] * Lm[j][k];
        Lm[j][j] = sqrt(sd > 1e-300 ? sd : 1e-300);
        for (int i = j + 1; i < 3; ++i) {
            double t = V[i][j];
            for (int k = 0; k < j; ++k) t -= Lm[i][k] * Lm[j][k];
            Lm[i][j] = t / Lm[j][j];
        }
    }
    double* Ls = q.lm_L + (size_t)r * 9;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) Ls[3 * i + j] = Lm[i][j];
    for (int i = 0; i < 3; ++i) q.lm_gp[(size_t)r * 3 + i] = gp[i];
    // y = L^-1 g_p ; Q_o rows = L^-1 W_o[row]^T
    double y[3];
    for (int i = 0; i < 3; ++i) {
        double t = gp[i];
        for (int k = 0; k < i; ++k) t -= Lm[i][k] * y[k];
        y[i] = t / Lm[i][i];
    }
    double* Q = q.Qt + (size_t)(3 * r) * 64;   // three k-columns of 64 rows
    for (int e = 0; e < 3 * 64; ++e) Q[e] = 0.0;
    for (int j = 0; j < 3; ++j) Q[j * 64 + 60] = y[j];
    for (int oi = o0; oi < o1; ++oi) {
        const int o = q.lm_obs[oi];
        const int ci = q.obs_cam[o];
        const double* W = q.obs_W + (size_t)o * 18;
        for (int rr = 0; rr < 6; ++rr) {
            double z[3];
            for (int i = 0; i < 3; ++i) {
                double t = W[3 * rr + i];
                for (int k = 0; k < i; ++k) t -= Lm[i][k] * z[k];
                z[i] = t / Lm[i][i];
            }
            for (int j = 0; j < 3; ++j) Q[j * 64 + 6 * ci + rr] = z[j];
        }
    }
}

__global__ __launch_bounds__(256) void k_ba_camred(BatchCtx c, BaArgs a) {
    __shared__ double s_red[256];
    BaPair q = ba_pair(c, a, a.pair);
    const int ci = blockIdx.x;
    const int o0 = q.cam_off[ci], o1 = q.cam_off[ci + 1];
    for (int e = 0; e < 27; ++e) {
        double s = 0.0;
        for (int o = o0 + (int)threadIdx.x; o < o1; o += blockDim.x) s += q.obs_Ug[(size_t)o * 27 + e];
        s_red[threadIdx.x] = s;
        __syncthreads();
        for (int w = 128; w > 0; w >>= 1) {
            if ((int)threadIdx.x < w) s_red[threadIdx.x] += s_red[threadIdx.x + w];
            __syncthreads();
        }
        if (threadIdx.x == 0) q.cam_U[(size_t)ci * 27 + e] = s_red[0];
        __syncthreads();
    }
}

typedef double d4v __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_ba_gemm(BatchCtx c, BaArgs a) {
    BaPair q = ba_pair(c, a, a.pair);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int L = q.counts[1];
    const int kt = ((3 * L + 3) & ~3) / 4;            // k-steps of 4
    const int per = (kt + gridDim.x - 1) / gridDim.x;
    const int s0 = blockIdx.x * per, s1 = min(kt, s0 + per);
    d4v acc[4];
    for (int t = 0; t < 4; ++t) acc[t] = (d4v){0.0, 0.0, 0.0, 0.0};
    const int a0 = 16 * wave, kk = lane >> 4, rc = lane & 15;
    for (int st = s0; st < s1; ++st) {
        const double* col = q.Qt + (size_t)(4 * st + kk) * 64;
        const double av = col[a0 + rc];
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, col[16 * t + rc], acc[t], 0, 0, 0);
    }
    double* out = q.part + (size_t)blockIdx.x * 64 * 64;
    // C/D layout of v_mfma_f64_16x16x4f64: col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) out[(size_t)(a0 + kk + 4 * rg) * 64 + 16 * t + rc] = acc[t][rg];
}

__global__ __launch_bounds__(1024) void k_ba_solve(BatchCtx c, BaArgs a) {
    __shared__ double s_S[TS_BA_MAXD * TS_BA_MAXD];
    __shared__ double s_b[TS_BA_MAXD], s_x[TS_BA_MAXD];
    __shared__ int s_ok;
    BaPair q = ba_pair(c, a, a.pair);
    const int n = a.n_order;
    const int m = 6 * (n - 1);   // camera 0 is the gauge
    if (q.counts[1] == 0 || n < 2) {
        if (threadIdx.x == 0) q.counts[2] = 0;
        return;
    }
    for (int i = threadIdx.x; i < m * m; i += blockDim.x) {
        const int rr = i / m, cc = i % m;
        const int R = rr + 6, Cc = cc + 6;   // full-system indices
        double sum = 0.0;
        for (int bk = 0; bk < a.nsplit; ++bk) sum += q.part[(size_t)bk * 4096 + R * 64 + Cc];
        double v = -sum;
        if (R / 6 == Cc / 6) {
            const int ci = R / 6, i0 = R % 6, j0 = Cc % 6;
            const int lo = min(i0, j0), hi = max(i0, j0);
            const int e = lo * 6 - lo * (lo - 1) / 2 + (hi - lo);   // upper-triangular index
            v += q.cam_U[(size_t)ci * 27 + e] + (i0 == j0 ? a.lam : 0.0);
        }
        s_S[rr * m + cc] = v;
    }
    for (int rr = threadIdx.x; rr < m; rr += blockDim.x) {
        const int R = rr + 6;
        double sum = 0.0;
        for (int bk = 0; bk < a.nsplit; ++bk) sum += q.part[(size_t)bk * 4096 + R * 64 + 60];
        s_b[rr] = -q.cam_U[(size_t)(R / 6) * 27 + 21 + R % 6] + sum;
    }
    if (threadIdx.x == 0) s_ok = 1;
    __syncthreads();
    // right-looking Cholesky in LDS (lower triangle)
    for (int j = 0; j < m; ++j) {
        if (threadIdx.x == 0) {
            const double dj = s_S[j * m + j];
            if (!(dj > 0.0)) s_ok = 0;
            s_S[j * m + j] = sqrt(dj > 0.0 ? dj : 1.0);
        }
        __syncthreads();
        const double ljj = s_S[j * m + j];
        for (int i = j + 1 + (int)threadIdx.x; i < m; i += blockDim.x) s_S[i * m + j] /= ljj;
        __syncthreads();
        const int nt = m - j - 1;
        for (int t = threadIdx.x; t < nt * nt; t += blockDim.x) {
            const int i = j + 1 + t / nt, k = j + 1 + t % nt;
            if (k <= i) s_S[i * m + k] -= s_S[i * m + j] * s_S[k * m + j];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        for (int i = 0; i < m; ++i) {   // L y = b
            double t = s_b[i];
            for (int k = 0; k < i; ++k) t -= s_S[i * m + k] * s_x[k];
            s_x[i] = t / s_S[i * m + i];
        }
        for (int i = m - 1; i >= 0; --i) {   // L^T x = y
            double t = s_x[i];
            for (int k = i + 1; k < m; ++k) t -= s_S[k * m + i] * s_x[k];
            s_x[i] = t / s_S[i * m + i];
        }
        q.counts[2] = s_ok;
    }
    __syncthreads();
    // dc (camera 0: zero) and camera updates: R <- cayley(w) R, t <- cayley(w) t + rho
    for (int i = threadIdx.x; i < 6 * n; i += blockDim.x) q.dc[i] = (i < 6 || !s_ok) ? 0.0 : s_x[i - 6];
    if (s_ok && (int)threadIdx.x >= 1 && (int)threadIdx.x < n) {
        const int ci = threadIdx.x;
        const double* x = s_x + 6 * (ci - 1);
        const double w0 = x[3], w1 = x[4], w2 = x[5];
        const double A[9] = {0.0, -w2, w1, w2, 0.0, -w0, -w1, w0, 0.0};
        double A2[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) A2[3 * i + j] = (A[3 * i] * A[j] + A[3 * i + 1] * A[3 + j]) + A[3 * i + 2] * A[6 + j];
        const double n2 = (w0 * w0 + w1 * w1) + w2 * w2;
        const double sc = 4.0 / (4.0 + n2);
        double RU[9];
        for (int e = 0; e < 9; ++e) RU[e] = ((e % 4) == 0 ? 1.0 : 0.0) + sc * (A[e] + 0.5 * A2[e]);
        double* T = q.T + (size_t)a.order[ci] * 16;
        double Rn[9], tn[3];
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) Rn[3 * i + j] = (RU[3 * i] * T[j] + RU[3 * i + 1] * T[4 + j]) + RU[3 * i + 2] * T[8 + j];
            tn[i] = ((RU[3 * i] * T[3] + RU[3 * i + 1] * T[7]) + RU[3 * i + 2] * T[11]) + x[i];
        }
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) T[4 * i + j] = Rn[3 * i + j];
            T[4 * i + 3] = tn[i];
        }
    }
}

__global__ __launch_bounds__(256) void k_ba_backsub(BatchCtx c, BaArgs a) {
    BaPair q = ba_pair(c, a, a.pair);
    const int L = q.counts[1];
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= L || !q.counts[2]) return;
    double rhs[3];
    for (int i = 0; i < 3; ++i) rhs[i] = -q.lm_gp[(size_t)r * 3 + i];
    for (int oi = q.lm_off[r]; oi < q.lm_off[r + 1]; ++oi) {
        const int o = q.lm_obs[oi];
        const double* W = q.obs_W + (size_t)o * 18;
        const double* dc = q.dc + 6 * q.obs_cam[o];
        for (int j = 0; j < 3; ++j) {
            double t = 0.0;
            for (int i = 0; i < 6; ++i) t += W[3 * i + j] * dc[i];
            rhs[j] -= t;
        }
    }
    const double* Lm = q.lm_L + (size_t)r * 9;
    double y[3], x[3];
    for (int i = 0; i < 3; ++i) {
        double t = rhs[i];
        for (int k = 0; k < i; ++k) t -= Lm[3 * i + k] * y[k];
        y[i] = t / Lm[3 * i + i];
    }
    for (int i = 2; i >= 0; --i) {
        double t = y[i];
        for (int k = i + 1; k < 3; ++k) t -= Lm[3 * k + i] * x[k];
        x[i] = t / Lm[3 * i + i];
    }
    const int id = q.lm_id[r];
    for (int i = 0; i < 3; ++i) q.X[(size_t)id * 3 + i] += x[i];
}

// ---------------------------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------------------------
void launch_ba_keyframe(const BatchCtx& c, const BaArgs& a, bool evict, hipStream_t s) {
    if (evict) hipLaunchKernelGGL(k_ba_evict, dim3(1), dim3(1024), 0, s, c, a);
    hipLaunchKernelGGL(k_ba_insert, dim3(1), dim3(1024), 0, s, c, a);
}

void launch_ba_solve(const BatchCtx& c, const BaArgs& a, hipStream_t s) {
    const int maxL = a.W * c.g.K;
    hipLaunchKernelGGL(k_ba_gather, dim3(1), dim3(1024), 0, s, c, a);
    for (int it = 0; it < a.iters; ++it) {
        hipLaunchKernelGGL(k_ba_lin, dim3((maxL + 4 + 255) / 256), dim3(256), 0, s, c, a);
        hipLaunchKernelGGL(k_ba_camred, dim3(a.n_order), dim3(256), 0, s, c, a);
        hipLaunchKernelGGL(k_ba_gemm, dim3(a.nsplit), dim3(256), 0, s, c, a);
        hipLaunchKernelGGL(k_ba_solve, dim3(1), dim3(1024), 0, s, c, a);
        hipLaunchKernelGGL(k_ba_backsub, dim3((maxL + 255) / 256), dim3(256), 0, s, c, a);
    }
}
