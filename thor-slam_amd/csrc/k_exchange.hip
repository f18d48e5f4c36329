// k_exchange.hip — the per-batch block of SURVEY.md §8e that the ranks all-gather over RCCL:
// per (frame, camera) K*8 B keypoints | K*32 B descriptors | L*4 B level counts, then per
// (frame, pair) T_rel (16 f64) | covariance (36 f64) | stats (8 i32).  One kernel gathers it from
// the ring buffers with 16-byte copies (a memcpy per piece would be ~2,300 API calls per batch).
#include "tslam_common.h"

__global__ __launch_bounds__(256) void k_pack(BatchCtx c, uint8_t* dst) {
    const int64_t K = c.g.K, L = c.g.n_levels;
    const int64_t per_cam = K * 40 + L * 4;
    const int item = blockIdx.x;   // f * C + cam, then trailer blocks
    if (item < c.n * c.C) {
        const int f = item / c.C, cam = item % c.C;
        const int slot = ring_slot(c, c.g0 + f);
        const size_t sc = (size_t)slot * c.C + cam;
        uint8_t* o = dst + (int64_t)item * per_cam;
        const uint4* kp = reinterpret_cast<const uint4*>(c.kps + sc * K * 2);
        const uint4* de = reinterpret_cast<const uint4*>(c.desc + sc * K * 8);
        // keypoints: K*8 B = K/2 uint4 (K even) ; descriptors: K*32 B = 2K uint4
        if ((K & 1) == 0 && (per_cam & 15) == 0) {
            uint4* ok = reinterpret_cast<uint4*>(o);
            for (int64_t i = threadIdx.x; i < K / 2; i += blockDim.x) ok[i] = kp[i];
            uint4* od = reinterpret_cast<uint4*>(o + K * 8);
            for (int64_t i = threadIdx.x; i < 2 * K; i += blockDim.x) od[i] = de[i];
        } else {
            const uint32_t* k32 = c.kps + sc * K * 2;
            const uint32_t* d32 = c.desc + sc * K * 8;
            for (int64_t i = threadIdx.x; i < 2 * K; i += blockDim.x) reinterpret_cast<uint32_t*>(o)[i] = k32[i];
            for (int64_t i = threadIdx.x; i < 8 * K; i += blockDim.x) reinterpret_cast<uint32_t*>(o + K * 8)[i] = d32[i];
        }
        for (int64_t i = threadIdx.x; i < L; i += blockDim.x)
            reinterpret_cast<int32_t*>(o + K * 40)[i] = c.kcount[sc * L + i];
        return;
    }
    // pose trailer: one block covers up to 256 (frame, pair) records, 52 doubles + 8 ints each
    const int64_t feat = (int64_t)c.n * c.C * per_cam;
    const int nrec = c.n * c.P;
    const int r0 = (item - c.n * c.C) * 4;
    for (int r = r0; r < min(r0 + 4, nrec); ++r) {
        uint8_t* o = dst + feat + (int64_t)r * (52 * 8 + TS_STATS_INTS * 4);
        const double* pz = c.pose + (size_t)r * TS_POSE_DOUBLES;
        for (int i = threadIdx.x; i < 52; i += blockDim.x)
            reinterpret_cast<double*>(o)[i] = i < 16 ? pz[i] : pz[32 + (i - 16)];
        for (int i = threadIdx.x; i < TS_STATS_INTS; i += blockDim.x)
            reinterpret_cast<int32_t*>(o + 52 * 8)[i] = c.stats[(size_t)r * TS_STATS_INTS + i];
    }
}

void launch_pack(const BatchCtx& c, uint8_t* dst, hipStream_t s) {
    const int trailer_blocks = (c.n * c.P + 3) / 4;
    hipLaunchKernelGGL(k_pack, dim3(c.n * c.C + trailer_blocks), dim3(256), 0, s, c, dst);
}

// ---- rig fusion across ranks (the rig-level solve after the all-gather) ---------
// Every rank holds one (or P) stereo pair(s); after the gather it has every pair's relative pose
// and covariance of the batch.  Per frame, each tracked pair's motion is moved to the body frame,
// M_q = (E_q T_q) E_q^-1 (the k_rig_pose convention), its covariance rotated with E_q's rotation
// (blockdiag(R, R) C blockdiag(R, R)^T) and inverted into an information matrix; the motions are
// combined in the tangent space of the first tracked pair: xi = (sum L_q)^-1 sum L_q xi_q with
// xi_q = (translation, rotation vector) of M_ref^-1 M_q, M = M_ref [exp(xi_w) | xi_rho].
// One thread per frame (the work is a few hundred flops per pair).
__device__ bool chol6_inv_solve(const double* A, double* L) {
    for (int j = 0; j < 6; ++j) {
        double s = A[j * 6 + j];
        for (int k = 0; k < j; ++k) s -= L[j * 6 + k] * L[j * 6 + k];
        if (!(s > 0.0)) return false;
        L[j * 6 + j] = sqrt(s);
        for (int i = j + 1; i < 6; ++i) {
            double t = A[i * 6 + j];
            for (int k = 0; k < j; ++k) t -= L[i * 6 + k] * L[j * 6 + k];
            L[i * 6 + j] = t / L[j * 6 + j];
        }
    }
    return true;
}
__device__ void chol6_apply(const double* L, const double* b, double* x) {   // (L L^T) x = b
    double y[6];
    for (int i = 0; i < 6; ++i) {
        double s = b[i];
        for (int k = 0; k < i; ++k) s -= L[i * 6 + k] * y[k];
        y[i] = s / L[i * 6 + i];
    }
    for (int i = 5; i >= 0; --i) {
        double s = y[i];
        for (int k = i + 1; k < 6; ++k) s -= L[k * 6 + i] * x[k];
        x[i] = s / L[i * 6 + i];
    }
}
__device__ void mul4_x(const double* A, const double* B, double* out) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            out[4 * i + j] = ((A[4 * i] * B[j] + A[4 * i + 1] * B[4 + j]) + A[4 * i + 2] * B[8 + j]) + A[4 * i + 3] * B[12 + j];
}
__device__ void inv4_rigid(const double* T, double* out) {
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) out[4 * i + j] = T[4 * j + i];
        out[4 * i + 3] = -((T[i] * T[3] + T[4 + i] * T[7]) + T[8 + i] * T[11]);
    }
    out[12] = out[13] = out[14] = 0.0;
    out[15] = 1.0;
}
__device__ void so3_log(const double* T, double* w) {   // rotation part of a 4x4
    const double v0 = 0.5 * (T[9] - T[6]), v1 = 0.5 * (T[2] - T[8]), v2 = 0.5 * (T[4] - T[1]);
    const double s = sqrt((v0 * v0 + v1 * v1) + v2 * v2);
    const double cth = 0.5 * (((T[0] + T[5]) + T[10]) - 1.0);
    const double th = atan2(s, cth);
    const double k = s > 1e-12 ? th / s : 1.0;
    w[0] = v0 * k; w[1] = v1 * k; w[2] = v2 * k;
}
__device__ void so3_exp(const double* w, double* R) {
    const double th = sqrt((w[0] * w[0] + w[1] * w[1]) + w[2] * w[2]);
    double a, b;
    if (th > 1e-9) {
        a = sin(th) / th;
        b = (1.0 - cos(th)) / (th * th);
    } else {
        a = 1.0 - th * th / 6.0;
        b = 0.5 - th * th / 24.0;
    }
    const double K[9] = {0.0, -w[2], w[1], w[2], 0.0, -w[0], -w[1], w[0], 0.0};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            const double k2 = (K[3 * i] * K[j] + K[3 * i + 1] * K[3 + j]) + K[3 * i + 2] * K[6 + j];
            R[3 * i + j] = (i == j ? 1.0 : 0.0) + a * K[3 * i + j] + b * k2;
        }
}

__global__ __launch_bounds__(64) void k_rig_fuse(BatchCtx c, const uint8_t* gathered, int64_t rank_bytes, int world) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= c.n) return;
    const int64_t K = c.g.K, L = c.g.n_levels;
    const int64_t feat = (int64_t)c.n * c.C * (K * 40 + L * 4);
    const int64_t rec = 52 * 8 + TS_STATS_INTS * 4;
    const int Q = world * c.P;   // pairs of the whole rig, rank-major
    double* pout = c.rig_pose + (size_t)f * TS_POSE_DOUBLES;
    int32_t* sout = c.rig_stats + (size_t)f * TS_STATS_INTS;
    for (int i = 0; i < TS_POSE_DOUBLES; ++i) pout[i] = (i < 16 && (i % 5) == 0) ? 1.0 : 0.0;
    double Mref[16], Minv[16];
    double sumL[36], sumLx[6];
    for (int i = 0; i < 36; ++i) sumL[i] = 0.0;
    for (int i = 0; i < 6; ++i) sumLx[i] = 0.0;
    int used = 0, init = 0;
    for (int q = 0; q < Q; ++q) {
        const int r = q / c.P, p = q % c.P;
        const uint8_t* o = gathered + r * rank_bytes + feat + (int64_t)(f * c.P + p) * rec;
        const double* T = reinterpret_cast<const double*>(o);
        const double* cov = T + 16;
        const int st = reinterpret_cast<const int32_t*>(o + 52 * 8)[0];
        if (st == 2) init = 1;
        if (st != 0) continue;
        const double* E = c.rig_E + 16 * q;
        const double* Ei = c.rig_Einv + 16 * q;
        double ET[16], M[16];
        mul4_x(E, T, ET);
        mul4_x(ET, Ei, M);
        // body-frame covariance with the rotation of E (blockdiag(R, R))
        double R6[36], tmp[36], cb[36], Lc[36], Lam[36];
        for (int i = 0; i < 36; ++i) R6[i] = 0.0;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) R6[i * 6 + j] = R6[(i + 3) * 6 + j + 3] = E[4 * i + j];
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j) {
                double s = 0.0;
                for (int k = 0; k < 6; ++k) s += R6[i * 6 + k] * cov[k * 6 + j];
                tmp[i * 6 + j] = s;
            }
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j) {
                double s = 0.0;
                for (int k = 0; k < 6; ++k) s += tmp[i * 6 + k] * R6[j * 6 + k];
                cb[i * 6 + j] = s;
            }
        for (int i = 0; i < 36; ++i) Lc[i] = 0.0;
        if (!chol6_inv_solve(cb, Lc)) continue;
        for (int k = 0; k < 6; ++k) {   // information = cov^-1, column by column
            double e[6], x[6];
            for (int i = 0; i < 6; ++i) e[i] = i == k ? 1.0 : 0.0;
            chol6_apply(Lc, e, x);
            for (int i = 0; i < 6; ++i) Lam[i * 6 + k] = x[i];
        }
        if (used == 0) {
            for (int i = 0; i < 16; ++i) Mref[i] = M[i];
            inv4_rigid(Mref, Minv);
        }
        double D[16], xi[6];
        mul4_x(Minv, M, D);
        xi[0] = D[3]; xi[1] = D[7]; xi[2] = D[11];
        so3_log(D, xi + 3);
        for (int i = 0; i < 6; ++i) {
            double s = 0.0;
            for (int k = 0; k < 6; ++k) {
                sumL[i * 6 + k] += Lam[i * 6 + k];
                s += Lam[i * 6 + k] * xi[k];
            }
            sumLx[i] += s;
        }
        ++used;
    }
    if (used == 0) {
        sout[0] = init ? 2 : 1;
        for (int i = 1; i < TS_STATS_INTS; ++i) sout[i] = 0;
        sout[5] = (int)(c.g0 + f);
        return;
    }
    double Ls[36], xi[6];
    for (int i = 0; i < 36; ++i) Ls[i] = 0.0;
    const bool ok = chol6_inv_solve(sumL, Ls);
    if (ok) chol6_apply(Ls, sumLx, xi);
    else for (int i = 0; i < 6; ++i) xi[i] = 0.0;
    double Rx[9], X[16], M[16];
    so3_exp(xi + 3, Rx);
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) X[4 * i + j] = Rx[3 * i + j];
        X[4 * i + 3] = xi[i];
    }
    X[12] = X[13] = X[14] = 0.0;
    X[15] = 1.0;
    mul4_x(Mref, X, M);
    for (int i = 0; i < 12; ++i) pout[i] = M[i];
    if (ok)
        for (int k = 0; k < 6; ++k) {
            double e[6], x[6];
            for (int i = 0; i < 6; ++i) e[i] = i == k ? 1.0 : 0.0;
            chol6_apply(Ls, e, x);
            for (int i = 0; i < 6; ++i) pout[32 + i * 6 + k] = x[i];
        }
    sout[0] = 0;
    sout[1] = used;
    for (int i = 2; i < TS_STATS_INTS; ++i) sout[i] = 0;
    sout[5] = (int)(c.g0 + f);
}

void launch_rig_fuse(const BatchCtx& c, const uint8_t* gathered, int64_t rank_bytes, int world, hipStream_t s) {
    hipLaunchKernelGGL(k_rig_fuse, dim3((c.n + 63) / 64), dim3(64), 0, s, c, gathered, rank_bytes, world);
    launch_rig_chain(c, s);
}
