// k_posegraph.hip — keyframe pose-graph optimisation ("plus a keyframe pose
// graph"; loop edges from k_loop.hip, item 3).  CPU restatement: oracle/numpy_loop.py (optimize).
//
// Nodes T_i = world_T_cam_i (4x4 f64 row-major), edges (a, b, Z_ab = measured T_a^-1 T_b, Omega
// 6x6).  se(3) vectors are (rho, phi); residual e = Log(Z^-1 T_a^-1 T_b); right perturbations give
// J_b = Jr^-1(e), J_a = -Jr^-1(e) Ad(T_b^-1 T_a), Jr^-1(e) ~ I + ad(e)/2.  One Gauss-Newton
// iteration on the device:
//
//   k_pg_edges     thread per edge: e, J_a, J_b -> H_aa, H_ab, H_bb, g_a, g_b, e^T Omega e;
//   k_pg_assemble  thread per element of the dense normal matrix (free nodes 1..N-1, padded to a
//                  multiple of 32 with identity): fixed-order sums over the node's incident edges
//                  (CSR built on the host, sorted by edge) — deterministic, no atomics;
//   k_pg_potrf     right-looking blocked Cholesky, panel k: every block factors the 32x32 diagonal
//                  tile in registers from its lower triangle, blocks 1.. solve their tile row of the
//                  panel, and block 0 stores L_kk where no block of the launch reads: the strict
//                  lower part transposed into the tile's upper triangle, the diagonal into Ld (the
//                  blocks of one launch need not be resident together, so L_kk written in place
//                  would race with a late block's read of A_kk); tiles outside the matrix profile
//                  (zero, no fill-in) are skipped;
//   k_pg_syrk      trailing update A_IJ -= L_Ik L_Jk^T, one 32x32 tile per block, four waves of
//                  v_mfma_f64_16x16x4f64 (the dense J^T J work on the FP64 matrix cores);
//   k_pg_trsv      one block: blocked forward / backward substitution (wave 0 solves the 32x32
//                  diagonal systems with lane broadcasts, the block updates the rest);
//   k_pg_update    thread per free node: T_i <- T_i Exp(delta_i).
#include "tslam_common.h"
#include <atomic>

#define PG_TILE 32
#define PG_TERMS 128   // doubles per edge: H_aa 36, H_ab 36, H_bb 36, g_a 6, g_b 6, cost 1
#define PG_TRSV_THREADS 1024
#define PG_MAX_N 6144  // padded unknowns held in LDS by k_pg_trsv (1024 nodes)

typedef double pg_d4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------------------------
// SE(3) helpers (same formulas as oracle/numpy_loop.py)
// ---------------------------------------------------------------------------------------------
// A = sin t / t, B = 2 sin^2(t/2) / t^2, C = (t - sin t) / t^3; four Taylor terms below t^2 = 1e-3
__device__ void pg_abc(double th2, double* A, double* B, double* C) {
    if (th2 < 1e-3) {
        const double t4 = th2 * th2, t6 = th2 * th2 * th2;
        *A = 1.0 - th2 / 6.0 + t4 / 120.0 - t6 / 5040.0;
        *B = 0.5 - th2 / 24.0 + t4 / 720.0 - t6 / 40320.0;
        *C = 1.0 / 6.0 - th2 / 120.0 + t4 / 5040.0 - t6 / 362880.0;
        return;
    }
    const double th = sqrt(th2), s = sin(th), h = sin(0.5 * th);
    *A = s / th;
    *B = 2.0 * h * h / th2;
    *C = (th - s) / (th2 * th);
}

__device__ void pg_hat(const double* w, double* W) {
    W[0] = 0.0;   W[1] = -w[2]; W[2] = w[1];
    W[3] = w[2];  W[4] = 0.0;   W[5] = -w[0];
    W[6] = -w[1]; W[7] = w[0];  W[8] = 0.0;
}

__device__ void pg_mul3(const double* a, const double* b, double* o) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) o[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
}

__device__ void pg_mul4(const double* a, const double* b, double* o) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            o[4 * i + j] = a[4 * i] * b[j] + a[4 * i + 1] * b[4 + j] + a[4 * i + 2] * b[8 + j] + a[4 * i + 3] * b[12 + j];
}

__device__ void pg_inv(const double* T, double* o) {
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) o[4 * i + j] = T[4 * j + i];
        o[4 * i + 3] = -(T[i] * T[3] + T[4 + i] * T[7] + T[8 + i] * T[11]);
    }
    o[12] = o[13] = o[14] = 0.0;
    o[15] = 1.0;
}

__device__ void pg_exp(const double* xi, double* T) {
    const double* rho = xi;
    const double* phi = xi + 3;
    const double th2 = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
    double A, B, C, W[9], W2[9];
    pg_abc(th2, &A, &B, &C);
    pg_hat(phi, W);
    pg_mul3(W, W, W2);
    for (int i = 0; i < 3; ++i) {
        double t = 0.0;
        for (int j = 0; j < 3; ++j) {
            const double id = i == j ? 1.0 : 0.0;
            T[4 * i + j] = id + A * W[3 * i + j] + B * W2[3 * i + j];
            t += (id + B * W[3 * i + j] + C * W2[3 * i + j]) * rho[j];
        }
        T[4 * i + 3] = t;
    }
    T[12] = T[13] = T[14] = 0.0;
    T[15] = 1.0;
}

__device__ void pg_log(const double* T, double* xi) {
    // theta = atan2(|v| / 2, (tr R - 1) / 2), v = vee(R - R^T): accurate at small angles too
    const double v[3] = {T[9] - T[6], T[2] - T[8], T[4] - T[1]};
    const double s = 0.5 * sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    const double c = (T[0] + T[5] + T[10] - 1.0) * 0.5;
    const double th = atan2(s, c);
    const double f = th < 1e-5 ? 0.5 * (1.0 + th * th / 6.0) : th / (2.0 * s);
    double phi[3] = {v[0] * f, v[1] * f, v[2] * f};
    const double th2 = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
    double k;
    if (th2 < 1e-3) {   // k = (1 - A / 2B) / t^2
        k = 1.0 / 12.0 + th2 / 720.0 + th2 * th2 / 30240.0 + th2 * th2 * th2 / 1209600.0;
    } else {
        double A, B, C;
        pg_abc(th2, &A, &B, &C);
        k = (1.0 - A / (2.0 * B)) / th2;
    }
    double W[9], W2[9];
    pg_hat(phi, W);
    pg_mul3(W, W, W2);
    for (int i = 0; i < 3; ++i) {
        double r = 0.0;
        for (int j = 0; j < 3; ++j) r += ((i == j ? 1.0 : 0.0) - 0.5 * W[3 * i + j] + k * W2[3 * i + j]) * T[4 * j + 3];
        xi[i] = r;
        xi[3 + i] = phi[i];
    }
}

// ---------------------------------------------------------------------------------------------
// k_pg_edges: per-edge normal-equation blocks
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_pg_edges(const double* T, const int32_t* edges, const double* Z,
                                                 const double* info, int E, double* terms) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= E) return;
    const int a = edges[2 * k], b = edges[2 * k + 1];
    double Ta_inv[16], Tab[16], Zinv[16], M[16], e[6];
    pg_inv(T + 16 * (size_t)a, Ta_inv);
    pg_mul4(Ta_inv, T + 16 * (size_t)b, Tab);
    pg_inv(Z + 16 * (size_t)k, Zinv);
    pg_mul4(Zinv, Tab, M);
    pg_log(M, e);
    // Jr^-1(e) = I + ad(e)/2, ad(rho, phi) = [[phi^, rho^], [0, phi^]]
    double Jr[36], P[9], R[9];
    pg_hat(e + 3, P);
    pg_hat(e, R);
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
            double ad = 0.0;
            if (i < 3 && j < 3) ad = P[3 * i + j];
            else if (i < 3) ad = R[3 * i + j - 3];
            else if (j >= 3) ad = P[3 * (i - 3) + j - 3];
            Jr[6 * i + j] = (i == j ? 1.0 : 0.0) + 0.5 * ad;
        }
    // Ad(T_b^-1 T_a) = [[R, t^ R], [0, R]]
    double Tba[16], Ad[36], th[9], tR[9];
    pg_inv(Tab, Tba);
    const double rr[9] = {Tba[0], Tba[1], Tba[2], Tba[4], Tba[5], Tba[6], Tba[8], Tba[9], Tba[10]};
    const double tt[3] = {Tba[3], Tba[7], Tba[11]};
    pg_hat(tt, th);
    pg_mul3(th, rr, tR);
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
            double v = 0.0;
            if (i < 3 && j < 3) v = rr[3 * i + j];
            else if (i < 3) v = tR[3 * i + j - 3];
            else if (j >= 3) v = rr[3 * (i - 3) + j - 3];
            Ad[6 * i + j] = v;
        }
    double Ja[36];
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
            double s = 0.0;
            for (int m = 0; m < 6; ++m) s += Jr[6 * i + m] * Ad[6 * m + j];
            Ja[6 * i + j] = -s;
        }
    const double* W = info + 36 * (size_t)k;
    double WJa[36], WJb[36], We[6];
    for (int i = 0; i < 6; ++i) {
        double s = 0.0;
        for (int m = 0; m < 6; ++m) s += W[6 * i + m] * e[m];
        We[i] = s;
        for (int j = 0; j < 6; ++j) {
            double sa = 0.0, sb = 0.0;
            for (int m = 0; m < 6; ++m) {
                sa += W[6 * i + m] * Ja[6 * m + j];
                sb += W[6 * i + m] * Jr[6 * m + j];
            }
            WJa[6 * i + j] = sa;
            WJb[6 * i + j] = sb;
        }
    }
    double* o = terms + (size_t)k * PG_TERMS;
    for (int i = 0; i < 6; ++i) {
        for (int j = 0; j < 6; ++j) {
            double haa = 0.0, hab = 0.0, hbb = 0.0;
            for (int m = 0; m < 6; ++m) {
                haa += Ja[6 * m + i] * WJa[6 * m + j];
                hab += Ja[6 * m + i] * WJb[6 * m + j];
                hbb += Jr[6 * m + i] * WJb[6 * m + j];
            }
            o[6 * i + j] = haa;
            o[36 + 6 * i + j] = hab;
            o[72 + 6 * i + j] = hbb;
        }
        double ga = 0.0, gb = 0.0;
        for (int m = 0; m < 6; ++m) {
            ga += Ja[6 * m + i] * We[m];
            gb += Jr[6 * m + i] * We[m];
        }
        o[108 + i] = ga;
        o[114 + i] = gb;
    }
    double cost = 0.0;
    for (int m = 0; m < 6; ++m) cost += e[m] * We[m];
    o[120] = cost;
}

// ---------------------------------------------------------------------------------------------
// k_pg_assemble: H (np x np, row-major) and g (np); node p >= 1 owns rows 6(p-1) .. 6(p-1)+5
// adj_off[N+1], adj[...] = (edge << 1) | role, role 0: the node is the edge's a, 1: its b
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pg_assemble(const double* terms, const int32_t* edges, const int32_t* adj_off,
                                                     const int32_t* adj, int n, int np, double* H, double* g) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    const int r = blockIdx.y;
    if (c >= np) return;
    double v = 0.0;
    if (r >= n || c >= n) {
        v = r == c ? 1.0 : 0.0;
    } else {
        const int p = r / 6 + 1, q = c / 6 + 1, lr = r % 6, lc = c % 6;
        for (int i = adj_off[p]; i < adj_off[p + 1]; ++i) {
            const int k = adj[i] >> 1, role = adj[i] & 1;
            const double* o = terms + (size_t)k * PG_TERMS;
            if (p == q) {
                v += o[(role ? 72 : 0) + 6 * lr + lc];
            } else {
                const int other = edges[2 * k + (role ? 0 : 1)];
                if (other == q) v += role ? o[36 + 6 * lc + lr] : o[36 + 6 * lr + lc];
            }
        }
    }
    H[(size_t)r * np + c] = v;
    if (c == 0) {
        double gv = 0.0;
        if (r < n) {
            const int p = r / 6 + 1, lr = r % 6;
            for (int i = adj_off[p]; i < adj_off[p + 1]; ++i) {
                const int k = adj[i] >> 1, role = adj[i] & 1;
                gv += terms[(size_t)k * PG_TERMS + (role ? 114 : 108) + lr];
            }
        }
        g[r] = gv;
    }
}

// ---------------------------------------------------------------------------------------------
// blocked Cholesky over the profile: ftile[I] = first tile column holding a nonzero of tile row
// I (host-computed from the graph; Cholesky fill-in stays inside the profile), so tiles (I, J)
// with J < ftile[I] are zero throughout and are skipped everywhere.
// ---------------------------------------------------------------------------------------------

// lane `l` (compile-time) of a wave-wide double, through v_readlane (no LDS round trip)
__device__ __forceinline__ double pg_lane(double v, int l) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, l), hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// The 32x32 diagonal tile at (d0, d0) factored in registers: lane t (mod 32) holds row t; column j
// of step j is broadcast by v_readlane.  Returns row t of L (lower part valid).
__device__ __forceinline__ void pg_factor_tile(const double* H, int np, size_t d0, int t, double* r) {
#pragma unroll
    for (int c = 0; c < PG_TILE; ++c) r[c] = H[(d0 + t) * np + d0 + c];
#pragma unroll
    for (int j = 0; j < PG_TILE; ++j) {
        const double ljj = sqrt(pg_lane(r[j], j));   // a non-positive pivot gives NaN (host check)
        r[j] = t == j ? ljj : (t > j ? r[j] / ljj : r[j]);
#pragma unroll
        for (int c = j + 1; c < PG_TILE; ++c) {
            const double lcj = pg_lane(r[j], c);
            if (t >= c) r[c] -= r[j] * lcj;
        }
    }
}

// panel k: block 0 stores L_kk (strict lower part as the tile's upper triangle, L^T, the diagonal
// in Ld); block b >= 1 solves tile row I = k + b (X L_kk^T = A_Ik), unless that tile row is
// outside the profile of column k.
// `delay` (0 on every product path; tslam_test_potrf_delay) holds blocks >= 1 back by delay x
// 127 x 64 cycles before they read A_kk, so block 0's stores have landed by then: the read order
// that made the pre-round-5 in-place store of L_kk fail, forced (tests/test_gpu_loop.py).
__global__ __launch_bounds__(64) void k_pg_potrf(double* H, int np, int k, const int32_t* ftile, double* Ld, int delay) {
    __shared__ double s_L[PG_TILE][PG_TILE + 1];
    const int I = k + blockIdx.x;
    if (blockIdx.x > 0 && ftile[I] > k) return;
    if (blockIdx.x > 0)
        for (int i = 0; i < delay; ++i) __builtin_amdgcn_s_sleep(127);
    const int t = threadIdx.x & (PG_TILE - 1);
    const size_t d0 = (size_t)k * PG_TILE;
    double r[PG_TILE];
    pg_factor_tile(H, np, d0, t, r);
    if (blockIdx.x == 0) {
        if (threadIdx.x < PG_TILE) {
            double dg = 0.0;
#pragma unroll
            for (int c = 0; c < PG_TILE; ++c) {
                if (c < t) H[(d0 + c) * np + d0 + t] = r[c];   // L[t][c] at (c, t): coalesced over t
                if (c == t) dg = r[c];   // (a run-time index into r would put it in scratch)
            }
            Ld[d0 + t] = dg;
        }
        return;
    }
    if (threadIdx.x < PG_TILE)
#pragma unroll
        for (int c = 0; c < PG_TILE; ++c) s_L[t][c] = r[c];
    __syncthreads();
    if (threadIdx.x >= PG_TILE) return;
    // row t of the tile in registers; L_kk read as LDS broadcasts (no dependent LDS round trips)
    const size_t r0 = (size_t)I * PG_TILE + t;
    double a[PG_TILE];
#pragma unroll
    for (int c = 0; c < PG_TILE; ++c) a[c] = H[r0 * np + d0 + c];
#pragma unroll
    for (int c = 0; c < PG_TILE; ++c) {
        double x = a[c];
#pragma unroll
        for (int m = 0; m < c; ++m) x -= a[m] * s_L[c][m];
        a[c] = x / s_L[c][c];
    }
#pragma unroll
    for (int c = 0; c < PG_TILE; ++c) H[r0 * np + d0 + c] = a[c];
}

// trailing tiles (I, J), k < J <= I < nt, dealt as a lower triangle: block b -> (ti, tj)
__global__ __launch_bounds__(256) void k_pg_syrk(double* H, int np, int k, const int32_t* ftile) {
    int ti = (int)((sqrt(8.0 * blockIdx.x + 1.0) - 1.0) * 0.5);
    while ((ti + 1) * (ti + 2) / 2 <= (int)blockIdx.x) ++ti;
    while (ti * (ti + 1) / 2 > (int)blockIdx.x) --ti;
    const int tj = blockIdx.x - ti * (ti + 1) / 2;
    const int I = k + 1 + ti, J = k + 1 + tj;
    if (ftile[I] > k || ftile[J] > k) return;   // L_Ik or L_Jk is zero
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int qi = wave >> 1, qj = wave & 1;
    const int rc = lane & 15, kk = lane >> 4;
    const double* La = H + ((size_t)I * PG_TILE + 16 * qi + rc) * np + (size_t)k * PG_TILE;
    const double* Lb = H + ((size_t)J * PG_TILE + 16 * qj + rc) * np + (size_t)k * PG_TILE;
    pg_d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < PG_TILE / 4; ++s)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(La[4 * s + kk], Lb[4 * s + kk], acc, 0, 0, 0);
    // C/D layout: col = lane & 15, row = (lane >> 4) + 4 * reg
    double* C = H + ((size_t)I * PG_TILE + 16 * qi) * np + (size_t)J * PG_TILE + 16 * qj + rc;
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) C[(size_t)(kk + 4 * rg) * np] -= acc[rg];
}

// ---------------------------------------------------------------------------------------------
// k_pg_trsv: delta = -(L L^T)^-1 g in one block (np <= PG_MAX_N).  Wave 0 solves each diagonal
// tile from registers (lane shuffles); the off-diagonal updates skip tiles outside the profile:
// forward rows two per wave-instruction (32 lanes read a contiguous 256-B row segment, then a
// 32-lane sum), backward one column element per thread (consecutive threads, consecutive bytes).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(PG_TRSV_THREADS) void k_pg_trsv(const double* H, int np, const double* g, double* delta,
                                                             const int32_t* ftile, const double* Ld) {
    __shared__ double s_r[PG_MAX_N];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int nt = np / PG_TILE;
    const int tl = lane & (PG_TILE - 1), half = lane >> 5;
    for (int i = t; i < np; i += PG_TRSV_THREADS) s_r[i] = -g[i];
    __syncthreads();
    for (int k = 0; k < nt; ++k) {   // forward: L y = -g
        const int d0 = k * PG_TILE;
        if (wave == 0) {
            double l[PG_TILE];   // row tl of L_kk: L[tl][c] is stored at (c, tl), the diagonal in Ld
#pragma unroll
            for (int c = 0; c < PG_TILE; ++c) l[c] = c == tl ? Ld[d0 + tl] : H[(size_t)(d0 + c) * np + d0 + tl];
            double y = s_r[d0 + tl];
#pragma unroll
            for (int c = 0; c < PG_TILE; ++c) {
                if (tl == c) y /= l[c];
                const double yc = pg_lane(y, c);
                if (tl > c) y -= l[c] * yc;
            }
            if (lane < PG_TILE) s_r[d0 + tl] = y;
        }
        __syncthreads();
        const double yk = s_r[d0 + tl];
        for (int I = k + 1; I < nt; ++I) {
            if (ftile[I] > k) continue;   // uniform
            for (int rr = 2 * wave + half; rr < PG_TILE; rr += 2 * (PG_TRSV_THREADS / 64)) {
                const int m = I * PG_TILE + rr;
                double v = H[(size_t)m * np + d0 + tl] * yk;
#pragma unroll
                for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 32);
                if (tl == 0) s_r[m] -= v;
            }
        }
        __syncthreads();
    }
    for (int k = nt - 1; k >= 0; --k) {   // backward: L^T x = y
        const int d0 = k * PG_TILE;
        if (wave == 0) {
            double lc[PG_TILE];   // column tl of L_kk: lc[c] = L[c][tl], stored at (tl, c)
#pragma unroll
            for (int c = 0; c < PG_TILE; ++c) lc[c] = c == tl ? Ld[d0 + tl] : H[(size_t)(d0 + tl) * np + d0 + c];
            double x = s_r[d0 + tl];
#pragma unroll
            for (int c = PG_TILE - 1; c >= 0; --c) {
                if (tl == c) x /= lc[c];
                const double xc = pg_lane(x, c);
                if (tl < c) x -= lc[c] * xc;
            }
            if (lane < PG_TILE) s_r[d0 + tl] = x;
        }
        __syncthreads();
        for (int m = ftile[k] * PG_TILE + t; m < d0; m += PG_TRSV_THREADS) {
            double acc = s_r[m];
            for (int c = 0; c < PG_TILE; ++c) acc -= H[(size_t)(d0 + c) * np + m] * s_r[d0 + c];
            s_r[m] = acc;
        }
        __syncthreads();
    }
    for (int i = t; i < np; i += PG_TRSV_THREADS) delta[i] = s_r[i];
}

__global__ __launch_bounds__(64) void k_pg_update(double* T, const double* delta, int N) {
    const int a = blockIdx.x * blockDim.x + threadIdx.x + 1;
    if (a >= N) return;
    double X[16], O[16];
    pg_exp(delta + 6 * (size_t)(a - 1), X);
    double* Ta = T + 16 * (size_t)a;
    pg_mul4(Ta, X, O);
    for (int i = 0; i < 16; ++i) Ta[i] = O[i];
}

static std::atomic<int> g_potrf_delay{0};
void pose_graph_test_delay(int spins) { g_potrf_delay.store(spins < 0 ? 0 : spins); }

void launch_pose_graph_iteration(double* T, const int32_t* edges, const double* Z, const double* info, int N, int E,
                                 const int32_t* adj_off, const int32_t* adj, const int32_t* ftile, double* terms,
                                 double* H, double* g, double* delta, double* Ld, hipStream_t s) {
    const int n = 6 * (N - 1), np = (n + PG_TILE - 1) / PG_TILE * PG_TILE, nt = np / PG_TILE;
    hipLaunchKernelGGL(k_pg_edges, dim3((E + 63) / 64), dim3(64), 0, s, T, edges, Z, info, E, terms);
    hipLaunchKernelGGL(k_pg_assemble, dim3((np + 255) / 256, np), dim3(256), 0, s, terms, edges, adj_off, adj, n, np, H, g);
    for (int k = 0; k < nt; ++k) {
        hipLaunchKernelGGL(k_pg_potrf, dim3(nt - k), dim3(64), 0, s, H, np, k, ftile, Ld, g_potrf_delay.load());
        const int m = nt - k - 1;
        if (m > 0) hipLaunchKernelGGL(k_pg_syrk, dim3(m * (m + 1) / 2), dim3(256), 0, s, H, np, k, ftile);
    }
    hipLaunchKernelGGL(k_pg_trsv, dim3(1), dim3(PG_TRSV_THREADS), 0, s, H, np, g, delta, ftile, Ld);
    hipLaunchKernelGGL(k_pg_update, dim3((N + 62) / 64), dim3(64), 0, s, T, delta, N);
}

// the cost sum_k e_k^T info_k e_k in edge order (one lane: the order the host summed in before)
__global__ __launch_bounds__(64) void k_pg_cost_sum(const double* terms, int E, double* cost) {
    if (threadIdx.x) return;
    double cs = 0.0;
    for (int k = 0; k < E; ++k) cs += terms[(size_t)128 * k + 120];
    *cost = cs;
}

void launch_pose_graph_cost(const double* T, const int32_t* edges, const double* Z, const double* info, int E,
                            double* terms, double* cost, hipStream_t s) {
    if (E > 0) hipLaunchKernelGGL(k_pg_edges, dim3((E + 63) / 64), dim3(64), 0, s, T, edges, Z, info, E, terms);
    hipLaunchKernelGGL(k_pg_cost_sum, dim3(1), dim3(64), 0, s, terms, E, cost);
}
