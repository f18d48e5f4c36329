// k_ba.hip — row A8 of SURVEY.md §8a: sliding-window local bundle adjustment (config C4).
//
// Follows oracle/numpy_ba.py (the spec: keyframes, association by chained temporal matches,
// landmark homes slot*K + k with re-homing on eviction, stereo reprojection residuals, Schur
// complement on the cameras, Gauss-Newton with Levenberg damping, gauge = oldest keyframe).
//
// Per window solve: k_ba_insert_gate inserts the new keyframe (after k_ba_evict_* re-homed the
// evicted slot's landmarks), gates the observations at the current estimate and counts them per
// landmark; a tiled scan (k_ba_tilecount, k_ba_tilescatter) keeps landmarks seen >= 2 times,
// ranks them (compact index) and writes the dense (landmark, camera) slot table that every
// iteration reads with one level of indexing (k_ba_insert_gate clears the last solve's rows, k_ba_backsub
// re-zeroes the gate counts).
// Then per Gauss-Newton iteration:
//   k_ba_schur   per chunk of 32 landmarks: the previous iteration's landmark update (fused back
//                substitution), then J_c, J_p, r per observation -> W_o, J_c^T J_c | J_c^T r;
//                V_i = sum J_p^T J_p + lam I, g_p,i, L_i = chol(V_i), y_i = L_i^-1 g_p,i; the
//                chunk's Schur columns Q_i = [W_o L_i^-T] (rows of the observing camera) with y_i
//                in row 60 in an LDS tile; C += Q^T Q on the FP64 matrix cores
//                (v_mfma_f64_16x16x4f64), blocks striding the chunks (split-K partials);
//   k_ba_reduce  fixed-order sum of the split partials, and the camera blocks U_c, g_c;
//   k_ba_solve   one block: S = blockdiag(U + lam) - C, b = -g_c + C[:,60] without camera 0,
//                blocked LDL^T + back substitution, camera updates (Cayley);
// and after the last one k_ba_backsub: dp = V^-1 (-g_p - sum W_o^T dc), X = Xc + dp.
// Every reduction has a fixed order, so a solve is deterministic run to run.  Floating-point
// results differ from the oracle's (LU solves, numpy summation order) at the 1e-14 level.
#include "tslam_ba.h"
#include <cstring>

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

// The BA chain is latency-bound (small grids, dependent launches) and shares the SIMDs with the
// next batches' front-end waves: its waves raise their issue priority (s_setprio) so the SIMD
// arbiter serves them first.
#define BA_PRIO __builtin_amdgcn_s_setprio(3)

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

// The *_rec entry points read the batch context and the arguments from a device record
// (BaRec, graph replays) through constant-address-space pointers: the record is immutable during
// the launch, so its fields come in through scalar loads and the pointers loaded from it stay
// global (a generic pointer to the record would turn every access through them into flat ones).
typedef const __attribute__((address_space(4))) BatchCtx* __restrict__ BaCtxRef;
typedef const __attribute__((address_space(4))) BaArgs* __restrict__ BaArgsRef;

// ---------------------------------------------------------------------------------------------
// keyframe insertion (after the batch that contains frame g) and eviction
// ---------------------------------------------------------------------------------------------
// Eviction of slot a.slot: each landmark homed there moves to its observation in the oldest
// remaining keyframe (a.order, oldest first).  Pass 1 takes the minimum (rank, keypoint) key per
// landmark (remap pre-filled with a large value), pass 2 rewrites the ids and copies the position.
__device__ __forceinline__ void d_ba_evict_min(const BatchCtx& c, const BaArgs& a) {
    BA_PRIO;
    const int K = c.g.K;
    BaPair q = ba_pair(c, a, a.pair);
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n_order * K) return;
    const int r = i / K, k = i - r * K;
    const int id = q.lm[(size_t)a.order[r] * K + k], lo = a.slot * K;
    if (id >= lo && id < lo + K) atomicMin(&q.remap[id - lo], i);
}
__global__ __launch_bounds__(256) void k_ba_evict_min(BatchCtx c, BaArgs a) { d_ba_evict_min(c, a); }
__global__ __launch_bounds__(256) void k_ba_evict_min_rec(BaCtxRef c, BaArgsRef a) {
    d_ba_evict_min(*(const BatchCtx*)c, *(const BaArgs*)a);
}

__device__ __forceinline__ void d_ba_evict_move(const BatchCtx& c, const BaArgs& a) {
    BA_PRIO;
    const int K = c.g.K;
    BaPair q = ba_pair(c, a, a.pair);
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n_order * K) return;
    const int r = i / K, k = i - r * K;
    const size_t o = (size_t)a.order[r] * K + k;
    const int id = q.lm[o], lo = a.slot * K;
    if (id < lo || id >= lo + K) return;
    const int key = q.remap[id - lo];
    const int hr = key / K;
    const int nid = a.order[hr] * K + (key - hr * K);
    q.lm[o] = nid;
    if (key == i) {   // the new home copies the position and global id (sources: the evicted slot)
        for (int e = 0; e < 3; ++e) q.X[(size_t)nid * 3 + e] = q.X[(size_t)id * 3 + e];
        q.gid[nid] = q.gid[id];
    }
}
__global__ __launch_bounds__(256) void k_ba_evict_move(BatchCtx c, BaArgs a) { d_ba_evict_move(c, a); }
__global__ __launch_bounds__(256) void k_ba_evict_move_rec(BaCtxRef c, BaArgsRef a) {
    d_ba_evict_move(*(const BatchCtx*)c, *(const BaArgs*)a);
}

// ---------------------------------------------------------------------------------------------
// observation set of a solve (one block): gate at the current estimate, >= 2 observations per
// landmark, compact landmark index (= rank of the id), camera x landmark observation table
// ---------------------------------------------------------------------------------------------
#define BA_SCAN_ITEMS 8

// Exclusive scan of one int per thread over the block; *total = block sum.
__device__ int block_scan_excl(int v, int* s_tmp, int* total) {
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

// Insertion of frame a.frame into slot a.slot, fused with the gate of the solve that follows (one
// launch instead of two).  a.order is the solve's window (the new slot is in it).  Every block
// derives the new keyframe's pose (block 0 stores it); a thread of the new slot's items inserts its
// keypoint — landmark by the chained temporal matches to the previous keyframe, else a new one from
// the disparity — and gates that observation from its registers; the other items are gated as
// stored (positive depth, reprojection error <= outlier_px) and every gated observation counts
// towards its landmark (cnt pre-zeroed).  No other item reads what an inserting thread writes: the
// new slot's landmarks are observed by the new keyframe only (eviction re-homed the slot's old ones).
// A new keyframe's bias component k (accelerometer 0-2, gyroscope 3-5; oracle new_keyframe_bias):
// its inertial record's linearisation point, else the previous keyframe's, else 0.
__device__ __forceinline__ double ba_new_bias(const BaArgs& a, const double* bias, int k) {
    if (a.ine[28] > 0.0) return k < 3 ? a.ine[24 + k] : a.ine[68 + k - 3];
    return a.prev >= 0 ? bias[(size_t)a.prev * 6 + k] : 0.0;
}

__device__ __forceinline__ void d_ba_insert_gate(const BatchCtx& c, const BaArgs& a) {
    BA_PRIO;
    __shared__ double s_T[TS_BA_MAXW][12];   // cam_T_world of the window
    __shared__ double s_Tn[16];              // the new keyframe's
    const int K = c.g.K, p = a.pair, n = a.n_order;
    BaPair q = ba_pair(c, a, p);
    const int64_t g = a.frame;
    const int f = (int)(g - c.g0);   // frame of the current batch
    const int rslot = ring_slot(c, g);
    if (threadIdx.x == 0 && a.pose_given) {   // rig-level A8: E_p^-1 B set by k_ba_rig_insert
        for (int e = 0; e < 16; ++e) s_Tn[e] = q.T[(size_t)a.slot * 16 + e];
        if (blockIdx.x == 0)
            for (int e = 0; e < 16; ++e) q.Tfe[(size_t)a.slot * 16 + e] = a.fe[(size_t)(f * c.P + p) * 16 + e];
    } else if (threadIdx.x == 0) {
        const double* Tfe = a.fe + (size_t)(f * c.P + p) * 16;   // world_T_cam (front-end snapshot)
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
        double Tcw[16];
        inv_rigid(Twc, Tcw);
        for (int e = 0; e < 16; ++e) s_Tn[e] = Tcw[e];
        if (blockIdx.x == 0)
            for (int e = 0; e < 16; ++e) {
                q.Tfe[(size_t)a.slot * 16 + e] = Tfe[e];
                q.T[(size_t)a.slot * 16 + e] = Tcw[e];
            }
    }
    if (blockIdx.x == 0 && threadIdx.x < 10) q.imu[(size_t)a.slot * 10 + threadIdx.x] = a.imu[threadIdx.x];
    if (blockIdx.x == 0 && threadIdx.x < TS_BA_INE) q.ine[(size_t)a.slot * TS_BA_INE + threadIdx.x] = a.ine[threadIdx.x];
    if (blockIdx.x == 0 && threadIdx.x < 3) q.vel[(size_t)a.slot * 3 + threadIdx.x] = a.vel0[threadIdx.x];
    if (blockIdx.x == 0 && threadIdx.x < 6) q.bias[(size_t)a.slot * 6 + threadIdx.x] = ba_new_bias(a, q.bias, threadIdx.x);
    // the slot table back to all -1: the rows the last solve filled (k_ba_tilescatter fills this one's)
    const int Lp = q.counts[1];
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < Lp * TS_BA_MAXW; t += gridDim.x * blockDim.x) q.lo_o[t] = -1;
    __syncthreads();
    for (int i = threadIdx.x; i < n * 12; i += blockDim.x)
        s_T[i / 12][i % 12] = a.order[i / 12] == a.slot ? s_Tn[i % 12] : q.T[(size_t)a.order[i / 12] * 16 + i % 12];
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * K) return;
    const PairCalib cal = c.calib[p];
    const int ci = i / K, k = i - ci * K;
    const size_t o = (size_t)a.order[ci] * K + k;
    int id;
    double u, v, X[3];
    if (a.order[ci] == a.slot) {   // insert keypoint k of the new keyframe
        q.remap[k] = 0x7F7F7F7F;   // for the next eviction (k_ba_evict_* have run)
        u = __builtin_nan("");
        v = __builtin_nan("");
        const bool valid = kp_obs(c, rslot, c.cpp * p, k, &u, &v);
        const double dd = c.disp[((size_t)rslot * c.P + p) * K + k];
        const bool has_d = __builtin_isfinite(dd) && dd > 0.0;
        int lm = -1;
        if (valid && a.prev >= 0) {   // the temporal matches chained back to the previous keyframe
            const int j = a.kf_assoc[((size_t)f * c.P + p) * K + k];
            if (j >= 0) lm = q.lm[(size_t)a.prev * K + j];
        }
        if (valid && lm < 0 && has_d) {
            lm = a.slot * K + k;
            q.gid[lm] = g * K + k;
            const double z = cal.fxb / dd;
            const double xc[3] = {(u - cal.cx) * z / cal.fx, (v - cal.cy) * z / cal.fy, z};
            for (int e = 0; e < 3; ++e) {   // R^T (xc - t)
                X[e] = ((s_Tn[e] * (xc[0] - s_Tn[3]) + s_Tn[4 + e] * (xc[1] - s_Tn[7])) + s_Tn[8 + e] * (xc[2] - s_Tn[11]));
                q.X[(size_t)lm * 3 + e] = X[e];
            }
        } else if (lm >= 0) {
            for (int e = 0; e < 3; ++e) X[e] = q.X[(size_t)lm * 3 + e];
        }
        const uint4* dsrc = reinterpret_cast<const uint4*>(c.desc + (((size_t)rslot * c.C + c.cpp * p) * K + k) * 8);
        uint4* ddst = reinterpret_cast<uint4*>(q.kf_desc + o * 8);
        ddst[0] = dsrc[0];
        ddst[1] = dsrc[1];
        if (!valid) {
            u = __builtin_nan("");
            v = __builtin_nan("");
        }
        q.u[o] = u;
        q.v[o] = v;
        q.d[o] = has_d ? dd : __builtin_nan("");
        q.lm[o] = lm;
        id = lm;
    } else {
        id = q.lm[o];
        u = q.u[o];
        v = q.v[o];
        if (id >= 0)
            for (int e = 0; e < 3; ++e) X[e] = q.X[(size_t)id * 3 + e];
    }
    int keep = 0;
    if (id >= 0) {
        const double* T = s_T[ci];
        const double lim = a.outlier_px * a.outlier_px;
        const double xc = ((T[0] * X[0] + T[1] * X[1]) + T[2] * X[2]) + T[3];
        const double yc = ((T[4] * X[0] + T[5] * X[1]) + T[6] * X[2]) + T[7];
        const double zc = ((T[8] * X[0] + T[9] * X[1]) + T[10] * X[2]) + T[11];
        const double pu = cal.fx * xc / zc + cal.cx, pv = cal.fy * yc / zc + cal.cy;
        const double du = pu - u, dv = pv - v;
        keep = zc > 0.0 && du * du + dv * dv <= lim;
        if (keep) atomicAdd(&q.cnt[id], 1);
    }
    q.keep[i] = (uint8_t)keep;
}
__global__ __launch_bounds__(256) void k_ba_insert_gate(BatchCtx c, BaArgs a) { d_ba_insert_gate(c, a); }
__global__ __launch_bounds__(256) void k_ba_insert_gate_rec(BaCtxRef c, BaArgsRef a) {
    d_ba_insert_gate(*(const BatchCtx*)c, *(const BaArgs*)a);
}

// Compaction after the gate, as a deterministic tiled scan (tiles of BA_TILE items):
//   landmark tiles over the ids (flag: >= 2 gated observations) -> compact index li = rank of the
//   id, lm_id = its inverse;  observation tiles per window camera over its keypoints (flag: gated
//   and its landmark kept) -> the observation list in (camera, keypoint) order.
// k_ba_tilecount counts every tile (and keeps each landmark tile's flag words), k_ba_tilescatter
// scans the counts and writes the compact landmarks and the dense slot table directly: an
// observation's compact landmark index is its id's tile offset + the flagged ids before its word +
// a popcount in the word.
#define BA_TILE (256 * BA_SCAN_ITEMS)
static_assert(BA_TILE == 2048 && BA_SCAN_ITEMS == 8, "tc_ids / tc_fl layout (tslam_ba.h)");

struct BaTiles {
    int n_lm_tiles, per_cam;   // landmark tiles; observation tiles per camera
};
__device__ __forceinline__ BaTiles ba_tiles(const BatchCtx& c, const BaArgs& a) {
    return BaTiles{(a.W * c.g.K + BA_TILE - 1) / BA_TILE, (c.g.K + BA_TILE - 1) / BA_TILE};
}

// Flags of the BA_SCAN_ITEMS items of this thread in tile b; *ids gets the landmark id of each
// flagged observation (observation tiles) or the id itself (landmark tiles).
__device__ __forceinline__ void ba_tile_flags(const BatchCtx& c, const BaArgs& a, const BaPair& q, int b, int* fl,
                                              int* ids, int* ci_out, int* k0_out) {
    const int K = c.g.K;
    const BaTiles t = ba_tiles(c, a);
    if (b < t.n_lm_tiles) {
        const int NID = a.W * K;
        const int i0 = b * BA_TILE + threadIdx.x * BA_SCAN_ITEMS;
        *ci_out = -1;
        *k0_out = i0;
#pragma unroll
        for (int it = 0; it < BA_SCAN_ITEMS; ++it) {   // unconditional (clamped) loads, no branches
            ids[it] = i0 + it;
            const int cn = q.cnt[min(i0 + it, NID - 1)];
            fl[it] = i0 + it < NID && cn >= 2;
        }
    } else {
        const int bb = b - t.n_lm_tiles, ci = bb / t.per_cam;
        const int k0 = (bb - ci * t.per_cam) * BA_TILE + threadIdx.x * BA_SCAN_ITEMS;
        *ci_out = ci;
        *k0_out = k0;
        const size_t base = (size_t)a.order[ci] * K;
        // the items' gate bytes and ids first, then the count gathers (a kept observation has an id)
        uint32_t kp[BA_SCAN_ITEMS];
        int lmv[BA_SCAN_ITEMS];
#pragma unroll
        for (int it = 0; it < BA_SCAN_ITEMS; ++it) {
            const int k = min(k0 + it, K - 1);
            kp[it] = k0 + it < K ? q.keep[ci * K + k] : 0u;
            lmv[it] = q.lm[base + k];
        }
#pragma unroll
        for (int it = 0; it < BA_SCAN_ITEMS; ++it) {
            const int cn = q.cnt[kp[it] ? lmv[it] : 0];
            ids[it] = kp[it] ? lmv[it] : -1;
            fl[it] = kp[it] && cn >= 2;
        }
    }
}

__device__ __forceinline__ void d_ba_tilecount(const BatchCtx& c, const BaArgs& a) {
    BA_PRIO;
    __shared__ int s_tmp[32];
    __shared__ __attribute__((aligned(4))) uint8_t s_fl[256];   // thread t's flags: bits 8t .. 8t+7 of the tile
    BaPair q = ba_pair(c, a, a.pair);
    int fl[BA_SCAN_ITEMS], ids[BA_SCAN_ITEMS], ci, k0, cnt = 0;
    ba_tile_flags(c, a, q, blockIdx.x, fl, ids, &ci, &k0);
    uint32_t bits = 0;
#pragma unroll
    for (int it = 0; it < BA_SCAN_ITEMS; ++it) {
        cnt += fl[it];
        bits |= (uint32_t)fl[it] << it;
    }
    s_fl[threadIdx.x] = (uint8_t)bits;
    // this thread's flags and (observation tiles) ids for the scatter
    q.tc_fl[blockIdx.x * 256 + threadIdx.x] = (uint8_t)bits;
    if (ci >= 0) {
        int4* dst = reinterpret_cast<int4*>(q.tc_ids + (size_t)blockIdx.x * BA_TILE + threadIdx.x * BA_SCAN_ITEMS);
        dst[0] = int4{ids[0], ids[1], ids[2], ids[3]};
        dst[1] = int4{ids[4], ids[5], ids[6], ids[7]};
    }
    int tot;
    block_scan_excl(cnt, s_tmp, &tot);   // its barriers order the s_fl stores
    if (threadIdx.x == 0) q.tiles[blockIdx.x] = tot;
    // a landmark tile's 64 flag words and the flagged ids before each (wave 0: a word per lane)
    if (ci < 0 && threadIdx.x < 64) {
        const uint32_t w = reinterpret_cast<const uint32_t*>(s_fl)[threadIdx.x];
        const int pc = __popc(w);
        int x = pc;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if ((int)threadIdx.x >= o) x += y;
        }
        q.lmask[blockIdx.x * 64 + threadIdx.x] = w;
        q.lpre[blockIdx.x * 64 + threadIdx.x] = x - pc;
    }
}
__global__ __launch_bounds__(256) void k_ba_tilecount(BatchCtx c, BaArgs a) { d_ba_tilecount(c, a); }
__global__ __launch_bounds__(256) void k_ba_tilecount_rec(BaCtxRef c, BaArgsRef a) {
    d_ba_tilecount(*(const BatchCtx*)c, *(const BaArgs*)a);
}

// Scatter after the tile counts; each block takes its tile's offset from the counts of the tiles
// before it (landmark tiles and observation tiles are scanned separately), and block 0 also
// publishes the totals and the per-camera observation ranges (no separate scan launch).
__device__ __forceinline__ void d_ba_tilescatter(const BatchCtx& c, const BaArgs& a) {
    BA_PRIO;
    __shared__ int s_tmp[32];
    __shared__ int s_cnt[TS_BA_TILES];
    __shared__ int s_lbase[TS_BA_TILES];   // compact index of each landmark tile's first flagged id
    BaPair q = ba_pair(c, a, a.pair);
    const BaTiles t = ba_tiles(c, a);
    const int ntiles = t.n_lm_tiles + a.n_order * t.per_cam;
    for (int j = threadIdx.x; j < ntiles; j += blockDim.x) s_cnt[j] = q.tiles[j];
    __syncthreads();
    if (threadIdx.x == 0) {
        int run = 0;
        for (int b = 0; b < t.n_lm_tiles; ++b) {
            s_lbase[b] = run;
            run += s_cnt[b];
        }
    }
    // the tile count's flags and ids (k_ba_tilecount stored them; same tiles, same threads)
    int fl[BA_SCAN_ITEMS], ids[BA_SCAN_ITEMS], ci, k0, cnt = 0;
    {
        const int b = blockIdx.x;
        if (b < t.n_lm_tiles) {
            ci = -1;
            k0 = b * BA_TILE + threadIdx.x * BA_SCAN_ITEMS;
#pragma unroll
            for (int it = 0; it < BA_SCAN_ITEMS; ++it) ids[it] = k0 + it;
        } else {
            const int bb = b - t.n_lm_tiles;
            ci = bb / t.per_cam;
            k0 = (bb - ci * t.per_cam) * BA_TILE + threadIdx.x * BA_SCAN_ITEMS;
            const int4* src = reinterpret_cast<const int4*>(q.tc_ids + (size_t)b * BA_TILE + threadIdx.x * BA_SCAN_ITEMS);
            const int4 u0 = src[0], u1 = src[1];
            ids[0] = u0.x; ids[1] = u0.y; ids[2] = u0.z; ids[3] = u0.w;
            ids[4] = u1.x; ids[5] = u1.y; ids[6] = u1.z; ids[7] = u1.w;
        }
        const uint32_t bits = q.tc_fl[b * 256 + threadIdx.x];
#pragma unroll
        for (int it = 0; it < BA_SCAN_ITEMS; ++it) fl[it] = (bits >> it) & 1u;
    }
#pragma unroll
    for (int it = 0; it < BA_SCAN_ITEMS; ++it) cnt += fl[it];
    int tot;
    const int within = block_scan_excl(cnt, s_tmp, &tot);   // its barriers order the s_lbase stores
    const int first = (int)blockIdx.x < t.n_lm_tiles ? 0 : t.n_lm_tiles;
    int base = 0;
    for (int j = first; j < (int)blockIdx.x; ++j) base += s_cnt[j];   // LDS broadcast reads
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        int run = 0;
        for (int b = 0; b < t.n_lm_tiles; ++b) run += s_cnt[b];
        q.counts[1] = run;
        run = 0;
        for (int cc = 0; cc < a.n_order; ++cc) {
            q.cam_off[cc] = run;
            for (int tt = 0; tt < t.per_cam; ++tt) run += s_cnt[t.n_lm_tiles + cc * t.per_cam + tt];
        }
        q.cam_off[a.n_order] = run;
        q.counts[0] = run;
    }
    int pos = base + within;
    // every item's loads are issued before the first store (indices clamped for the unflagged
    // ones), so a thread waits on one round of gathers instead of one per item
    if (ci < 0) {   // compact landmark pos: its id and its position during the solve
        double x[BA_SCAN_ITEMS][3];
#pragma unroll
        for (int it = 0; it < BA_SCAN_ITEMS; ++it) {
            const size_t id = fl[it] ? (size_t)(k0 + it) : 0;
#pragma unroll
            for (int e = 0; e < 3; ++e) x[it][e] = q.X[id * 3 + e];
        }
#pragma unroll
        for (int it = 0; it < BA_SCAN_ITEMS; ++it)
            if (fl[it]) {
                q.lm_id[pos] = k0 + it;
#pragma unroll
                for (int e = 0; e < 3; ++e) q.Xc[(size_t)pos * 3 + e] = x[it][e];
                ++pos;
            }
    } else {   // observation pos of window camera ci: its slot (compact landmark r, ci) and (u, v, d)
        const size_t ob = (size_t)a.order[ci] * c.g.K;
        uint32_t mw[BA_SCAN_ITEMS];
        int pw[BA_SCAN_ITEMS], rb[BA_SCAN_ITEMS];
        double uvd[BA_SCAN_ITEMS][3];
#pragma unroll
        for (int it = 0; it < BA_SCAN_ITEMS; ++it) {
            const int id = fl[it] ? ids[it] : 0;
            const int tl = id / BA_TILE, item = id - tl * BA_TILE, w = tl * 64 + (item >> 5);
            mw[it] = q.lmask[w] & ((1u << (item & 31)) - 1u);
            pw[it] = q.lpre[w];
            rb[it] = s_lbase[tl];
            const size_t so = fl[it] ? ob + k0 + it : ob;
            uvd[it][0] = q.u[so];
            uvd[it][1] = q.v[so];
            uvd[it][2] = q.d[so];
        }
#pragma unroll
        for (int it = 0; it < BA_SCAN_ITEMS; ++it)
            if (fl[it]) {
                const int r = rb[it] + pw[it] + __popc(mw[it]);
                const size_t sl = (size_t)r * TS_BA_MAXW + ci;
                q.lo_o[sl] = pos;
                double* d = q.lo_uvd + sl * 4;
                d[0] = uvd[it][0];
                d[1] = uvd[it][1];
                d[2] = uvd[it][2];
                d[3] = 0.0;
                ++pos;
            }
    }
}
__global__ __launch_bounds__(256) void k_ba_tilescatter(BatchCtx c, BaArgs a) { d_ba_tilescatter(c, a); }
__global__ __launch_bounds__(256) void k_ba_tilescatter_rec(BaCtxRef c, BaArgsRef a) {
    d_ba_tilescatter(*(const BatchCtx*)c, *(const BaArgs*)a);
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
    double iz = __builtin_amdgcn_rcp(zc);   // + one Newton step instead of the division chain (error ~e0^2, e0 the estimate's)
    iz = iz * (2.0 - zc * iz);
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

typedef double d4v __attribute__((ext_vector_type(4)));

// Workgroup barrier ordering LDS only: waits for this wave's LDS operations, not for its HBM
// stores (a __syncthreads() would wait for those too), so stores drain behind the barrier.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
#ifdef TS_BA_STAMPS   // experiment builds: phase durations (s_memrealtime, 100 MHz) printed by one thread
#define BST_DECL uint64_t bst_prev = wall_clock64(), bst[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define BST(i)                              \
    do {                                    \
        const uint64_t n_ = wall_clock64(); \
        bst[i] += n_ - bst_prev;            \
        bst_prev = n_;                      \
    } while (0)
#define BST_PRINT(tag, cond) \
    if (cond) printf(tag " %lu %lu %lu %lu %lu %lu %lu %lu (x10ns)\n", bst[0], bst[1], bst[2], bst[3], bst[4], bst[5], bst[6], bst[7])
#else
#define BST_DECL \
    do {         \
    } while (0)
#define BST(i) \
    do {       \
    } while (0)
#define BST_PRINT(tag, cond) \
    do {                     \
    } while (0)
#endif
#define BA_CHUNK 32          // landmarks per LDS tile (96 Schur columns)
#define BA_QPITCH 80         // doubles per tile column: 160 dwords = 32 mod 64 banks, so the four
                             // columns one MFMA operand read touches fall in disjoint bank halves
#define BA_SCHUR_THREADS (BA_CHUNK * TS_BA_MAXW)   // 320: one thread per (landmark, window camera)

// The landmark side of one Gauss-Newton step, fused; per chunk of BA_CHUNK landmarks:
//   1. one thread per (landmark, camera) with an observation: J_c, J_p, r (ba_obs_jac) ->
//      W_o = J_c^T J_p and J_p^T J_p | J_p^T r into LDS; W_o (for the back substitution) and
//      J_c^T J_c | J_c^T r into LDS;
//   2. one thread per landmark: V = lam I + sum_c J_p^T J_p (camera order), g_p, L = chol(V),
//      y = L^-1 g_p (L, g_p to HBM for the back substitution); beside them one thread per (camera,
//      element) sums the chunk's J_c^T J_c | J_c^T r over its landmarks (landmark order) into the
//      block's camera partial;
//   3. the chunk's Schur columns into an LDS tile Q[3 * BA_CHUNK][64]: column 3l + j holds
//      (W_o L^-T)[:, j] in the 6 rows of the observing camera (0 when unobserved), y_j in row 60;
//   4. C += Q^T Q on the FP64 matrix cores (v_mfma_f64_16x16x4f64), waves 0-3 own 16 rows each.
// Blocks stride the chunks; each block that had a chunk writes its 64 x 64 partial and its camera
// partial (TS_BA_PART doubles per block: C, then [camera][27]), which k_ba_reduce sums in a fixed
// order.  The camera sums stay in the block instead of 27 scattered 8-byte stores per observation.
__device__ __forceinline__ void d_ba_schur(const BatchCtx& c, const BaArgs& a, int fused) {
#pragma clang fp contract(fast)   // single FMAs in the landmark chains (held to 1e-9, as k_ba_solve)
    BA_PRIO;
    // the Schur tile Q (phases 3-4) and the observations' camera blocks (phases 1-2) share LDS
    constexpr int QN = 3 * BA_CHUNK * BA_QPITCH, CN = BA_CHUNK * TS_BA_MAXW * 27;
    __shared__ double s_buf[QN > CN ? QN : CN];
    double* const s_Q = s_buf;
    double(*const s_cu)[TS_BA_MAXW][27] = reinterpret_cast<double(*)[TS_BA_MAXW][27]>(s_buf);
    __shared__ double s_Vg[BA_CHUNK][TS_BA_MAXW][9];
    __shared__ int s_has[BA_CHUNK][TS_BA_MAXW];
    __shared__ double s_L[BA_CHUNK][9];   // inverse-diagonal Cholesky factor | y
    __shared__ double s_T[TS_BA_MAXW][12];
    __shared__ double s_bs[BA_CHUNK][TS_BA_MAXW][3];
    __shared__ double s_X[BA_CHUNK][3];
    const int K = c.g.K, WK = a.W * K, n = a.n_order;
    BaPair q = ba_pair(c, a, a.pair);
    const int L = q.counts[1];
    const PairCalib cal = c.calib[a.pair];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int kk = lane >> 4, rc = lane & 15;
    BST_DECL;
    for (int i = threadIdx.x; i < n * 12; i += blockDim.x) s_T[i / 12][i % 12] = q.T[(size_t)a.order[i / 12] * 16 + i % 12];
    // wave w's two tiles (row block, column block) of the lower triangle of C, as the first rows /
    // columns: (0,0) (3,0) | (1,0) (3,1) | (1,1) (3,2) | (2,0) (3,3) | (2,1) (2,2)
    static_assert(BA_SCHUR_THREADS == 5 * 64, "five waves share the ten lower tiles");
    const int ta[4] = {16 * ((0x22110 >> (4 * wave)) & 15), 16 * ((0x10100 >> (4 * wave)) & 15),
                       16 * ((0x23333 >> (4 * wave)) & 15), 16 * ((0x23210 >> (4 * wave)) & 15)};
    d4v acc[2];
    for (int t = 0; t < 2; ++t) acc[t] = (d4v){0.0, 0.0, 0.0, 0.0};
    const bool bsub = fused && q.counts[2];   // the previous solve succeeded
    const int cu_item = (int)threadIdx.x - BA_CHUNK;     // (camera, element) of the camera sums
    double cam_acc = 0.0;
    for (int l0 = blockIdx.x * BA_CHUNK; l0 < L; l0 += gridDim.x * BA_CHUNK) {
        const int nl = min(BA_CHUNK, L - l0);
        lds_barrier();
        BST(0);
        // every global read of the chunk is one level of indexing (the slot table of k_ba_tilescatter), issued
        // up front: slot (li, ci) = thread / TS_BA_MAXW, thread % TS_BA_MAXW; landmark li = thread
        const int li = threadIdx.x / TS_BA_MAXW, ci = threadIdx.x - li * TS_BA_MAXW;
        const int r = l0 + li;
        const size_t sl = (size_t)r * TS_BA_MAXW + ci;
        const bool in = li < nl && ci < n;
        const int o = in ? q.lo_o[sl] : -1;
        double uvd[3] = {0.0, 0.0, 0.0};
        if (in) {
            const double* pu = q.lo_uvd + sl * 4;
            uvd[0] = pu[0]; uvd[1] = pu[1]; uvd[2] = pu[2];
        }
        const bool lmt = (int)threadIdx.x < nl;   // landmark thread of landmark l0 + threadIdx.x
        const int rl = l0 + threadIdx.x;
        double Xl[3] = {0.0, 0.0, 0.0};
        if (lmt) {
            Xl[0] = q.Xc[(size_t)rl * 3]; Xl[1] = q.Xc[(size_t)rl * 3 + 1]; Xl[2] = q.Xc[(size_t)rl * 3 + 2];
        }
        // 0. the previous iteration's landmark update for the chunk (this block factored these
        //    landmarks then): dp = V^-1 (-g_p - sum_c W_o^T dc_c), Xc += dp
        if (bsub) {
            double t[3] = {0.0, 0.0, 0.0};
            if (in && ci >= 1) {   // dc of camera 0 is zero
                double Wv[18], dcv[6];
                const double* W = q.lo_W + sl * 18;
#pragma unroll
                for (int e = 0; e < 18; ++e) Wv[e] = W[e];
#pragma unroll
                for (int e = 0; e < 6; ++e) dcv[e] = q.dc[6 * ci + e];
                if (o >= 0) {
#pragma unroll
                    for (int j = 0; j < 3; ++j) {
                        double acc = 0.0;
#pragma unroll
                        for (int e = 0; e < 6; ++e) acc += Wv[3 * e + j] * dcv[e];
                        t[j] = acc;
                    }
                }
            }
            double gp[3] = {0.0, 0.0, 0.0}, Lf[6] = {1.0, 0.0, 1.0, 0.0, 0.0, 1.0};
            if (lmt) {
#pragma unroll
                for (int j = 0; j < 3; ++j) gp[j] = q.lm_gp[(size_t)j * WK + rl];
#pragma unroll
                for (int j = 0; j < 6; ++j) Lf[j] = q.lm_L[(size_t)j * WK + rl];
            }
            if (li < BA_CHUNK) {
#pragma unroll
                for (int j = 0; j < 3; ++j) s_bs[li][ci][j] = t[j];
            }
            lds_barrier();
            if (lmt) {
                double rhs[3];
                for (int j = 0; j < 3; ++j) {
                    double sum = 0.0;
                    for (int cj = 1; cj < n; ++cj) sum += s_bs[threadIdx.x][cj][j];
                    rhs[j] = -gp[j] - sum;
                }
                const double L0 = Lf[0], L1 = Lf[1], L2 = Lf[2], L3 = Lf[3], L4 = Lf[4], L5 = Lf[5];
                // L0, L2, L5 are the inverse diagonal (lm_L)
                const double y0 = rhs[0] * L0, y1 = (rhs[1] - L1 * y0) * L2, y2 = ((rhs[2] - L3 * y0) - L4 * y1) * L5;
                const double x2 = y2 * L5, x1 = (y1 - L4 * x2) * L2, x0 = ((y0 - L1 * x1) - L3 * x2) * L0;
                Xl[0] += x0;
                Xl[1] += x1;
                Xl[2] += x2;
#pragma unroll
                for (int j = 0; j < 3; ++j) q.Xc[(size_t)rl * 3 + j] = Xl[j];
            }
        }
        if (lmt) {
#pragma unroll
            for (int j = 0; j < 3; ++j) s_X[threadIdx.x][j] = Xl[j];
        }
        lds_barrier();
        BST(1);
        // 1. Jacobians of every (landmark, camera) observation of the chunk; W_o stays in this
        //    thread's registers for step 3 (and goes to HBM for the next pass's landmark update)
        double Wr[18];
#pragma unroll
        for (int e = 0; e < 18; ++e) Wr[e] = 0.0;
        s_has[li][ci] = o >= 0;
        if (o >= 0) {
            double Jc[3][6], Jp[3][3], res[3];
            ba_obs_jac(s_T[ci], s_X[li], uvd[0], uvd[1], uvd[2], cal, Jc, Jp, res);
            double* Wg = q.lo_W + sl * 18;
#pragma unroll
            for (int i = 0; i < 6; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const double w = (Jc[0][i] * Jp[0][j] + Jc[1][i] * Jp[1][j]) + Jc[2][i] * Jp[2][j];
                    Wr[3 * i + j] = w;
                    Wg[3 * i + j] = w;
                }
            double* cu = s_cu[li][ci];
            int e = 0;
            for (int i = 0; i < 6; ++i)
                for (int j = i; j < 6; ++j) cu[e++] = (Jc[0][i] * Jc[0][j] + Jc[1][i] * Jc[1][j]) + Jc[2][i] * Jc[2][j];
            for (int i = 0; i < 6; ++i) cu[21 + i] = (Jc[0][i] * res[0] + Jc[1][i] * res[1]) + Jc[2][i] * res[2];
            double* vg = s_Vg[li][ci];
            e = 0;
            for (int i = 0; i < 3; ++i)
                for (int j = i; j < 3; ++j) vg[e++] = (Jp[0][i] * Jp[0][j] + Jp[1][i] * Jp[1][j]) + Jp[2][i] * Jp[2][j];
            for (int i = 0; i < 3; ++i) vg[6 + i] = (Jp[0][i] * res[0] + Jp[1][i] * res[1]) + Jp[2][i] * res[2];
        } else if (li < BA_CHUNK) {
#pragma unroll
            for (int e = 0; e < 27; ++e) s_cu[li][ci][e] = 0.0;
        }
        lds_barrier();   // LDS only: the HBM stores above drain behind it
        BST(2);
        // 2. per-landmark factor
        if (threadIdx.x < BA_CHUNK) {
            const int li = threadIdx.x, r = l0 + li;
            const bool live = li < nl;
            double vg[9] = {a.lam, 0.0, 0.0, a.lam, 0.0, a.lam, 0.0, 0.0, 0.0};   // V00 V01 V02 V11 V12 V22 g
            for (int ci = 0; ci < n; ++ci)
                if (s_has[li][ci])
#pragma unroll
                    for (int e = 0; e < 9; ++e) vg[e] += s_Vg[li][ci][e];
            // one reciprocal square root per pivot, multiplications after it (the chain had 9
            // divisions, then 3 sqrt + division pairs): v_rsq_f64 + one Newton step; the hardware estimate is
            // good to roughly 2^-22..2^-26, so the result is within ~2^-44..2^-52 relative (not correctly
            // rounded; the oracle bar is 1e-9)
            auto rsqrt_nr = [](double x) {
                x = x > 1e-300 ? x : 1e-300;
                const double y = __builtin_amdgcn_rsq(x);
                return y * (1.5 - (0.5 * x) * (y * y));
            };
            const double i00 = rsqrt_nr(vg[0]);
            const double l10 = vg[1] * i00, l20 = vg[2] * i00;
            const double d11 = vg[3] - l10 * l10;
            const double i11 = rsqrt_nr(d11);
            const double l21 = (vg[4] - l20 * l10) * i11;
            const double d22 = (vg[5] - l20 * l20) - l21 * l21;
            const double i22 = rsqrt_nr(d22);
            const double y0 = vg[6] * i00, y1 = (vg[7] - l10 * y0) * i11, y2 = ((vg[8] - l20 * y0) - l21 * y1) * i22;
            s_L[li][0] = i00; s_L[li][1] = l10; s_L[li][2] = i11; s_L[li][3] = l20; s_L[li][4] = l21;
            s_L[li][5] = i22;
            s_L[li][6] = live ? y0 : 0.0;   // row 60 of the landmark's three columns (phase 3)
            s_L[li][7] = live ? y1 : 0.0;
            s_L[li][8] = live ? y2 : 0.0;
            if (live) {
                q.lm_L[r] = i00; q.lm_L[(size_t)WK + r] = l10; q.lm_L[(size_t)2 * WK + r] = i11;
                q.lm_L[(size_t)3 * WK + r] = l20; q.lm_L[(size_t)4 * WK + r] = l21; q.lm_L[(size_t)5 * WK + r] = i22;
                q.lm_gp[r] = vg[6]; q.lm_gp[(size_t)WK + r] = vg[7]; q.lm_gp[(size_t)2 * WK + r] = vg[8];
            }
        } else if (cu_item < n * 27) {   // the chunk's camera sums, landmark order
            const int cc = cu_item / 27, e = cu_item - 27 * cc;
            double sum = 0.0;
            for (int l = 0; l < nl; ++l) sum += s_cu[l][cc][e];
            cam_acc += sum;
        }
        lds_barrier();
        BST(3);
        // 3. Schur columns: thread (landmark, camera) writes the camera's 6 rows of the landmark's
        //    3 columns, (W_o L^-T) or zeros
        {
            const double* Lm = s_L[li];
            const double i0 = Lm[0], m1 = Lm[1], i2 = Lm[2], m3 = Lm[3], m4 = Lm[4], i5 = Lm[5];
#pragma unroll
            for (int rr = 0; rr < 6; ++rr) {
                const double* W = Wr + 3 * rr;
                const double z0 = W[0] * i0;
                const double z1 = (W[1] - m1 * z0) * i2;
                const double z2 = ((W[2] - m3 * z0) - m4 * z1) * i5;
                const int row = 6 * ci + rr;
                s_Q[(3 * li) * BA_QPITCH + row] = o >= 0 ? z0 : 0.0;
                s_Q[(3 * li + 1) * BA_QPITCH + row] = o >= 0 ? z1 : 0.0;
                s_Q[(3 * li + 2) * BA_QPITCH + row] = o >= 0 ? z2 : 0.0;
            }
            if (ci == 0) {
#pragma unroll
                for (int j = 0; j < 3; ++j) {   // rows 60 (y) .. 63 of the landmark's three columns
                    double* colq = s_Q + (3 * li + j) * BA_QPITCH;
                    colq[60] = Lm[6 + j];
                    colq[61] = 0.0;
                    colq[62] = 0.0;
                    colq[63] = 0.0;
                }
            }
        }
        lds_barrier();
        BST(4);
        // 4. C += Q^T Q over the chunk's columns (zero columns past nl contribute nothing): only
        //    the 10 lower-triangle 16 x 16 tiles, two per wave (the upper ones are their transposes)
        {
            const int ksteps = (3 * nl + 3) >> 2;
            // the next k-step's operands load while this one's two MFMAs run
            const double* col = s_Q + kk * BA_QPITCH + rc;
            double n0 = col[ta[0]], n1 = col[ta[1]], n2 = col[ta[2]], n3 = col[ta[3]];
            for (int st = 0; st < ksteps; ++st) {
                const double a0v = n0, b0v = n1, a1v = n2, b1v = n3;
                const double* nx = col + 4 * min(st + 1, ksteps - 1) * BA_QPITCH;
                n0 = nx[ta[0]];
                n1 = nx[ta[1]];
                n2 = nx[ta[2]];
                n3 = nx[ta[3]];
                acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0v, b0v, acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1v, b1v, acc[1], 0, 0, 0);
            }
        }
        BST(5);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {   // algorithmic flops of the symmetric Schur product
        const double rows = 6.0 * n + 1.0;          // (SYRK: the lower triangle with its diagonal)
        q.flops[0] += rows * (rows + 1.0) * 3.0 * L;
    }
    BST_PRINT("schur b0: stage+T, lm update, jacobians, factor, columns, mfma, -, -", blockIdx.x == 0 && threadIdx.x == 0);
    if (blockIdx.x * BA_CHUNK >= L) return;   // no chunk: no partial
    if (cu_item >= 0 && cu_item < n * 27) q.part[(size_t)blockIdx.x * TS_BA_PART + 4096 + cu_item] = cam_acc;
    double* out = q.part + (size_t)blockIdx.x * TS_BA_PART;
    // C/D layout of v_mfma_f64_16x16x4f64: col = lane & 15, row = (lane >> 4) + 4 * reg; an
    // off-diagonal tile is stored twice, as itself and as its transpose (the symmetric partner;
    // a diagonal tile is symmetric bit for bit)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int r0 = ta[2 * t], c0 = ta[2 * t + 1];
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) {
            out[(size_t)(r0 + kk + 4 * rg) * 64 + c0 + rc] = acc[t][rg];
            if (r0 != c0) out[(size_t)(c0 + rc) * 64 + r0 + kk + 4 * rg] = acc[t][rg];
        }
    }
}
__global__ __launch_bounds__(BA_SCHUR_THREADS) void k_ba_schur(BatchCtx c, BaArgs a) { d_ba_schur(c, a, a.fused_backsub); }
__global__ __launch_bounds__(BA_SCHUR_THREADS) void k_ba_schur_rec(BaCtxRef c, BaArgsRef a,
    int fused) {
    d_ba_schur(*(const BatchCtx*)c, *(const BaArgs*)a, fused);
}

// Fixed-order sum of the partials of the blocks that had a chunk: block = 64 elements of a
// partial, BA_SOLVE_WAVES waves each summing every BA_SOLVE_WAVES-th partial, then the wave sums
// in order (k_ba_reduce_solve sums in the same order: the split and the fused launch agree bit for
// bit).  Elements 0..4095 are C, 4096.. the camera blocks U_c, g_c ([camera][27]).
#define BA_SOLVE_WAVES 8
__device__ __forceinline__ double ba_reduce_elem(const BaPair& q, const BaArgs& a, int e, bool live,
                                                 double (*s_p)[64]) {
    const int L = q.counts[1];
    const int np = min(a.nsplit, (L + BA_CHUNK - 1) / BA_CHUNK);
    const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
    double sum = 0.0;
    if (live) {
#pragma unroll 8
        for (int b = grp; b < np; b += BA_SOLVE_WAVES) sum += q.part[(size_t)b * TS_BA_PART + e];
    }
    s_p[grp][lane] = sum;
    __syncthreads();
    double v = s_p[0][lane];
#pragma unroll
    for (int g = 1; g < BA_SOLVE_WAVES; ++g) v += s_p[g][lane];
    return v;   // meaningful in wave 0
}

__device__ __forceinline__ void d_ba_reduce(const BatchCtx& c, const BaArgs& a) {
    BA_PRIO;
    __shared__ double s_p[BA_SOLVE_WAVES][64];
    BaPair q = ba_pair(c, a, a.pair);
    const int e = blockIdx.x * 64 + (threadIdx.x & 63);
    const bool live = e < 4096 + a.n_order * 27;
    const double v = ba_reduce_elem(q, a, e, live, s_p);
    if ((threadIdx.x >> 6) != 0 || !live) return;
    if (e < 4096) q.C[e] = v;
    else q.cam_U[e - 4096] = v;
}
__global__ __launch_bounds__(64 * BA_SOLVE_WAVES) void k_ba_reduce(BatchCtx c, BaArgs a) { d_ba_reduce(c, a); }
__global__ __launch_bounds__(64 * BA_SOLVE_WAVES) void k_ba_reduce_rec(BaCtxRef c, BaArgsRef a) {
    d_ba_reduce(*(const BatchCtx*)c, *(const BaArgs*)a);
}

// Reduced camera system (camera 0 = gauge): S = blockdiag(U + lam) - C, b = -g_c + C[:, 60].
// Blocked right-looking LDL^T over the 6-wide camera blocks (m = 6 (n - 1) <= 54), one block of
// 8 waves, the lower triangle of S in LDS:
//   * wave 0 factors the panels: lane i = row i holds the 6 columns of block b and the right-hand
//     side; column step jj takes the pivot d_jj from lane jj (v_readlane), the multipliers
//     l_ij = S_ij / d_jj, and updates the block's later columns and the right-hand side in
//     registers (forward substitution fused); the panel (l_ij and l_ij d_jj) goes to LDS;
//   * look-ahead: during step b wave 0 applies panel b to block column b + 1 and factors panel
//     b + 1 at once, while waves 1-7 apply panel b to the trailing columns >= 6 (b + 2) (lane =
//     row, wave = every 7th column); one barrier per block step (9 at a full window instead of
//     the 54 of a column-by-column elimination), panels double-buffered;
//   * wave 0 then solves D L^T x = y (x_i by readlane, l_ki from the upper triangle, where the
//     panel wave left them).
// Camera updates R <- cayley(w) R, t <- ... + rho follow.
#define BA_SP 65   // LDS row pitch of S (doubles)
// ---------------------------------------------------------------------------------------------
// Inertial factors (oracle/numpy_ba.py inertial_system): per window-consecutive pair (i, j) =
// (c - 1, c) whose later keyframe carries a factor, the velocity, position and gyro-rotation
// residuals of the IMU preintegration against the cameras, the velocities and the earlier
// keyframe's biases, plus the random walks of both biases between the two keyframes.  Every
// keyframe c has TS_BA_INEY unknowns y_c = (v_c, ba_c, bg_c) (9n in all, block tridiagonal Hyy),
// eliminated into the camera system in LDS:
//   phase 0: factor t (= c - 1) on thread t: r (15), J (15 x 30: rho_i, omega_i, rho_j, omega_j,
//            y_i, y_j), the five row weights;
//   phase 1: per factor (in order, a barrier each), thread (a, b) of J^T W J scatters into S
//            (lower triangle), Hxy or Hyy (packed lower) and 30 threads the gradient into b_x or
//            b_y; then the priors on y_0's biases and lam I on Hyy;
//   phase 2: wave 0 factors Hyy = L L^T (two rows per lane; fill-in stays in the block band);
//   phase 3: thread i < m: Z_i = L^-1 Hxy_i (in place, banded forward substitution); thread m:
//            zb = L^-1 b_y;
//   phase 4: S -= Z Z^T (lower), b_x -= Z zb;
//   after the camera solve (ba_inertial_update): dy = L^-T (zb - Z^T dc) (banded), then every
//   keyframe's velocity and biases move by its dy.
// ---------------------------------------------------------------------------------------------
#define BA_INE_R 15   // residual rows: r_v, r_p, r_R, r_ba, r_bg
#define BA_INE_C 30   // Jacobian columns: rho_i, omega_i, rho_j, omega_j, y_i, y_j
struct BaIneLds {
    double J[TS_BA_MAXW - 1][BA_INE_R][BA_INE_C];
    double r[TS_BA_MAXW - 1][BA_INE_R];
    double w[TS_BA_MAXW - 1][5];
    double Y[TS_BA_MAXY * (TS_BA_MAXY + 1) / 2];   // Hyy (lower, packed by rows), then its Cholesky factor
    double X[TS_BA_MAXD][TS_BA_MAXY + 1];           // row i: Hxy_i, then Z_i = (L^-1 Hyx)^T_i
    double by[TS_BA_MAXY];                          // b_y, then zb = L^-1 b_y, then dy
    double ld[TS_BA_MAXY];                          // 1 / L_yy
    int any, good;
};
__device__ __forceinline__ int ine_yi(int i, int k) { return i * (i + 1) / 2 + k; }   // (i, k <= i)
// last row + 1 of the band of column j (L_ij = 0 for i >= this: Hyy is block tridiagonal)
__device__ __forceinline__ int ine_band_end(int j, int my) { return min(my, TS_BA_INEY * (j / TS_BA_INEY + 2)); }
// first column of the band of row y
__device__ __forceinline__ int ine_band_start(int y) { return max(0, TS_BA_INEY * (y / TS_BA_INEY - 1)); }

template <bool INE>
__device__ __forceinline__ BaIneLds* ine_lds() {
    return nullptr;
}
template <>
__device__ __forceinline__ BaIneLds* ine_lds<true>() {
    __shared__ BaIneLds s;
    return &s;
}

// global unknown of factor t's column col: x index (camera rows without the gauge, -1 = camera 0)
// for col < 12, else y index
__device__ __forceinline__ int ine_col(int t, int col) {
    const int c = t + 1;
    if (col < 6) return c - 1 >= 1 ? 6 * (c - 2) + col : -1;
    if (col < 12) return 6 * (c - 1) + col - 6;
    if (col < 21) return TS_BA_INEY * (c - 1) + col - 12;
    return TS_BA_INEY * c + col - 21;
}

// 3x3 row-major helpers (in-kernel: registers)
__device__ __forceinline__ void ine_mv(const double* M, const double* x, double* y) {
    for (int r = 0; r < 3; ++r) y[r] = (M[3 * r] * x[0] + M[3 * r + 1] * x[1]) + M[3 * r + 2] * x[2];
}

// phases 0-4; returns whether any factor acts (block-uniform)
__device__ bool ba_inertial_reduce(const BaPair& q, const BaArgs& a, int n, int m, double* s_S, double* s_x, BaIneLds* L) {
#pragma clang fp contract(fast)
    const int tid = threadIdx.x, nthr = blockDim.x;
    const int nf = n - 1, my = TS_BA_INEY * n;
    if (tid < 5 * nf) {   // phase 0: thread (t, grp) = factor t's row group grp (r_v, r_p, r_R, r_ba, r_bg)
        const int t = tid / 5, grp = tid - 5 * t, c = t + 1;
        const double* f = q.ine + (size_t)a.order[c] * TS_BA_INE;
        const bool on = f[28] > 0.0;
        double (*J)[BA_INE_C] = L->J[t] + 3 * grp;   // this group's 3 rows
        double* rr = L->r[t] + 3 * grp;
        for (int r = 0; r < 3; ++r) {
            rr[r] = 0.0;
            for (int k = 0; k < BA_INE_C; ++k) J[r][k] = 0.0;
        }
        const int wi[5] = {28, 29, 30, 31, 71};
        L->w[t][grp] = on ? f[wi[grp]] : 0.0;
        if (on) {
            const double* Ti = q.T + (size_t)a.order[c - 1] * 16;
            const double* Tj = q.T + (size_t)a.order[c] * 16;
            const double* bi = q.bias + (size_t)a.order[c - 1] * 6;
            const double* bj = q.bias + (size_t)a.order[c] * 6;
            const double dt = f[27];
            double dbg[3];
            for (int k = 0; k < 3; ++k) dbg[k] = bi[3 + k] - f[68 + k];
            if (grp <= 1) {   // r_v / r_p: R_i u - (d + J_a dba + J_g dbg)
                const double* vi = q.vel + (size_t)a.order[c - 1] * 3;
                const double* vj = q.vel + (size_t)a.order[c] * 3;
                double dba[3], u[3];
                for (int k = 0; k < 3; ++k) dba[k] = bi[k] - f[24 + k];
                for (int k = 0; k < 3; ++k) {
                    const double g = a.icfg[k];
                    if (grp == 0) {
                        u[k] = ((vj[k] - vi[k]) - g * dt);
                    } else {
                        const double pik = -((Ti[k] * Ti[3] + Ti[4 + k] * Ti[7]) + Ti[8 + k] * Ti[11]);
                        const double pjk = -((Tj[k] * Tj[3] + Tj[4 + k] * Tj[7]) + Tj[8 + k] * Tj[11]);
                        u[k] = (((pjk - pik) - vi[k] * dt) - 0.5 * g * dt * dt);
                    }
                }
                double ru[3], ja[3], jg[3];
                for (int r = 0; r < 3; ++r) ru[r] = (Ti[4 * r] * u[0] + Ti[4 * r + 1] * u[1]) + Ti[4 * r + 2] * u[2];
                const double* Ja = f + (grp == 0 ? 6 : 15);
                const double* Jg = f + (grp == 0 ? 50 : 59);
                ine_mv(Ja, dba, ja);
                ine_mv(Jg, dbg, jg);
                for (int r = 0; r < 3; ++r) rr[r] = ru[r] - ((f[3 * grp + r] + ja[r]) + jg[r]);
                // -[ru]x rows: (0, a2, -a1), (-a2, 0, a0), (a1, -a0, 0)
                const double sk[3][3] = {{0.0, ru[2], -ru[1]}, {-ru[2], 0.0, ru[0]}, {ru[1], -ru[0], 0.0}};
                for (int r = 0; r < 3; ++r)
                    for (int k = 0; k < 3; ++k) {
                        const double Rrk = Ti[4 * r + k];
                        J[r][3 + k] = sk[r][k];
                        J[r][15 + k] = -Ja[3 * r + k];
                        J[r][18 + k] = -Jg[3 * r + k];
                        if (grp == 0) {
                            J[r][12 + k] = -Rrk;
                            J[r][21 + k] = Rrk;
                        } else {
                            J[r][k] = r == k ? 1.0 : 0.0;
                            // -R_cw,i R_cw,j^T
                            J[r][6 + k] = -((Ti[4 * r] * Tj[4 * k] + Ti[4 * r + 1] * Tj[4 * k + 1]) + Ti[4 * r + 2] * Tj[4 * k + 2]);
                            J[r][12 + k] = -Rrk * dt;
                        }
                    }
            } else if (grp == 2) {   // r_R = vee-asym(M^T Q) + JRe dbg, Q = R_j R_i^T
                double Qm[9], A[9], jr[3];
                for (int r = 0; r < 3; ++r)
                    for (int k = 0; k < 3; ++k)
                        Qm[3 * r + k] = (Tj[4 * r] * Ti[4 * k] + Tj[4 * r + 1] * Ti[4 * k + 1]) + Tj[4 * r + 2] * Ti[4 * k + 2];
                for (int r = 0; r < 3; ++r)
                    for (int k = 0; k < 3; ++k)
                        A[3 * r + k] = (f[32 + r] * Qm[k] + f[35 + r] * Qm[3 + k]) + f[38 + r] * Qm[6 + k];
                ine_mv(f + 41, dbg, jr);
                rr[0] = 0.5 * (A[7] - A[5]) + jr[0];
                rr[1] = 0.5 * (A[2] - A[6]) + jr[1];
                rr[2] = 0.5 * (A[3] - A[1]) + jr[2];
                for (int r = 0; r < 3; ++r)
                    for (int k = 0; k < 3; ++k) {
                        J[r][3 + k] = r == k ? -1.0 : 0.0;
                        J[r][9 + k] = Qm[3 * k + r];   // Q^T
                        J[r][18 + k] = f[41 + 3 * r + k];
                    }
            } else {   // random walk of the accelerometer (grp 3) / gyroscope (grp 4) bias
                const int o = grp == 3 ? 0 : 3, col = grp == 3 ? 15 : 18;
                for (int r = 0; r < 3; ++r) {
                    rr[r] = bj[o + r] - bi[o + r];
                    J[r][col + r] = -1.0;
                    J[r][col + 9 + r] = 1.0;
                }
            }
        }
    }
    for (int e = tid; e < TS_BA_MAXY * (TS_BA_MAXY + 1) / 2; e += nthr) L->Y[e] = 0.0;
    for (int e = tid; e < TS_BA_MAXD * (TS_BA_MAXY + 1); e += nthr) (&L->X[0][0])[e] = 0.0;
    if (tid < TS_BA_MAXY) L->by[tid] = 0.0;
    __syncthreads();
    if (tid == 0) {
        int any = 0;
        for (int t = 0; t < nf; ++t) any |= L->w[t][0] > 0.0;
        L->any = any;
    }
    __syncthreads();
    if (!L->any) return false;
    for (int t = 0; t < nf; ++t) {   // phase 1, one factor at a time
        if (!(L->w[t][0] > 0.0)) continue;   // (uniform)
        const double (*J)[BA_INE_C] = L->J[t];
        const double* wt = L->w[t];
        for (int e = tid; e < BA_INE_C * BA_INE_C + BA_INE_C; e += nthr) {
            if (e < BA_INE_C * BA_INE_C) {
                const int ca = e / BA_INE_C, cb = e - BA_INE_C * ca;
                const int ga = ine_col(t, ca), gb = ine_col(t, cb);
                const bool xa = ca < 12, xb = cb < 12;
                if (ga < 0 || gb < 0) continue;        // the gauge camera's columns
                if (xa && xb && ga < gb) continue;     // S: lower triangle
                if (!xa && xb) continue;               // Hyx: from (b, a)
                if (!xa && !xb && ga < gb) continue;   // Hyy: lower triangle
                double h = 0.0;
#pragma unroll
                for (int g5 = 0; g5 < 5; ++g5) {
                    const double wg = wt[g5];
                    h += (wg * (J[3 * g5][ca] * J[3 * g5][cb]) + wg * (J[3 * g5 + 1][ca] * J[3 * g5 + 1][cb])) +
                         wg * (J[3 * g5 + 2][ca] * J[3 * g5 + 2][cb]);
                }
                if (xa && xb) s_S[ga * BA_SP + gb] += h;
                else if (xa) L->X[ga][gb] += h;
                else L->Y[ine_yi(ga, gb)] += h;
            } else {
                const int ca = e - BA_INE_C * BA_INE_C;
                const int ga = ine_col(t, ca);
                if (ga < 0) continue;
                double gsum = 0.0;
#pragma unroll
                for (int rr = 0; rr < BA_INE_R; ++rr) gsum += wt[rr / 3] * (J[rr][ca] * L->r[t][rr]);
                if (ca < 12) s_x[ga] -= gsum;
                else L->by[ga] -= gsum;
            }
        }
        __syncthreads();
    }
    if (tid < my) {   // the priors on the oldest keyframe's biases, lam on every y unknown
        L->Y[ine_yi(tid, tid)] += a.lam;
        const double* b0 = q.bias + (size_t)a.order[0] * 6;
        if (tid >= 3 && tid < 6) {
            L->Y[ine_yi(tid, tid)] += a.icfg[6];
            L->by[tid] -= a.icfg[6] * (b0[tid - 3] - a.icfg[tid]);
        } else if (tid >= 6 && tid < 9) {
            L->Y[ine_yi(tid, tid)] += a.icfg[10];
            L->by[tid] -= a.icfg[10] * (b0[tid - 3] - a.icfg[tid + 1]);
        }
    }
    __syncthreads();
    if (tid < 64) {   // phase 2: wave 0, rows lane and lane + 64
        bool good = true;
        for (int j = 0; j < my; ++j) {
            const int iend = ine_band_end(j, my);
            const double d = L->Y[ine_yi(j, j)];
            good = good && d > 0.0;
            const double l = sqrt(d), inv = 1.0 / l;
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            for (int i = tid; i < TS_BA_MAXY; i += 64) {
                if (i > j && i < iend) L->Y[ine_yi(i, j)] *= inv;
                if (i == j) {
                    L->Y[ine_yi(j, j)] = l;
                    L->ld[j] = inv;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            for (int i = tid; i < TS_BA_MAXY; i += 64) {
                if (i > j && i < iend) {
                    const double lij = L->Y[ine_yi(i, j)];
                    for (int k = j + 1; k <= i; ++k) L->Y[ine_yi(i, k)] -= lij * L->Y[ine_yi(k, j)];
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        }
        if (tid == 0) L->good = good;
    }
    __syncthreads();
    if (tid <= m) {   // phase 3: banded forward substitutions (thread m: the right-hand side)
        double* z = tid < m ? L->X[tid] : L->by;
        for (int y = 0; y < my; ++y) {
            double v = z[y];
            for (int k = ine_band_start(y); k < y; ++k) v -= L->Y[ine_yi(y, k)] * z[k];
            z[y] = v * L->ld[y];
        }
    }
    __syncthreads();
    for (int e = tid; e < m * m + m; e += nthr) {   // phase 4
        if (e < m * m) {
            const int i = e / m, k = e - m * i;
            if (k > i) continue;
            double sum = 0.0;
            for (int y = 0; y < my; ++y) sum += L->X[i][y] * L->X[k][y];
            s_S[i * BA_SP + k] -= sum;
        } else {
            const int i = e - m * m;
            double sum = 0.0;
            for (int y = 0; y < my; ++y) sum += L->X[i][y] * L->by[y];
            s_x[i] -= sum;
        }
    }
    __syncthreads();
    return true;
}

// after the camera solve (dc = s_x[0 .. m)): dy = L^-T (zb - Z^T dc); every keyframe's velocity
// and biases move by its dy
__device__ void ba_inertial_update(const BaPair& q, const BaArgs& a, int n, int m, const double* s_x, BaIneLds* L) {
#pragma clang fp contract(fast)
    const int tid = threadIdx.x, my = TS_BA_INEY * n;
    if (tid < my) {
        double v = L->by[tid];
        for (int i = 0; i < m; ++i) v -= L->X[i][tid] * s_x[i];
        L->by[tid] = v;
    }
    __syncthreads();
    if (tid == 0)   // banded back substitution L^T x = by, in place
        for (int y = my - 1; y >= 0; --y) {
            double v = L->by[y];
            const int kend = ine_band_end(y, my);
            for (int k = y + 1; k < kend; ++k) v -= L->Y[ine_yi(k, y)] * L->by[k];
            L->by[y] = v * L->ld[y];
        }
    __syncthreads();
    if (tid < my) {
        const int c = tid / TS_BA_INEY, k = tid - TS_BA_INEY * c;
        const int s = a.order[c];
        if (k < 3) q.vel[(size_t)s * 3 + k] += L->by[tid];
        else q.bias[(size_t)s * 6 + k - 3] += L->by[tid];
    }
}

// `handoff`: C and the camera blocks were published by other workgroups of this launch with
// write-through stores (k_ba_reduce_solve), so they are read with agent-scope loads that bypass
// this CU's caches.
template <bool handoff, bool INE>
__device__ __forceinline__ void ba_solve_block(const BatchCtx& c, const BaArgs& a) {
    // the elimination's a - l * b updates as single FMAs (the library builds with contraction off
    // for the bit-exact pose kernels; this solve is only held to 1e-9 against the oracle's LU)
#pragma clang fp contract(fast)
    static_assert(TS_BA_MAXW * 27 <= 64 * BA_SOLVE_WAVES, "one camera-block load per thread");
    __shared__ double s_S[64 * BA_SP];             // lower: S; upper (row j, column i > j): l_ij
    __shared__ double s_U[TS_BA_MAXW * 27];
    __shared__ double s_iw[TS_BA_MAXW];            // IMU rotation factor weight per window camera
    __shared__ __attribute__((aligned(16))) double s_pl[2][64][6];   // panel multipliers l_ij
    __shared__ __attribute__((aligned(16))) double s_pq[2][64][6];   // l_ij d_j
    __shared__ double s_d[64];
    __shared__ double s_x[64];
    __shared__ int s_ok;
    BaPair q = ba_pair(c, a, a.pair);
    const int n = a.n_order;
    const int m = 6 * (n - 1), nb = n - 1;
    if (q.counts[1] == 0 || n < 2) {
        if (threadIdx.x == 0) q.counts[2] = 0;
        return;
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    BST_DECL;
    // stage C (every thread's 8 loads in flight at once) and the camera blocks
    constexpr int NL = 4096 / (64 * BA_SOLVE_WAVES);
    double cv[NL];
#pragma unroll
    for (int k = 0; k < NL; ++k) {
        const double* src = q.C + threadIdx.x + 64 * BA_SOLVE_WAVES * k;
        cv[k] = handoff ? __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *src;
    }
    if ((int)threadIdx.x < n * 27)
        s_U[threadIdx.x] = handoff ? __hip_atomic_load(q.cam_U + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                   : q.cam_U[threadIdx.x];
    if ((int)threadIdx.x < n) s_iw[threadIdx.x] = q.imu[(size_t)a.order[threadIdx.x] * 10 + 9];   // factor weights
    __syncthreads();
    BST(0);
    // S_ik = -C[i+6][k+6] (+ U + lam inside a camera block), lower triangle; row i's right-hand
    // side -g_c + C[i+6][60] into s_x[i] (read back by wave 0)
#pragma unroll
    for (int k8 = 0; k8 < NL; ++k8) {
        const int e = threadIdx.x + 64 * BA_SOLVE_WAVES * k8;
        const int R = e >> 6, Cc = e & 63;
        const int i = R - 6, k = Cc - 6;
        if (i < 0 || i >= m) continue;
        if (Cc == 60) {
            s_x[i] = -s_U[(R / 6) * 27 + 21 + R % 6] + cv[k8];
            continue;
        }
        if (k < 0 || k > i) continue;
        double v = -cv[k8];
        if (R / 6 == Cc / 6) {
            const int ci = R / 6, i0 = R % 6, j0 = Cc % 6;
            const int lo = min(i0, j0), hi = max(i0, j0);
            v += s_U[ci * 27 + lo * 6 - lo * (lo - 1) / 2 + (hi - lo)] + (i0 == j0 ? a.lam : 0.0);
        }
        s_S[i * BA_SP + k] = v;
    }
    __syncthreads();
    BST(1);
    bool any_imu = false;
    for (int cc = 1; cc < n; ++cc) any_imu = any_imu || s_iw[cc] > 0.0;   // (uniform: LDS broadcast)
    if (any_imu && threadIdx.x == 0) {
        // IMU rotation factors between window-consecutive keyframes (oracle imu_terms): with
        // Q = R_c R_{c-1}^T, e = vee((A - A^T) / 2), A = M^T Q — S_cc, S_{c-1,c-1} += w I,
        // S_{c,c-1} -= w Q (rotation blocks, lower triangle), b_c -= w Q e, b_{c-1} += w e; camera 0
        // (the gauge) has no rows
        for (int cc = 1; cc < n; ++cc) {
            const double w = s_iw[cc];
            if (!(w > 0.0)) continue;
            const double* f = q.imu + (size_t)a.order[cc] * 10;
            const double* Tc = q.T + (size_t)a.order[cc] * 16;
            const double* Tp = q.T + (size_t)a.order[cc - 1] * 16;
            double Q[9], A[9];
            for (int r = 0; r < 3; ++r)
                for (int k = 0; k < 3; ++k) Q[3 * r + k] = Tc[4 * r] * Tp[4 * k] + Tc[4 * r + 1] * Tp[4 * k + 1] + Tc[4 * r + 2] * Tp[4 * k + 2];
            for (int r = 0; r < 3; ++r)
                for (int k = 0; k < 3; ++k) A[3 * r + k] = f[r] * Q[k] + f[3 + r] * Q[3 + k] + f[6 + r] * Q[6 + k];   // M^T Q
            const double e[3] = {0.5 * (A[7] - A[5]), 0.5 * (A[2] - A[6]), 0.5 * (A[3] - A[1])};
            const int rc = 6 * (cc - 1) + 3, rp = 6 * (cc - 2) + 3;
            for (int r = 0; r < 3; ++r) {
                s_S[(rc + r) * BA_SP + rc + r] += w;
                s_x[rc + r] -= w * ((Q[3 * r] * e[0] + Q[3 * r + 1] * e[1]) + Q[3 * r + 2] * e[2]);
                if (cc >= 2) {
                    s_S[(rp + r) * BA_SP + rp + r] += w;
                    s_x[rp + r] += w * e[r];
                    for (int k = 0; k < 3; ++k) s_S[(rc + r) * BA_SP + rp + k] -= w * Q[3 * r + k];
                }
            }
        }
    }
    if (any_imu) __syncthreads();
    BaIneLds* ine = ine_lds<INE>();
    bool ine_on = false;
    if constexpr (INE) ine_on = ba_inertial_reduce(q, a, n, m, s_S, s_x, ine);
    const bool live = lane < m;
    double rhs = (w == 0 && live) ? s_x[lane] : 0.0;   // wave 0: right-hand side of row `lane`
    bool good = true;   // wave 0: every pivot positive
    double cl[6];       // wave 0: this lane's multipliers of the current panel
    // wave 0: factor panel b from its 6 columns col[] (rows >= 6b current), into buffer b & 1
    auto factor = [&](int b, double* col) {
        const int b6 = 6 * b;
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            const int jj = b6 + j;
            const double d = readlane_f64(col[j], jj);
            good = good && d > 0.0;
            double inv = __builtin_amdgcn_rcp(d);   // + one Newton step (~2^-44..2^-52 relative), off the division chain
            inv = inv * (2.0 - d * inv);
            const double pre = col[j];
            const double l = lane > jj ? pre * inv : 0.0;
#pragma unroll
            for (int k = j + 1; k < 6; ++k) col[k] -= l * readlane_f64(pre, b6 + k);
            rhs -= l * readlane_f64(rhs, jj);
            cl[j] = l;
            s_pl[b & 1][lane][j] = l;
            s_pq[b & 1][lane][j] = lane > jj ? pre : 0.0;
            if (lane > jj && live) s_S[jj * BA_SP + lane] = l;   // upper triangle: for D L^T x = y
            if (lane == jj) s_d[jj] = d;
        }
    };
    if (w == 0) {
        double col[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) col[k] = live ? s_S[lane * BA_SP + k] : 0.0;
        factor(0, col);
    }
    __syncthreads();
    BST(2);
#ifdef TS_BA_STAMPS
    uint64_t ls_work = 0, ls_wait = 0;   // per thread: the block steps' own work and barrier waits
#endif
    for (int b = 0; b < nb; ++b) {
#ifdef TS_BA_STAMPS
        const uint64_t ls_t0 = wall_clock64();
#endif
        const int pb = b & 1;
        if (w == 0) {
            if (b + 1 < nb) {
                // block column b + 1, rows >= 6 (b + 1): apply panel b, then factor it
                const int c0 = 6 * (b + 1);
                double col[6];
#pragma unroll
                for (int k = 0; k < 6; ++k) {
                    const double* qk = s_pq[pb][c0 + k];
                    double s = (lane >= c0 + k && live) ? s_S[lane * BA_SP + c0 + k] : 0.0;
#pragma unroll
                    for (int j = 0; j < 6; ++j) s -= cl[j] * qk[j];
                    col[k] = s;
                }
                factor(b + 1, col);
            }
        } else {
            // trailing columns k >= 6 (b + 2) with panel b: lane = row i, waves 1-7 deal the columns
            const int c0 = 6 * (b + 2);
            const int i = lane;
            if (i >= c0 && i < m) {
                double li[6];
#pragma unroll
                for (int j = 0; j < 6; ++j) li[j] = s_pl[pb][i][j];
                // two columns per iteration, so their LDS reads are in flight together
                int k = c0 + (w - 1);
                for (; k + (BA_SOLVE_WAVES - 1) <= i; k += 2 * (BA_SOLVE_WAVES - 1)) {
                    const int k2 = k + (BA_SOLVE_WAVES - 1);
                    const double* qa = s_pq[pb][k];
                    const double* qb = s_pq[pb][k2];
                    double sa = s_S[i * BA_SP + k], sb = s_S[i * BA_SP + k2];
#pragma unroll
                    for (int j = 0; j < 6; ++j) {
                        sa -= li[j] * qa[j];
                        sb -= li[j] * qb[j];
                    }
                    s_S[i * BA_SP + k] = sa;
                    s_S[i * BA_SP + k2] = sb;
                }
                if (k <= i) {
                    const double* qk = s_pq[pb][k];
                    double sa = s_S[i * BA_SP + k];
#pragma unroll
                    for (int j = 0; j < 6; ++j) sa -= li[j] * qk[j];
                    s_S[i * BA_SP + k] = sa;
                }
            }
        }
#ifdef TS_BA_STAMPS
        const uint64_t ls_t1 = wall_clock64();
        ls_work += ls_t1 - ls_t0;
#endif
        __syncthreads();
#ifdef TS_BA_STAMPS
        ls_wait += wall_clock64() - ls_t1;
#endif
    }
    BST(3);
    if (w == 0) {
        // D L^T x = y: x_i = y_i / d_i - sum_{k > i} l_ki x_k (the row's l_ki preloaded, so the
        // chain is readlane -> FMA only)
        double lr[TS_BA_MAXD];
#pragma unroll
        for (int k = 0; k < TS_BA_MAXD; ++k) lr[k] = (lane < k && k < m) ? s_S[lane * BA_SP + k] : 0.0;
        double x = live ? rhs / s_d[lane] : 0.0;
#pragma unroll
        for (int i2 = TS_BA_MAXD - 1; i2 > 0; --i2) {
            if (i2 >= m) continue;   // uniform
            const double xi = readlane_f64(x, i2);
            x -= lr[i2] * xi;
        }
        s_x[lane] = x;
        if (lane == 0) s_ok = good;
    }
    __syncthreads();
    BST(4);
    const bool good_all = s_ok != 0;
    const bool ok = good_all && (!ine_on || ine->good);
    if (threadIdx.x == 0) q.counts[2] = ok;
    for (int e = threadIdx.x; e < 6 * n; e += blockDim.x) q.dc[e] = (e < 6 || !ok) ? 0.0 : s_x[e - 6];
    if (ok && (int)threadIdx.x >= 1 && (int)threadIdx.x < n) {
        const int cj = threadIdx.x;
        const double* x = s_x + 6 * (cj - 1);
        const double w0 = x[3], w1 = x[4], w2 = x[5];
        const double A[9] = {0.0, -w2, w1, w2, 0.0, -w0, -w1, w0, 0.0};
        double A2[9];
        for (int ii = 0; ii < 3; ++ii)
            for (int jj = 0; jj < 3; ++jj) A2[3 * ii + jj] = (A[3 * ii] * A[jj] + A[3 * ii + 1] * A[3 + jj]) + A[3 * ii + 2] * A[6 + jj];
        const double n2 = (w0 * w0 + w1 * w1) + w2 * w2;
        const double sc = 4.0 / (4.0 + n2);
        double RU[9];
        for (int e = 0; e < 9; ++e) RU[e] = ((e % 4) == 0 ? 1.0 : 0.0) + sc * (A[e] + 0.5 * A2[e]);
        double* T = q.T + (size_t)a.order[cj] * 16;
        double Rn[9], tn[3];
        for (int ii = 0; ii < 3; ++ii) {
            for (int jj = 0; jj < 3; ++jj) Rn[3 * ii + jj] = (RU[3 * ii] * T[jj] + RU[3 * ii + 1] * T[4 + jj]) + RU[3 * ii + 2] * T[8 + jj];
            tn[ii] = ((RU[3 * ii] * T[3] + RU[3 * ii + 1] * T[7]) + RU[3 * ii + 2] * T[11]) + x[ii];
        }
        for (int ii = 0; ii < 3; ++ii) {
            for (int jj = 0; jj < 3; ++jj) T[4 * ii + jj] = Rn[3 * ii + jj];
            T[4 * ii + 3] = tn[ii];
        }
    }
    if constexpr (INE)
        if (ine_on && ok) ba_inertial_update(q, a, n, m, s_x, ine);
    BST(5);
    BST_PRINT("solve: stage C, build S, panel 0, block steps, backsub, update, -, -", threadIdx.x == 1);
#ifdef TS_BA_STAMPS
    if (threadIdx.x == 0 || threadIdx.x == 64 || threadIdx.x == 448)
        printf("solve steps thread %d: work %lu wait %lu (x10ns)\n", (int)threadIdx.x, ls_work, ls_wait);
#endif
}

__device__ __forceinline__ void d_ba_solve(const BatchCtx& c, const BaArgs& a) {
    BA_PRIO;
    ba_solve_block<false, false>(c, a);
}
__global__ __launch_bounds__(64 * BA_SOLVE_WAVES) void k_ba_solve(BatchCtx c, BaArgs a) { d_ba_solve(c, a); }
__global__ __launch_bounds__(64 * BA_SOLVE_WAVES) void k_ba_solve_rec(BaCtxRef c, BaArgsRef a) {
    d_ba_solve(*(const BatchCtx*)c, *(const BaArgs*)a);
}

__device__ __forceinline__ void d_ba_solve_ine(const BatchCtx& c, const BaArgs& a) {
    BA_PRIO;
    ba_solve_block<false, true>(c, a);
}
__global__ __launch_bounds__(64 * BA_SOLVE_WAVES) void k_ba_solve_ine(BatchCtx c, BaArgs a) { d_ba_solve_ine(c, a); }
__global__ __launch_bounds__(64 * BA_SOLVE_WAVES) void k_ba_solve_ine_rec(BaCtxRef c, BaArgsRef a) {
    d_ba_solve_ine(*(const BatchCtx*)c, *(const BaArgs*)a);
}

// k_ba_reduce and k_ba_solve in one launch (a stereo pair's own solve): the reduction's blocks
// (k_ba_reduce's fixed order, waves 0-3) publish their sums with write-through (agent-scope)
// stores, drain them (vmcnt(0)) and count themselves in; the block that arrives last runs the
// solve, reading the sums with agent-scope loads.  No agent-scope release fence: on this GPU it
// writes back the whole L2 of the XCD (the iteration's Schur partials and Jacobian blocks), which
// cost more than the launch it saves (measured: 0.300 against 0.260 ms per keyframe).
template <bool INE>
__device__ __forceinline__ void ba_reduce_solve_body(const BatchCtx& c, const BaArgs& a) {
    // all BA_SOLVE_WAVES waves sum (every 8th partial each), then the 8 wave sums in order
    __shared__ double s_p[BA_SOLVE_WAVES][64];
    __shared__ int s_last;
    BaPair q = ba_pair(c, a, a.pair);
    const int e = blockIdx.x * 64 + (threadIdx.x & 63);
    const bool live = e < 4096 + a.n_order * 27;
    const double v = ba_reduce_elem(q, a, e, live, s_p);
    if ((threadIdx.x >> 6) == 0 && live)
        __hip_atomic_store(e < 4096 ? q.C + e : q.cam_U + (e - 4096), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the write-through stores have landed
    __syncthreads();
    if (threadIdx.x == 0)
        s_last = __hip_atomic_fetch_add(q.done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1;
    __syncthreads();
    if (!s_last) return;
    if (threadIdx.x == 0) __hip_atomic_store(q.done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // next launch
    ba_solve_block<true, INE>(c, a);
}

__device__ __forceinline__ void d_ba_reduce_solve(const BatchCtx& c, const BaArgs& a) {
    BA_PRIO;
    ba_reduce_solve_body<false>(c, a);
}
__global__ __launch_bounds__(64 * BA_SOLVE_WAVES) void k_ba_reduce_solve(BatchCtx c, BaArgs a) { d_ba_reduce_solve(c, a); }
__global__ __launch_bounds__(64 * BA_SOLVE_WAVES) void k_ba_reduce_solve_rec(BaCtxRef c, BaArgsRef a) {
    d_ba_reduce_solve(*(const BatchCtx*)c, *(const BaArgs*)a);
}

// with the window's inertial factors (velocities + accelerometer bias eliminated into S)
__device__ __forceinline__ void d_ba_reduce_solve_ine(const BatchCtx& c, const BaArgs& a) {
    BA_PRIO;
    ba_reduce_solve_body<true>(c, a);
}
__global__ __launch_bounds__(64 * BA_SOLVE_WAVES) void k_ba_reduce_solve_ine(BatchCtx c, BaArgs a) { d_ba_reduce_solve_ine(c, a); }
__global__ __launch_bounds__(64 * BA_SOLVE_WAVES) void k_ba_reduce_solve_ine_rec(BaCtxRef c, BaArgsRef a) {
    d_ba_reduce_solve_ine(*(const BatchCtx*)c, *(const BaArgs*)a);
}


// The last iteration's landmark update and the write-back of the window's landmarks: 16 lanes
// per landmark (lane = window camera): W_o^T dc_o of each observation (slot table), summed over
// the 16 lanes by a fixed xor-butterfly; the first lane then solves dp = V^-1 (-g_p - sum) with
// the stored Cholesky factor and stores X[lm_id[r]] = Xc[r] + dp (Xc[r] alone when the last
// solve failed).
__device__ __forceinline__ void d_ba_backsub(const BatchCtx& c, const BaArgs& a) {
    BA_PRIO;
    const int WK = a.W * c.g.K;
    BaPair q = ba_pair(c, a, a.pair);
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid < WK) q.cnt[gid] = 0;   // the gate counts, for the next solve (the tile kernels have run)
    const int r = gid >> 4, ci = gid & 15;
    const int L = q.counts[1];
    if ((r & ~15) >= L) return;   // whole 16-landmark groups exit together
    const bool live = r < L;
    const bool upd = q.counts[2] != 0;
    const int rc = min(r, L - 1);
    const size_t sl = (size_t)rc * TS_BA_MAXW + min(ci, TS_BA_MAXW - 1);
    const int o = upd && ci >= 1 && ci < a.n_order ? q.lo_o[sl] : -1;   // dc of camera 0 is zero
    const double* W = q.lo_W + sl * 18;
    double wv[18];
#pragma unroll
    for (int e = 0; e < 18; ++e) wv[e] = W[e];
    const double* dc = q.dc + 6 * min(ci, TS_BA_MAXW - 1);
    double t[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        double acc = 0.0;
#pragma unroll
        for (int i = 0; i < 6; ++i) acc += wv[3 * i + j] * dc[i];
        t[j] = o >= 0 ? acc : 0.0;
    }
#pragma unroll
    for (int sh = 8; sh > 0; sh >>= 1)
#pragma unroll
        for (int j = 0; j < 3; ++j) t[j] += __shfl_xor(t[j], sh, 64);
    if (ci != 0 || !live) return;
    double x[3] = {0.0, 0.0, 0.0};
    if (upd) {
        double rhs[3];
        for (int i = 0; i < 3; ++i) rhs[i] = -q.lm_gp[(size_t)i * WK + r] - t[i];
        double Lm[3][3] = {{q.lm_L[r], 0.0, 0.0}, {q.lm_L[(size_t)WK + r], q.lm_L[(size_t)2 * WK + r], 0.0},
                           {q.lm_L[(size_t)3 * WK + r], q.lm_L[(size_t)4 * WK + r], q.lm_L[(size_t)5 * WK + r]}};
        double y[3];
        for (int i = 0; i < 3; ++i) {
            double v = rhs[i];
            for (int k = 0; k < i; ++k) v -= Lm[i][k] * y[k];
            y[i] = v * Lm[i][i];   // the diagonal is stored inverted
        }
        for (int i = 2; i >= 0; --i) {
            double v = y[i];
            for (int k = i + 1; k < 3; ++k) v -= Lm[k][i] * x[k];
            x[i] = v * Lm[i][i];
        }
    }
    const int id = q.lm_id[r];
    for (int i = 0; i < 3; ++i) q.X[(size_t)id * 3 + i] = upd ? q.Xc[(size_t)r * 3 + i] + x[i] : q.Xc[(size_t)r * 3 + i];
}
__global__ __launch_bounds__(256) void k_ba_backsub(BatchCtx c, BaArgs a) { d_ba_backsub(c, a); }
__global__ __launch_bounds__(256) void k_ba_backsub_rec(BaCtxRef c, BaArgsRef a) {
    d_ba_backsub(*(const BatchCtx*)c, *(const BaArgs*)a);
}

// ---------------------------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------------------------
// The batch's front-end poses (T_abs) copied out of the per-batch pose buffer on the front-end
// stream, so the BA of this batch may run on another stream while the next batch reuses it.
__global__ __launch_bounds__(256) void k_ba_snapshot(BatchCtx c, double* dst) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= c.n * c.P * 16) return;
    dst[i] = c.pose[(size_t)(i / 16) * TS_POSE_DOUBLES + 16 + i % 16];
}

void launch_ba_snapshot(const BatchCtx& c, double* dst, hipStream_t s) {
    hipLaunchKernelGGL(k_ba_snapshot, dim3((c.n * c.P * 16 + 255) / 256), dim3(256), 0, s, c, dst);
}

// Keypoint k of every keyframe g (g % iv == 0) of the batch chained through the temporal matches
// of frames g, g - 1, .., g - iv + 1 to its keypoint in frame g - iv (-1 where a link is missing):
// the association k_ba_insert_gate needs, computed on the stream of the batch's last stage beside
// the pose snapshot, so the BA chain itself starts from one load instead of iv dependent ones.
__global__ __launch_bounds__(256) void k_ba_kf_assoc(BatchCtx c, int32_t* dst, int iv) {
    const int K = c.g.K;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= c.n * c.P * K) return;
    const int f = i / (c.P * K), r = i - f * c.P * K, p = r / K, k = r - p * K;
    const int64_t g = c.g0 + f;
    if (g % iv != 0) return;
    int j = k;
    for (int st = 0; st < iv && j >= 0; ++st) j = c.temporal[((size_t)ring_slot(c, g - st) * c.P + p) * K + j];
    dst[i] = j;
}

void launch_ba_kf_assoc(const BatchCtx& c, int32_t* dst, int iv, hipStream_t s) {
    hipLaunchKernelGGL(k_ba_kf_assoc, dim3((c.n * c.P * c.g.K + 255) / 256), dim3(256), 0, s, c, dst, iv);
}

void launch_ba_keyframe(const BatchCtx& c, const BaArgs& a, bool evict, hipStream_t s) {
    const int K = c.g.K;
    if (evict) {   // the insertion itself is the first launch of the solve (k_ba_insert_gate)
        const int nb = (a.n_order * K + 255) / 256;
        hipLaunchKernelGGL(k_ba_evict_min, dim3(nb), dim3(256), 0, s, c, a);
        hipLaunchKernelGGL(k_ba_evict_move, dim3(nb), dim3(256), 0, s, c, a);
    }
}

void launch_ba_schur(const BatchCtx& c, const BaArgs& a, hipStream_t s) {
    BaArgs ai = a;
    ai.fused_backsub = 0;   // a replay must not move the landmarks
    hipLaunchKernelGGL(k_ba_schur, dim3(a.nsplit), dim3(BA_SCHUR_THREADS), 0, s, c, ai);
}

// A solve's observation set of pair a.pair (gate, compaction, slot table).
static void launch_ba_prepare(const BatchCtx& c, const BaArgs& a, hipStream_t s) {
    // grids sized for the window's maximum (counts live on the device; threads past them exit)
    const int WK = a.W * c.g.K;
    hipLaunchKernelGGL(k_ba_insert_gate, dim3((a.n_order * c.g.K + 255) / 256), dim3(256), 0, s, c, a);
    const int ntiles = (WK + BA_TILE - 1) / BA_TILE + a.n_order * ((c.g.K + BA_TILE - 1) / BA_TILE);
    hipLaunchKernelGGL(k_ba_tilecount, dim3(ntiles), dim3(256), 0, s, c, a);
    hipLaunchKernelGGL(k_ba_tilescatter, dim3(ntiles), dim3(256), 0, s, c, a);
}

// One linearisation of pair a.pair: the Schur pass (+ iteration it - 1's landmark update when
// `it` > 0) and the reduction to C, U_c, g_c.
static void launch_ba_linearize(const BatchCtx& c, const BaArgs& a, int it, hipStream_t s, BaTiming* timing,
                                bool reduce = true) {
    BaArgs ai = a;
    const bool rec = timing && timing->used < timing->cap;
    ai.fused_backsub = it > 0;   // iteration it - 1's landmark update happens inside this Schur pass
    if (rec) (void)hipEventRecord(timing->ev[2 * timing->used], s);
    hipLaunchKernelGGL(k_ba_schur, dim3(a.nsplit), dim3(BA_SCHUR_THREADS), 0, s, c, ai);
    if (rec) (void)hipEventRecord(timing->ev[2 * timing->used++ + 1], s);
    if (!reduce) return;   // k_ba_reduce_solve follows
    hipLaunchKernelGGL(k_ba_reduce, dim3(64 + (a.n_order * 27 + 63) / 64), dim3(64 * BA_SOLVE_WAVES), 0, s, c, a);
}

static void launch_ba_backsub(const BatchCtx& c, const BaArgs& a, hipStream_t s) {
    const int nb = (a.W * c.g.K + 255) / 256;
    hipLaunchKernelGGL(k_ba_backsub, dim3(16 * nb), dim3(256), 0, s, c, a);   // the last iteration's
}

void launch_ba_solve(const BatchCtx& c, const BaArgs& a, hipStream_t s, BaTiming* timing, bool split, bool inertial) {
    launch_ba_prepare(c, a, s);
    const dim3 grid(64 + (a.n_order * 27 + 63) / 64), block(64 * BA_SOLVE_WAVES);
    for (int it = 0; it < a.iters; ++it) {
        launch_ba_linearize(c, a, it, s, timing, split);
        if (split)   // the kernel boundary instead of the in-launch hand-off (tslam_ba_split_solve)
            hipLaunchKernelGGL(inertial ? k_ba_solve_ine : k_ba_solve, dim3(1), block, 0, s, c, a);
        else
            hipLaunchKernelGGL(inertial ? k_ba_reduce_solve_ine : k_ba_reduce_solve, grid, block, 0, s, c, a);
    }
    launch_ba_backsub(c, a, s);
}

// ---------------------------------------------------------------------------------------------
// the keyframe chain by record (graph replays, tslam_api.cpp ba_chain)
// ---------------------------------------------------------------------------------------------
struct BaRecWords {
    uint64_t w[(sizeof(BaRec) + 7) / 8];
};
static_assert(sizeof(BaRecWords) + sizeof(void*) <= 4096, "k_ba_setrec's record must fit the kernel arguments");

__global__ __launch_bounds__(64) void k_ba_setrec(BaRecWords r, BaRecWords* d) {
    for (int i = threadIdx.x; i < (int)(sizeof(BaRecWords) / 8); i += 64) d->w[i] = r.w[i];
}

void launch_ba_setrec(const BaRec& r, BaRec* d, hipStream_t s) {
    BaRecWords w{};
    memcpy(&w, &r, sizeof(BaRec));
    hipLaunchKernelGGL(k_ba_setrec, dim3(1), dim3(64), 0, s, w, reinterpret_cast<BaRecWords*>(d));
}

hipError_t ba_graph_set_record(hipGraphExec_t exec, hipGraphNode_t node, const BaRec& r, BaRec* d) {
    BaRecWords w{};
    memcpy(&w, &r, sizeof(BaRec));
    BaRecWords* dw = reinterpret_cast<BaRecWords*>(d);
    void* args[] = {&w, &dw};
    hipKernelNodeParams p{};
    p.func = reinterpret_cast<void*>(k_ba_setrec);
    p.gridDim = dim3(1);
    p.blockDim = dim3(64);
    p.sharedMemBytes = 0;
    p.kernelParams = args;
    p.extra = nullptr;
    return hipGraphExecKernelNodeSetParams(exec, node, &p);
}

void launch_ba_chain_rec(const BaRec& r, const BaRec* d, bool evict, bool split, bool inertial, hipStream_t s) {
    const BaCtxRef c = (BaCtxRef)&d->c;
    const BaArgsRef a = (BaArgsRef)&d->a;
    const BaArgsRef ev = (BaArgsRef)&d->evict;
    const int K = r.c.g.K;
    if (evict) {
        const int nb = (r.evict.n_order * K + 255) / 256;
        hipLaunchKernelGGL(k_ba_evict_min_rec, dim3(nb), dim3(256), 0, s, c, ev);
        hipLaunchKernelGGL(k_ba_evict_move_rec, dim3(nb), dim3(256), 0, s, c, ev);
    }
    const BaArgs& ha = r.a;
    const int WK = ha.W * K;
    hipLaunchKernelGGL(k_ba_insert_gate_rec, dim3((ha.n_order * K + 255) / 256), dim3(256), 0, s, c, a);
    const int ntiles = (WK + BA_TILE - 1) / BA_TILE + ha.n_order * ((K + BA_TILE - 1) / BA_TILE);
    hipLaunchKernelGGL(k_ba_tilecount_rec, dim3(ntiles), dim3(256), 0, s, c, a);
    hipLaunchKernelGGL(k_ba_tilescatter_rec, dim3(ntiles), dim3(256), 0, s, c, a);
    const dim3 grid(64 + (ha.n_order * 27 + 63) / 64), block(64 * BA_SOLVE_WAVES);
    for (int it = 0; it < ha.iters; ++it) {
        hipLaunchKernelGGL(k_ba_schur_rec, dim3(ha.nsplit), dim3(BA_SCHUR_THREADS), 0, s, c, a, it > 0 ? 1 : 0);
        if (split) {
            hipLaunchKernelGGL(k_ba_reduce_rec, grid, block, 0, s, c, a);
            hipLaunchKernelGGL(inertial ? k_ba_solve_ine_rec : k_ba_solve_rec, dim3(1), block, 0, s, c, a);
        } else {
            hipLaunchKernelGGL(inertial ? k_ba_reduce_solve_ine_rec : k_ba_reduce_solve_rec, grid, block, 0, s, c, a);
        }
    }
    hipLaunchKernelGGL(k_ba_backsub_rec, dim3(16 * ((WK + 255) / 256)), dim3(256), 0, s, c, a);
}

// ---------------------------------------------------------------------------------------------
// rig-level A8 (oracle RigKeyframeWindow): one body pose per keyframe, storage pair c.P
// ---------------------------------------------------------------------------------------------
// Adjoint of rigid T = [R | t] for left perturbations in (rho, omega) order:
// (I + (Ad d)^) T = T (I + d^), Ad = [[R, [t]x R], [0, R]].
__device__ __forceinline__ void adjoint_rl(const double* T, double A[6][6]) {
    const double t0 = T[3], t1 = T[7], t2 = T[11];
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) A[i][j] = 0.0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            A[i][j] = T[4 * i + j];
            A[3 + i][3 + j] = T[4 * i + j];
        }
    // [t]x R: row 0 = -t2 R1 + t1 R2, row 1 = t2 R0 - t0 R2, row 2 = -t1 R0 + t0 R1
    for (int j = 0; j < 3; ++j) {
        const double r0 = T[j], r1 = T[4 + j], r2 = T[8 + j];
        A[0][3 + j] = -t2 * r1 + t1 * r2;
        A[1][3 + j] = t2 * r0 - t0 * r2;
        A[2][3 + j] = -t1 * r0 + t0 * r1;
    }
}

// The batch's rig front-end body poses (T_abs of the rig records: world_T_body).
__global__ __launch_bounds__(256) void k_ba_snapshot_rig(BatchCtx c, double* dst) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= c.n * 16) return;
    dst[i] = c.rig_pose[(size_t)(i / 16) * TS_POSE_DOUBLES + 16 + i % 16];
}

// Keyframe a.frame's body pose into slot a.slot of the body window: B = inv(W_ba(prev)
// inv(W_fe(prev)) W_fe(g)) (body terms, RigBATracker), and every pair's camera E_p^-1 B.
__global__ void k_ba_rig_insert(BatchCtx c, BaArgs a) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    BaPair qb = ba_pair(c, a, c.P);
    const int f = (int)(a.frame - c.g0);
    const double* fe = a.fe_body + (size_t)f * 16;   // world_T_body
    double Twb[16], Tbw[16];
    if (a.prev < 0) {
        for (int e = 0; e < 16; ++e) Twb[e] = fe[e];
    } else {
        double Wba[16], ifp[16], tmp[16];
        inv_rigid(qb.T + (size_t)a.prev * 16, Wba);
        inv_rigid(qb.Tfe + (size_t)a.prev * 16, ifp);
        mul4(Wba, ifp, tmp);
        mul4(tmp, fe, Twb);
    }
    inv_rigid(Twb, Tbw);
    for (int e = 0; e < 16; ++e) {
        qb.T[(size_t)a.slot * 16 + e] = Tbw[e];
        qb.Tfe[(size_t)a.slot * 16 + e] = fe[e];
    }
    for (int p = 0; p < c.P; ++p) mul4(c.rig_Einv + 16 * p, Tbw, a.st.T + ((size_t)p * a.W + a.slot) * 16);
    for (int e = 0; e < TS_BA_INE; ++e) qb.ine[(size_t)a.slot * TS_BA_INE + e] = a.ine[e];   // the body's inertial factor
    for (int e = 0; e < 3; ++e) qb.vel[(size_t)a.slot * 3 + e] = a.vel0[e];
    for (int e = 0; e < 6; ++e) qb.bias[(size_t)a.slot * 6 + e] = ba_new_bias(a, qb.bias, e);
}

// The body system of an iteration from every pair's reduced system (block r = row, thread = column):
// S = sum_p Ad_p^T S_p Ad_p with S_p = blockdiag(U_c) - C_p (undamped), b = sum_p Ad_p^T b_p with
// b_p = -g_c + C_p[:, 60], Ad_p = adjoint_rl(E_p^-1); written as the body pair's C = -S (column 60:
// b) and U = 0, so k_ba_solve on the body pair solves (lam I + S) dB = b.
__global__ __launch_bounds__(64) void k_ba_rig_combine(BatchCtx c, BaArgs a) {
    // Ad_p is the same for every thread of the block: built once per pair into LDS (a per-thread
    // array read at the runtime column j would live in scratch)
    __shared__ double sA[6][6];
    const int n = a.n_order, r = blockIdx.x, col = threadIdx.x;
    BaPair qb = ba_pair(c, a, c.P);
    double v = 0.0;
    const bool live = r < 6 * n && (col < 6 * n || col == 60);
    const int ci = r / 6, i = r - 6 * ci;
    for (int p = 0; p < c.P; ++p) {
        __syncthreads();   // the previous pair's reads are done
        if (col == 0) {
            double A[6][6];
            adjoint_rl(c.rig_Einv + 16 * p, A);
            for (int aa = 0; aa < 6; ++aa)
                for (int bb = 0; bb < 6; ++bb) sA[aa][bb] = A[aa][bb];
        }
        __syncthreads();
        if (live) {
            BaPair q = ba_pair(c, a, p);
            const double(*A)[6] = sA;
            const double* U = q.cam_U + (size_t)ci * 27;
            if (col == 60) {   // (Ad^T b_p)[i]
                double acc = 0.0;
                for (int aa = 0; aa < 6; ++aa) acc += A[aa][i] * (-U[21 + aa] + q.C[(6 * ci + aa) * 64 + 60]);
                v += acc;
                continue;
            }
            const int cj = col / 6, j = col - 6 * cj;
            double acc = 0.0;
            for (int aa = 0; aa < 6; ++aa) {
                double sb = 0.0;   // (S_p Ad)[aa][j]
                for (int bb = 0; bb < 6; ++bb) {
                    double sab = -q.C[(6 * ci + aa) * 64 + 6 * cj + bb];
                    if (ci == cj) {
                        const int lo = aa < bb ? aa : bb, hi = aa < bb ? bb : aa;
                        sab += U[lo * 6 - lo * (lo - 1) / 2 + (hi - lo)];
                    }
                    sb += sab * A[bb][j];
                }
                acc += A[aa][i] * sb;
            }
            v += acc;
        }
    }
    if (live && col != 60) v = -v;
    qb.C[r * 64 + col] = v;
    if (r == 0) {
        for (int e = col; e < a.W * 27; e += 64) qb.cam_U[e] = 0.0;
        if (col == 0) {
            int nobs = 0, L = 0;
            for (int p = 0; p < c.P; ++p) {
                nobs += a.st.counts[4 * p];
                L += a.st.counts[4 * p + 1];
            }
            qb.counts[0] = nobs;
            qb.counts[1] = L;
        }
    }
}

// After the body solve: every pair's cameras E_p^-1 B, its camera updates dc_p = Ad_p dB (for the
// landmark back substitution) and the solve's status (block = pair, thread = window camera).
__global__ __launch_bounds__(64) void k_ba_rig_expand(BatchCtx c, BaArgs a) {
    const int p = blockIdx.x, cj = threadIdx.x;
    BaPair q = ba_pair(c, a, p), qb = ba_pair(c, a, c.P);
    if (cj < a.n_order) {
        const int slot = a.order[cj];
        mul4(c.rig_Einv + 16 * p, qb.T + (size_t)slot * 16, q.T + (size_t)slot * 16);
        double A[6][6];
        adjoint_rl(c.rig_Einv + 16 * p, A);
        for (int i = 0; i < 6; ++i) {
            double acc = 0.0;
            for (int j = 0; j < 6; ++j) acc += A[i][j] * qb.dc[6 * cj + j];
            q.dc[6 * cj + i] = acc;
        }
    }
    if (cj == 0) q.counts[2] = qb.counts[2];
}

void launch_ba_snapshot_rig(const BatchCtx& c, double* dst, hipStream_t s) {
    hipLaunchKernelGGL(k_ba_snapshot_rig, dim3((c.n * 16 + 255) / 256), dim3(256), 0, s, c, dst);
}

void launch_ba_rig_keyframe(const BatchCtx& c, const BaArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_ba_rig_insert, dim3(1), dim3(64), 0, s, c, a);
}

void launch_ba_rig_solve(const BatchCtx& c, const BaArgs& a, hipStream_t s, BaTiming* timing, bool inertial) {
    BaArgs ap = a, ab = a;
    ab.pair = c.P;
    for (int p = 0; p < c.P; ++p) {
        ap.pair = p;
        launch_ba_prepare(c, ap, s);
    }
    for (int it = 0; it < a.iters; ++it) {
        for (int p = 0; p < c.P; ++p) {
            ap.pair = p;
            launch_ba_linearize(c, ap, it, s, timing);
        }
        hipLaunchKernelGGL(k_ba_rig_combine, dim3(64), dim3(64), 0, s, c, ab);
        hipLaunchKernelGGL(inertial ? k_ba_solve_ine : k_ba_solve, dim3(1), dim3(64 * BA_SOLVE_WAVES), 0, s, c, ab);
        hipLaunchKernelGGL(k_ba_rig_expand, dim3(c.P), dim3(64), 0, s, c, ab);
    }
    for (int p = 0; p < c.P; ++p) {
        ap.pair = p;
        launch_ba_backsub(c, ap, s);
    }
}
