// k_loop.hip — keyframe database and loop detection (SURVEY.md §8f items 1 + 3; the reference's
// SlamConfig.enable_loop_closure, thor_slam/slam/interface.py:155-156, forwarded to cuVSLAM).
// CPU restatement: oracle/numpy_loop.py.
//
// Per keyframe (a resident frame of one stereo pair) the database holds its stereo landmarks in
// the rectified left camera frame, compacted in keypoint order: xyz f64 [K][3] (z = fx*B / d,
// x = (u - cx) z / fx, y = (v - cy) z / fy, the A8 insertion formula) and rBRIEF-256 [K][8].
// The first S landmarks are the keyframe's signature (the strongest level-0 corners with depth).
//
//   k_loop_store  one block: valid keypoints with a disparity d > 0 -> compacted landmarks;
//   k_loop_store_auto  the same for every keyframe of a batch (grid keyframes x pairs, on the
//                 batch's back stream after its pose stage; tslam_loop_auto), plus a snapshot of
//                 the keyframe image's keypoint records, level counts and descriptors, so a later
//                 verification needs no ring slot;
//   k_loop_vote   block per candidate keyframe: each of the query's S signature descriptors is
//                 matched by brute-force Hamming against the candidate's signature (LDS
//                 broadcasts, best / second by (distance, index)); ratio + max_hamming votes;
// geometric verification reuses the relocalisation matcher + A7 RANSAC (launch_reloc) with the
// candidate's landmarks as the map: its result is cam_q_T_cam_c.
#include "tslam_common.h"

#define LP_THREADS 256

__device__ __forceinline__ void loop_store_block(const BatchCtx& c, int pair, int rslot, double* xyz, uint32_t* desc,
                                                 int32_t* n_out) {
    __shared__ int s_tmp[LP_THREADS / 64];
    const int K = c.g.K, cam = c.cpp * pair;
    const size_t ib = (size_t)rslot * c.C + cam;
    const PairCalib cal = c.calib[pair];
    const double* disp = c.disp + ((size_t)rslot * c.P + pair) * K;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int n = 0;
    for (int base = 0; base < K; base += LP_THREADS) {
        const int k = base + threadIdx.x;
        double u = 0.0, v = 0.0, dd = 0.0;
        int flag = 0;
        if (k < K) {
            const uint32_t xy = c.kps[(ib * K + k) * 2], meta = c.kps[(ib * K + k) * 2 + 1];
            const int l = (int)(meta & 0xFF);
            const bool valid = k - c.g.koff[l] < (int)c.kcount[ib * c.g.n_levels + l];
            dd = disp[k];
            flag = valid && __builtin_isfinite(dd) && dd > 0.0;
            const double sc = (double)(1 << l);
            u = ((double)(xy & 0xFFFF) + 0.5) * sc - 0.5;
            v = ((double)(xy >> 16) + 0.5) * sc - 0.5;
        }
        // block exclusive scan of the flags (keypoint order)
        int x = flag;
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) s_tmp[wave] = x;
        __syncthreads();
        int off = 0, tot = 0;
        for (int w = 0; w < LP_THREADS / 64; ++w) {
            if (w < wave) off += s_tmp[w];
            tot += s_tmp[w];
        }
        if (flag) {
            const int o = n + off + x - 1;
            const double z = cal.fxb / dd;
            xyz[(size_t)o * 3] = (u - cal.cx) * z / cal.fx;
            xyz[(size_t)o * 3 + 1] = (v - cal.cy) * z / cal.fy;
            xyz[(size_t)o * 3 + 2] = z;
            const uint4* src = reinterpret_cast<const uint4*>(c.desc + (ib * K + k) * 8);
            uint4* dst = reinterpret_cast<uint4*>(desc + (size_t)o * 8);
            dst[0] = src[0];
            dst[1] = src[1];
        }
        n += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) *n_out = n;
}

__global__ __launch_bounds__(LP_THREADS) void k_loop_store(BatchCtx c, int pair, int rslot, double* xyz, uint32_t* desc,
                                                           int32_t* n_out) {
    loop_store_block(c, pair, rslot, xyz, desc, n_out);
}

// Tracked keyframes of a batch (tslam_loop_auto): keyframe frames g = k * interval of the batch
// whose pose status is 0 (the rig's with `rig`, pair 0's otherwise) take the next database
// positions in frame order, position i -> entry (i mod capk) * P + pair; *count holds the
// positions taken by earlier batches (k_loop_count_commit adds this batch's after the stores).
__device__ __forceinline__ bool kf_tracked(const BatchCtx& c, int64_t g, bool rig) {
    const int64_t f = g - c.g0;
    return (rig ? c.rig_stats[f * TS_STATS_INTS] : c.stats[f * c.P * TS_STATS_INTS]) == 0;
}

// grid (keyframes of the batch, pairs): keyframe k_first + x is frame (k_first + x) * interval
__global__ __launch_bounds__(LP_THREADS) void k_loop_store_auto(BatchCtx c, int interval, int64_t k_first, int capk,
                                                                bool rig, const int64_t* count, LoopDb db) {
    __shared__ int s_before;
    const int x = blockIdx.x;
    const int pair = blockIdx.y, K = c.g.K, L = c.g.n_levels;
    if (!kf_tracked(c, (k_first + x) * interval, rig)) return;
    if (threadIdx.x == 0) s_before = 0;
    __syncthreads();
    int mine = 0;   // tracked keyframes of this batch before x
    for (int i = threadIdx.x; i < x; i += LP_THREADS) mine += kf_tracked(c, (k_first + i) * interval, rig);
    if (mine) atomicAdd(&s_before, mine);   // integer count: order-free
    __syncthreads();
    const int64_t pos = *count + s_before;
    const int rslot = ring_slot(c, (k_first + x) * interval);
    const size_t e = (size_t)(pos % capk) * c.P + pair;
    loop_store_block(c, pair, rslot, db.xyz + e * K * 3, db.desc + e * K * 8, db.n + e);
    const size_t ib = (size_t)rslot * c.C + c.cpp * pair;
    const uint2* kp = reinterpret_cast<const uint2*>(c.kps + ib * K * 2);   // one 8-byte record per keypoint
    uint2* skp = reinterpret_cast<uint2*>(db.snap_kps + e * K * 2);
    for (int i = threadIdx.x; i < K; i += LP_THREADS) skp[i] = kp[i];
    const uint4* dsrc = reinterpret_cast<const uint4*>(c.desc + ib * K * 8);
    uint4* ddst = reinterpret_cast<uint4*>(db.snap_desc + e * K * 8);
    for (int i = threadIdx.x; i < K * 2; i += LP_THREADS) ddst[i] = dsrc[i];
    if ((int)threadIdx.x < L) db.snap_kcount[e * TS_MAX_LEVELS + threadIdx.x] = c.kcount[ib * L + threadIdx.x];
}

// one wave: *count += the batch's tracked keyframes (after the stores read it)
__global__ __launch_bounds__(64) void k_loop_count_commit(BatchCtx c, int interval, int64_t k_first, int nkf, bool rig,
                                                          int64_t* count) {
    int n = 0;
    for (int i = threadIdx.x; i < nkf; i += 64) n += kf_tracked(c, (k_first + i) * interval, rig);
    for (int o = 32; o; o >>= 1) n += __shfl_xor(n, o, 64);
    if (threadIdx.x == 0) *count += n;
}

// grid = candidates, block = LP_THREADS (S <= LP_THREADS): thread t owns query signature entry t.
// Candidate b is entry ((k0 + b / P) mod capk) * P + b mod P (keyframe-major, every pair's entry;
// the manual database passes k0 = 0, P = 1 and a capk above the count: entry b).
__global__ __launch_bounds__(LP_THREADS) void k_loop_vote(const uint32_t* db_desc, const int32_t* db_n, int K, int S,
                                                          int q_slot, int64_t k0, int capk, int P, int max_hamming,
                                                          int ratio_pct, int32_t* votes) {
    __shared__ uint4 s_d[LP_THREADS][2];
    __shared__ int s_votes;
    const int t = threadIdx.x;
    const int cand = (int)(((k0 + blockIdx.x / P) % capk) * P + blockIdx.x % P);
    const int nc = min(S, db_n[cand]), nq = min(S, db_n[q_slot]);
    if (t == 0) s_votes = 0;
    for (int i = t; i < 2 * nc; i += LP_THREADS)
        s_d[i >> 1][i & 1] = reinterpret_cast<const uint4*>(db_desc + ((size_t)cand * K + (i >> 1)) * 8)[i & 1];
    __syncthreads();
    if (t < nq && nc > 0) {
        const uint4* qp = reinterpret_cast<const uint4*>(db_desc + ((size_t)q_slot * K + t) * 8);
        const uint4 qa = qp[0], qb = qp[1];
        uint32_t best = 0xFFFFFFFFu, second = 0xFFFFFFFFu;   // (distance << 20) | index
        for (int j = 0; j < nc; ++j) {
            const uint4 a = s_d[j][0], b = s_d[j][1];
            const uint32_t dist = __builtin_popcount(qa.x ^ a.x) + __builtin_popcount(qa.y ^ a.y) +
                                  __builtin_popcount(qa.z ^ a.z) + __builtin_popcount(qa.w ^ a.w) +
                                  __builtin_popcount(qb.x ^ b.x) + __builtin_popcount(qb.y ^ b.y) +
                                  __builtin_popcount(qb.z ^ b.z) + __builtin_popcount(qb.w ^ b.w);
            const uint32_t key = (dist << 20) | (uint32_t)j;
            if (key < best) {
                second = best;
                best = key;
            } else if (key < second) {
                second = key;
            }
        }
        const uint32_t bd = best >> 20, sd = second >> 20;
        if ((int)bd <= max_hamming && (second == 0xFFFFFFFFu || 100u * bd < (uint32_t)ratio_pct * sd))
            atomicAdd(&s_votes, 1);   // integer count: order-free
    }
    __syncthreads();
    if (t == 0) votes[blockIdx.x] = s_votes;
}

void launch_loop_store(const BatchCtx& c, int pair, int64_t frame, double* xyz, uint32_t* desc, int32_t* n_out,
                       hipStream_t s) {
    hipLaunchKernelGGL(k_loop_store, dim3(1), dim3(LP_THREADS), 0, s, c, pair, ring_slot(c, frame), xyz, desc, n_out);
}

void launch_loop_store_auto(const BatchCtx& c, int interval, const LoopDb& db, int capk, bool rig, int64_t* count,
                            hipStream_t s) {
    const int64_t k_first = (c.g0 + interval - 1) / interval, k_last = (c.g0 + c.n - 1) / interval;
    if (k_last < k_first) return;
    const int nkf = (int)(k_last - k_first + 1);
    hipLaunchKernelGGL(k_loop_store_auto, dim3(nkf, c.P), dim3(LP_THREADS), 0, s, c, interval, k_first, capk, rig,
                       (const int64_t*)count, db);
    hipLaunchKernelGGL(k_loop_count_commit, dim3(1), dim3(64), 0, s, c, interval, k_first, nkf, rig, count);
}

void launch_loop_vote(const uint32_t* db_desc, const int32_t* db_n, int K, int S, int q_slot, int64_t k0, int capk, int P,
                      int n_cand, int max_hamming, int ratio_pct, int32_t* votes, hipStream_t s) {
    hipLaunchKernelGGL(k_loop_vote, dim3(n_cand), dim3(LP_THREADS), 0, s, db_desc, db_n, K, S, q_slot, k0, capk, P,
                       max_hamming, ratio_pct, votes);
}
