// k_exchange.hip — the blocks a sharded rig moves between ranks.
//
// A rank owns camera streams (front end: rectify .. describe of those cameras for every frame of
// the batch) and a range of the batch's frames (back end: A6/A7 of every pair + the rig pose for
// those frames).  Two device-side gathers/scatters feed the RCCL collectives:
//
//   stream block, per (frame, camera): the feature side of one image in the ring, i.e. what the
//     back end reads of it (keypoints, level counts, y-sorted records, y-sorted descriptors,
//     row-start table), 16-byte aligned pieces:
//       kps u32[K][2] | kcount i32[L] (padded to 16 B) | ys u32x4[K] | desc_ys u32[K][8] | rowstart u16[rs_total]
//   pose record, per frame: pose f64[P][68] | rig pose f64[68] | stats i32[P][8] | rig stats i32[8]
//
// Pixels travel as the raw images (the back end re-runs rectify + pyramid on them, cheaper than
// moving the 1.33x larger pyramid).  One block per item, 16-byte copies.
#include "tslam_common.h"

struct StreamBlock {
    int64_t kps, kcount, ys, desc, rowstart, bytes;   // byte offsets of the pieces, block size
};

static inline __host__ __device__ StreamBlock stream_block(const LevelGeom& g) {
    StreamBlock b;
    const int64_t K = g.K;
    b.kps = 0;
    b.kcount = K * 8;
    b.ys = b.kcount + ((int64_t)g.n_levels * 4 + 15) / 16 * 16;
    b.desc = b.ys + K * 16;
    b.rowstart = b.desc + K * 32;
    b.bytes = (b.rowstart + (int64_t)g.rs_total * 2 + 15) / 16 * 16;
    return b;
}

int64_t stream_block_bytes(const LevelGeom& g) { return stream_block(g).bytes; }

// 16-byte copy of n bytes when both ends and n are 16-byte aligned, else bytes
__device__ __forceinline__ void copy_piece(uint8_t* dst, const uint8_t* src, int64_t n) {
    if ((((uintptr_t)dst | (uintptr_t)src | (uintptr_t)n) & 15) == 0) {
        uint4* d = reinterpret_cast<uint4*>(dst);
        const uint4* s = reinterpret_cast<const uint4*>(src);
        for (int64_t i = threadIdx.x; i < n / 16; i += blockDim.x) d[i] = s[i];
    } else {
        for (int64_t i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
    }
}

// item = k * ncam + s: frame first + k, camera cam_lo + s.  pack: ring -> block (zeros for frames
// before the sequence start); unpack: block -> ring (frames before the start are skipped).
template <bool PACK>
__global__ __launch_bounds__(256) void k_stream_blocks(BatchCtx c, int64_t first, int cam_lo, int ncam, uint8_t* blk) {
    const int item = blockIdx.x;
    const int k = item / ncam, cam = cam_lo + item % ncam;
    const int64_t g = first + k;
    const StreamBlock sb = stream_block(c.g);
    uint8_t* b = blk + (int64_t)item * sb.bytes;
    if (g < 0) {
        if (PACK)
            for (int64_t i = threadIdx.x; i < sb.bytes / 16; i += blockDim.x) reinterpret_cast<uint4*>(b)[i] = uint4{0, 0, 0, 0};
        return;
    }
    const size_t sc = (size_t)ring_slot(c, g) * c.C + cam;
    const int64_t K = c.g.K;
    uint8_t* ring[5] = {reinterpret_cast<uint8_t*>(c.kps + sc * K * 2), reinterpret_cast<uint8_t*>(c.kcount + sc * c.g.n_levels),
                        reinterpret_cast<uint8_t*>(c.ys + sc * K), reinterpret_cast<uint8_t*>(c.desc_ys + sc * K * 8),
                        reinterpret_cast<uint8_t*>(c.rowstart + sc * c.g.rs_total)};
    const int64_t off[5] = {sb.kps, sb.kcount, sb.ys, sb.desc, sb.rowstart};
    const int64_t len[5] = {K * 8, (int64_t)c.g.n_levels * 4, K * 16, K * 32, (int64_t)c.g.rs_total * 2};
    for (int p = 0; p < 5; ++p) {
        if (PACK) copy_piece(b + off[p], ring[p], len[p]);
        else copy_piece(ring[p], b + off[p], len[p]);
    }
}

// the per-item copy of k_stream_blocks (frame g, camera cam <-> block b)
template <bool PACK>
__device__ __forceinline__ void stream_block_item(const BatchCtx& c, int64_t g, int cam, uint8_t* b) {
    const StreamBlock sb = stream_block(c.g);
    if (g < 0) {
        if (PACK)
            for (int64_t i = threadIdx.x; i < sb.bytes / 16; i += blockDim.x) reinterpret_cast<uint4*>(b)[i] = uint4{0, 0, 0, 0};
        return;
    }
    const size_t sc = (size_t)ring_slot(c, g) * c.C + cam;
    const int64_t K = c.g.K;
    uint8_t* ring[5] = {reinterpret_cast<uint8_t*>(c.kps + sc * K * 2), reinterpret_cast<uint8_t*>(c.kcount + sc * c.g.n_levels),
                        reinterpret_cast<uint8_t*>(c.ys + sc * K), reinterpret_cast<uint8_t*>(c.desc_ys + sc * K * 8),
                        reinterpret_cast<uint8_t*>(c.rowstart + sc * c.g.rs_total)};
    const int64_t off[5] = {sb.kps, sb.kcount, sb.ys, sb.desc, sb.rowstart};
    const int64_t len[5] = {K * 8, (int64_t)c.g.n_levels * 4, K * 16, K * 32, (int64_t)c.g.rs_total * 2};
    for (int p = 0; p < 5; ++p) {
        if (PACK) copy_piece(b + off[p], ring[p], len[p]);
        else copy_piece(ring[p], b + off[p], len[p]);
    }
}

// item over the world-1 peers' slots: (peer q != me, frame k, camera s) of [world][cap][S][block];
// the frames past a peer's count (a shorter or empty range) are not touched
template <bool PACK>
__global__ __launch_bounds__(256) void k_stream_blocks_peers(BatchCtx c, int64_t g0, int n, int world, int cap, int me, int S,
                                                             uint8_t* blk) {
    const int item = blockIdx.x, per = cap * S;
    const int qq = item / per, q = qq < me ? qq : qq + 1;
    const int r = item - qq * per, k = r / S, s = r - k * S;
    const int owner = PACK ? q : me;   // whose frame range the slot carries
    int lo, hi;
    peer_range(owner, n, world, &lo, &hi);
    if (k >= peer_frames(owner, n, world)) return;
    uint8_t* b = blk + ((int64_t)q * per + r) * stream_block(c.g).bytes;
    if (PACK) stream_block_item<true>(c, g0 + lo - 1 + k, me * S + s, b);   // my cameras, q's frames
    else stream_block_item<false>(c, g0 + lo - 1 + k, q * S + s, b);        // q's cameras, my frames
}

void launch_stream_blocks_peers(const BatchCtx& c, bool pack, int64_t g0, int n, int world, int cap, int me, int S,
                                uint8_t* blk, hipStream_t s) {
    const dim3 grid((world - 1) * cap * S);
    if (grid.x == 0) return;
    if (pack) hipLaunchKernelGGL(k_stream_blocks_peers<true>, grid, dim3(256), 0, s, c, g0, n, world, cap, me, S, blk);
    else hipLaunchKernelGGL(k_stream_blocks_peers<false>, grid, dim3(256), 0, s, c, g0, n, world, cap, me, S, blk);
}

void launch_stream_blocks(const BatchCtx& c, bool pack, int64_t first, int n_frames, int cam_lo, int ncam, uint8_t* blk,
                          hipStream_t s) {
    const dim3 grid(n_frames * ncam);
    if (pack) hipLaunchKernelGGL(k_stream_blocks<true>, grid, dim3(256), 0, s, c, first, cam_lo, ncam, blk);
    else hipLaunchKernelGGL(k_stream_blocks<false>, grid, dim3(256), 0, s, c, first, cam_lo, ncam, blk);
}

// pose records of batch frames f0 .. f0+n-1 (record k <-> batch frame f0 + k)
static inline __host__ __device__ int64_t pose_record_size(int P) { return (int64_t)(P + 1) * (TS_POSE_DOUBLES * 8 + TS_STATS_INTS * 4); }
int64_t pose_record_bytes(int P) { return pose_record_size(P); }

template <bool PACK>
__global__ __launch_bounds__(256) void k_pose_records(BatchCtx c, int f0, uint8_t* rec) {
    const int k = blockIdx.x, f = f0 + k;
    const int P = c.P;
    uint8_t* r = rec + (int64_t)k * pose_record_size(P);
    double* rd = reinterpret_cast<double*>(r);
    int32_t* ri = reinterpret_cast<int32_t*>(r + (int64_t)(P + 1) * TS_POSE_DOUBLES * 8);
    for (int i = threadIdx.x; i < (P + 1) * TS_POSE_DOUBLES; i += blockDim.x) {
        const int p = i / TS_POSE_DOUBLES, e = i % TS_POSE_DOUBLES;
        double* src = p < P ? c.pose + ((size_t)f * P + p) * TS_POSE_DOUBLES + e
                            : (c.rig_pose ? c.rig_pose + (size_t)f * TS_POSE_DOUBLES + e : nullptr);
        if (PACK) rd[i] = src ? *src : 0.0;
        else if (src) *src = rd[i];
    }
    for (int i = threadIdx.x; i < (P + 1) * TS_STATS_INTS; i += blockDim.x) {
        const int p = i / TS_STATS_INTS, e = i % TS_STATS_INTS;
        int32_t* src = p < P ? c.stats + ((size_t)f * P + p) * TS_STATS_INTS + e
                             : (c.rig_stats ? c.rig_stats + (size_t)f * TS_STATS_INTS + e : nullptr);
        if (PACK) ri[i] = src ? *src : 0;
        else if (src) *src = ri[i];
    }
}

// unpack of the all-gather's padded layout: frame f of the batch is record (f - lo) of range q's
// owner's slot (peer_records(n, world) records per rank), [lo, hi) = range q the one holding f
// (the owner of range q is rank q, or rig_rank(q) under the pair split)
__global__ __launch_bounds__(256) void k_pose_records_gathered(BatchCtx c, int world, int pairs, const uint8_t* rec) {
    const int f = blockIdx.x, per = peer_records(c.n, world);
    int q = 0, lo = 0, hi = 0;
    for (; q < world; ++q) {
        peer_range(q, c.n, world, &lo, &hi);
        if (f < hi) break;
    }
    const int P = c.P;
    const uint8_t* r = rec + ((int64_t)rig_rank(q, world, pairs) * per + (f - lo)) * pose_record_size(P);
    const double* rd = reinterpret_cast<const double*>(r);
    const int32_t* ri = reinterpret_cast<const int32_t*>(r + (int64_t)(P + 1) * TS_POSE_DOUBLES * 8);
    for (int i = threadIdx.x; i < (P + 1) * TS_POSE_DOUBLES; i += blockDim.x) {
        const int p = i / TS_POSE_DOUBLES, e = i % TS_POSE_DOUBLES;
        double* dst = p < P ? c.pose + ((size_t)f * P + p) * TS_POSE_DOUBLES + e
                            : (c.rig_pose ? c.rig_pose + (size_t)f * TS_POSE_DOUBLES + e : nullptr);
        if (dst) *dst = rd[i];
    }
    for (int i = threadIdx.x; i < (P + 1) * TS_STATS_INTS; i += blockDim.x) {
        const int p = i / TS_STATS_INTS, e = i % TS_STATS_INTS;
        int32_t* dst = p < P ? c.stats + ((size_t)f * P + p) * TS_STATS_INTS + e
                             : (c.rig_stats ? c.rig_stats + (size_t)f * TS_STATS_INTS + e : nullptr);
        if (dst) *dst = ri[i];
    }
}

void launch_pose_records_gathered(const BatchCtx& c, int world, bool pairs, const uint8_t* rec, hipStream_t s) {
    hipLaunchKernelGGL(k_pose_records_gathered, dim3(c.n), dim3(256), 0, s, c, world, pairs ? 1 : 0, rec);
}

void launch_pose_records(const BatchCtx& c, bool pack, int f0, int n, uint8_t* rec, hipStream_t s) {
    if (n <= 0) return;
    if (pack) hipLaunchKernelGGL(k_pose_records<true>, dim3(n), dim3(256), 0, s, c, f0, rec);
    else hipLaunchKernelGGL(k_pose_records<false>, dim3(n), dim3(256), 0, s, c, f0, rec);
}

// pair block, per (batch frame, pair), for the rig pose of a frame range on another rank (a
// camera-sharded RGB-D rig, or the pair split of a stereo rig): pose f64[68] | stats i32[8] |
// corr f64[K][5] — the columns k_rig_pose reads of a correspondence (X, Y, Z, cx - u, cy - v; the
// bearing columns 5..7 serve P3P on the pair's own rank), rows past stats[1] not copied.  The rig
// pose reads nothing else of a pair.
#define TS_PAIR_CORR 5
static inline __host__ __device__ int64_t pair_block_size(int K) {
    return (int64_t)TS_POSE_DOUBLES * 8 + TS_STATS_INTS * 4 + (int64_t)K * TS_PAIR_CORR * 8;
}
int64_t pair_block_bytes(const LevelGeom& g) { return pair_block_size(g.K); }

// item = k * np + s: batch frame f0 + k, pair p0 + s
template <bool PACK>
__global__ __launch_bounds__(256) void k_pair_blocks(BatchCtx c, int f0, int p0, int np, uint8_t* blk) {
    const int item = blockIdx.x;
    const int f = f0 + item / np, p = p0 + item % np;
    const int64_t K = c.g.K;
    uint8_t* b = blk + (int64_t)item * pair_block_size((int)K);
    const size_t fp = (size_t)f * c.P + p;
    uint8_t* pose = reinterpret_cast<uint8_t*>(c.pose + fp * TS_POSE_DOUBLES);
    uint8_t* stats = reinterpret_cast<uint8_t*>(c.stats + fp * TS_STATS_INTS);
    double* corr = c.corr + fp * K * TS_CORR_DOUBLES;
    const int64_t so = (int64_t)TS_POSE_DOUBLES * 8, co = so + TS_STATS_INTS * 4;
    double* bc = reinterpret_cast<double*>(b + co);   // 16-byte aligned: 544 + 32 bytes in
    if (PACK) {
        copy_piece(b, pose, so);
        copy_piece(b + so, stats, TS_STATS_INTS * 4);
        const int n = min(max(c.stats[fp * TS_STATS_INTS + 1], 0), (int)K);
        for (int i = threadIdx.x; i < n * TS_PAIR_CORR; i += blockDim.x) {
            const int row = i / TS_PAIR_CORR, col = i - row * TS_PAIR_CORR;
            bc[i] = corr[(size_t)row * TS_CORR_DOUBLES + col];
        }
    } else {
        copy_piece(pose, b, so);
        copy_piece(stats, b + so, TS_STATS_INTS * 4);
        const int n = min(max(reinterpret_cast<const int32_t*>(b + so)[1], 0), (int)K);
        for (int i = threadIdx.x; i < n * TS_PAIR_CORR; i += blockDim.x) {
            const int row = i / TS_PAIR_CORR, col = i - row * TS_PAIR_CORR;
            corr[(size_t)row * TS_CORR_DOUBLES + col] = bc[i];
        }
    }
}

void launch_pair_blocks(const BatchCtx& c, bool pack, int f0, int n_frames, int p0, int np, uint8_t* blk, hipStream_t s) {
    const dim3 grid(n_frames * np);
    if (pack) hipLaunchKernelGGL(k_pair_blocks<true>, grid, dim3(256), 0, s, c, f0, p0, np, blk);
    else hipLaunchKernelGGL(k_pair_blocks<false>, grid, dim3(256), 0, s, c, f0, p0, np, blk);
}

// Raw images of this rank's cameras for every peer (alltoall layout [world][cap][S][H*W]): slot q
// = frames lo_q - 1 .. hi_q - 1 of the batch (frame -1 = `prev`, the previous batch's last frame);
// one block per (peer, frame, camera) image, 16-byte copies.  (The library's driver sends these
// straight from the input instead: tslam_shard.cpp; this staging serves the host-framework path.)
__global__ __launch_bounds__(256) void k_stage_raw_peers(const uint8_t* images, const uint8_t* prev, uint8_t* dst, int n,
                                                         int world, int cap, int me, int S, int64_t img_bytes) {
    const int item = blockIdx.x, per = cap * S;
    const int qq = item / per, q = qq < me ? qq : qq + 1;
    const int r = item - qq * per, k = r / S, s = r - k * S;
    int lo, hi;
    peer_range(q, n, world, &lo, &hi);
    if (k >= peer_frames(q, n, world)) return;
    const int f = lo - 1 + k;   // batch frame
    const uint8_t* src = f < 0 ? prev + (int64_t)s * img_bytes : images + ((int64_t)f * S + s) * img_bytes;
    uint8_t* out = dst + ((int64_t)q * per + r) * img_bytes;
    copy_piece(out, src, img_bytes);
}

void launch_stage_raw_peers(const uint8_t* images, const uint8_t* prev, uint8_t* dst, int n, int world, int cap, int me,
                            int S, int64_t img_bytes, hipStream_t s) {
    if (world < 2) return;
    hipLaunchKernelGGL(k_stage_raw_peers, dim3((world - 1) * cap * S), dim3(256), 0, s, images, prev, dst, n, world, cap, me,
                       S, img_bytes);
}

// ---- state blocks to rank 0 (local BA, loop closure, relocalisation on a sharded rig) ----------
//   range block, per (frame of the sender's range, pair): temporal i32[K] | disp f64[K]
//   camera block, per (batch frame, left camera of the sender): kps u32[K][2] | kcount i32[L]
//     (padded to 16 B) | desc u32[K][8]
// Payload of sender r: its range blocks (frame-major, pairs inner), then its camera blocks
// (frame-major, cameras inner).
static inline __host__ __device__ int64_t range_block_size(const LevelGeom& g) { return (int64_t)g.K * 12; }
static inline __host__ __device__ int64_t camera_block_size(const LevelGeom& g) {
    return (int64_t)g.K * 8 + ((int64_t)g.n_levels * 4 + 15) / 16 * 16 + (int64_t)g.K * 32;
}
int64_t state_range_block_bytes(const LevelGeom& g) { return range_block_size(g); }
int64_t state_camera_block_bytes(const LevelGeom& g) { return camera_block_size(g); }

template <bool PACK>
__global__ __launch_bounds__(256) void k_state_blocks(BatchCtx c, int lo, int nrange, int cam_lo, int nleft, uint8_t* blk) {
    const int item = blockIdx.x;
    const int64_t K = c.g.K;
    if (item < nrange * c.P) {
        const int f = lo + item / c.P, p = item % c.P;
        const size_t sp = (size_t)ring_slot(c, c.g0 + f) * c.P + p;
        uint8_t* b = blk + (int64_t)item * range_block_size(c.g);
        uint8_t* t = reinterpret_cast<uint8_t*>(c.temporal + sp * K);
        uint8_t* d = reinterpret_cast<uint8_t*>(c.disp + sp * K);
        if (PACK) {
            copy_piece(b, t, K * 4);
            copy_piece(b + K * 4, d, K * 8);
        } else {
            copy_piece(t, b, K * 4);
            copy_piece(d, b + K * 4, K * 8);
        }
        return;
    }
    const int j = item - nrange * c.P, f = j / nleft, cam = cam_lo + 2 * (j % nleft);   // left cameras: even
    const size_t sc = (size_t)ring_slot(c, c.g0 + f) * c.C + cam;
    uint8_t* b = blk + (int64_t)nrange * c.P * range_block_size(c.g) + (int64_t)j * camera_block_size(c.g);
    const int64_t kc = K * 8, de = kc + ((int64_t)c.g.n_levels * 4 + 15) / 16 * 16;
    uint8_t* ring[3] = {reinterpret_cast<uint8_t*>(c.kps + sc * K * 2), reinterpret_cast<uint8_t*>(c.kcount + sc * c.g.n_levels),
                        reinterpret_cast<uint8_t*>(c.desc + sc * K * 8)};
    const int64_t off[3] = {0, kc, de}, len[3] = {K * 8, (int64_t)c.g.n_levels * 4, K * 32};
    for (int q = 0; q < 3; ++q) {
        if (PACK) copy_piece(b + off[q], ring[q], len[q]);
        else copy_piece(ring[q], b + off[q], len[q]);
    }
}

// the state blocks of sender `rank` (its frame range and its stereo cameras [cam_lo, cam_hi)):
// pack on the sender, unpack on rank 0
void launch_state_blocks(const BatchCtx& c, bool pack, int n, int world, int rank, int cam_lo, int cam_hi, uint8_t* blk,
                         hipStream_t s) {
    int lo, hi;
    peer_range(rank, n, world, &lo, &hi);
    const int left0 = (cam_lo + 1) & ~1, nleft = cam_hi > left0 ? (cam_hi - left0 + 1) / 2 : 0;
    const dim3 grid((hi - lo) * c.P + n * nleft);
    if (grid.x == 0) return;
    if (pack) hipLaunchKernelGGL(k_state_blocks<true>, grid, dim3(256), 0, s, c, lo, hi - lo, left0, nleft, blk);
    else hipLaunchKernelGGL(k_state_blocks<false>, grid, dim3(256), 0, s, c, lo, hi - lo, left0, nleft, blk);
}
