// tslam_shard.cpp — the library's own driver of a sharded rig (one camera stream per
// GPU; replaces cuVSLAM's multicam mode, launch/thor_visual_slam.launch.py:49,81).
//
// A driver owns, per local rank, the exchange buffers (two sets, by batch parity), three streams and
// the events between them, and runs one batch of every local rank through the stages of a sharded
// handle (tslam_set_shard) with the exchanges in between:
//
//   stereo rig                                         camera-sharded RGB-D rig
//   x : raw images of the frames each peer solves ──┐   f : RECTIFY .. DESCRIBE (own cameras)
//   f : RECTIFY, DETECT, DESCRIBE, pack streams      │   b : MATCH, POSE (own cameras, whole batch),
//   x : ── exchange 1 (raw images, stream blocks) ◄──┘       pack pair blocks per peer range
//   b : import raw + unpack streams, MATCH, POSE(+rig)  b : ── exchange 1 (pair blocks)
//   b : [state blocks ── gather to rank 0 ── unpack]    b : unpack pairs, KERNEL_RIG (own range)
//   b : pack pose records ── exchange 2 (all-gather) ── unpack, CHAIN  (both)
//   b : [rank 0: local BA]; [results into pinned slots]
//
// f = front stream (high priority), x = exchange stream, b = back stream.  Batch s's raw exchange
// overlaps its front end and batch s+1's front end overlaps batch s's back end; a parity's receive
// buffers are reused once the imports of batch s-2 are done (event), its send buffers once the
// collectives that read them are.  Nothing here synchronises the host.
//
// Any batch of 1 .. max_batch frames: rank q's back end owns frames [q n / N, (q + 1) n / N) (ranges
// may differ by a frame or be empty), exchange slots are sized for a full batch (peer_cap frames),
// the pose all-gather pads every range to peer_records(n, N) records.  Raw images go straight from
// the caller's input (and the previous batch's last frame) to the peers: no staging copy.
//
// Pair split (TSLAM_SHARD_PAIRS, one camera per rank): rank r's back end solves pair r / 2 over
// half r & 1 of the batch, so the raw images and stream blocks go to the partner (r ^ 1) only —
// half a batch + 1 frame instead of a range + 1 frame to each of world - 1 peers; the rig pose of a
// rank's rig range (tslam_ranges.h rig_slot, inside its half) then takes the other pairs' pair
// blocks (pose, stats, the 5 correspondence columns it reads) from the ranks of the same half.
// Fewer bytes per rank, all of the image traffic on the one partner link.
//
// State gather (TSLAM_SHARD_GATHER, implied by local BA): every rank sends rank 0 the temporal
// matches and disparities of its range and the keypoints + descriptors of its left cameras, so
// rank 0's ring holds what the one-handle path's local BA, loop closure and relocalisation read;
// rank 0 then runs the local BA itself (the other ranks keep no window).
//
// Transports: RCCL (ncclSend / ncclRecv / ncclAllGather over xGMI; two communicators per rank so
// the pose all-gather of batch s, on the back stream, never shares a communicator with batch s+1's
// exchange on the exchange stream), created per process (tslam_comm_init: one local rank) or for
// all devices of one process (tslam_group_create: ncclCommInitAll); or COPY (device-to-device
// copies pushed on the sender's stream: a group of ranks in one process, also several on one device
// — the same packing and ordering as RCCL, used to test world > 1 on one GPU).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "tslam_common.h"
#include "tslam_internal.h"

#define SHCHK(expr)                                                                                            \
    do {                                                                                                       \
        hipError_t e__ = (expr);                                                                               \
        if (e__ != hipSuccess)                                                                                 \
            return tslam_internal_fail(TSLAM_EHIP, (std::string(#expr) + ": " + hipGetErrorString(e__)).c_str()); \
    } while (0)
#define NCCLCHK(expr)                                                                                          \
    do {                                                                                                       \
        ncclResult_t r__ = (expr);                                                                             \
        if (r__ != ncclSuccess)                                                                                \
            return tslam_internal_fail(TSLAM_EHIP, (std::string(#expr) + ": " + ncclGetErrorString(r__)).c_str()); \
    } while (0)
#define RC(expr)                          \
    do {                                  \
        const int rc__ = (expr);          \
        if (rc__ != TSLAM_OK) return rc__; \
    } while (0)

namespace {
struct Span {   // one timed segment of one batch (TSLAM_SHARD_PROFILE)
    int seg;
    hipEvent_t a, b;
};

struct Rank {
    tslam_handle* h = nullptr;
    int rank = 0, device = 0;
    ncclComm_t comm_x = nullptr, comm_p = nullptr;
    hipStream_t fs = nullptr, xs = nullptr, bs = nullptr;
    hipStream_t serial = nullptr;   // TSLAM_SHARD_SERIAL: the device's one stream (owned by its first rank)
    bool serial_owner = false;
    hipEvent_t ev_in = nullptr, ev_front = nullptr, ev_x = nullptr, ev_push = nullptr, ev_done = nullptr;
    hipEvent_t consumed[2] = {nullptr, nullptr};   // this parity's receive buffers were read
    bool consumed_armed[2] = {false, false};
    bool done_armed = false;
    uint8_t* raw_recv[2] = {nullptr, nullptr};
    uint8_t* feat_send[2] = {nullptr, nullptr};    // stream blocks (stereo) or pair blocks (RGB-D)
    uint8_t* feat_recv[2] = {nullptr, nullptr};
    uint8_t* pose_send[2] = {nullptr, nullptr};
    uint8_t* pose_recv[2] = {nullptr, nullptr};
    uint8_t* state_buf[2] = {nullptr, nullptr};    // gather: the payload (sender) / all payloads (rank 0)
    uint8_t* pb_send[2] = {nullptr, nullptr};      // pair split: pair blocks per rig-range owner
    uint8_t* pb_recv[2] = {nullptr, nullptr};
    uint8_t* prev_raw = nullptr;   // the previous batch's last frame of this rank's cameras
    std::vector<void*> allocs;
    // profiling
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    std::vector<Span> spans;
    double seg_us[TSLAM_SEG_COUNT] = {};
    int64_t timed_batches = 0;
};

enum Which { RAW = 0, FEAT = 1, POSE = 2, STATE = 3, PAIRB = 4 };
}  // namespace

struct tslam_shard_driver {
    int world = 1, transport = TSLAM_TRANSPORT_RCCL;
    bool rgbd = false, rig = false, ba = false;
    int flags = 0;                       // TSLAM_SHARD_* options
    int S = 0, B = 0, cap = 0;           // cameras per rank, max_batch, frames per peer slot
    int P = 0;                           // stereo pairs (RGB-D: cameras)
    int n = 0, maxr = 0;                 // this batch: frames, pose records per rank in the all-gather
    size_t img = 0, rec = 0, sblk = 0, pblk = 0;   // bytes: image, pose record, stream block, pair block
    size_t state_cap = 0;                // bytes of one sender's state payload slot (full batch)
    bool pb_ready = false;               // pair split: pair-block buffers allocated
    int64_t batches = 0;
    std::vector<Rank> ranks;   // local ranks: all of a group, one after tslam_comm_init
    bool gather() const { return world > 1 && !rgbd && (ba || (flags & TSLAM_SHARD_GATHER)); }
    // TSLAM_SHARD_PAIRS: rank r's back end solves pair r / 2 over half r & 1 of the batch; the
    // stereo exchange goes to the partner (r ^ 1) only, the rig pose gathers pair blocks
    bool pairs() const { return (flags & TSLAM_SHARD_PAIRS) != 0; }
};

// The rank's streams: its own three, or with TSLAM_SHARD_SERIAL one stream per device shared by
// every rank on it (each kernel and copy then runs alone: the per-rank profile of a one-GPU
// rehearsal reports isolated durations)
static hipStream_t FS(const tslam_shard_driver* d, const Rank& r) { return (d->flags & TSLAM_SHARD_SERIAL) ? r.serial : r.fs; }
static hipStream_t XS(const tslam_shard_driver* d, const Rank& r) { return (d->flags & TSLAM_SHARD_SERIAL) ? r.serial : r.xs; }
static hipStream_t BS(const tslam_shard_driver* d, const Rank& r) { return (d->flags & TSLAM_SHARD_SERIAL) ? r.serial : r.bs; }

static void destroy_driver(tslam_shard_driver* d) {
    if (!d) return;
    for (Rank& r : d->ranks) {
        (void)hipSetDevice(r.device);
        (void)hipDeviceSynchronize();
        if (r.comm_p) (void)ncclCommDestroy(r.comm_p);
        if (r.comm_x) (void)ncclCommDestroy(r.comm_x);
        for (hipEvent_t e : {r.ev_in, r.ev_front, r.ev_x, r.ev_push, r.ev_done, r.consumed[0], r.consumed[1]})
            if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : r.ev_pool) (void)hipEventDestroy(e);
        for (hipStream_t s : {r.fs, r.xs, r.bs})
            if (s) (void)hipStreamDestroy(s);
        if (r.serial && r.serial_owner) (void)hipStreamDestroy(r.serial);
        for (void* p : r.allocs) (void)hipFree(p);
        r.allocs.clear();
    }
    delete d;
}

extern "C" void tslam_internal_driver_destroy(tslam_shard_driver* d) { destroy_driver(d); }

static int alloc(Rank& r, uint8_t** p, size_t bytes) {
    void* q = nullptr;
    const hipError_t e = hipMalloc(&q, bytes ? bytes : 16);
    if (e != hipSuccess) return tslam_internal_fail(TSLAM_ENOMEM, (std::string("hipMalloc: ") + hipGetErrorString(e)).c_str());
    r.allocs.push_back(q);
    *p = (uint8_t*)q;
    SHCHK(hipMemset(q, 0, bytes ? bytes : 16));
    return TSLAM_OK;
}

// Geometry of the driver from its ranks' handles (all the same rig, sharded by tslam_set_shard).
static int plan(tslam_shard_driver* d, tslam_handle* h, int world) {
    tslam_handle_info in{};
    RC(tslam_internal_info(h, &in));
    if (in.ba && in.rgbd) return tslam_internal_fail(TSLAM_EINVAL, "a camera-sharded RGB-D rig runs without local BA");
    if (in.C % world) return tslam_internal_fail(TSLAM_EINVAL, "the cameras must divide by world");
    if (world > in.B) return tslam_internal_fail(TSLAM_EINVAL, "world must be <= max_batch");
    d->world = world;
    d->rgbd = in.rgbd != 0;
    d->rig = in.rig != 0;
    d->ba = in.ba != 0;
    d->S = in.C / world;
    d->P = in.P;
    d->B = in.B;
    d->cap = peer_cap(in.B, world);
    d->img = (size_t)in.W * in.H;
    d->rec = (size_t)in.pose_record;
    d->sblk = (size_t)in.stream_block;
    d->pblk = (size_t)in.pair_block;
    return TSLAM_OK;
}

// The frames rank q's stereo back end solves: its frame range, or under the pair split its pair's
// half of the batch; it reads the other cameras of frames lo - 1 .. hi - 1 (none when empty).
static void back_range(const tslam_shard_driver* d, int q, int* lo, int* hi) {
    if (d->pairs()) peer_range(q & 1, d->n, 2, lo, hi);
    else peer_range(q, d->n, d->world, lo, hi);
}
static int back_frames(const tslam_shard_driver* d, int q) {
    int lo, hi;
    back_range(d, q, &lo, &hi);
    return hi > lo ? hi - lo + 1 : 0;
}
// does rank src send rank dst its raw images and stream blocks (pair split: the partner only)
static bool stereo_peer(const tslam_shard_driver* d, int src, int dst) { return src != dst && (!d->pairs() || dst == (src ^ 1)); }

// bytes rank `q`'s slot carries for this batch: raw images / stream blocks of the frames q's back end
// reads (lo_q - 1 .. hi_q - 1) of S cameras; pair blocks (RGB-D) of q's range; slot capacities
static size_t raw_bytes(const tslam_shard_driver* d, int q) { return (size_t)back_frames(d, q) * d->S * d->img; }
static size_t feat_bytes(const tslam_shard_driver* d, int q) {
    if (!d->rgbd) return (size_t)back_frames(d, q) * d->S * d->sblk;
    int lo, hi;
    peer_range(q, d->n, d->world, &lo, &hi);
    return (size_t)(hi - lo) * d->S * d->pblk;
}
static size_t raw_cap(const tslam_shard_driver* d) { return (size_t)d->cap * d->S * d->img; }
static size_t feat_cap(const tslam_shard_driver* d) {
    return d->rgbd ? (size_t)(d->cap - 1) * d->S * d->pblk : (size_t)d->cap * d->S * d->sblk;
}

static int setup_rank(tslam_shard_driver* d, Rank& r) {
    tslam_handle_info in{};
    RC(tslam_internal_info(r.h, &in));
    r.device = in.device;
    SHCHK(hipSetDevice(r.device));
    int lo = 0, hi = 0;
    SHCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    SHCHK(hipStreamCreateWithPriority(&r.fs, hipStreamNonBlocking, hi));   // the front end is the critical path
    SHCHK(hipStreamCreateWithFlags(&r.xs, hipStreamNonBlocking));
    SHCHK(hipStreamCreateWithFlags(&r.bs, hipStreamNonBlocking));
    for (hipEvent_t* e : {&r.ev_in, &r.ev_front, &r.ev_x, &r.ev_push, &r.ev_done, &r.consumed[0], &r.consumed[1]})
        SHCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
    const size_t N = d->world, maxr = (size_t)peer_records(d->B, d->world);
    for (int k = 0; k < 2; ++k) {
        if (!d->rgbd) RC(alloc(r, &r.raw_recv[k], N * raw_cap(d)));
        RC(alloc(r, &r.feat_send[k], N * feat_cap(d)));
        RC(alloc(r, &r.feat_recv[k], N * feat_cap(d)));
        RC(alloc(r, &r.pose_send[k], maxr * d->rec));
        RC(alloc(r, &r.pose_recv[k], N * maxr * d->rec));
    }
    if (!d->rgbd) RC(alloc(r, &r.prev_raw, (size_t)d->S * d->img));
    SHCHK(hipDeviceSynchronize());   // the zeroing (null stream) lands before the rank's streams use them
    return TSLAM_OK;
}

// The state-gather buffers (allocated when the gather is first needed): a sender's payload slot
// holds its largest payload (a full batch); rank 0 keeps one slot per rank.
static int setup_gather(tslam_shard_driver* d) {
    if (!d->gather() || d->state_cap) return TSLAM_OK;
    size_t cap = 0;
    for (int q = 0; q < d->world; ++q)
        cap = std::max(cap, (size_t)tslam_internal_state_bytes(d->ranks[0].h, d->B, q, q * d->S, (q + 1) * d->S));
    d->state_cap = (cap + 255) / 256 * 256;
    for (Rank& r : d->ranks) {
        SHCHK(hipSetDevice(r.device));
        for (int k = 0; k < 2; ++k) RC(alloc(r, &r.state_buf[k], (r.rank == 0 ? d->world : 1) * d->state_cap));
        SHCHK(hipDeviceSynchronize());
    }
    return TSLAM_OK;
}

// The pair split's pair-block buffers (allocated when first needed): a slot per rank of the rig
// range it owns (peer_records(max_batch, world) frames), sent to / received from the ranks of the
// same half.  The stereo receive buffers need no change: world slots of peer_cap frames hold the
// partner's half (max_batch / 2 + 1 frames) from offset 0.
static int setup_pairs(tslam_shard_driver* d) {
    if (!d->pairs() || d->pb_ready) return TSLAM_OK;
    const size_t bytes = (size_t)d->world * peer_records(d->B, d->world) * d->pblk;
    for (Rank& r : d->ranks) {
        SHCHK(hipSetDevice(r.device));
        for (int k = 0; k < 2; ++k) {
            RC(alloc(r, &r.pb_send[k], bytes));
            RC(alloc(r, &r.pb_recv[k], bytes));
        }
        SHCHK(hipDeviceSynchronize());
    }
    d->pb_ready = true;
    return TSLAM_OK;
}
// pair split: rank q's rig range (rig pose + pose records), inside its pair's half
static void rig_range(const tslam_shard_driver* d, int q, int* lo, int* hi) {
    peer_range(rig_slot(q, d->world, 1), d->n, d->world, lo, hi);
}
static size_t pb_slot(const tslam_shard_driver* d) { return (size_t)peer_records(d->B, d->world) * d->pblk; }
// does rank src send rank dst pair blocks (pair split: the other ranks of the same half)
static bool pair_peer(const tslam_shard_driver* d, int src, int dst) { return src != dst && ((src ^ dst) & 1) == 0; }
static size_t pb_bytes(const tslam_shard_driver* d, int dst) {   // one pair's blocks of dst's rig range
    int lo, hi;
    rig_range(d, dst, &lo, &hi);
    return (size_t)(hi - lo) * d->pblk;
}

// ---- profiling (TSLAM_SHARD_PROFILE) ------------------------------------------------------------
static int span_begin(tslam_shard_driver* d, Rank& r, int seg, hipStream_t s) {
    if (!(d->flags & TSLAM_SHARD_PROFILE)) return TSLAM_OK;
    SHCHK(hipSetDevice(r.device));
    while (r.ev_pool.size() < r.ev_used + 2) {
        hipEvent_t e;
        SHCHK(hipEventCreate(&e));
        r.ev_pool.push_back(e);
    }
    Span sp{seg, r.ev_pool[r.ev_used], r.ev_pool[r.ev_used + 1]};
    r.ev_used += 2;
    SHCHK(hipEventRecord(sp.a, s));
    r.spans.push_back(sp);
    return TSLAM_OK;
}
static int span_end(tslam_shard_driver* d, Rank& r, hipStream_t s) {
    if (!(d->flags & TSLAM_SHARD_PROFILE)) return TSLAM_OK;
    SHCHK(hipEventRecord(r.spans.back().b, s));
    return TSLAM_OK;
}
// the span between an event already recorded on one stream and now on another
static int span_between(tslam_shard_driver* d, Rank& r, int seg, hipStream_t from, hipStream_t to) {
    RC(span_begin(d, r, seg, from));
    return span_end(d, r, to);
}
static int run_timed(tslam_shard_driver* d, Rank& r, int seg, int stage, hipStream_t s) {
    RC(span_begin(d, r, seg, s));
    RC(tslam_run_stage(r.h, stage, s));
    return span_end(d, r, s);
}

// ---- exchanges ----------------------------------------------------------------------------------
// The stream an exchange runs on (sender and receiver side): stereo raw images and stream blocks
// on the exchange stream, pair blocks, state blocks and pose records on the back stream.
static hipStream_t xstream(const tslam_shard_driver* d, const Rank& r, Which w) {
    return (w == POSE || w == STATE || w == PAIRB || d->rgbd) ? BS(d, r) : XS(d, r);
}

// The pieces rank `src` sends rank `dst` for exchange w (at most two: a raw image slot of peer 0
// starts with the previous batch's last frame), as (source pointer, destination offset, bytes).
struct Piece {
    const uint8_t* p;
    size_t off, bytes;
};
static int pieces(const tslam_shard_driver* d, const Rank& src, int dst, Which w, int k, const uint8_t* images,
                  Piece* out) {
    if (w == RAW) {
        const size_t frame = (size_t)d->S * d->img, total = raw_bytes(d, dst);
        if (total == 0) return 0;
        int lo, hi;
        back_range(d, dst, &lo, &hi);
        if (lo > 0) {   // frames lo-1 .. hi-1 are contiguous in the input
            out[0] = {images + (size_t)(lo - 1) * frame, 0, total};
            return 1;
        }
        out[0] = {src.prev_raw, 0, frame};   // frame -1: the previous batch's last frame
        out[1] = {images, frame, total - frame};
        return 2;
    }
    if (w == FEAT) {
        const size_t b = feat_bytes(d, dst);
        if (b == 0) return 0;
        out[0] = {src.feat_send[k] + (d->pairs() ? 0 : (size_t)dst * feat_cap(d)), 0, b};   // pair split: one slot
        return 1;
    }
    if (w == PAIRB) {
        const size_t b = pb_bytes(d, dst);
        if (b == 0) return 0;
        out[0] = {src.pb_send[k] + (size_t)dst * pb_slot(d), 0, b};
        return 1;
    }
    return 0;
}

static int exchange(tslam_shard_driver* d, Which w, int k, const uint8_t* const* images) {
    const int N = d->world;
    if (w == STATE && !d->gather()) return TSLAM_OK;
    const bool pairs = d->pairs();
    auto recv_buf = [&](Rank& r, int src) -> uint8_t* {   // where src's data lands in r's buffers
        if (w == RAW) return r.raw_recv[k] + (pairs ? 0 : (size_t)src * raw_cap(d));   // pair split: the partner's
        if (w == FEAT) return r.feat_recv[k] + (pairs ? 0 : (size_t)src * feat_cap(d));
        if (w == PAIRB) return r.pb_recv[k] + (size_t)src * pb_slot(d);
        return r.state_buf[k] + (size_t)src * d->state_cap;
    };
    auto recv_bytes = [&](const Rank& r, int src) -> size_t {   // what r receives from src
        if (w == RAW) return raw_bytes(d, r.rank);
        if (w == FEAT) return feat_bytes(d, r.rank);
        if (w == PAIRB) return pb_bytes(d, r.rank);
        return (size_t)tslam_internal_state_bytes(r.h, d->n, src, src * d->S, (src + 1) * d->S);
    };
    // the (src, dst) pairs exchange w connects
    auto linked = [&](int src, int dst) -> bool {
        if (w == PAIRB) return pair_peer(d, src, dst);
        if (w == RAW || (w == FEAT && !d->rgbd)) return stereo_peer(d, src, dst);
        return src != dst;
    };
    if (d->transport == TSLAM_TRANSPORT_RCCL) {
        NCCLCHK(ncclGroupStart());
        for (size_t i = 0; i < d->ranks.size(); ++i) {
            Rank& r = d->ranks[i];
            hipStream_t s = xstream(d, r, w);
            if (w == POSE) {
                NCCLCHK(ncclAllGather(r.pose_send[k], r.pose_recv[k], (size_t)d->maxr * d->rec, ncclUint8, r.comm_p, s));
                continue;
            }
            if (w == STATE) {   // every rank to rank 0
                if (r.rank != 0) {
                    const size_t b = recv_bytes(d->ranks[i], r.rank);
                    if (b) NCCLCHK(ncclSend(r.state_buf[k], b, ncclUint8, 0, r.comm_p, s));
                } else {
                    for (int q = 1; q < N; ++q) {
                        const size_t b = recv_bytes(r, q);
                        if (b) NCCLCHK(ncclRecv(recv_buf(r, q), b, ncclUint8, q, r.comm_p, s));
                    }
                }
                continue;
            }
            ncclComm_t comm = w == PAIRB ? r.comm_p : r.comm_x;   // PAIRB: the back stream's communicator
            for (int q = 0; q < N; ++q) {
                if (!linked(r.rank, q)) continue;
                Piece pc[2];
                const int np = pieces(d, r, q, w, k, images ? images[i] : nullptr, pc);
                for (int j = 0; j < np; ++j) NCCLCHK(ncclSend(pc[j].p, pc[j].bytes, ncclUint8, q, comm, s));
                // what q sends me, in the same pieces (q's view of my range)
                const size_t b = recv_bytes(r, q);
                if (b == 0) continue;
                int lo, hi;
                back_range(d, r.rank, &lo, &hi);
                if (w == RAW && lo == 0) {
                    const size_t frame = (size_t)d->S * d->img;
                    NCCLCHK(ncclRecv(recv_buf(r, q), frame, ncclUint8, q, comm, s));
                    NCCLCHK(ncclRecv(recv_buf(r, q) + frame, b - frame, ncclUint8, q, comm, s));
                } else {
                    NCCLCHK(ncclRecv(recv_buf(r, q), b, ncclUint8, q, comm, s));
                }
            }
        }
        NCCLCHK(ncclGroupEnd());
        return TSLAM_OK;
    }
    // COPY: each sender pushes into its peers' receive buffers on its own exchange-side stream,
    // once the peer has consumed the previous use of that parity; the receivers wait for every push
    for (size_t i = 0; i < d->ranks.size(); ++i) {
        Rank& src = d->ranks[i];
        SHCHK(hipSetDevice(src.device));
        hipStream_t s = xstream(d, src, w);
        for (Rank& dst : d->ranks) {
            if (w == POSE) {
                if (dst.done_armed && &dst != &src) SHCHK(hipStreamWaitEvent(s, dst.ev_done, 0));
                SHCHK(hipMemcpyAsync(dst.pose_recv[k] + (size_t)src.rank * d->maxr * d->rec, src.pose_send[k],
                                     (size_t)d->maxr * d->rec, hipMemcpyDeviceToDevice, s));
                continue;
            }
            if (&dst == &src) continue;
            if (w == STATE) {
                if (dst.rank != 0) continue;
                if (dst.done_armed) SHCHK(hipStreamWaitEvent(s, dst.ev_done, 0));   // rank 0 unpacked batch s-2
                const size_t b = recv_bytes(dst, src.rank);
                if (b) SHCHK(hipMemcpyAsync(recv_buf(dst, src.rank), src.state_buf[k], b, hipMemcpyDeviceToDevice, s));
                continue;
            }
            if (!linked(src.rank, dst.rank)) continue;
            if (w == PAIRB) {   // dst's back stream unpacked this parity's blocks (batch s-2) before its batch s-1 ended
                if (dst.done_armed) SHCHK(hipStreamWaitEvent(s, dst.ev_done, 0));
                Piece pc[2];
                if (pieces(d, src, dst.rank, w, k, nullptr, pc))
                    SHCHK(hipMemcpyAsync(recv_buf(dst, src.rank), pc[0].p, pc[0].bytes, hipMemcpyDeviceToDevice, s));
                continue;
            }
            if (dst.consumed_armed[k]) SHCHK(hipStreamWaitEvent(s, dst.consumed[k], 0));
            Piece pc[2];
            const int np = pieces(d, src, dst.rank, w, k, images ? images[i] : nullptr, pc);
            for (int j = 0; j < np; ++j)
                SHCHK(hipMemcpyAsync(recv_buf(dst, src.rank) + pc[j].off, pc[j].p, pc[j].bytes, hipMemcpyDeviceToDevice, s));
        }
        SHCHK(hipEventRecord(src.ev_push, s));
    }
    for (Rank& dst : d->ranks) {
        if (w == STATE && dst.rank != 0) continue;
        SHCHK(hipSetDevice(dst.device));
        hipStream_t s = xstream(d, dst, w);
        for (Rank& src : d->ranks)
            if (&src != &dst) SHCHK(hipStreamWaitEvent(s, src.ev_push, 0));
    }
    return TSLAM_OK;
}

static int submit(tslam_shard_driver* d, const uint8_t* const* images, int n, void* const* streams) {
    if (n < 1 || n > d->B) return tslam_internal_fail(TSLAM_EINVAL, "a sharded batch needs 1 <= n_frames <= max_batch");
    RC(setup_gather(d));
    RC(setup_pairs(d));
    d->n = n;
    d->maxr = peer_records(n, d->world);
    const int k = (int)(d->batches & 1), N = d->world, S = d->S;
    const bool prof = (d->flags & TSLAM_SHARD_PROFILE) != 0;
    // TSLAM_SHARD_SOLO: rank 0's work only, no exchange (the receive buffers keep what the last
    // full batch left): rank 0's step on a GPU of its own with the exchange hidden
    const bool solo = (d->flags & TSLAM_SHARD_SOLO) != 0;
    const bool xchg = N > 1 && !solo;
    auto idle = [&](const Rank& r) { return solo && r.rank != 0; };
    for (size_t i = 0; i < d->ranks.size(); ++i) {   // inputs, buffer reuse
        Rank& r = d->ranks[i];
        if (idle(r)) continue;
        SHCHK(hipSetDevice(r.device));
        SHCHK(hipEventRecord(r.ev_in, streams ? (hipStream_t)streams[i] : nullptr));
        for (hipStream_t s : {FS(d, r), XS(d, r), BS(d, r)}) SHCHK(hipStreamWaitEvent(s, r.ev_in, 0));
        if (r.consumed_armed[k])
            for (hipStream_t s : {FS(d, r), XS(d, r)}) SHCHK(hipStreamWaitEvent(s, r.consumed[k], 0));
        RC(tslam_begin_batch(r.h, images[i], n));
    }
    if (!d->rgbd && xchg) RC(exchange(d, RAW, k, images));   // straight from the inputs
    for (size_t i = 0; i < d->ranks.size(); ++i) {   // this batch's last frame becomes prev_raw (after the sends)
        Rank& r = d->ranks[i];
        if (d->rgbd || idle(r)) continue;
        SHCHK(hipSetDevice(r.device));
        const size_t frame = (size_t)S * d->img;
        SHCHK(hipMemcpyAsync(r.prev_raw, images[i] + (size_t)(n - 1) * frame, frame, hipMemcpyDeviceToDevice, XS(d, r)));
    }
    for (Rank& r : d->ranks) {   // front end of the rank's cameras (+ its stream blocks per peer)
        if (idle(r)) continue;
        if (prof) {
            RC(run_timed(d, r, TSLAM_SEG_RECTIFY, TSLAM_KERNEL_RECTIFY_PYRAMID, FS(d, r)));
            RC(run_timed(d, r, TSLAM_SEG_DETECT, TSLAM_KERNEL_DETECT, FS(d, r)));
            RC(run_timed(d, r, TSLAM_SEG_SELECT, TSLAM_KERNEL_SELECT, FS(d, r)));
            RC(run_timed(d, r, TSLAM_SEG_DESCRIBE, TSLAM_KERNEL_DESCRIBE, FS(d, r)));
        } else {
            for (int st : {TSLAM_STAGE_RECTIFY, TSLAM_STAGE_DETECT, TSLAM_STAGE_DESCRIBE}) RC(tslam_run_stage(r.h, st, FS(d, r)));
        }
        if (d->rgbd) continue;
        if (N > 1) {
            RC(span_begin(d, r, TSLAM_SEG_PACK, FS(d, r)));
            if (d->pairs()) RC(tslam_internal_pack_partner(r.h, r.feat_send[k], FS(d, r)));   // the partner's half
            else RC(tslam_pack_streams_peers(r.h, r.feat_send[k], FS(d, r)));   // every peer's frames, one launch
            RC(span_end(d, r, FS(d, r)));
        }
        SHCHK(hipSetDevice(r.device));
        SHCHK(hipEventRecord(r.ev_front, FS(d, r)));
        SHCHK(hipStreamWaitEvent(XS(d, r), r.ev_front, 0));
    }
    if (!d->rgbd && xchg) RC(exchange(d, FEAT, k, images));
    for (Rank& r : d->ranks) {   // back end
        if (idle(r)) continue;
        if (!d->rgbd) {
            // the other cameras of frames lo-1 .. hi-1 of this rank's range into the ring
            SHCHK(hipSetDevice(r.device));
            SHCHK(hipEventRecord(r.ev_x, XS(d, r)));
            SHCHK(hipStreamWaitEvent(BS(d, r), r.ev_x, 0));
            if (prof && N > 1) RC(span_between(d, r, TSLAM_SEG_EXCHANGE_WAIT, FS(d, r), BS(d, r)));   // front done -> data landed
            if (N > 1) {
                RC(span_begin(d, r, TSLAM_SEG_IMPORT, BS(d, r)));
                if (d->pairs()) RC(tslam_internal_import_partner(r.h, r.raw_recv[k], r.feat_recv[k], BS(d, r)));
                else RC(tslam_import_peers(r.h, r.raw_recv[k], r.feat_recv[k], BS(d, r)));
                RC(span_end(d, r, BS(d, r)));
            }
            SHCHK(hipEventRecord(r.consumed[k], BS(d, r)));
            r.consumed_armed[k] = true;
        }
        if (prof) {
            RC(run_timed(d, r, TSLAM_SEG_MATCH, TSLAM_KERNEL_MATCH, BS(d, r)));
            RC(run_timed(d, r, TSLAM_SEG_MATCH_REFINE, TSLAM_KERNEL_MATCH_REFINE, BS(d, r)));
            RC(run_timed(d, r, TSLAM_SEG_POSE, TSLAM_KERNEL_POSE, BS(d, r)));
            if (d->rig && !d->rgbd && !d->pairs()) RC(run_timed(d, r, TSLAM_SEG_RIG, TSLAM_KERNEL_RIG, BS(d, r)));
        } else {
            RC(tslam_run_stage(r.h, TSLAM_STAGE_MATCH, BS(d, r)));
            RC(tslam_run_stage(r.h, TSLAM_STAGE_POSE, BS(d, r)));
        }
        if (d->rgbd)   // this rank's cameras over every peer's frame range
            for (int q = 0; q < N; ++q) {
                int lo, hi;
                peer_range(q, n, N, &lo, &hi);
                if (q != r.rank && hi > lo)
                    RC(tslam_pack_pairs(r.h, lo, hi - lo, r.rank * S, (r.rank + 1) * S, r.feat_send[k] + (size_t)q * feat_cap(d),
                                        BS(d, r)));
            }
    }
    if (d->rgbd) {
        if (xchg) RC(exchange(d, FEAT, k, images));
        for (Rank& r : d->ranks) {
            if (idle(r)) continue;
            int lo, hi;
            peer_range(r.rank, n, N, &lo, &hi);
            for (int q = 0; q < N; ++q)
                if (q != r.rank && hi > lo)
                    RC(tslam_unpack_pairs(r.h, lo, hi - lo, q * S, (q + 1) * S, r.feat_recv[k] + (size_t)q * feat_cap(d), BS(d, r)));
            SHCHK(hipSetDevice(r.device));
            SHCHK(hipEventRecord(r.consumed[k], BS(d, r)));
            r.consumed_armed[k] = true;
            if (d->rig) RC(run_timed(d, r, TSLAM_SEG_RIG, TSLAM_KERNEL_RIG, BS(d, r)));
        }
    }
    if (d->pairs()) {   // every pair's blocks of a rank's rig range from the ranks of its half, then the rig pose
        const size_t slot = pb_slot(d);
        if (d->P > 1) {
            for (Rank& r : d->ranks) {
                if (idle(r)) continue;
                RC(span_begin(d, r, TSLAM_SEG_PAIR_BLOCKS, BS(d, r)));
                for (int q = 0; q < N; ++q) {
                    int lo, hi;
                    rig_range(d, q, &lo, &hi);
                    if (pair_peer(d, r.rank, q) && hi > lo)
                        RC(tslam_pack_pairs(r.h, lo, hi - lo, r.rank / 2, r.rank / 2 + 1, r.pb_send[k] + (size_t)q * slot, BS(d, r)));
                }
            }
            if (!solo) RC(exchange(d, PAIRB, k, images));
            for (Rank& r : d->ranks) {
                if (idle(r)) continue;
                int lo, hi;
                rig_range(d, r.rank, &lo, &hi);
                for (int q = 0; q < N; ++q)
                    if (pair_peer(d, q, r.rank) && hi > lo)
                        RC(tslam_unpack_pairs(r.h, lo, hi - lo, q / 2, q / 2 + 1, r.pb_recv[k] + (size_t)q * slot, BS(d, r)));
                RC(span_end(d, r, BS(d, r)));
            }
        }
        if (d->rig)
            for (Rank& r : d->ranks)
                if (!idle(r)) RC(run_timed(d, r, TSLAM_SEG_RIG, TSLAM_KERNEL_RIG, BS(d, r)));
    }
    if (d->gather()) {   // every rank's share of the pairs' state into rank 0's ring
        for (Rank& r : d->ranks) {
            if (r.rank == 0 || idle(r)) continue;
            RC(span_begin(d, r, TSLAM_SEG_STATE, BS(d, r)));
            RC(tslam_internal_state_blocks(r.h, 1, r.rank, r.rank * S, (r.rank + 1) * S, r.state_buf[k], BS(d, r)));
            RC(span_end(d, r, BS(d, r)));
        }
        if (!solo) RC(exchange(d, STATE, k, images));
        for (Rank& r : d->ranks) {
            if (r.rank != 0) continue;
            RC(span_begin(d, r, TSLAM_SEG_STATE, BS(d, r)));
            for (int q = 1; q < N; ++q)
                RC(tslam_internal_state_blocks(r.h, 0, q, q * S, (q + 1) * S, r.state_buf[k] + (size_t)q * d->state_cap, BS(d, r)));
            RC(span_end(d, r, BS(d, r)));
        }
    }
    for (Rank& r : d->ranks) {
        if (idle(r)) continue;
        RC(tslam_pack_poses(r.h, r.pose_send[k], BS(d, r)));
        RC(span_begin(d, r, TSLAM_SEG_POSE_GATHER, BS(d, r)));
    }
    if (!solo) RC(exchange(d, POSE, k, images));
    for (size_t i = 0; i < d->ranks.size(); ++i) {
        Rank& r = d->ranks[i];
        if (idle(r)) continue;
        RC(span_end(d, r, BS(d, r)));
        RC(tslam_unpack_poses(r.h, r.pose_recv[k], BS(d, r)));
        RC(run_timed(d, r, TSLAM_SEG_CHAIN, TSLAM_KERNEL_CHAIN, BS(d, r)));
        // local BA on rank 0 once its ring holds every pair (the back stream keeps it ordered before
        // the next batch's imports; tslam_run_stage orders it after the next-but-one front end)
        if (d->ba && (r.rank == 0 || N == 1) && (d->gather() || N == 1))
            RC(run_timed(d, r, TSLAM_SEG_BA, TSLAM_STAGE_BA, BS(d, r)));
        if (d->flags & TSLAM_SHARD_RESULTS) RC(tslam_internal_stash(r.h, BS(d, r)));
        RC(tslam_end_batch(r.h));
        SHCHK(hipSetDevice(r.device));
        SHCHK(hipEventRecord(r.ev_done, BS(d, r)));
        r.done_armed = true;
        // the caller's stream orders after the batch (results in stream order), or with
        // TSLAM_SHARD_PIPELINE after the batch's last read of its input and receive buffers, so
        // that the next batch's front end overlaps this batch's back end
        SHCHK(hipStreamWaitEvent(streams ? (hipStream_t)streams[i] : nullptr,
                                 (d->flags & TSLAM_SHARD_PIPELINE) ? r.consumed[k] : r.ev_done, 0));
        if (prof) r.timed_batches += 1;
    }
    d->batches += 1;
    return TSLAM_OK;
}

// Sum the finished spans into the per-segment totals (synchronises the rank's device).
static int collect(Rank& r) {
    if (r.spans.empty()) return TSLAM_OK;
    SHCHK(hipSetDevice(r.device));
    SHCHK(hipDeviceSynchronize());
    for (const Span& sp : r.spans) {
        float ms = 0.0f;
        SHCHK(hipEventElapsedTime(&ms, sp.a, sp.b));
        r.seg_us[sp.seg] += 1e3 * (double)ms;
    }
    r.spans.clear();
    r.ev_used = 0;
    return TSLAM_OK;
}

static Rank* rank_of(tslam_shard_driver* d, tslam_handle* h) {
    for (Rank& r : d->ranks)
        if (r.h == h) return &r;
    return nullptr;
}

extern "C" {

int tslam_comm_unique_id(void* id128) {
    if (!id128) return tslam_internal_fail(TSLAM_EINVAL, "null id");
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    ncclUniqueId id;
    NCCLCHK(ncclGetUniqueId(&id));
    memcpy(id128, &id, sizeof(id));
    return TSLAM_OK;
}

int tslam_comm_init(tslam_handle* h, const void* id128, int rank, int world) {
    if (!h || !id128) return tslam_internal_fail(TSLAM_EINVAL, "bad argument");
    if (tslam_internal_driver(h)) return tslam_internal_fail(TSLAM_ESTATE, "communicator already set");
    if (world < 1 || rank < 0 || rank >= world) return tslam_internal_fail(TSLAM_EINVAL, "need 0 <= rank < world");
    auto* d = new tslam_shard_driver();
    int rc = plan(d, h, world);
    if (rc == TSLAM_OK) rc = tslam_set_shard(h, rank * d->S, (rank + 1) * d->S, rank, world);
    if (rc != TSLAM_OK) {
        delete d;
        return rc;
    }
    d->transport = TSLAM_TRANSPORT_RCCL;
    d->ranks.resize(1);
    Rank& r = d->ranks[0];
    r.h = h;
    r.rank = rank;
    rc = setup_rank(d, r);
    if (rc == TSLAM_OK) {
        ncclUniqueId id;
        memcpy(&id, id128, sizeof(id));
        ncclResult_t nr = ncclCommInitRank(&r.comm_x, world, id, rank);
        // the pose all-gather's (and the state gather's) own communicator (same ranks)
        if (nr == ncclSuccess) nr = ncclCommSplit(r.comm_x, 0, rank, &r.comm_p, nullptr);
        if (nr != ncclSuccess) rc = tslam_internal_fail(TSLAM_EHIP, (std::string("RCCL communicator: ") + ncclGetErrorString(nr)).c_str());
    }
    if (rc == TSLAM_OK) rc = tslam_internal_attach_driver(h, d, true);
    if (rc != TSLAM_OK) {
        (void)tslam_set_shard(h, 0, (int)(d->S * world), 0, 1);
        destroy_driver(d);
    }
    return rc;
}

int tslam_submit_sharded(tslam_handle* h, const uint8_t* images, int n_frames, void* stream) {
    if (!h || !images) return tslam_internal_fail(TSLAM_EINVAL, "bad argument");
    tslam_shard_driver* d = tslam_internal_driver(h);
    if (!d || d->ranks.size() != 1) return tslam_internal_fail(TSLAM_ESTATE, "tslam_comm_init first");
    void* streams[1] = {stream};
    return submit(d, &images, n_frames, streams);
}

int tslam_shard_options(tslam_handle* h, int flags) {
    if (!h) return tslam_internal_fail(TSLAM_EINVAL, "null handle");
    tslam_shard_driver* d = tslam_internal_driver(h);
    if (!d) return tslam_internal_fail(TSLAM_ESTATE, "the handle is not driven (tslam_comm_init / tslam_group_create)");
    if (flags & ~(TSLAM_SHARD_GATHER | TSLAM_SHARD_RESULTS | TSLAM_SHARD_PROFILE | TSLAM_SHARD_SERIAL |
                  TSLAM_SHARD_PIPELINE | TSLAM_SHARD_SOLO | TSLAM_SHARD_PAIRS))
        return tslam_internal_fail(TSLAM_EINVAL, "unknown TSLAM_SHARD_* flag");
    if ((flags & TSLAM_SHARD_SOLO) && (int)d->ranks.size() != d->world)
        return tslam_internal_fail(TSLAM_EINVAL, "TSLAM_SHARD_SOLO needs every rank in this process (tslam_group_create)");
    if ((flags & TSLAM_SHARD_GATHER) && d->rgbd)
        return tslam_internal_fail(TSLAM_EINVAL, "the state gather describes a stereo rig");
    if ((flags & TSLAM_SHARD_PAIRS) && (d->rgbd || d->S != 1 || d->world < 2))
        return tslam_internal_fail(TSLAM_EINVAL, "the pair split shards a stereo rig with one camera per rank");
    if ((flags & TSLAM_SHARD_PAIRS) && (d->ba || (flags & TSLAM_SHARD_GATHER)))
        return tslam_internal_fail(TSLAM_EINVAL, "the pair split runs without the state gather (no local BA)");
    // the streams may change (TSLAM_SHARD_SERIAL): everything enqueued so far finishes first
    for (Rank& r : d->ranks) {
        SHCHK(hipSetDevice(r.device));
        SHCHK(hipDeviceSynchronize());
    }
    if (flags & TSLAM_SHARD_SERIAL)
        for (size_t i = 0; i < d->ranks.size(); ++i) {
            Rank& r = d->ranks[i];
            if (r.serial) continue;
            for (size_t j = 0; j < i && !r.serial; ++j)
                if (d->ranks[j].device == r.device) r.serial = d->ranks[j].serial;
            if (!r.serial) {
                SHCHK(hipSetDevice(r.device));
                SHCHK(hipStreamCreateWithFlags(&r.serial, hipStreamNonBlocking));
                r.serial_owner = true;
            }
        }
    for (Rank& r : d->ranks) RC(tslam_internal_set_pairs(r.h, (flags & TSLAM_SHARD_PAIRS) ? 1 : 0));
    d->flags = flags;
    return TSLAM_OK;
}

int tslam_shard_timing(tslam_handle* h, double* out_us, int n_out) {
    if (!h || !out_us || n_out < 1) return tslam_internal_fail(TSLAM_EINVAL, "bad argument");
    tslam_shard_driver* d = tslam_internal_driver(h);
    Rank* r = d ? rank_of(d, h) : nullptr;
    if (!r) return tslam_internal_fail(TSLAM_ESTATE, "the handle is not driven (tslam_comm_init / tslam_group_create)");
    RC(collect(*r));
    const int64_t nb = r->timed_batches;
    for (int i = 0; i < std::min(n_out, (int)TSLAM_SEG_COUNT); ++i) out_us[i] = nb ? r->seg_us[i] / (double)nb : 0.0;
    for (double& v : r->seg_us) v = 0.0;
    r->timed_batches = 0;
    return (int)nb;
}

struct tslam_group {
    tslam_shard_driver* d = nullptr;
};

int tslam_group_create(tslam_handle* const* handles, int n, int transport, tslam_group** out) {
    if (!handles || n < 1 || !out) return tslam_internal_fail(TSLAM_EINVAL, "bad argument");
    if (transport != TSLAM_TRANSPORT_RCCL && transport != TSLAM_TRANSPORT_COPY)
        return tslam_internal_fail(TSLAM_EINVAL, "transport must be TSLAM_TRANSPORT_RCCL or TSLAM_TRANSPORT_COPY");
    tslam_handle_info in0{};
    RC(tslam_internal_info(handles[0], &in0));
    std::vector<int> devs(n);
    for (int i = 0; i < n; ++i) {
        tslam_handle_info in{};
        if (!handles[i]) return tslam_internal_fail(TSLAM_EINVAL, "null handle");
        RC(tslam_internal_info(handles[i], &in));
        if (in.C != in0.C || in.P != in0.P || in.B != in0.B || in.W != in0.W || in.H != in0.H || in.rgbd != in0.rgbd ||
            in.rig != in0.rig || in.ba != in0.ba)
            return tslam_internal_fail(TSLAM_EINVAL, "a group's handles must describe the same rig and batch");
        if (tslam_internal_driver(handles[i])) return tslam_internal_fail(TSLAM_ESTATE, "handle already driven");
        devs[i] = in.device;
        for (int j = 0; j < i; ++j)
            if (transport == TSLAM_TRANSPORT_RCCL && devs[j] == devs[i])
                return tslam_internal_fail(TSLAM_EINVAL, "an RCCL group needs one device per handle (COPY allows sharing)");
    }
    auto* d = new tslam_shard_driver();
    int rc = plan(d, handles[0], n);
    d->transport = transport;
    d->ranks.resize(n);
    for (int i = 0; i < n && rc == TSLAM_OK; ++i) {
        d->ranks[i].h = handles[i];
        d->ranks[i].rank = i;
        rc = tslam_set_shard(handles[i], i * d->S, (i + 1) * d->S, i, n);
        if (rc == TSLAM_OK) rc = setup_rank(d, d->ranks[i]);
    }
    if (rc == TSLAM_OK && transport == TSLAM_TRANSPORT_RCCL) {
        std::vector<ncclComm_t> cx(n), cp(n);
        ncclResult_t nr = ncclCommInitAll(cx.data(), n, devs.data());
        if (nr == ncclSuccess) nr = ncclCommInitAll(cp.data(), n, devs.data());
        if (nr != ncclSuccess) {
            rc = tslam_internal_fail(TSLAM_EHIP, (std::string("ncclCommInitAll: ") + ncclGetErrorString(nr)).c_str());
        } else {
            for (int i = 0; i < n; ++i) {
                d->ranks[i].comm_x = cx[i];
                d->ranks[i].comm_p = cp[i];
            }
        }
    }
    for (int i = 0; i < n && rc == TSLAM_OK; ++i) rc = tslam_internal_attach_driver(handles[i], d, false);
    if (rc != TSLAM_OK) {
        for (int i = 0; i < n; ++i) {
            (void)tslam_internal_attach_driver(handles[i], nullptr, false);
            (void)tslam_set_shard(handles[i], 0, in0.C, 0, 1);
        }
        destroy_driver(d);
        return rc;
    }
    *out = new tslam_group{d};
    return TSLAM_OK;
}

int tslam_group_submit(tslam_group* g, const uint8_t* const* images, int n_frames, void* const* streams) {
    if (!g || !g->d || !images) return tslam_internal_fail(TSLAM_EINVAL, "bad argument");
    for (size_t i = 0; i < g->d->ranks.size(); ++i)
        if (!images[i]) return tslam_internal_fail(TSLAM_EINVAL, "null images");
    return submit(g->d, images, n_frames, streams);
}

int tslam_group_destroy(tslam_group* g) {
    if (!g) return TSLAM_OK;
    if (g->d) {
        const int C = g->d->S * g->d->world;
        for (Rank& r : g->d->ranks) {
            (void)tslam_internal_attach_driver(r.h, nullptr, false);
            (void)tslam_set_shard(r.h, 0, C, 0, 1);
        }
        destroy_driver(g->d);
    }
    delete g;
    return TSLAM_OK;
}

}  // extern "C"
